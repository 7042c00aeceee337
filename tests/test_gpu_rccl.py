"""T3 on one GPU: the framework's own RCCL communicator (csrc/runtime/rccl_comm.cpp) at world 1.

Multi-rank RCCL needs one GPU per rank (8-GPU runs belong to the round-end driver); here the
communicator is bootstrapped, and all-reduce / broadcast are checked at the DDP message sizes of
SURVEY.md §2.5 (1 element, the 75,264-B conv bucket, the 4,724,264-B fc bucket) in fp32 and bf16.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("numel", [1, 18816, 1181066])
def test_rccl_allreduce_and_broadcast_world1(cuda_device, dtype, numel):
    from pytorch_mnist_ddp_amd.ops import native
    C = native.load()
    assert C.RcclComm.available()
    comm = C.RcclComm(C.RcclComm.unique_id(), 1, 0, 0)
    assert comm.world_size == 1 and comm.rank == 0
    g = torch.Generator(device="cpu").manual_seed(numel)
    x = torch.randn(numel + 64, generator=g).to(dtype).to(cuda_device)
    ref = x.clone()
    s = torch.cuda.current_stream().cuda_stream
    code = 1 if dtype == torch.bfloat16 else 0
    comm.allreduce_sum(x.data_ptr(), numel, code, s)          # world 1: sum == identity
    comm.broadcast(x.data_ptr(), numel, code, 0, s)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)                                 # and the 64 guard elements untouched
