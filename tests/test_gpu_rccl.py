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


def test_pending_rccl_init_never_on_the_setup_path(gpu_box, tmp_path):
    """``bench.py --force-comm`` at world 1 under a launcher that does not say every rank is local (no
    LOCAL_WORLD_SIZE: RCCL's non-blocking init starts at once, as across nodes) with that init held
    back 60 s (MNIST_AMD_FAULT=rccl_init_delay): ``--allreduce auto`` validates the xGMI transport,
    cancels the pending RCCL init and trains - no rccl_comm_wait phase, setup far below the delay,
    and the cancelled init does not hold up the exit."""
    import json
    import os
    import socket
    import subprocess
    import sys
    import time
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if not k.startswith(("TORCHELASTIC", "LOCAL_WORLD"))}
    env.update(PYTHONPATH=ROOT, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), MNIST_AMD_FAULT="rccl_init_delay:0:60")
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-comm", "--no-full-run",
                        "--steps", "20", "--warmup", "5"], capture_output=True, text=True, timeout=110,
                       cwd=tmp_path, env=env)
    wall = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads(r.stdout.strip().splitlines()[-1])
    c = j["config"]
    assert c["allreduce"] == "xgmi" and c["rccl_init"] == "cancelled", c
    assert c["transport_report"]["rccl"]["ok"] is None, c["transport_report"]
    assert not any(k.startswith("rccl_comm_wait") or k.startswith("trainer.rccl") for k in j["setup_phases_s"])
    assert sum(j["setup_phases_s"].values()) < 20.0 and wall < 60.0, (j["setup_phases_s"], wall)
