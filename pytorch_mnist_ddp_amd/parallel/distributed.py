"""Process-group bootstrap: reference ``init_distributed_mode`` (mnist_ddp.py:13-37) + RCCL comm.

Rank discovery order and printed lines are the reference's:
  (a) ``RANK`` and ``WORLD_SIZE`` in the environment (torchrun / torch.distributed.launch)
      -> rank, world_size, gpu = ``LOCAL_RANK``;
  (b) ``SLURM_PROCID`` -> rank, gpu = rank % device_count, world_size from ``--world-size``;
  (c) an ``args.rank`` attribute set by the caller (unreachable from the reference CLI);
  (d) otherwise "Not using distributed mode".
Then ``set_device(gpu)``, print ``| distributed init (rank r): url, local rank:g, world size:w``
and ``init_process_group``.  The backend is ``"nccl"`` (= RCCL on ROCm) on GPU and ``"gloo"``
for ``--no-cuda`` runs (the reference hardcodes nccl, which cannot work without a GPU).

On top of that, :func:`create_rccl_comm` builds the framework's own RCCL communicator for the
native gradient all-reduce: rank 0 draws an ``ncclUniqueId`` and publishes it through the c10d
TCPStore that ``env://`` already created, every rank joins with ``ncclCommInitRank``.
"""
from __future__ import annotations

import os
from datetime import timedelta

import torch
import torch.distributed as dist


def init_distributed_mode(args) -> None:
    use_cuda = not getattr(args, "no_cuda", False) and torch.cuda.is_available()
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        args.rank = int(os.environ["RANK"])
        args.world_size = int(os.environ["WORLD_SIZE"])
        args.gpu = int(os.environ.get("LOCAL_RANK", "0"))
    elif "SLURM_PROCID" in os.environ:
        args.rank = int(os.environ["SLURM_PROCID"])
        ndev = torch.cuda.device_count() if use_cuda else 1
        args.gpu = args.rank % max(1, ndev)
    elif hasattr(args, "rank"):
        pass
    else:
        print("Not using distributed mode")
        args.distributed = False
        return

    args.distributed = True
    if use_cuda:
        torch.cuda.set_device(args.gpu)
        args.dist_backend = "nccl"
    else:
        args.dist_backend = "gloo"
    print(f"| distributed init (rank {args.rank}): {args.dist_url}, local rank:{args.gpu}, "
          f"world size:{args.world_size}", flush=True)
    kwargs = dict(backend=args.dist_backend, init_method=args.dist_url, world_size=args.world_size,
                  rank=args.rank, timeout=timedelta(minutes=10))
    if use_cuda:
        kwargs["device_id"] = torch.device("cuda", args.gpu)
    dist.init_process_group(**kwargs)


_UID_KEY = "pytorch_mnist_ddp_amd/rccl_unique_id"


def create_rccl_comm(world_size: int, rank: int, device: int, tag: str = "0"):
    """Framework-owned RCCL communicator (requires an initialised default process group)."""
    from ..ops import native
    C = native.load()
    if not C.RcclComm.available():
        raise RuntimeError("RCCL not found in this process")
    store = dist.distributed_c10d._get_default_store()
    key = f"{_UID_KEY}/{tag}"
    if rank == 0:
        uid = C.RcclComm.unique_id()
        store.set(key, uid)
    else:
        store.wait([key], timedelta(minutes=5))
        uid = store.get(key)
    return C.RcclComm(bytes(uid), world_size, rank, device)


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def create_rccl_comms(world_size: int, rank: int, device: int, n: int = 2):
    """``n`` independent framework communicators (the fused engine's DDP schedule 2 reduces the
    conv bucket on the first and the fc bucket on the second, concurrently)."""
    return [create_rccl_comm(world_size, rank, device, tag=str(i)) for i in range(n)]

