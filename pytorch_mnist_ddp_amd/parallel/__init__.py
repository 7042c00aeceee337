from .ddp import BucketReducer, DistributedDataParallel, compute_bucket_assignment
from .distributed import barrier, create_rccl_comm, get_rank, get_world_size, init_distributed_mode

__all__ = ["BucketReducer", "DistributedDataParallel", "compute_bucket_assignment", "barrier",
           "create_rccl_comm", "get_rank", "get_world_size", "init_distributed_mode"]
