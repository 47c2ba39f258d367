"""Distributed runtime: process-group API, launcher, DDP, sampler."""
from . import distributed
from .ddp import DistributedDataParallel
from .distributed import (ReduceOp, all_gather, all_gather_into_tensor, all_reduce, barrier, broadcast,
                          destroy_process_group, get_backend, get_rank, get_world_size, init_process_group,
                          is_initialized, new_group, reduce_scatter_tensor)
from .launch import (ProcessExitedException, ProcessRaisedException, env_rank_info, find_free_port, setup_rendezvous_env,
                     spawn)
from .sampler import DistributedSampler

__all__ = [
    "distributed", "DistributedDataParallel", "DistributedSampler", "ReduceOp", "all_gather", "all_gather_into_tensor",
    "all_reduce", "barrier", "broadcast", "destroy_process_group", "get_backend", "get_rank", "get_world_size",
    "init_process_group", "is_initialized", "new_group", "reduce_scatter_tensor", "spawn", "find_free_port",
    "setup_rendezvous_env", "env_rank_info", "ProcessRaisedException", "ProcessExitedException",
]
