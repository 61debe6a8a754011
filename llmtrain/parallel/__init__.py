"""Data parallelism over RCCL/xGMI (GPU) or gloo (CPU)."""

from llmtrain.parallel.ddp import unwrap, wrap_data_parallel
from llmtrain.parallel.dist import DDPState, resolve_backend, setup_ddp, teardown_ddp
from llmtrain.parallel.reducer import FlatDataParallel, plan_buckets

__all__ = [
    "DDPState",
    "FlatDataParallel",
    "plan_buckets",
    "resolve_backend",
    "setup_ddp",
    "teardown_ddp",
    "unwrap",
    "wrap_data_parallel",
]
