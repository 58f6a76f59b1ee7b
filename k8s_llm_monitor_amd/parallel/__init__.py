"""One-process-per-GPU parallelism over torch.distributed (RCCL on MI355X, gloo on CPU)."""
from .comm import shard_range, tp_all_gather_last, tp_all_reduce, tp_broadcast_object  # noqa: F401
from .state import ParallelState, get_state, init_parallel, set_state  # noqa: F401
