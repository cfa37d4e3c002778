from .comm import (barrier, tp_all_gather_last, tp_all_reduce, tp_all_to_all, tp_all_to_all_counts,
                   tp_broadcast_object, tp_broadcast_tensor)
from .state import ParallelState, destroy_parallel, get_state, init_parallel, set_state

__all__ = ["barrier", "tp_all_gather_last", "tp_all_reduce", "tp_all_to_all", "tp_all_to_all_counts",
           "tp_broadcast_object", "tp_broadcast_tensor", "ParallelState", "destroy_parallel", "get_state",
           "init_parallel", "set_state"]
