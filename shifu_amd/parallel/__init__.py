"""Distributed runtime (RCCL over xGMI; gloo on CPU for tests)."""
from .dist import (DistInfo, info, init_from_env, shutdown, barrier, all_reduce_, broadcast_,
                   all_gather_cat, BucketedAllReducer, DEFAULT_BUCKET_BYTES, set_info)

__all__ = ["DistInfo", "info", "init_from_env", "shutdown", "barrier", "all_reduce_",
           "broadcast_", "all_gather_cat", "BucketedAllReducer", "DEFAULT_BUCKET_BYTES",
           "set_info"]
