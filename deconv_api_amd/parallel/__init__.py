from .dist import (DistInfo, all_gather_rows, all_reduce_max, barrier, broadcast_state, init, shard_counts,
                   shard_sizes, shutdown)

__all__ = ["DistInfo", "all_gather_rows", "all_reduce_max", "barrier", "broadcast_state", "init", "shard_counts",
           "shard_sizes", "shutdown"]
