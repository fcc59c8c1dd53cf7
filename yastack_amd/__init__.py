"""yastack_amd — MI355X-native software-RSS engine for yastack / F-Stack.

The hot path (parse + Toeplitz hash + queue + per-queue FIFO lists) runs as
hand-written HIP kernels for gfx950 in ``_lib/libyrss.so``, behind the C ABI
of ``include/yrss.h``.  This package is the thin Python host side used by the
tests and ``bench.py``; C hosts (F-Stack itself) link the library directly
(see INTEGRATION.md).
"""
from . import abi
from .abi import YrssError, YrssLibraryError
from .dispatch import DispatchResult, FanOut, SoftRss
from .shard import merge_queue_lists, shard_range

__all__ = [
    "abi", "SoftRss", "FanOut", "DispatchResult", "YrssError", "YrssLibraryError",
    "shard_range", "merge_queue_lists",
]
