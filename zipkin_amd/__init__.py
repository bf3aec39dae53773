"""zipkin_amd — MI355X-native zipkin-aggregate dependency path.

The compute lives in libzkagg.so (HIP, gfx950) behind the C ABI of include/zkagg.h; this package
binds it (ctypes) and mirrors the reference's Aggregates store surface for the host side.
"""
from ._abi import ZkError, ZkLibraryError  # noqa: F401
from .columns import BYTES_PER_RECORD, DeviceColumns, SpanColumns, tracegen_host, tracegen_params  # noqa: F401
from .context import DepsContext, LinkTable  # noqa: F401
from . import table  # noqa: F401

__all__ = [
    "ZkError",
    "ZkLibraryError",
    "SpanColumns",
    "DeviceColumns",
    "tracegen_host",
    "tracegen_params",
    "DepsContext",
    "LinkTable",
    "BYTES_PER_RECORD",
]
