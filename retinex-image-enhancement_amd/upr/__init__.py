"""upr — MI355X (gfx950) runtime of the UP-Retinex hot path.

The C ABI (include/upr.h, lib/libupr.so) holds every kernel and the forward
executor; this package binds it with ctypes and hands it torch-allocated
device buffers and the current HIP stream.
"""
from ._lib import LIB_PATH, UprError, lib  # noqa: F401
from . import runtime  # noqa: F401
