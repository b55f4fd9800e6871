"""omr — MI355X-native OmniReduce sparse-block hot path (host-side mirror of the reference interface).

The compute path is libomr.so (HIP, gfx950) behind the C ABI in include/omr.h; this package only binds it
to torch-allocated device memory and HIP streams, and provides the multi-GPU exchange over RCCL.
"""
from .layout import Layout, MESSAGE_SIZE, NUM_SLOTS, NUM_THREADS  # noqa: F401
from . import _lib  # noqa: F401


def load():
    """Load libomr.so (raises if it is missing; there is no fallback)."""
    return _lib.load()
