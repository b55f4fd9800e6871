"""Light HIP timing events for kernel timing inside a timed loop.

torch.cuda.Event records with a system-scope release fence (an L2 write-back + invalidate): bracketing every
step of a ~50 us kernel with two of them measured ~7 us of extra time per step on MI355X.  These events are
created with hipEventDisableSystemFence, the flag HIP documents for timing-only events, through the HIP
runtime torch already loaded (same libamdhip64.so.7)."""
from __future__ import annotations

import ctypes

import torch  # noqa: F401  (loads the HIP runtime)

hipEventDisableSystemFence = 0x20000000
_hip = None


def _rt():
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        h.hipEventSynchronize.argtypes = [ctypes.c_void_p]
        h.hipEventDestroy.argtypes = [ctypes.c_void_p]
        _hip = h
    return _hip


class Event:
    def __init__(self, fence: bool = False):
        self._e = ctypes.c_void_p()
        rc = _rt().hipEventCreateWithFlags(ctypes.byref(self._e), 0 if fence else hipEventDisableSystemFence)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags failed: {rc}")

    def record(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream()
        rc = _rt().hipEventRecord(self._e, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"hipEventRecord failed: {rc}")

    def elapsed_time(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _rt().hipEventSynchronize(end._e)
        rc = _rt().hipEventElapsedTime(ctypes.byref(ms), self._e, end._e)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime failed: {rc}")
        return ms.value

    def __del__(self):
        try:
            if self._e:
                _rt().hipEventDestroy(self._e)
        except Exception:
            pass
