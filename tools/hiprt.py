"""Minimal ctypes access to the HIP runtime for device-pointer tests (no torch)."""
import ctypes

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
    return _hip


H2D, D2H = 1, 2


class DeviceBuffer:
    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.ptr = ctypes.c_void_p()
        rc = hip().hipMalloc(ctypes.byref(self.ptr), max(nbytes, 1))
        assert rc == 0, f"hipMalloc rc={rc}"

    @classmethod
    def from_array(cls, a: np.ndarray):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        assert hip().hipMemcpy(b.ptr, a.ctypes.data, a.nbytes, H2D) == 0
        return b

    def to_array(self, shape, dtype):
        out = np.empty(shape, dtype)
        assert hip().hipDeviceSynchronize() == 0
        assert hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H) == 0
        return out

    @property
    def addr(self) -> int:
        return self.ptr.value

    def free(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
