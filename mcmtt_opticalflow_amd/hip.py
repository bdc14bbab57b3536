"""The HIP runtime libpsn_lk.so is bound to, through ctypes: device selection,
device / pinned host memory, streams, events, copies.

The bench and the tests drive the library with these instead of torch.cuda, so
a process that runs the Tracker2D path initialises exactly one HIP runtime: the
one libpsn_lk.so resolved (ROCm's /opt/rocm/lib when the library loads first;
see psn_lk_runtime_info in include/psn_lk.h). torch stays plumbing for the
gloo control plane. The runtime is opened by its soname AFTER the library, so
the loader hands back the object the library already bound, never a second
copy.
"""
from __future__ import annotations

import ctypes
import re

import numpy as np

from . import _lib

_hip = None

H2D, D2H, D2D = 1, 2, 3
STREAM_NON_BLOCKING = 1
EVENT_DISABLE_TIMING = 2
HOST_MALLOC_COHERENT = 0x40000000


class HipError(RuntimeError):
    pass


def rt():
    """The HIP runtime libpsn_lk.so is bound to (ctypes.CDLL)."""
    global _hip
    if _hip is None:
        _lib.load()  # first: the soname below then resolves to the library's runtime
        h = ctypes.CDLL("libamdhip64.so.7")
        vp, sz, ip = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        h.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
        h.hipFree.argtypes = [vp]
        h.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
        h.hipHostFree.argtypes = [vp]
        h.hipMemcpy.argtypes = [vp, vp, sz, ip]
        h.hipMemcpyAsync.argtypes = [vp, vp, sz, ip, vp]
        h.hipMemset.argtypes = [vp, ip, sz]
        h.hipMemsetAsync.argtypes = [vp, ip, sz, vp]
        h.hipMemsetD32Async.argtypes = [vp, ip, sz, vp]
        h.hipDeviceSynchronize.argtypes = []
        h.hipSetDevice.argtypes = [ip]
        h.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        h.hipStreamDestroy.argtypes = [vp]
        h.hipStreamSynchronize.argtypes = [vp]
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        h.hipEventDestroy.argtypes = [vp]
        h.hipEventRecord.argtypes = [vp, vp]
        h.hipEventSynchronize.argtypes = [vp]
        h.hipGetErrorString.argtypes = [ip]
        h.hipGetErrorString.restype = ctypes.c_char_p
        _hip = h
    return _hip


def check(rc: int, what: str):
    if rc != 0:
        raise HipError(f"{what}: {rt().hipGetErrorString(rc).decode()} ({rc})")


def set_device(device: int):
    check(rt().hipSetDevice(device), "hipSetDevice")


def synchronize():
    check(rt().hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceBuffer:
    """hipMalloc'd device memory (`addr` = the device pointer)."""

    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.ptr = ctypes.c_void_p()
        check(rt().hipMalloc(ctypes.byref(self.ptr), max(nbytes, 1)), "hipMalloc")

    @classmethod
    def from_array(cls, a: np.ndarray):
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        check(rt().hipMemcpy(b.ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")
        return b

    def to_array(self, shape, dtype):
        out = np.empty(shape, dtype)
        check(rt().hipDeviceSynchronize(), "hipDeviceSynchronize")
        check(rt().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H), "hipMemcpy D2H")
        return out

    def zero(self):
        check(rt().hipMemset(self.ptr, 0, max(self.nbytes, 1)), "hipMemset")
        return self

    @property
    def addr(self) -> int:
        return self.ptr.value

    def free(self):
        if self.ptr:
            rt().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PinnedAllocator:
    """Page-locked host buffers (hipHostMalloc) as uint8 numpy arrays; the
    allocator keeps them alive and frees them on close()."""

    def __init__(self, coherent: bool = False):
        self.flags = HOST_MALLOC_COHERENT if coherent else 0
        self.keep = []

    def __call__(self, shape):
        n = int(np.prod(shape))
        p = ctypes.c_void_p()
        check(rt().hipHostMalloc(ctypes.byref(p), max(n, 1), self.flags), "hipHostMalloc")
        self.keep.append(p)
        return np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(p.value))[:n].reshape(shape)

    def close(self):
        for p in self.keep:
            rt().hipHostFree(p)
        self.keep = []


class Stream:
    def __init__(self):
        self.ptr = ctypes.c_void_p()
        check(rt().hipStreamCreateWithFlags(ctypes.byref(self.ptr), STREAM_NON_BLOCKING), "hipStreamCreate")

    @property
    def handle(self) -> int:
        return self.ptr.value

    def synchronize(self):
        check(rt().hipStreamSynchronize(self.ptr), "hipStreamSynchronize")

    def destroy(self):
        if self.ptr:
            rt().hipStreamDestroy(self.ptr)
            self.ptr = ctypes.c_void_p()


class Event:
    def __init__(self):
        self.ptr = ctypes.c_void_p()
        check(rt().hipEventCreateWithFlags(ctypes.byref(self.ptr), EVENT_DISABLE_TIMING), "hipEventCreate")

    def record(self, stream: Stream):
        check(rt().hipEventRecord(self.ptr, stream.ptr), "hipEventRecord")

    def synchronize(self):
        check(rt().hipEventSynchronize(self.ptr), "hipEventSynchronize")

    def destroy(self):
        if self.ptr:
            rt().hipEventDestroy(self.ptr)
            self.ptr = ctypes.c_void_p()


def memcpy_async(dst: int, src: int, nbytes: int, kind: int, stream: Stream):
    check(rt().hipMemcpyAsync(dst, src, nbytes, kind, stream.ptr), "hipMemcpyAsync")


def memset_d32_async(dst: int, value: int, count: int, stream: Stream):
    check(rt().hipMemsetD32Async(dst, value, count, stream.ptr), "hipMemsetD32Async")


RUNTIME_LIBS = ("libamdhip64", "libhsa-runtime64", "librccl", "libamd_comgr")


def mapped_runtimes() -> dict:
    """Every file of the HIP / HSA / RCCL / comgr runtimes mapped into this
    process (/proc/self/maps), per library: one entry each = one runtime."""
    out = {k: set() for k in RUNTIME_LIBS}
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) < 6:
                continue
            base = parts[-1].rsplit("/", 1)[-1]
            for k in RUNTIME_LIBS:
                if re.match(re.escape(k) + r"\.so(\.|$)", base):
                    out[k].add(parts[-1])
    return {k: sorted(v) for k, v in out.items()}
