"""ctypes binding of libpsn_lk.so (the C ABI declared in include/psn_lk.h).

The library is built in-tree (mcmtt_opticalflow_amd/lib/libpsn_lk.so) by
__graft_entry__.build(). There is NO fallback: if the HIP library is missing
every entry point raises, so a test can never pass on a CPU path.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpsn_lk.so")
# the instrumented build of the same sources (tools/ only: per-phase s_memtime stamps)
STAMPS_LIB_PATH = os.path.join(_HERE, "lib", "libpsn_lk_stamps.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "psn_lk.h")
# every header whose entry points libpsn_lk.so exports
HEADER_PATHS = [HEADER_PATH] + [os.path.join(os.path.dirname(_HERE), "include", h)
                                for h in ("psn_sgsmooth.h", "psn_t2d_device.h", "psn_jpeg.h")]

PSN_LK_OK = 0
ERRORS = {
    -1: "PSN_LK_ERR_ARG",
    -2: "PSN_LK_ERR_WINSIZE",
    -3: "PSN_LK_ERR_HIP",
    -4: "PSN_LK_ERR_NOMEM",
    -5: "PSN_LK_ERR_SLOT",
    -6: "PSN_LK_ERR_LEVEL_CAP",
    -7: "PSN_LK_ERR_COMM",
    -8: "PSN_LK_ERR_UNSUPPORTED",
}
USE_INITIAL_FLOW = 4
GET_MIN_EIGENVALS = 8
ACCUM_SCALAR = 0x100
OVERLAP_OFF, OVERLAP_STREAM, OVERLAP_FUSED = 0, 1, 2  # psn_lk_set_ingest_overlap modes
TERM_COUNT = 1
TERM_EPS = 2
MAX_WIN_WIDTH = 6400  # PSN_LK_MAX_WIN_WIDTH (any window height)
COMM_UNIQUE_ID_BYTES = 128
# psn_lk_debug_set_variant keys (tests / experiments; never read from the environment)
VARIANTS = {"threads": 1, "generic": 2, "onewave": 3, "box": 4, "tiled_lds": 5, "fused_helpers": 6,
            "large": 7, "lg_lds": 8, "lg_jr": 9, "st_ovl": 10, "poison_lds": 11}


class PsnLkError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")


class LkParams(ctypes.Structure):
    _fields_ = [
        ("win_w", ctypes.c_int),
        ("win_h", ctypes.c_int),
        ("max_level", ctypes.c_int),
        ("term_type", ctypes.c_int),
        ("max_count", ctypes.c_int),
        ("epsilon", ctypes.c_double),
        ("flags", ctypes.c_int),
        ("min_eig_threshold", ctypes.c_double),
    ]


class LkQuery(ctypes.Structure):
    _fields_ = [
        ("prev_slot", ctypes.c_int),
        ("next_slot", ctypes.c_int),
        ("first_pt", ctypes.c_int),
        ("num_pts", ctypes.c_int),
        ("params", LkParams),
    ]


class GridFastParams(ctypes.Structure):
    _fields_ = [
        ("threshold", ctypes.c_int),
        ("nonmax", ctypes.c_int),
        ("max_total", ctypes.c_int),
        ("grid_rows", ctypes.c_int),
        ("grid_cols", ctypes.c_int),
        ("cap", ctypes.c_int),
    ]


def header_functions() -> list[str]:
    """Names of every function declared in include/psn_lk.h and psn_sgsmooth.h."""
    src = "".join(open(p).read() for p in HEADER_PATHS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(psn_\w+)\s*\(", src)))


_lib = None


_lib_path = None


def timing_launches(L, ctx, cap: int):
    """psn_lk_timing_launches -> list of (ms, tag) per timed LK call."""
    ms = (ctypes.c_double * max(cap, 1))()
    tag = (ctypes.c_int * max(cap, 1))()
    n = ctypes.c_int()
    rc = L.psn_lk_timing_launches(ctx, cap, ms, tag, ctypes.byref(n))
    if rc != 0:
        raise PsnLkError(rc, "psn_lk_timing_launches")
    return [(ms[i], tag[i]) for i in range(n.value)]


def kernel_of_tag(tag: int) -> str:
    """psn_lk_timing_launches tag -> kernel name (a call split over several
    window-class launches: "mixed:" + the launch with the most window pixels)."""
    if tag >= 1000:
        return "mixed:" + kernel_of_tag(tag - 1000)
    if tag == 3:
        return "lk_kernel_lg"
    if tag == 1:
        return "lk_kernel_st"
    if tag == 2:
        return "lk_kernel"
    return f"lk_kernel_bx<{tag // 10}, {'true' if tag % 10 else 'false'}>"


def runtime_info() -> dict:
    """The ROCm runtime this process runs the library on: psn_lk_runtime_info
    (the file each HIP / HSA / RCCL / comgr symbol resolves to, versions) plus
    every runtime file mapped (`mapped`: one path per library = one runtime)."""
    import json

    from . import hip

    L = load()
    buf = ctypes.create_string_buffer(4096)
    rc = L.psn_lk_runtime_info(buf, len(buf))
    if rc != 0:
        raise PsnLkError(rc, "psn_lk_runtime_info")
    info = json.loads(buf.value.decode())
    info["mapped"] = hip.mapped_runtimes()
    info["one_runtime"] = all(len(v) <= 1 for v in info["mapped"].values())
    return info


def load(path: str | None = None):
    """The product library (mcmtt_opticalflow_amd/lib/libpsn_lk.so). Only the
    profiling tools pass path (STAMPS_LIB_PATH), before anything else loads it."""
    global _lib, _lib_path
    if _lib is not None:
        # load() without a path returns whatever is loaded (a tool's diagnostic
        # build, loaded first); an explicit different path is an error
        if path is not None and os.path.abspath(path) != os.path.abspath(_lib_path):
            raise RuntimeError(f"{_lib_path} is loaded already (asked for {path})")
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    L = ctypes.CDLL(path)
    vp, ip, u8p, fp = ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p
    L.psn_lk_abi_version.restype = ip
    L.psn_lk_default_params.argtypes = [ctypes.POINTER(LkParams)]
    L.psn_lk_default_params.restype = None
    L.psn_lk_effective_max_level.argtypes = [ip] * 5
    L.psn_lk_create.argtypes = [ip, ip, ip, ip, ip, ctypes.POINTER(vp)]
    L.psn_lk_destroy.argtypes = [vp]
    L.psn_lk_destroy.restype = None
    L.psn_lk_last_error.argtypes = [vp]
    L.psn_lk_last_error.restype = ctypes.c_char_p
    L.psn_lk_set_stream.argtypes = [vp, vp]
    L.psn_lk_get_stream.argtypes = [vp]
    L.psn_lk_get_stream.restype = vp
    L.psn_lk_sync.argtypes = [vp]
    L.psn_lk_push_frame.argtypes = [vp, ip, u8p, ip, ip]
    L.psn_lk_push_frame_device.argtypes = [vp, ip, vp, ip, ip]
    L.psn_lk_push_frame_async.argtypes = [vp, ip, u8p, ip, ip]
    L.psn_lk_push_frame_jpeg.argtypes = [vp, ip, vp, ctypes.c_size_t]
    L.psn_jpeg_info.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(ip), ctypes.POINTER(ip), ctypes.POINTER(ip)]
    L.psn_jpeg_create.argtypes = [ip, ctypes.POINTER(vp)]
    L.psn_jpeg_destroy.argtypes = [vp]
    L.psn_jpeg_destroy.restype = None
    L.psn_jpeg_last_error.argtypes = [vp]
    L.psn_jpeg_last_error.restype = ctypes.c_char_p
    L.psn_jpeg_set_stream.argtypes = [vp, vp]
    L.psn_jpeg_decode_device.argtypes = [vp, vp, ctypes.c_size_t, vp, ip]
    L.psn_jpeg_decode.argtypes = [vp, vp, ctypes.c_size_t, vp, ip]
    L.psn_lk_debug_set_variant.argtypes = [vp, ip, ip]
    L.psn_lk_track.argtypes = [vp, ctypes.POINTER(LkQuery), ip, fp, fp, u8p, fp]
    L.psn_lk_track_device.argtypes = [vp, ctypes.POINTER(LkQuery), ip, vp, vp, vp, vp]
    L.psn_lk_track_device_counted.argtypes = [vp, ctypes.POINTER(LkQuery), ip, vp, vp, vp, vp, vp]
    L.psn_lk_track_device_counted_strided.argtypes = [vp, ctypes.POINTER(LkQuery), ip, vp, ip, vp, vp, vp, vp]
    L.psn_calc_optical_flow_pyr_lk.argtypes = [vp, u8p, u8p, ip, fp, fp, u8p, fp, ip, ctypes.POINTER(LkParams)]
    L.psn_lk_read_level.argtypes = [vp, ip, ip, u8p, ip]
    L.psn_lk_level_size.argtypes = [vp, ip, ctypes.POINTER(ip), ctypes.POINTER(ip)]
    L.psn_lk_enable_timing.argtypes = [vp, ip, ip]
    L.psn_lk_timing_stats.argtypes = [vp, ctypes.POINTER(ip), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ip), ctypes.POINTER(ctypes.c_double)]
    L.psn_lk_timing_launches.argtypes = [vp, ip, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ip),
                                         ctypes.POINTER(ip)]
    L.psn_lk_debug_set_stamps.argtypes = [vp, vp]
    L.psn_lk_debug_count_samples.argtypes = [vp, ip]
    L.psn_lk_debug_read_samples.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong)]
    L.psn_lk_enable_timing.argtypes = [vp, ip, ip]
    L.psn_lk_set_ingest_overlap.argtypes = [vp, ip]
    L.psn_gridfast_default_params.argtypes = [ctypes.POINTER(GridFastParams)]
    L.psn_gridfast_default_params.restype = None
    gfa = [vp, ip, vp, ip, ctypes.POINTER(GridFastParams), ctypes.c_uint32, vp, vp, vp]
    L.psn_gridfast_detect.argtypes = gfa
    L.psn_gridfast_detect_device.argtypes = gfa
    if hasattr(L, "psn_gridfast_detect_device_sets"):  # (absent from the A/B experiments' older builds only)
        L.psn_gridfast_detect_device_sets.argtypes = [vp, ip, vp, vp, vp, ctypes.POINTER(GridFastParams),
                                                      ctypes.c_uint32, vp, vp, vp]
    L.psn_sg_create.argtypes = [ip, ip, ip, ip, ip, ctypes.POINTER(vp)]
    L.psn_sg_destroy.argtypes = [vp]
    L.psn_sg_destroy.restype = None
    L.psn_sg_reset.argtypes = [vp]
    L.psn_sg_set_stream.argtypes = [vp, vp]
    L.psn_sg_insert_device.argtypes = [vp, vp, ip, vp, vp, vp]
    L.psn_sg_insert.argtypes = [vp, vp, ip, vp, vp, vp]
    L.psn_sg_lengths.argtypes = [vp, vp]
    L.psn_comm_get_unique_id.argtypes = [vp]
    L.psn_comm_init.argtypes = [ip, ip, ip, vp, ctypes.POINTER(vp)]
    L.psn_comm_allgather.argtypes = [vp, vp, vp, ctypes.c_size_t, vp]
    L.psn_comm_destroy.argtypes = [vp]
    L.psn_comm_destroy.restype = None
    L.psn_lk_runtime_info.argtypes = [ctypes.c_char_p, ip]
    if hasattr(L, "psn_lk_sdma_warmup_ms"):  # (absent from the A/B experiments' older builds only)
        L.psn_lk_sdma_warmup_ms.argtypes = [ip, ctypes.POINTER(ctypes.c_double)]
    _lib, _lib_path = L, path
    return L


def default_params() -> LkParams:
    p = LkParams()
    load().psn_lk_default_params(ctypes.byref(p))
    return p
