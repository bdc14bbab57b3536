"""The binade-run model of an ordered float chain (oracle/chain_model.c) equals
the plain sequential float sum, bit for bit, on chains shaped like
LKTrackerInvoker's b sums (integer products of 14-bit diffs and 13-bit
gradients, SSE2 lane chains split into per-thread segments). CPU only: this
pins the argument recorded in DESIGN.md (the measured GPU evaluation of it was
slower than the ordered chains and is not in the kernel)."""
import ctypes
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402  (the checker)

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int)


def _lib():
    L = oracle.lib()
    L.oracle_chain_serial.argtypes = [_f32p, ctypes.c_int]
    L.oracle_chain_serial.restype = ctypes.c_float
    L.oracle_chain_binade.argtypes = [_f32p, ctypes.c_int, _i32p, ctypes.c_int, ctypes.c_int, _i32p]
    L.oracle_chain_binade.restype = ctypes.c_float
    return L


def _run(L, terms, seg_len):
    f = np.ascontiguousarray(terms, np.float32)
    n = len(f)
    off = np.arange(0, n + seg_len, seg_len, dtype=np.int32)
    off[-1] = n
    off = np.ascontiguousarray(np.minimum(off, n), np.int32)
    nseg = len(off) - 1
    st = np.zeros(8, np.int32)
    a = L.oracle_chain_serial(f.ctypes.data_as(_f32p), n)
    b = L.oracle_chain_binade(f.ctypes.data_as(_f32p), n, off.ctypes.data_as(_i32p), nseg, 64,
                              st.ctypes.data_as(_i32p))
    return np.float32(a), np.float32(b), st


@pytest.mark.parametrize("scale", [1, 30, 400, 4000])
@pytest.mark.parametrize("seg_len", [1, 4, 10, 40])
def test_binade_model_matches_sequential(scale, seg_len):
    L = _lib()
    rng = np.random.default_rng(1000 * scale + seg_len)
    for trial in range(40):
        n = int(rng.integers(1, 3000))
        d = rng.integers(-8160, 8161, n) // max(1, 4000 // scale)
        g = rng.integers(-4080, 4081, n)
        if trial % 3 == 0:  # a biased chain: the accumulator climbs through several binades
            g = np.abs(g) * np.sign(d)
        t = (d.astype(np.int64) * g).astype(np.float32)
        a, b, _ = _run(L, t, seg_len)
        assert a.tobytes() == b.tobytes(), (scale, seg_len, trial, a, b)


def test_binade_model_edges():
    L = _lib()
    cases = [np.zeros(0, np.float32), np.zeros(17, np.float32), np.full(1000, 16777215.0, np.float32),
             np.full(3000, 33333333.0, np.float32), np.array([2.0 ** 24, 1.0, 1.0, 3.0, -1.0] * 200, np.float32),
             np.tile(np.array([3.3e7, -3.3e7, 1.0], np.float32), 500)]
    for t in cases:
        for seg in (1, 3, 16):
            a, b, _ = _run(L, t, seg)
            assert a.tobytes() == b.tobytes(), (t[:5], seg, a, b)


def _runs(L, terms, seg_len, fs):
    """oracle_chain_runs (the per-thread parity records with local HARD runs of
    psn_lk_xb.h) from segment fs, whose exact start every earlier prefix must
    allow: None when the chain is not exact before fs or the model aborts."""
    L.oracle_chain_runs.argtypes = [_f32p, _i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p]
    L.oracle_chain_runs.restype = ctypes.c_float
    f = np.ascontiguousarray(terms, np.float32)
    n = len(f)
    off = np.ascontiguousarray(np.minimum(np.arange(0, n + seg_len, seg_len), n), np.int32)
    nseg = len(off) - 1
    fs = min(fs, nseg)
    P = np.cumsum(f[:off[fs]].astype(np.int64))
    if len(P) and np.abs(P).max() > (1 << 24):
        return None
    st = np.zeros(5, np.int32)
    b = L.oracle_chain_runs(f.ctypes.data_as(_f32p), off.ctypes.data_as(_i32p), nseg, fs,
                            int(P[-1]) if len(P) else 0, st.ctypes.data_as(_i32p))
    if np.isnan(b):
        return None
    return np.float32(b), st


@pytest.mark.parametrize("seg_len", [1, 7, 25, 64])
def test_parity_record_model_matches_sequential(seg_len):
    """The b fallback by parity records (psn_lk_xb.h, build parameter PSN_LG_XB):
    bit for bit the sequential float sum, on biased and unbiased chains of
    LK-sized integer products, started at several segments."""
    L = _lib()
    rng = np.random.default_rng(77 + seg_len)
    checked = 0
    for trial in range(60):
        n = int(rng.integers(1, 6000))
        d = rng.integers(-8160, 8161, n) // int(rng.choice([1, 8, 64]))
        g = rng.integers(-4080, 4081, n)
        if trial % 3 == 0:
            g = np.abs(g) * np.sign(d)
        t = (d.astype(np.int64) * g).astype(np.float32)
        a = np.float32(L.oracle_chain_serial(np.ascontiguousarray(t).ctypes.data_as(_f32p), n))
        for fs in (0, 3, 40):
            r = _runs(L, t, seg_len, fs)
            if r is None:
                continue
            assert a.tobytes() == r[0].tobytes(), (seg_len, trial, fs, a, r)
            checked += 1
    assert checked > 40
