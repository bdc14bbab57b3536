"""Savitzky-Golay trajectory post-filter (BASELINE configs[4]
"SGSmooth post-filter"): the reference's online smoother CPSNWhere_SGSmooth
(psn_where/PSNWhere_SGSmooth.cpp) batched over many series on the GPU
(include/psn_sgsmooth.h, libpsn_lk.so).

Oracle: oracle/sgsmooth_oracle.py restates the reference; it is pinned
bit-for-bit against the reference's OWN code (oracle/_ref/libsgsmooth_ref.so,
compiled from psn_where/PSNWhere_SGSmooth.cpp by `make -C oracle ref`) when
that library is present. Bar: bit-exact doubles (same operations, same order).
"""
import ctypes
import os

import numpy as np
import pytest

import sgsmooth_oracle as sgo

CASES = [(9, 1), (7, 2), (4, 1), (1, 1), (15, 3), (2, 0)]


def _ref_or_skip():
    L = sgo.ref_lib()
    if L is None:
        pytest.skip("oracle/_ref/libsgsmooth_ref.so not built (needs /root/reference)")
    return L


@pytest.mark.parametrize("w,degree", [(3, 1), (5, 1), (9, 1), (7, 2), (11, 3), (9, 0), (31, 2)])
def test_calculate_q_matches_reference(w, degree):
    L = _ref_or_skip()
    hf = (w - 1) // 2
    qb = (ctypes.c_double * max(hf * w, 1))()
    qm = (ctypes.c_double * w)()
    qe = (ctypes.c_double * max(hf * w, 1))()
    L.sgref_q(w, degree, qb, qm, qe)
    b, m, e = sgo.calculate_q(w, degree)
    assert list(qb)[:hf * w] == b and list(qm) == m and list(qe)[:hf * w] == e


@pytest.mark.parametrize("span,degree", CASES)
def test_restatement_matches_reference(span, degree):
    L = _ref_or_skip()
    rng = np.random.default_rng(span * 10 + degree)
    h = L.sgref_create(span, degree)
    try:
        s = sgo.SGSmooth(span, degree)
        for k, v in enumerate((rng.normal(0, 50, 40) + 300).astype(np.float32)):
            assert L.sgref_insert(h, float(v)) == s.insert(float(v))
            # the smoothed series always has one value per inserted value (the
            # reference's size() is stale after a bypass insert and starts
            # uninitialised, so the count is taken from the inserts)
            assert [L.sgref_result(h, i) for i in range(k + 1)] == s.smoothed
    finally:
        L.sgref_destroy(h)


def test_known_values():
    # degree 1, window 3: Qmid = 1/3 each; a linear ramp is reproduced exactly
    # at the ends (local line fit) and in the middle (moving average of a line)
    s = sgo.SGSmooth(3, 1)
    for v in (0.0, 3.0, 6.0, 9.0):
        s.insert(v)
    assert np.allclose(s.smoothed, [0.0, 3.0, 6.0, 9.0], atol=1e-12)
    s = sgo.SGSmooth(9, 1)
    assert s.insert(5.0) == 0 and s.insert(7.0) == 1  # bypass while the window <= degree
    assert s.smoothed == [5.0, 7.0]


@pytest.mark.gpu
@pytest.mark.parametrize("span,degree,dims", [(9, 1, 2), (7, 2, 3), (4, 1, 2), (15, 3, 1)])
def test_sg_gpu_matches_oracle(span, degree, dims):
    from mcmtt_opticalflow_amd import lk as glk

    n, T = 300, 24
    rng = np.random.default_rng(span + 100 * degree)
    sm = glk.SGSmoother(n, dims, span, degree)
    oracles = [[sgo.SGSmooth(span, degree) for _ in range(dims)] for _ in range(n)]
    try:
        for t in range(T):
            vals = (rng.normal(0, 30, (n, dims)) + 500).astype(np.float32)
            active = (rng.random(n) < 0.8).astype(np.uint8) if t % 3 == 2 else None
            ref, out = sm.insert(vals, active)
            for i in range(n):
                if active is not None and not active[i]:
                    assert ref[i] == -1
                    continue
                rs = [oracles[i][d].insert(float(vals[i, d])) for d in range(dims)]
                assert ref[i] == rs[0], (t, i)
                m = len(oracles[i][0].smoothed) - rs[0]
                for d in range(dims):
                    exp = oracles[i][d].smoothed[rs[0]:]
                    assert out[i, :m, d].tolist() == exp, (t, i, d)
        lens = sm.lengths()
        assert (lens == [len(o[0].data) for o in oracles]).all()
    finally:
        sm.close()
