"""Seeded random sweep of the HIP LK path against the CPU oracle (bit-exact).

Each case draws its own frame size, window (every kernel class: single-tile,
box with and without a scalar tail, large window), pyramid depth, flags,
termination criteria, kernel variant (LDS poisoning among them) and point set
(points inside, on and past the border), then compares nextPts / status / err
with oracle/lk_oracle.c bit for bit. The fixed cases in test_lk_gpu.py cover
the shapes the reference calls with; this sweep covers the combinations in
between (a stale-LDS read this round showed only in such a combination).
Reference behaviour: cv::calcOpticalFlowPyrLK as called at
PSNWhere_Tracker2D.cpp:776-782 and :871-877.
"""
import numpy as np
import pytest

from mcmtt_opticalflow_amd import lk as glk
from mcmtt_opticalflow_amd import synth
from mcmtt_opticalflow_amd._lib import ACCUM_SCALAR, GET_MIN_EIGENVALS, USE_INITIAL_FLOW

from test_lk_gpu import assert_same, oracle_ref

pytestmark = pytest.mark.gpu

_VARIANTS = [{}, {}, {"poison_lds": 1}, {"st_ovl": 0}, {"onewave": 0}, {"poison_lds": 1, "lg_jr": 0},
             {"large": 1}, {"threads": 128}]
_CRITERIA = [(3, 30, 0.01), (3, 10, 0.03), (1, 7, 0.0), (2, 30, 0.3), (3, 20, 0.0)]


def _window(rng):
    k = rng.integers(0, 4)
    if k == 0:  # single-tile kernel (<= 1024 px)
        w = int(rng.integers(3, 33))
        return w, int(rng.integers(3, max(4, min(64, 1024 // w) + 1)))
    if k == 1:  # box kernel, no scalar tail (w % 8 == 0)
        return 8 * int(rng.integers(4, 11)), int(rng.integers(33, 180))
    if k == 2:  # box kernel with a tail
        return int(rng.integers(33, 90)) | 1, int(rng.integers(20, 160))
    return int(rng.integers(90, 170)), int(rng.integers(90, 260))  # large-window kernel


def _case(seed):
    rng = np.random.default_rng(7100 + seed)
    win = _window(rng)
    W = int(rng.integers(max(2 * win[0], 200), 1400))
    H = int(rng.integers(max(2 * win[1], 160), 900))
    ml = int(rng.integers(0, 6))
    npts = int(rng.integers(8, 40))
    sc = synth.make_scene(seed % 17, W, H, npts, box_w=max(8, min(win[0], W // 3)),
                          box_h=max(8, min(win[1], H // 3)), max_speed=float(rng.uniform(0.5, 6.0)))
    f0, f1 = sc.frame(0), sc.frame(int(rng.integers(1, 3)))
    if rng.random() < 0.25:  # lower contrast: more exact fast paths
        f1 = (f1.astype(np.int32) // 2 + 64).astype(np.uint8)
        f0 = (f0.astype(np.int32) // 2 + 64).astype(np.uint8)
    border = np.array([[0.0, 0.0], [W - 0.5, H - 0.75], [-win[0] / 2.0, H / 2.0], [W / 2.0, H + 3.0],
                       [1.25, H - 2.5], [W - 1.5, 0.5]], np.float32)
    pts = np.concatenate([sc.points_at(0), border[rng.permutation(len(border))[:3]]]).astype(np.float32)
    flags = int(rng.choice([0, 0, ACCUM_SCALAR, USE_INITIAL_FLOW, GET_MIN_EIGENVALS]))
    guess = None
    if flags & USE_INITIAL_FLOW:
        guess = (pts + rng.uniform(-3, 3, pts.shape)).astype(np.float32)
    crit = _CRITERIA[int(rng.integers(0, len(_CRITERIA)))]
    var = _VARIANTS[int(rng.integers(0, len(_VARIANTS)))]
    return f0, f1, pts, win, ml, flags, guess, crit, var


@pytest.mark.parametrize("seed", range(40))
def test_lk_random_sweep(oracle_mod, seed):
    f0, f1, pts, win, ml, flags, guess, crit, var = _case(seed)
    kw = dict(criteria=crit, flags=flags)
    if guess is not None:
        kw["next_pts"] = guess
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, ml, **kw)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, ml, variants=var, **kw)
    assert_same(gpu, ref, f"seed {seed}: {f0.shape[::-1]} win {win} ml {ml} flags {flags} crit {crit} {var}")


@pytest.mark.parametrize("seed", range(12))
def test_lk_random_batched_queries(oracle_mod, seed):
    """Several random queries (each its own window, depth, flags, criteria and
    direction between the two ring slots) in ONE track call: the per-class
    launches of a mixed call, as Tracker2D issues its backward / forward calls;
    runs of repeated queries (contiguous points) merge into sub-queries."""
    rng = np.random.default_rng(9100 + seed)
    W, H = int(rng.integers(640, 1500)), int(rng.integers(480, 1000))
    sc = synth.make_scene(seed % 13, W, H, 200, max_speed=float(rng.uniform(1.0, 5.0)))
    frames = [sc.frame(0), sc.frame(1)]
    specs, first = [], 0
    for _ in range(int(rng.integers(2, 9))):
        if specs and rng.random() < 0.4:  # the previous query again: merged into sub-queries
            a, b, _, n, win, ml, flags, crit = specs[-1]
            specs.append((a, b, first, n, win, ml, flags, crit))
            first += n
            continue
        win = _window(rng)
        n = int(rng.integers(0, 30))
        ml = glk.effective_max_level(W, H, win[0], win[1], int(rng.integers(0, 5)))
        flags = int(rng.choice([0, ACCUM_SCALAR, GET_MIN_EIGENVALS]))
        crit = _CRITERIA[int(rng.integers(0, len(_CRITERIA)))]
        a = int(rng.integers(0, 2))
        specs.append((a, 1 - a, first, n, win, ml, flags, crit))
        first += n
    pool = np.concatenate([sc.points_at(0), sc.points_at(1)])
    pts = pool[rng.permutation(len(pool))[:max(first, 1)] % len(pool)]
    var = _VARIANTS[int(rng.integers(0, len(_VARIANTS)))]
    with glk.LKContext(W, H, ring_slots=2, max_level_cap=4, variants=var) as ctx:
        for s, f in enumerate(frames):
            ctx.push_frame(s, f)
        qs = [glk.make_query(a, b, f0, n, glk.make_params(win, ml, crit, flags))
              for a, b, f0, n, win, ml, flags, crit in specs]
        gn, gs, ge = ctx.track(qs, pts)
    for a, b, f0, n, win, ml, flags, crit in specs:
        sl = slice(f0, f0 + n)
        ref = oracle_ref(oracle_mod, frames[a], frames[b], pts[sl], win, ml, criteria=crit, flags=flags)
        assert_same((gn[sl], gs[sl], ge[sl]), ref, f"seed {seed}: query {win} ml {ml} flags {flags} {crit} {var}")
