"""GridFAST feature extraction: the keypoints
CPSNWhere_Tracker2D extracts per detection before its backward LK chain
(psn_where/PSNWhere_Tracker2D.cpp:142 "GridFAST", :734-757 mask + detect +
random_shuffle + cap 100).

CPU part: known-answer tests of the oracle (oracle/gridfast_oracle.c), which
restates OpenCV 2.4.6's FAST_t<16> / cornerScore<16> / GridAdaptedFeatureDetector
/ keepStrongest. OpenCV is absent and the reference has no fixtures, so parity
with OpenCV itself is UNPINNED; the oracle is pinned here by hand-derived
answers and by an independent brute-force restatement (arc test + closed-form
score) written in numpy below.

GPU part: psn_gridfast_detect (libpsn_lk.so, C ABI) must return exactly the
oracle's points (integer work: bit-exact), for the seeded shuffle and for the
full keypoint sets, over edge-case rois.
"""
import numpy as np
import pytest

from mcmtt_opticalflow_amd import synth

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def brute_fast(img, t=10, nonmax=True):
    """Independent numpy restatement: arc of >= 9 contiguous circle pixels all
    > v + t or all < v - t; response = max(t, best 9-arc min of |x - v| on the
    corner's side) - 1; strict 8-neighbour non-max on responses."""
    img = img.astype(np.int32)
    h, w = img.shape
    resp = np.full((h, w), -1, np.int32)
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            v = img[y, x]
            e = np.array([img[y + dy, x + dx] - v for dx, dy in CIRCLE])
            ee = np.concatenate([e, e])
            arcs = np.array([ee[k:k + 9] for k in range(16)])
            corner = (arcs > t).all(1).any() or (arcs < -t).all(1).any()
            if not corner:
                continue
            best = max(t, arcs.min(1).max(), (-arcs).min(1).max())
            resp[y, x] = best - 1 if nonmax else 0
    out = []
    for y in range(3, h - 3):
        for x in range(3, w - 3):
            s = resp[y, x]
            if s < 0:
                continue
            if nonmax:
                nb = np.maximum(resp[y - 1:y + 2, x - 1:x + 2], 0).ravel().tolist()
                del nb[4]
                if not all(s > q for q in nb):
                    continue
            out.append((x, y, s))
    return np.array(out, np.int32).reshape(-1, 3)


def test_single_dot_known_answer(oracle_mod):
    img = np.full((32, 32), 20, np.uint8)
    img[15, 17] = 120
    k = oracle_mod.fast16(img, 10)
    # all 16 circle pixels are 100 darker: one corner, response 100 - 1
    assert k.tolist() == [[17, 15, 99]]
    img[15, 17] = 31  # 11 brighter than the ring: corner at threshold 10 with response 10
    assert oracle_mod.fast16(img, 10).tolist() == [[17, 15, 10]]
    img[15, 17] = 30  # exactly threshold: not a corner (strict >)
    assert oracle_mod.fast16(img, 10).tolist() == []


def test_arc_length_known_answer(oracle_mod):
    base = np.full((16, 16), 100, np.uint8)
    for run, expect in ((8, 0), (9, 1), (12, 1)):
        img = base.copy()
        for k in range(run):  # a run of `run` bright circle pixels from position 5
            dx, dy = CIRCLE[(5 + k) % 16]
            img[8 + dy, 8 + dx] = 200
        k = oracle_mod.fast16(img, 10, nonmax=False)
        assert int(((k[:, 0] == 8) & (k[:, 1] == 8)).sum()) == expect, run


@pytest.mark.parametrize("seed,t", [(0, 10), (1, 10), (2, 25), (3, 0)])
def test_fast_matches_bruteforce(oracle_mod, seed, t):
    rng = np.random.default_rng(seed)
    img = (rng.random((40, 56)) * 255).astype(np.uint8)
    if seed == 1:
        img = synth.texture(56, 40, 7)
    for nm in (True, False):
        np.testing.assert_array_equal(oracle_mod.fast16(img, t, nm), brute_fast(img, t, nm))


def test_grid_cells_and_mask(oracle_mod):
    # isolated dots on a lattice: a dot within 3 px of a cell border is not
    # detected (each cell is its own sub-image); the mask keeps the roi only
    img = np.full((64, 64), 50, np.uint8)
    pts = [(x, y) for y in range(2, 64, 6) for x in range(2, 64, 6)]
    for x, y in pts:
        img[y, x] = 200
    xy, resp = oracle_mod.gridfast(img, (0, 0, 64, 64))
    got = {tuple(map(int, p)) for p in xy}
    exp = {(x, y) for x, y in pts if 3 <= x % 16 < 13 and 3 <= y % 16 < 13}
    assert got == exp and (resp == 149).all()
    xy2, _ = oracle_mod.gridfast(img, (10, 20, 30, 15))
    assert {tuple(map(int, p)) for p in xy2} == {p for p in exp if 10 <= p[0] < 40 and 20 <= p[1] < 35}
    # cell order: keypoints of cell (0, 0) first
    assert tuple(map(int, xy[0])) == (8, 8)


def test_keep_strongest_ties(oracle_mod):
    # 4 x 4 grid, max_total 32 -> 2 per cell; one cell holds 5 dots of
    # responses 59, 99, 99, 79, 99: keep the two 99s that come first
    img = np.full((128, 128), 20, np.uint8)
    dots = [(5, 5, 80), (12, 5, 120), (19, 5, 120), (26, 12, 100), (5, 19, 120)]
    for x, y, v in dots:
        img[y, x] = v
    xy, resp = oracle_mod.gridfast(img, (0, 0, 128, 128), max_total=32)
    assert [tuple(map(int, p)) for p in xy] == [(12, 5), (19, 5)] and resp.tolist() == [99, 99]


def test_select_is_seeded_permutation(oracle_mod):
    cand = np.stack([np.arange(300), np.arange(300) * 2], 1).astype(np.float32)
    a = oracle_mod.gridfast_select(cand, 7, 0, 100)
    b = oracle_mod.gridfast_select(cand, 7, 0, 100)
    c = oracle_mod.gridfast_select(cand, 8, 0, 100)
    np.testing.assert_array_equal(a, b)
    assert len(a) == 100 and len({tuple(p) for p in a.tolist()}) == 100 and not np.array_equal(a, c)
    full = oracle_mod.gridfast_select(cand, 7, 3, 1000)
    assert sorted(map(tuple, full.tolist())) == sorted(map(tuple, cand.tolist()))


# ------------------------------------------------------------------- GPU parity

ROIS_1080 = [
    (900, 400, 64, 160),     # a 1080p pedestrian box (Tracker2D box size)
    (470, 260, 20, 30),      # straddles four cells
    (0, 0, 1919, 1079),      # full frame (cropWithSize: w - 1, h - 1)
    (1850, 1000, 69, 79),    # bottom-right border
    (0, 0, 3, 3),            # inside a cell's 3-px border: nothing
    (500, 500, 0, 40),       # empty
    (-20, -10, 60, 50),      # partly outside (clipped)
    (1200, 100, 240, 600),   # tall, spans two cell rows
]


def _compare(g_pts, g_tot, r_pts, r_tot, rois):
    np.testing.assert_array_equal(g_tot, r_tot)
    for i, (a, b) in enumerate(zip(g_pts, r_pts)):
        np.testing.assert_array_equal(a, b, err_msg=f"roi {i} {rois[i]}")


@pytest.mark.gpu
@pytest.mark.parametrize("cam,seed", [(0, 1), (3, 99)])
def test_gridfast_gpu_matches_oracle(oracle_mod, cam, seed):
    from mcmtt_opticalflow_amd import lk as glk

    sc = synth.make_scene(cam, 1920, 1080, 64)
    f = sc.frame(0)
    r_pts, r_tot = oracle_mod.gridfast_detect(f, ROIS_1080, seed=seed)
    with glk.LKContext(1920, 1080, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame(1, f)
        g_pts, g_tot = ctx.gridfast_detect(1, ROIS_1080, seed=seed)
    assert r_tot[0] > 50 and r_tot[2] > 500  # the synthetic texture has corners
    _compare(g_pts, g_tot, r_pts, r_tot, ROIS_1080)


@pytest.mark.gpu
@pytest.mark.parametrize("thr,nonmax,max_total,grid", [(10, True, 1000, (4, 4)), (5, True, 64, (4, 4)),
                                                       (10, False, 1000, (4, 4)), (0, True, 300, (3, 5)),
                                                       (40, True, 4096, (2, 2))])
def test_gridfast_gpu_params_full_sets(oracle_mod, thr, nonmax, max_total, grid):
    """Every keypoint (cap = max_total) for non-default detector settings:
    keepStrongest cuts with ties, no non-max, threshold 0, other grids."""
    from mcmtt_opticalflow_amd import lk as glk

    rng = np.random.default_rng(thr + max_total)
    w, h = 333, 257
    img = np.clip(synth.texture(w, h, 5).astype(np.int32) + rng.integers(-30, 30, (h, w)), 0, 255).astype(np.uint8)
    rois = [(0, 0, w - 1, h - 1), (40, 30, 100, 120), (200, 100, 133, 157), (5, 200, 300, 40)]
    p = glk.gridfast_params(thr, nonmax, max_total, grid, cap=max_total)
    r_pts, r_tot = oracle_mod.gridfast_detect(img, rois, seed=3, threshold=thr, nonmax=nonmax,
                                              max_total=max_total, grid=grid, cap=max_total)
    with glk.LKContext(w, h, ring_slots=1, max_level_cap=0) as ctx:
        ctx.push_frame(0, img)
        g_pts, g_tot = ctx.gridfast_detect(0, rois, p, seed=3)
    _compare(g_pts, g_tot, r_pts, r_tot, rois)


@pytest.mark.gpu
def test_gridfast_gpu_many_rois(oracle_mod):
    """More rois than one launch's table (64), random boxes, 4K frame."""
    from mcmtt_opticalflow_amd import lk as glk

    w, h = 3840, 2160
    f = synth.texture(w, h, 11)
    rng = np.random.default_rng(5)
    rois = [(int(x), int(y), 128, 320) for x, y in zip(rng.integers(0, w - 129, 70), rng.integers(0, h - 321, 70))]
    r_pts, r_tot = oracle_mod.gridfast_detect(f, rois, seed=42)
    with glk.LKContext(w, h, ring_slots=1, max_level_cap=0) as ctx:
        ctx.push_frame(0, f)
        g_pts, g_tot = ctx.gridfast_detect(0, rois, seed=42)
    _compare(g_pts, g_tot, r_pts, r_tot, rois)


@pytest.mark.gpu
def test_gridfast_gpu_sets_match_per_frame(oracle_mod):
    """psn_gridfast_detect_device_sets (every camera's detections in one launch,
    as the tracker runs them): per set, exactly the oracle on that set's frame
    with the set-local shuffle keys. Sets of 30, 0, 45 and 3 rois: the 64-roi
    launch boundary falls inside the third set."""
    from mcmtt_opticalflow_amd import lk as glk

    w, h = 1920, 1080
    rng = np.random.default_rng(17)
    frames = [synth.make_scene(c, w, h, 64).frame(0) for c in range(4)]
    sizes = [30, 0, 45, 3]
    sets = [[(int(x), int(y), int(bw), int(bh)) for x, y, bw, bh in
             zip(rng.integers(-30, w - 40, n), rng.integers(-30, h - 60, n), rng.integers(8, 260, n),
                 rng.integers(8, 400, n))] for n in sizes]
    sets[3][0] = (0, 0, 0, 0)  # empty roi
    with glk.LKContext(w, h, ring_slots=4, max_level_cap=0) as ctx:
        for s, f in enumerate(frames):
            ctx.push_frame(s, f)
        got = ctx.gridfast_detect_sets([2, 0, 1, 3], [sets[0], sets[1], sets[2], sets[3]], seed=77)
        one = ctx.gridfast_detect(1, sets[2], seed=77)
    for (g_pts, g_tot), slot, rois in zip(got, [2, 0, 1, 3], sets):
        r_pts, r_tot = oracle_mod.gridfast_detect(frames[slot], rois, seed=77) if rois else ([], np.zeros(0))
        _compare(g_pts, g_tot, r_pts, r_tot, rois)
    _compare(got[2][0], got[2][1], one[0], one[1], sets[2])
