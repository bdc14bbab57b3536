"""GPU parity of the HIP path (libpsn_lk.so, through the C ABI) against the
CPU oracle (oracle/lk_oracle.c) on identical seeded inputs.

Bar: the LK outputs are integer-exact fixed-point + IEEE float arithmetic in
OpenCV 2.4.6's order, so nextPts, status and err must be BIT-IDENTICAL to the
oracle (EPE == 0, which is inside north_star's "EPE < 1e-4 px" tolerance);
pyramid levels are exact u8. Calls that rebuild pyramids on the CPU mimic the
reference call schedule (PSNWhere_Tracker2D.cpp:776-782, :871-877).
"""
import numpy as np
import pytest

from mcmtt_opticalflow_amd import lk as glk
from mcmtt_opticalflow_amd import synth
from mcmtt_opticalflow_amd._lib import ACCUM_SCALAR, GET_MIN_EIGENVALS, MAX_WIN_WIDTH, USE_INITIAL_FLOW, PsnLkError

pytestmark = pytest.mark.gpu

EPE_TOL = 1e-4  # north_star tolerance; the check below is the stricter bit-exact one


def assert_same(gpu, ref, what=""):
    (gn, gs, ge), (rn, rs, re_) = gpu, ref
    epe = np.linalg.norm(gn.astype(np.float64) - rn, axis=1)
    bad = np.nonzero((epe > 0) | (gs != rs))[0]
    assert bad.size == 0, (f"{what}: {bad.size} points differ; first {bad[:8]} max EPE {epe.max():.3g}; "
                           f"gpu {gn[bad[:3]]} {gs[bad[:3]]} ref {rn[bad[:3]]} {rs[bad[:3]]}")
    assert epe.max(initial=0.0) < EPE_TOL
    if re_ is not None:
        np.testing.assert_array_equal(ge, re_, err_msg=f"{what}: err differs")


def oracle_ref(oracle_mod, f0, f1, pts, win, ml, **kw):
    accum = oracle_mod.ACCUM_SCALAR if kw.get("flags", 0) & ACCUM_SCALAR else oracle_mod.ACCUM_SSE2
    flags = kw.pop("flags", 0) & ~ACCUM_SCALAR
    return oracle_mod.calc_optical_flow_pyr_lk(f0, f1, pts, win, ml, flags=flags, accum=accum, **kw)


def scene_pair(cam, w, h, n, **kw):
    sc = synth.make_scene(cam, w, h, n, **kw)
    return sc, sc.frame(0), sc.frame(1)


# --------------------------------------------------------------------- pyramid

@pytest.mark.parametrize("w,h,cap", [(640, 480, 3), (1920, 1080, 3), (37, 23, 2), (5, 3, 2), (1, 1, 0),
                                     (3840, 2160, 4), (101, 67, 5), (64, 64, 0)])
def test_pyramid_bit_exact(oracle_mod, w, h, cap):
    rng = np.random.default_rng(w * 7 + h)
    img = rng.integers(0, 256, (h, w), dtype=np.uint8) if w < 1000 else synth.texture(w, h, 3)
    ref = oracle_mod.build_pyramid(img, cap + 1)
    with glk.LKContext(w, h, ring_slots=2, max_level_cap=cap) as ctx:
        ctx.push_frame(1, img)
        for l in range(cap + 1):
            np.testing.assert_array_equal(ctx.read_level(1, l), ref[l], err_msg=f"level {l}")


def test_bgr_ingest_bit_exact(oracle_mod):
    rng = np.random.default_rng(11)
    bgr = rng.integers(0, 256, (97, 131, 3), dtype=np.uint8)
    gray = oracle_mod.bgr2gray(bgr)
    ref = oracle_mod.build_pyramid(gray, 3)
    with glk.LKContext(131, 97, ring_slots=1, max_level_cap=2) as ctx:
        ctx.push_frame(0, bgr)
        for l in range(3):
            np.testing.assert_array_equal(ctx.read_level(0, l), ref[l])


# --------------------------------------------------------------------- LK parity

@pytest.mark.parametrize("flags", [0, ACCUM_SCALAR])
def test_lk_21x21_parity(oracle_mod, flags):
    sc, f0, f1 = scene_pair(1, 640, 480, 256)
    pts = sc.points_at(0)
    # add border / outside points (status 0 paths, reflect-101 reads)
    extra = np.array([[0, 0], [639.9, 479.9], [-5, 100], [700, 10], [320, -30], [2.5, 477.25], [636.75, 1.5]],
                     np.float32)
    pts = np.concatenate([pts, extra])
    ref = oracle_ref(oracle_mod, f0, f1, pts, (21, 21), 3, flags=flags)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (21, 21), 3, flags=flags)
    assert_same(gpu, ref, "21x21")
    assert ref[1].sum() > 200


def test_lk_config2_full_size(oracle_mod):
    """configs[1]: 1 camera 1920x1080, 512 points, 4-level pyramid, 21x21."""
    sc, f0, f1 = scene_pair(0, 1920, 1080, 512)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (21, 21), 3)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (21, 21), 3)
    assert_same(gpu, ref, "1080p")
    # analytic flow sanity: most points track their box
    gt = sc.points_at(1)
    assert np.median(np.linalg.norm(gpu[0] - gt, axis=1)[gpu[1] == 1]) < 0.1


@pytest.mark.parametrize("win", [(32, 32), (32, 80), (3, 3), (8, 5), (21, 7), (13, 40)])
def test_lk_box_windows_640(oracle_mod, win):
    sc, f0, f1 = scene_pair(2, 640, 480, 48)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3)
    assert_same(gpu, ref, f"win {win}")


@pytest.mark.parametrize("win", [(64, 64), (64, 160), (100, 100)])
def test_lk_box_windows_1080p(oracle_mod, win):
    """Tracker2D-faithful windows at 1080p (box 64x160): multi-tile LDS path."""
    sc, f0, f1 = scene_pair(5, 1920, 1080, 24)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3)
    assert_same(gpu, ref, f"win {win}")


def test_lk_err_sequential_path(oracle_mod):
    """Random (uncorrelated) frames with a large window push sum|diff| over 2^24,
    forcing the sequential float chain for err."""
    rng = np.random.default_rng(9)
    f0 = rng.integers(0, 256, (400, 400), dtype=np.uint8)
    f1 = rng.integers(0, 256, (400, 400), dtype=np.uint8)
    pts = rng.uniform(100, 300, (16, 2)).astype(np.float32)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (100, 100), 1, criteria=(1, 2, 0.0))
    assert np.any(ref[2] * 32 * 100 * 100 > 2 ** 24)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (100, 100), 1, criteria=(1, 2, 0.0))
    assert_same(gpu, ref, "err chain")


@pytest.mark.parametrize("criteria", [(3, 0, 0.01), (1, 5, 0.0), (2, 30, 0.5), (3, 100, 0.0), (3, 30, 0.01)])
def test_lk_criteria(oracle_mod, criteria):
    sc, f0, f1 = scene_pair(4, 320, 240, 64)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (15, 15), 2, criteria=criteria)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (15, 15), 2, criteria=criteria)
    assert_same(gpu, ref, f"criteria {criteria}")


def test_lk_flags(oracle_mod):
    sc, f0, f1 = scene_pair(6, 320, 240, 64)
    pts = sc.points_at(0)
    guess = sc.points_at(1) + 0.7
    ref = oracle_ref(oracle_mod, f0, f1, pts, (15, 15), 2, flags=USE_INITIAL_FLOW, next_pts=guess)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (15, 15), 2, flags=USE_INITIAL_FLOW, next_pts=guess)
    assert_same(gpu, ref, "initial flow")
    ref = oracle_ref(oracle_mod, f0, f1, pts, (15, 15), 2, flags=GET_MIN_EIGENVALS)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (15, 15), 2, flags=GET_MIN_EIGENVALS)
    assert_same(gpu, ref, "min eig")


def test_lk_degenerate_inputs(oracle_mod):
    flat = np.full((120, 160), 77, np.uint8)
    tex = synth.texture(160, 120, 8)
    pts = np.array([[80, 60], [0, 0], [159, 119], [-21, 5], [10, -30], [500, 60]], np.float32)
    for a, b in [(flat, flat), (tex, flat), (tex, np.roll(tex, 40, axis=1))]:
        ref = oracle_ref(oracle_mod, a, b, pts, (9, 9), 3)
        gpu = glk.calc_optical_flow_pyr_lk(a, b, pts, (9, 9), 3)
        assert_same(gpu, ref, "degenerate")


def test_lk_empty_and_errors():
    f = synth.texture(64, 48, 1)
    nxt, st, er = glk.calc_optical_flow_pyr_lk(f, f, np.zeros((0, 2), np.float32), (9, 9), 1)
    assert nxt.shape == (0, 2) and st.shape == (0,)
    with pytest.raises(PsnLkError) as e:
        glk.calc_optical_flow_pyr_lk(f, f, np.zeros((3, 2), np.float32), (2, 9), 1)
    assert e.value.code == -2
    with glk.LKContext(64, 48, ring_slots=2, max_level_cap=1) as ctx:
        ctx.push_frame(0, f)
        ctx.push_frame(1, f)
        q = glk.make_query(0, 1, 0, 1, glk.make_params((9, 9), 3))
        with pytest.raises(PsnLkError) as e:  # 64x48 with 9x9 window needs level 2 > cap 1
            ctx.track([q], np.array([[30, 20]], np.float32))
        assert e.value.code == -6
        q = glk.make_query(0, 5, 0, 1, glk.make_params((9, 9), 1))
        with pytest.raises(PsnLkError) as e:
            ctx.track([q], np.array([[30, 20]], np.float32))
        assert e.value.code == -5
        q = glk.make_query(0, 1, 0, 1, glk.make_params((MAX_WIN_WIDTH + 1, 100), 0))
        with pytest.raises(PsnLkError) as e:  # wider than one LDS row band
            ctx.track([q], np.array([[30, 20]], np.float32))
        assert e.value.code == -8
        q = glk.make_query(0, 1, 0, 1, glk.make_params((4096, 4097), 0))
        with pytest.raises(PsnLkError) as e:  # 2^22 quads: past the kernel's exact quad division
            ctx.track([q], np.array([[30, 20]], np.float32))
        assert e.value.code == -8


def test_lk_batched_queries_ring(oracle_mod):
    """Several calcOpticalFlowPyrLK calls (different windows, slot pairs,
    directions) in ONE launch over a 4-slot ring, as Tracker2D issues them."""
    sc = synth.make_scene(3, 640, 480, 120)
    frames = [sc.frame(t) for t in range(4)]
    pts = np.concatenate([sc.points_at(2), sc.points_at(3), sc.points_at(1)])
    specs = [(2, 3, 0, 40, (21, 21)), (2, 3, 40, 40, (32, 80)), (3, 2, 120, 30, (32, 32)),
             (1, 0, 160, 50, (11, 11)), (0, 1, 210, 150, (21, 21))]
    with glk.LKContext(640, 480, ring_slots=4, max_level_cap=3) as ctx:
        for s, f in enumerate(frames):
            ctx.push_frame(s, f)
        allpts = np.concatenate([pts, sc.points_at(0)[:150]])
        qs = [glk.make_query(a, b, first, n, glk.make_params(win, 3)) for a, b, first, n, win in specs]
        gn, gs, ge = ctx.track(qs, allpts)
    for a, b, first, n, win in specs:
        ref = oracle_ref(oracle_mod, frames[a], frames[b], allpts[first:first + n], win, 3)
        assert_same((gn[first:first + n], gs[first:first + n], ge[first:first + n]), ref, f"query {win}")


@pytest.mark.parametrize("overlap", [False, True])
def test_lk_propagation_sequence(oracle_mod, overlap):
    """Tracklet propagation: frame t's outputs are frame t+1's inputs (with and
    without the ingest stream overlapping pyramid builds with LK)."""
    sc = synth.make_scene(8, 640, 480, 128)
    frames = [sc.frame(t) for t in range(6)]
    p_ref = sc.points_at(0)
    p_gpu = p_ref.copy()
    with glk.LKContext(640, 480, ring_slots=2, max_level_cap=3) as ctx:
        ctx.set_ingest_overlap(overlap)
        ctx.push_frame(0, frames[0])
        for t in range(1, 6):
            ctx.push_frame(t % 2, frames[t])
            q = glk.make_query((t - 1) % 2, t % 2, 0, len(p_gpu), glk.make_params((21, 21), 3))
            g = ctx.track([q], p_gpu)
            r = oracle_ref(oracle_mod, frames[t - 1], frames[t], p_ref, (21, 21), 3)
            assert_same(g, r, f"frame {t}")
            p_gpu, p_ref = g[0], r[0]


@pytest.mark.parametrize("overlap", [0, 1, 2])
def test_lk_device_pointer_path(oracle_mod, overlap):
    import hiprt

    sc, f0, f1 = scene_pair(9, 640, 480, 200)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (21, 21), 3)
    d_f0, d_f1 = hiprt.DeviceBuffer.from_array(f0), hiprt.DeviceBuffer.from_array(f1)
    d_p = hiprt.DeviceBuffer.from_array(pts)
    d_n, d_s, d_e = hiprt.DeviceBuffer(pts.nbytes), hiprt.DeviceBuffer(len(pts)), hiprt.DeviceBuffer(4 * len(pts))
    with glk.LKContext(640, 480, ring_slots=2, max_level_cap=3) as ctx:
        ctx.set_ingest_overlap(overlap)
        ctx.push_frame_device(0, d_f0.addr, 640, 1)
        ctx.push_frame_device(1, d_f1.addr, 640, 1)
        q = glk.make_query(0, 1, 0, len(pts), glk.make_params((21, 21), 3))
        ctx.track_device([q], d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        ctx.sync()
    gpu = (d_n.to_array(pts.shape, np.float32), d_s.to_array(len(pts), np.uint8), d_e.to_array(len(pts), np.float32))
    assert_same(gpu, ref, "device path")


def test_lk_device_empty_query_forms_agree():
    """No queries: the list [] and a prebuilt query_array([]) (one zeroed
    placeholder element, nq = 0) are both a no-op, and the outputs stay untouched."""
    import hiprt

    sc, f0, f1 = scene_pair(9, 640, 480, 16)
    d_f0, d_f1 = hiprt.DeviceBuffer.from_array(f0), hiprt.DeviceBuffer.from_array(f1)
    sentinel = np.full((16, 2), -7.0, np.float32)
    d_p, d_n = hiprt.DeviceBuffer.from_array(sc.points_at(0)), hiprt.DeviceBuffer.from_array(sentinel)
    d_s, d_e = hiprt.DeviceBuffer.from_array(np.full(16, 9, np.uint8)), hiprt.DeviceBuffer(64)
    with glk.LKContext(640, 480, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame_device(0, d_f0.addr, 640, 1)
        ctx.push_frame_device(1, d_f1.addr, 640, 1)
        for qs in ([], glk.query_array([])):
            ctx.track_device(qs, d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        ctx.sync()
    assert np.array_equal(d_n.to_array((16, 2), np.float32), sentinel)
    assert np.all(d_s.to_array(16, np.uint8) == 9)


@pytest.mark.parametrize("env", [{}, {"threads": 128}, {"threads": 64}, {"threads": 512}])
@pytest.mark.parametrize("win", [(21, 21), (9, 9), (64, 64)])
def test_lk_fused_ingest_pipeline(oracle_mod, env, win):
    """Fused ingest (PSN_LK_OVERLAP_FUSED): frame t+1 is pushed before frame t
    is tracked, so its pyramid is built by the tail workgroups of the t-1 -> t
    launch (or, for windows the single-tile kernel does not take, by its own
    launch). Pyramids and propagated points must match the oracle bit for bit."""
    import hiprt

    W, H, R, T = 640, 480, 4, 7
    sc = synth.make_scene(12, W, H, 96)
    frames = [sc.frame(t) for t in range(T)]
    d_frames = [hiprt.DeviceBuffer.from_array(f) for f in frames]
    p_ref = sc.points_at(0)
    n = len(p_ref)
    d_pts = [hiprt.DeviceBuffer.from_array(p_ref), hiprt.DeviceBuffer(p_ref.nbytes)]
    d_s, d_e = hiprt.DeviceBuffer(n), hiprt.DeviceBuffer(4 * n)
    with glk.LKContext(W, H, ring_slots=R, max_level_cap=3, variants=env) as ctx:
        ctx.set_ingest_overlap(2)
        ctx.push_frame_device(0, d_frames[0].addr, W, 1)
        ctx.push_frame_device(1, d_frames[1].addr, W, 1)
        ctx.sync()
        for t in range(1, T):
            if t + 1 < T:
                ctx.push_frame_device((t + 1) % R, d_frames[t + 1].addr, W, 1)  # deferred
            q = glk.make_query((t - 1) % R, t % R, 0, n, glk.make_params(win, 3))
            ctx.track_device([q], d_pts[(t - 1) % 2].addr, d_pts[t % 2].addr, d_s.addr, d_e.addr)
            ctx.sync()
            gpu = (d_pts[t % 2].to_array(p_ref.shape, np.float32), d_s.to_array(n, np.uint8), d_e.to_array(n, np.float32))
            r = oracle_ref(oracle_mod, frames[t - 1], frames[t], p_ref, win, 3)
            assert_same(gpu, r, f"{env} {win} frame {t}")
            p_ref = r[0]
            if t + 1 < T:  # the pyramid built in this launch's tail
                eff = oracle_mod.effective_max_level(W, H, 1, 1, 3)
                for lvl, ref_l in enumerate(oracle_mod.build_pyramid(frames[t + 1], eff + 1)):
                    np.testing.assert_array_equal(ctx.read_level((t + 1) % R, lvl), ref_l, f"pyr {t + 1} level {lvl}")


@pytest.mark.parametrize("ml", [0, 1, 4, 5])
def test_lk_st_overlapped_a_phase_levels(oracle_mod, ml):
    """One-wave single-tile launches at two workgroups per CU compute the finer
    levels' A phase on waves 1-3 beside the iterations (wave 1 takes two levels
    from 5 levels on); bit-identical to the oracle and to the prologue-only
    variant (st_ovl 0) at every level count."""
    sc, f0, f1 = scene_pair(13, 3840, 2160, 200)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (21, 21), ml)
    for env in [{}, {"st_ovl": 0}, {"poison_lds": 1}]:
        gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (21, 21), ml, variants=env)
        assert_same(gpu, ref, f"maxLevel {ml} {env}")


@pytest.mark.parametrize("win", [(24, 24), (16, 40), (32, 32), (24, 16), (21, 21), (9, 15)])
def test_lk_st_unwritten_lds_never_read(oracle_mod, win):
    """With the single-tile launch's LDS filled with pseudo-random words first
    (PSN_LK_VARIANT_POISON_LDS), every window shape -- widths that are multiples
    of 8 (no SSE2 tail class) included -- gives the oracle's bits in both A-phase
    modes: no path reads LDS it did not write."""
    sc, f0, f1 = scene_pair(14, 640, 480, 160)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3)
    for env in [{"poison_lds": 1}, {"poison_lds": 1, "st_ovl": 0}]:
        gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, variants=env)
        assert_same(gpu, ref, f"{win} {env}")


def test_lk_config5_4k_5level(oracle_mod):
    """configs[4] shape on one GPU: 3840x2160, 4096 points, 5-level pyramid."""
    sc, f0, f1 = scene_pair(7, 3840, 2160, 4096)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (21, 21), 4)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (21, 21), 4)
    assert_same(gpu, ref, "4k")


@pytest.mark.parametrize("env", [{}, {"st_ovl": 0}, {"poison_lds": 1}, {"poison_lds": 1, "st_ovl": 0},
                                 {"poison_lds": 1, "onewave": 0}, {"onewave": 0}, {"generic": 1}, {"threads": 64},
                                 {"threads": 128}, {"threads": 512},
                                 {"generic": 1, "threads": 64}])
@pytest.mark.parametrize("flags", [0, ACCUM_SCALAR])
def test_lk_kernel_variants(oracle_mod, env, flags):
    """The single-tile and the tiled kernel, at every workgroup size, give the
    same bits (both are checked against the oracle)."""
    sc, f0, f1 = scene_pair(10, 640, 480, 96)
    pts = sc.points_at(0)
    # one-wave mode row counts: 21x21 -> 7 rows/lane, 9x15 -> 4, 32x32 -> 16,
    # 24x16 -> 8, 7x7 -> 4 (no SSE2 lanes), 12x70 -> 16 (4 px/thread A phase),
    # 40x20 -> 20 rows: multi-wave iterations
    for win in [(21, 21), (9, 15), (32, 32), (24, 16), (7, 7), (12, 70), (40, 20)]:
        ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
        gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags, variants=env)
        assert_same(gpu, ref, f"{env} {win}")


@pytest.mark.parametrize("win", [(21, 21), (64, 64)])
def test_lk_counted_launch(oracle_mod, win):
    """psn_lk_track_device_counted: queries sized for 50 points each process
    the count found on the device (0, 17, 50); the points inside a count match
    the oracle bit for bit, the rest of the outputs stay untouched (single-tile
    and tiled kernels)."""
    import hiprt

    sc, f0, f1 = scene_pair(12, 640, 480, 150)
    pts = sc.points_at(0)
    counts = np.array([0, 17, 50], np.int32)
    d_f0, d_f1 = hiprt.DeviceBuffer.from_array(f0), hiprt.DeviceBuffer.from_array(f1)
    d_p = hiprt.DeviceBuffer.from_array(pts)
    sentinel = np.full(pts.shape, -7.0, np.float32)
    d_n = hiprt.DeviceBuffer.from_array(sentinel)
    d_s, d_e = hiprt.DeviceBuffer.from_array(np.full(len(pts), 9, np.uint8)), hiprt.DeviceBuffer(4 * len(pts))
    d_c = hiprt.DeviceBuffer.from_array(counts)
    with glk.LKContext(640, 480, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame_device(0, d_f0.addr, 640, 1)
        ctx.push_frame_device(1, d_f1.addr, 640, 1)
        qs = [glk.make_query(0, 1, 50 * i, 50, glk.make_params(win, 3)) for i in range(3)]
        ctx.track_device_counted(qs, d_c.addr, d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        ctx.sync()
    g_n, g_s = d_n.to_array(pts.shape, np.float32), d_s.to_array(len(pts), np.uint8)
    g_e = d_e.to_array(len(pts), np.float32)
    for i, c in enumerate(counts):
        lo = 50 * i
        if c:
            ref = oracle_ref(oracle_mod, f0, f1, pts[lo:lo + c], win, 3)
            assert_same((g_n[lo:lo + c], g_s[lo:lo + c], g_e[lo:lo + c]), ref, f"query {i}")
        np.testing.assert_array_equal(g_n[lo + c:lo + 50], sentinel[lo + c:lo + 50])
        assert (g_s[lo + c:lo + 50] == 9).all()


@pytest.mark.parametrize("kernel", ["box", "tiled"])
@pytest.mark.parametrize("win,flags", [((33, 33), 0), ((37, 50), 0), ((70, 45), 0), ((66, 100), 0), ((45, 120), 0),
                                       ((64, 160), 0), ((96, 128), 0), ((64, 64), ACCUM_SCALAR),
                                       ((45, 120), ACCUM_SCALAR), ((64, 64), GET_MIN_EIGENVALS)])
def test_lk_box_kernel_windows(oracle_mod, kernel, win, flags):
    """Box windows above the single-tile size: lk_kernel_bx (units of 4 pixels,
    per-chain prefix exactness) and the row-tiled kernel (variant box=0) against
    the oracle -- SSE2 tails (w % 8), partial quads (w % 4), the scalar build,
    border points."""
    sc, f0, f1 = scene_pair(6, 1920, 1080, 40)
    pts = np.concatenate([sc.points_at(0), np.array([[3, 4], [1915.5, 1077.25], [-20, 500], [960, 1079.5]],
                                                     np.float32)])
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags, variants={"box": int(kernel == "box")})
    assert_same(gpu, ref, f"{kernel} win {win} flags {flags}")


@pytest.mark.parametrize("win", [(21, 21), (64, 64), (64, 160)])
def test_configs2_four_cameras_one_context(oracle_mod, win):
    """BASELINE.json configs[2] on one GPU: 4 cameras x 1920x1080 x 512 points in
    ONE context (camera k owns ring slots [kR, kR+R)), every camera's query in one
    launch, with the OpenCV default window and the Tracker2D box windows
    (64x64 backward, 64x160 forward); each camera against the oracle."""
    W, H, R, C, N = 1920, 1080, 4, 4, 512
    scenes = [synth.make_scene(20 + k, W, H, N) for k in range(C)]
    with glk.LKContext(W, H, ring_slots=R * C, max_level_cap=3) as ctx:
        for k, sc in enumerate(scenes):
            ctx.push_frame(k * R + 1, synth.to_bgr(sc.frame(1)))  # BGR ingest
            ctx.push_frame(k * R + 2, sc.frame(2))
        pts = np.concatenate([sc.points_at(1) for sc in scenes])
        qs = [glk.make_query(k * R + 1, k * R + 2, k * N, N, glk.make_params(win, 3)) for k in range(C)]
        gn, gs, ge = ctx.track(qs, pts)
    for k, sc in enumerate(scenes):
        sl = slice(k * N, (k + 1) * N)
        ref = oracle_ref(oracle_mod, sc.frame(1), sc.frame(2), pts[sl], win, 3)
        assert_same((gn[sl], gs[sl], ge[sl]), ref, f"camera {k} win {win}")


@pytest.mark.parametrize("win", [(21, 21), (64, 64)])
def test_configs3_2048_points(oracle_mod, win):
    """configs[3]'s per-GPU slice: 1 camera x 1920x1080 x 2048 points."""
    sc, f0, f1 = scene_pair(31, 1920, 1080, 2048)
    pts = sc.points_at(0)
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3)
    assert_same(gpu, ref, f"2048 points win {win}")


# ------------------------------------------------------------ large windows

BORDER_PTS_1080 = np.array([[3, 4], [1915.5, 1077.25], [-20, 500], [960, 1079.5], [40, 1060]], np.float32)


@pytest.mark.parametrize("jr", [1, 0])
@pytest.mark.parametrize("win,flags", [((100, 250), 0), ((160, 400), 0), ((200, 200), 0), ((130, 130), 0),
                                       ((111, 277), 0), ((100, 250), ACCUM_SCALAR), ((150, 375), GET_MIN_EIGENVALS)])
def test_lk_large_windows_1080p(oracle_mod, win, flags, jr):
    """Tracker2D box windows above the LDS-resident sizes (PETS-scale pedestrians
    at 1080p: forward w x h, backward w x w) run lk_kernel_lg, bit for bit the
    oracle -- SSE2 tails, the scalar build, min-eigenvalue output, border points;
    with the iterations' J region in LDS where it fits (jr=1) and from the level
    (jr=0, variant lg_jr=0)."""
    sc, f0, f1 = scene_pair(13, 1920, 1080, 24, box_w=win[0], box_h=win[1])
    pts = np.concatenate([sc.points_at(0), BORDER_PTS_1080])
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags, variants={"lg_jr": jr})
    assert_same(gpu, ref, f"win {win} flags {flags} jr {jr}")
    assert ref[1].sum() >= 12


def test_lk_large_window_4k_5level(oracle_mod):
    """SURVEY 8(d)'s 4K tracker box: 128 x 320 windows, 5-level pyramid."""
    sc, f0, f1 = scene_pair(14, 3840, 2160, 16, box_w=128, box_h=320)
    pts = np.concatenate([sc.points_at(0), np.array([[1, 1], [3838.5, 2158.5]], np.float32)])
    ref = oracle_ref(oracle_mod, f0, f1, pts, (128, 320), 4)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (128, 320), 4)
    assert_same(gpu, ref, "4k 128x320")


@pytest.mark.parametrize("win", [(1024, 300), (2048, 200), (212, 300), (4093, 40)])
def test_lk_large_windows_4k_wide(oracle_mod, win):
    """Wide windows at 4K near the large-window kernel's plan limits: 1024 and
    2048 px wide (J from the level: the LDS J region would pass its cap; long
    quad runs per thread and lg_div over 10^5 quads), 212 x 300 (just past the
    80 KB cap where the planner turns the LDS J-region copy off), and 4093 px
    wide (a row band of ~4 KB per I-patch row, quad rows of 1024 + a tail)."""
    sc, f0, f1 = scene_pair(16, 3840, 2160, 4, box_w=min(win[0], 3000), box_h=win[1])
    pts = np.concatenate([sc.points_at(0), np.array([[1920, 1080], [5, 2150]], np.float32)])
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 4)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 4)
    assert_same(gpu, ref, f"4k wide {win}")


@pytest.mark.parametrize("lg_lds,jr", [(0, 1), (4096, 1), (0, 0)])
@pytest.mark.parametrize("flags", [0, ACCUM_SCALAR])
def test_lk_large_kernel_all_shapes(oracle_mod, lg_lds, jr, flags):
    """The large-window kernel forced for every window (variant large=1), with
    its default row bands and with 4 KB bands (many bands per window), the J
    region in LDS and from the level (lg_jr=0)."""
    sc, f0, f1 = scene_pair(15, 640, 480, 40)
    pts = np.concatenate([sc.points_at(0), np.array([[0, 0], [639.5, 479.5], [-8, 200], [320, 485]], np.float32)])
    env = {"large": 1, "lg_jr": jr}
    if lg_lds:
        env["lg_lds"] = lg_lds
    for win in [(21, 21), (3, 3), (9, 15), (33, 33), (64, 64), (45, 120), (37, 50), (100, 60)]:
        ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
        gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags, variants=env)
        assert_same(gpu, ref, f"{env} {win}")


@pytest.mark.parametrize("win,flags,env", [((37, 50), 0, {}), ((64, 160), 0, {}), ((64, 64), ACCUM_SCALAR, {}),
                                           ((45, 120), 0, {}), ((100, 250), 0, {}), ((130, 130), 0, {"lg_jr": 0}),
                                           ((111, 277), GET_MIN_EIGENVALS, {}), ((64, 64), 0, {"large": 1}),
                                           ((33, 33), ACCUM_SCALAR, {"large": 1})])
def test_lk_box_and_large_unwritten_lds_never_read(oracle_mod, win, flags, env):
    """The box and large-window kernels with their LDS filled with pseudo-random
    words first (PSN_LK_VARIANT_POISON_LDS): the oracle's bits -- no path reads
    LDS it did not write (pads, tile ends, record slots, J regions)."""
    sc, f0, f1 = scene_pair(17, 1920, 1080, 24, box_w=win[0], box_h=win[1])
    pts = np.concatenate([sc.points_at(0), BORDER_PTS_1080])
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags, variants={"poison_lds": 1, **env})
    assert_same(gpu, ref, f"poisoned LDS win {win} flags {flags} {env}")


def test_lk_large_err_sequential_path(oracle_mod):
    """Uncorrelated frames and a 160 x 160 window: sum|diff| > 2^24, so err takes
    the ordered chain of the large-window kernel; b and A chains as well."""
    rng = np.random.default_rng(19)
    f0 = rng.integers(0, 256, (480, 480), dtype=np.uint8)
    f1 = rng.integers(0, 256, (480, 480), dtype=np.uint8)
    pts = rng.uniform(100, 380, (12, 2)).astype(np.float32)
    ref = oracle_ref(oracle_mod, f0, f1, pts, (160, 160), 1, criteria=(1, 2, 0.0))
    assert np.any(ref[2] * 32 * 160 * 160 > 2 ** 24)
    gpu = glk.calc_optical_flow_pyr_lk(f0, f1, pts, (160, 160), 1, criteria=(1, 2, 0.0))
    assert_same(gpu, ref, "large err chain")


def test_lk_mixed_window_classes_one_call(oracle_mod):
    """One track call whose queries need four kernel classes (single-tile 21x21,
    box kernel no-tail 64x64 and tail 45x120, large 100x250 and 130x130): each
    class is its own launch; every query matches the oracle, also counted."""
    import hiprt

    W, H = 1920, 1080
    sc = synth.make_scene(16, W, H, 240)
    f0, f1 = sc.frame(0), sc.frame(1)
    pts = sc.points_at(0)
    specs = [(0, 40, (100, 250)), (40, 40, (21, 21)), (80, 40, (64, 64)), (120, 40, (45, 120)),
             (160, 40, (130, 130)), (200, 40, (21, 21))]
    with glk.LKContext(W, H, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame(0, f0)
        ctx.push_frame(1, f1)
        qs = [glk.make_query(0, 1, first, n, glk.make_params(win, 3)) for first, n, win in specs]
        gn, gs, ge = ctx.track(qs, pts)
        counts = np.array([40, 0, 17, 40, 5, 40], np.int32)
        d_p = hiprt.DeviceBuffer.from_array(pts)
        sentinel = np.full(pts.shape, -7.0, np.float32)
        d_n = hiprt.DeviceBuffer.from_array(sentinel)
        d_s, d_e = hiprt.DeviceBuffer.from_array(np.full(len(pts), 9, np.uint8)), hiprt.DeviceBuffer(4 * len(pts))
        d_c = hiprt.DeviceBuffer.from_array(counts)
        ctx.track_device_counted(qs, d_c.addr, d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        ctx.sync()
        cn, cs_ = d_n.to_array(pts.shape, np.float32), d_s.to_array(len(pts), np.uint8)
        ce = d_e.to_array(len(pts), np.float32)
    for (first, n, win), c in zip(specs, counts):
        sl = slice(first, first + n)
        ref = oracle_ref(oracle_mod, f0, f1, pts[sl], win, 3)
        assert_same((gn[sl], gs[sl], ge[sl]), ref, f"query {win}")
        assert_same((cn[first:first + c], cs_[first:first + c], ce[first:first + c]),
                    tuple(r[:c] if r is not None else None for r in ref), f"counted {win}")
        np.testing.assert_array_equal(cn[first + c:first + n], sentinel[first + c:first + n])


@pytest.mark.parametrize("W,H,win,flags,env,kern", [
    (3840, 2160, (128, 128), 0, {}, "lk_kernel_bx<16, true>"),       # configs[4] Run, backward windows
    (3840, 2160, (128, 128), 0, {"poison_lds": 1}, "lk_kernel_bx<16, true>"),
    (1920, 1080, (80, 200), 0, {}, "lk_kernel_bx<16, true>"),        # PETS-sized boxes
    (1920, 1080, (100, 160), 0, {}, "lk_kernel_bx<16, false>"),      # 100 % 8: the scalar-tail chain
    (1920, 1080, (100, 160), 0, {"poison_lds": 1}, "lk_kernel_bx<16, false>"),
    (1920, 1080, (90, 170), ACCUM_SCALAR, {}, "lk_kernel_bx<16, false>"),
    (1920, 1080, (52, 300), GET_MIN_EIGENVALS, {}, "lk_kernel_bx<16, false>"),
    (1920, 1080, (64, 200), 0, {}, "lk_kernel_bx<16, true>"),        # 3,200 units: 12.5 per thread
    (1920, 1080, (72, 160), 0, {}, "lk_kernel_bx<12, true>"),        # 2,880 units: still the 12-unit build
])
def test_lk_box_kernel_16_units(oracle_mod, W, H, win, flags, env, kern):
    """Box windows of 12-16 units of 4 px per thread (<= 4,096 units, two
    workgroups per CU, 208/242 VGPRs, no scratch) run the 16-unit box kernel
    instead of the large-window kernel: the oracle's bits, border points
    included, and the launch's kernel is the one named."""
    from mcmtt_opticalflow_amd import _lib

    sc, f0, f1 = scene_pair(18, W, H, 96, box_w=win[0], box_h=win[1])
    border = BORDER_PTS_1080 * np.float32([W / 1920, H / 1080])
    pts = np.concatenate([sc.points_at(0), border.astype(np.float32)])
    ref = oracle_ref(oracle_mod, f0, f1, pts, win, 3, flags=flags)
    L = _lib.load()
    with glk.LKContext(W, H, ring_slots=1, max_level_cap=3, variants=env) as ctx:
        ctx.enable_timing(4, 1)
        gpu = ctx.calc_optical_flow_pyr_lk(f0, f1, pts, win, 3, flags=flags)
        ctx.sync()
        tags = {_lib.kernel_of_tag(t) for _, t in _lib.timing_launches(L, ctx.handle, 4)}
    assert_same(gpu, ref, f"box16 {win} flags {flags} {env}")
    assert tags == {kern}, tags


@pytest.mark.parametrize("stride", [1, 3])
def test_lk_merged_counted_queries(oracle_mod, stride):
    """Many counted queries of one plan (more than the 32 of a launch's table)
    merge into sub-queries of one launch (LkQueryDev::sub_pts): blocks of 12-point
    capacity 16 points apart, device counts 0..12 at stride `stride`, a window
    change in the middle (a second merged run), an empty query between runs
    (no merge across it), windows of the single-tile, box and large kernels.
    Every point inside a count matches the oracle bit for bit; the rest of every
    block and the gaps stay untouched."""
    import hiprt

    W, H, CAP, GAP = 1920, 1080, 12, 16
    sc, f0, f1 = scene_pair(19, W, H, 1500, box_w=100, box_h=250)
    wins = [(21, 21)] * 30 + [(64, 160)] * 40 + [(100, 250)] * 6 + [(64, 160)] * 14
    nq = len(wins)
    pts = sc.points_at(0)[:GAP * nq]
    rng = np.random.default_rng(5)
    counts = rng.integers(0, CAP + 1, nq).astype(np.int32)
    counts[[3, 31, 77]] = [0, CAP, CAP]
    dc = np.zeros(nq * stride, np.int32)
    dc[::stride] = counts
    sentinel = np.full(pts.shape, -7.0, np.float32)
    d_f0, d_f1 = hiprt.DeviceBuffer.from_array(f0), hiprt.DeviceBuffer.from_array(f1)
    d_p, d_n = hiprt.DeviceBuffer.from_array(pts), hiprt.DeviceBuffer.from_array(sentinel)
    d_s, d_e = hiprt.DeviceBuffer.from_array(np.full(len(pts), 9, np.uint8)), hiprt.DeviceBuffer(4 * len(pts))
    d_c = hiprt.DeviceBuffer.from_array(dc)
    qs = [glk.make_query(0, 1, GAP * i, CAP if i != 50 else 0, glk.make_params(w, 3)) for i, w in enumerate(wins)]
    with glk.LKContext(W, H, ring_slots=2, max_level_cap=3) as ctx:
        ctx.push_frame_device(0, d_f0.addr, W, 1)
        ctx.push_frame_device(1, d_f1.addr, W, 1)
        if stride == 1:
            ctx.track_device_counted(qs, d_c.addr, d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        else:
            ctx.track_device_counted_strided(qs, d_c.addr, stride, d_p.addr, d_n.addr, d_s.addr, d_e.addr)
        ctx.sync()
    g_n, g_s = d_n.to_array(pts.shape, np.float32), d_s.to_array(len(pts), np.uint8)
    g_e = d_e.to_array(len(pts), np.float32)
    for i, (w, c) in enumerate(zip(wins, counts)):
        lo = GAP * i
        c = 0 if i == 50 else int(c)
        if c:
            ref = oracle_ref(oracle_mod, f0, f1, pts[lo:lo + c], w, 3)
            assert_same((g_n[lo:lo + c], g_s[lo:lo + c], g_e[lo:lo + c]), ref, f"query {i} {w}")
        np.testing.assert_array_equal(g_n[lo + c:lo + GAP], sentinel[lo + c:lo + GAP], f"query {i} untouched")
        assert (g_s[lo + c:lo + GAP] == 9).all(), i
