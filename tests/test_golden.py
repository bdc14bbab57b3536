"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

They come from this repo's oracle -- the reference holds no fixtures and
OpenCV 2.4.6 is absent, so parity with OpenCV itself is UNPINNED. CPU: the
oracle reproduces them bit for bit (regression pin). GPU: the HIP path
reproduces them bit for bit through the C ABI.
"""
import glob
import os

import numpy as np
import pytest

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if not os.path.basename(p).startswith("jpeg_"))  # LK fixtures (JPEG: tests/test_jpeg.py)


def load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _crit(d):
    c = d["criteria"]
    return (int(c[0]), int(c[1]), float(c[2]))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(oracle_mod, path):
    d = load(path)
    win = tuple(int(x) for x in d["win"])
    nxt, st, err = oracle_mod.calc_optical_flow_pyr_lk(d["prev_img"], d["next_img"], d["prev_pts"], win,
                                                       int(d["max_level"]), criteria=_crit(d), flags=int(d["flags"]),
                                                       accum=int(d["accum"]))
    np.testing.assert_array_equal(nxt, d["next_pts"])
    np.testing.assert_array_equal(st, d["status"])
    np.testing.assert_array_equal(err, d["err"])
    n = len([k for k in d if k.startswith("pyr")])
    for i, lv in enumerate(oracle_mod.build_pyramid(d["prev_img"], n)):
        np.testing.assert_array_equal(lv, d[f"pyr{i}"])


def test_golden_present():
    assert len(GOLDEN) >= 4


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_gpu_reproduces_golden(path):
    from mcmtt_opticalflow_amd import lk
    from mcmtt_opticalflow_amd._lib import ACCUM_SCALAR

    d = load(path)
    win = tuple(int(x) for x in d["win"])
    flags = int(d["flags"]) | (ACCUM_SCALAR if int(d["accum"]) == 1 else 0)
    h, w = d["prev_img"].shape
    n = len([k for k in d if k.startswith("pyr")])
    with lk.LKContext(w, h, ring_slots=2, max_level_cap=n - 1) as ctx:
        ctx.push_frame(0, d["prev_img"])
        for i in range(n):
            np.testing.assert_array_equal(ctx.read_level(0, i), d[f"pyr{i}"])
        nxt, st, err = ctx.calc_optical_flow_pyr_lk(d["prev_img"], d["next_img"], d["prev_pts"], win,
                                                    int(d["max_level"]), _crit(d), flags)
    np.testing.assert_array_equal(nxt, d["next_pts"])
    np.testing.assert_array_equal(st, d["status"])
    np.testing.assert_array_equal(err, d["err"])
