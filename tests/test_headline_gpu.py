"""The headline workload itself under oracle parity: bench.py's own Tracker2D
run (BASELINE.json configs[2] per GPU: 1920x1080 BGR, 4 cameras, 8 detections
x 64 points, box windows, frames pipelined by psn_t2d_group_complete_next,
packed result slots), every frame's stTrack2DResult of every camera compared
bit for bit with oracle/tracker2d_oracle.py's CameraTracker replay of the same
frames (the reference schedule of CPSNWhere_Tracker2D::Run,
psn_where/PSNWhere_Tracker2D.cpp:251-373, with the reference's Munkres).
Also the GridFAST Run and JPEG ingest, and configs[3]'s per-GPU shape.
Parity with OpenCV itself is unpinned."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _verify(*argv, steps, warmup):
    import bench

    args = bench.parse_args(["--verify", "--no-legs", "--no-secondary", "--no-cpu-baseline", "--no-isolated", *argv])
    r = bench.tracker_run(args, steps=steps, warmup=warmup)
    v = bench.verify_tracker(args, r)
    assert v["frames"] == steps + warmup
    return v


def test_headline_configs2_matches_oracle(oracle_mod):
    v = _verify(steps=3, warmup=2)
    assert v["cameras"] == 4 and v["camera_frames_checked"] == 20
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] >= 4 * 8 * 4  # every detection is reported every frame


def test_headline_gridfast_matches_oracle(oracle_mod):
    v = _verify("--features", "gridfast", "--cameras", "2", steps=2, warmup=2)
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] > 0


def test_headline_jpeg_ingest_matches_oracle(oracle_mod):
    pytest.importorskip("PIL")
    v = _verify("--ingest", "jpeg", "--cameras", "2", steps=2, warmup=1)
    assert v["mismatches"] == 0, v["first_mismatch"]


def test_configs3_shape_matches_oracle(oracle_mod):
    """configs[3] per GPU at N = 4: 2 cameras x 32 detections x 64 points (2048 per camera)."""
    v = _verify("--cameras", "2", "--points", "2048", "--boxes", "32", steps=2, warmup=1)
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] >= 2 * 32 * 2


def test_headline_mixed_boxes_matches_oracle(oracle_mod):
    """bench.py --box-dist pets (the mixed_boxes leg): PETS-like per-detection
    boxes, so every frame's LK launches span the box-kernel builds and the
    large-window kernel."""
    v = _verify("--box-dist", "pets", "--cameras", "2", steps=2, warmup=2)
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] >= 2 * 8 * 3


def test_headline_realistic_run_matches_oracle(oracle_mod):
    """bench.py --features gridfast --box-dist pets (the realistic leg): the
    reference Run's per-frame work together -- a masked GridFAST detection per
    detection (PSNWhere_Tracker2D.cpp:735-757) feeding the backward chains with
    box.w x box.w windows (:776-782) and the forward calls with box.w x box.h
    windows (:871-877) on PETS-sized boxes (box kernel and large-window kernel)."""
    v = _verify("--features", "gridfast", "--box-dist", "pets", "--cameras", "2", steps=2, warmup=2)
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] >= 2 * 8 * 2


def test_4k_tracker_run_matches_oracle(oracle_mod):
    """The 4K Tracker2D Run (legs.config4_tracker's shape, scaled down): 3840x2160
    BGR, 128x320 boxes -- the backward chains' 128x128 windows on the 16-unit box
    kernel, the forward 128x320 windows on the large-window kernel, the
    detections of a camera merged into one sub-query launch per class."""
    v = _verify("--width", "3840", "--height", "2160", "--cameras", "2", "--points", "64", "--boxes", "4",
                steps=2, warmup=2)
    assert v["mismatches"] == 0, v["first_mismatch"]
    assert v["objects_checked"] >= 2 * 4 * 3
