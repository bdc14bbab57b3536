"""bench.py's multi-GPU plumbing on CPU: `--gpus N` starts N rank processes
itself (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE set before anything touches
a GPU), the ranks join the gloo control plane, shard the cameras (weak: C per
GPU; strong, SURVEY 8(e): --total-cameras M split over the ranks, index ==
camID order as Associator3D requires, PSNWhere_Associator3D.cpp:1105-1116) and
time with barrier + max-over-ranks. --dry-run skips the GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*argv, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=240, env=e, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    return json.loads(lines[0])


def test_launcher_world2_weak():
    out = _run("--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "1")
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["steps"] == 3
    assert out["cameras_by_rank"] == [[0, 1, 2, 3], [4, 5, 6, 7]]  # configs[2] per GPU


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_strong_configs3(n):
    out = _run("--gpus", str(n), "--dry-run", "--total-cameras", "8", "--points", "2048", "--boxes", "32")
    assert out["n_gpus"] == n and out["scaling"] == "strong"
    per = 8 // n
    assert out["cameras_by_rank"] == [list(range(r * per, r * per + per)) for r in range(n)]


def test_launcher_single_and_bad_split():
    out = _run("--dry-run", "--total-cameras", "8")
    assert out["n_gpus"] == 1 and out["cameras_by_rank"] == [list(range(8))]
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-run",
                        "--total-cameras", "8"], capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert p.returncode != 0  # 8 cameras do not split over 3 ranks: every rank fails, the launcher reports it


def test_algorithmic_bytes_match_survey():
    """SURVEY 8(d)'s per-camera-frame figures (gray input)."""
    sys.path.insert(0, ROOT)
    import bench

    for (w, h, lv, n), exp in [((640, 480, 3, 64), 1902144), ((1920, 1080, 4, 512), 13067952),
                               ((1920, 1080, 4, 2048), 13100208), ((3840, 2160, 5, 4096), 52541616)]:
        pyr, lk = bench.algorithmic_bytes(w, h, lv, n)
        assert pyr + lk == exp
