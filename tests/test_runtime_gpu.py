"""On the device: the runtime a process runs the library on, and the RCCL
hand-off class the multi-GPU bench uses.

* A fresh process that loads libpsn_lk.so FIRST runs bench.tracker_run (the
  headline Run, verified bit for bit against the oracle) on ROCm's runtime, and
  torch imported afterwards runs on that same runtime (before psn_runtime.cpp,
  torch mapped a second HIP runtime and its init failed: "No HIP GPUs are
  available"). The reverse order (torch first) binds the library to torch's
  copies; both map one runtime.
* ResultExchange(backend="psn_comm") -- psn_comm_init / psn_comm_allgather on a
  one-rank RCCL communicator, pinned staging, the exchange stream and its events
  -- through the bench's pipelined hand-off (start at step t, wait at t+1),
  every frame's gathered slots checked (PSNWhere.cpp:253-269,
  PSNWhere_Associator3D.cpp:1105-1116: index == camID)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

RUN = r"""
import json, sys
sys.path.insert(0, {root!r})
order = {order!r}
if order == "torch":
    import torch
from mcmtt_opticalflow_amd import _lib
_lib.load()
import bench
args = bench.parse_args(["--verify", "--no-legs", "--no-secondary", "--no-cpu-baseline", "--no-isolated",
                         "--width", "640", "--height", "480", "--cameras", "2", "--points", "128", "--boxes", "2",
                         "--period", "4"])
r = bench.tracker_run(args, steps=3, warmup=2)
v = bench.verify_tracker(args, r)
out = {{"verify": v, "runtime": _lib.runtime_info()}}
if order == "lib":
    import torch  # after the library: binds to the library's runtime
    x = torch.arange(16, dtype=torch.float32, device="cuda")
    out["torch_sum"] = float(x.sum().item())
    out["runtime_after_torch"] = _lib.runtime_info()
print(json.dumps(out, default=str))
"""


def _run(order):
    p = subprocess.run([sys.executable, "-u", "-c", RUN.format(root=ROOT, order=order)], capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_library_first_then_tracker_run_and_torch():
    out = _run("lib")
    v = out["verify"]
    assert v["mismatches"] == 0 and v["camera_frames_checked"] == 2 * 5, v
    rt = out["runtime_after_torch"]
    assert rt["one_runtime"], rt["mapped"]
    assert rt["libamdhip64"].startswith("/opt/rocm"), rt
    assert out["torch_sum"] == 120.0


def test_torch_first_then_tracker_run():
    out = _run("torch")
    v = out["verify"]
    assert v["mismatches"] == 0 and v["camera_frames_checked"] == 2 * 5, v
    assert out["runtime"]["one_runtime"], out["runtime"]["mapped"]


def test_result_exchange_psn_comm_pipelined_one_rank():
    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import tracker2d as t2d

    C, F, depth = 3, 9, 3
    slot = t2d.result_slot_bytes(4, 1)
    ex = pdist.ResultExchange(1, 0, C * slot, device=0, backend="psn_comm", depth=depth)
    send = np.zeros((C, slot), np.uint8)
    want, got, pending = {}, {}, []
    try:
        for t in range(F):
            for cam in range(C):
                objs = [{"id": 100 * cam + t, "box": (float(cam), float(t), 8.0, 16.0),
                         "head": (0.0, 0.0, 0.0, 0.0), "score": 0.25 * cam,
                         "prev": np.full((cam + 1, 2), cam + 0.25 * t, np.float32),
                         "curr": np.full((cam + 2, 2), t + 0.5, np.float32)}]
                t2d.pack_result({"cam_id": cam, "frame_idx": t, "objects": objs, "detection_rects": [],
                                 "tracker_rects": []}, send[cam])
            want[t] = send.copy()
            pending.append((t, ex.start(send)))
            send[:] = 0xEE  # copied by start: the caller's buffer is free at once
            if t == 4:
                with pytest.raises(ValueError):  # a failed start leaves the tickets in flight intact
                    ex.start(np.zeros(7, np.uint8))
            if len(pending) > 1:  # frame t-1's slots consumed at step t
                tt, tk = pending.pop(0)
                got[tt] = np.array(ex.wait(tk), copy=True)
        while pending:
            tt, tk = pending.pop(0)
            got[tt] = np.array(ex.wait(tk), copy=True)
    finally:
        ex.close()
    assert sorted(got) == list(range(F))
    for t in range(F):
        np.testing.assert_array_equal(got[t].reshape(C, slot), want[t])
        rows = got[t].reshape(C, slot)
        for cam in range(C):
            r = t2d.unpack_result(rows[cam], 4, 1)
            assert r["cam_id"] == cam and r["frame_idx"] == t


def test_bench_exchange_flag_one_rank(oracle_mod):
    """bench.py --exchange at N = 1: every frame's result slots go through the
    RCCL exchange (pipelined) and the gathered slots equal the oracle's Run."""
    import bench

    args = bench.parse_args(["--verify", "--exchange", "--no-legs", "--no-secondary", "--no-cpu-baseline",
                             "--no-isolated", "--width", "640", "--height", "480", "--cameras", "2", "--points",
                             "128", "--boxes", "2", "--period", "4"])
    r = bench.tracker_run(args, steps=4, warmup=2)
    v = bench.verify_tracker(args, r)
    assert v["frames"] == 6 and v["mismatches"] == 0, v


WARM = r"""
import ctypes, json, sys
sys.path.insert(0, {root!r})
import numpy as np
from mcmtt_opticalflow_amd import lk as glk, _lib, synth
L = _lib.load()
sc = synth.make_scene(0, 640, 480, 64)
pts = sc.points_at(0).astype(np.float32)
nxt, st, err = glk.calc_optical_flow_pyr_lk(sc.frame(0), sc.frame(1), pts, (21, 21), 3)
ms = ctypes.c_double(-1.0)
rc = L.psn_lk_sdma_warmup_ms(0, ctypes.byref(ms))
print(json.dumps({{"rc": rc, "ms": ms.value, "tracked": int(st.sum()), "n": len(pts)}}))
"""


@pytest.mark.parametrize("warm", ["1", "0"])
def test_sdma_warmup_recorded_and_optional(warm):
    """The first psn_lk_create of a process sets up the SDMA engines and records
    the wall time it took (bounded); PSN_LK_SDMA_WARMUP=0 skips it (the path a
    device whose HSA agent cannot be matched takes) and the context still
    creates and tracks."""
    env = dict(os.environ, PSN_LK_SDMA_WARMUP=warm)
    p = subprocess.run([sys.executable, "-u", "-c", WARM.format(root=ROOT)], capture_output=True, text=True,
                       timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["rc"] == 0, out
    assert 0.0 <= out["ms"] < (5000.0 if warm == "1" else 5.0), out
    assert out["tracked"] > out["n"] // 2, out
