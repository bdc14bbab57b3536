#!/usr/bin/env python3
"""Tracker2D benchmark (BASELINE.json metric) on MI355X.

Default workload = BASELINE.json configs[2] on every GPU (north_star's target
shape, "4x1080p cameras with 512 tracked points/camera at 1 GPU"): C = 4
cameras per rank, 1920x1080 BGR frames, 8 detections per camera (64x160 boxes,
SURVEY 8(d)) with 64 feature points each (512 per camera; SURVEY 8(d) point
recipe: uniform inside the boxes, seed 3000+cam), box-derived LK windows
(64x64 backward, 64x160 forward), maxLevel 3.

One step = one frame of every camera through CPSNWhere_Tracker2D::Run
(psn_where/PSNWhere_Tracker2D.cpp:251-373) as psn_t2d_group runs it:
  1. upload of frame t+1 of every camera from pinned host memory (copy engine)
     + BGR->gray + pyramid build, overlapping frame t's work (:256-263);
  2. backward chains of every detection: 3 LK steps (64x64) with LocalSearchKLT
     between them, all cameras in one launch per step (:763-811);
  3. forward LK of every active tracker (64x160) + matching cost (:851-1025);
  4. assignment, tracker update, ResultWithTracker (:1038-1164, :1231-1257);
  5. every camera's stTrack2DResult packed into its binary slot in host memory.
     Frames are pipelined as psn_t2d_group_complete_next allows: frame t+1's
     backward chains are enqueued as soon as frame t's device work is done, and
     run while the host does frame t's step 4-5 (same results as launch/complete);
     N > 1: one RCCL all-gather of the slots over xGMI (psn_comm_allgather, the
     hand-off into Associator3D, PSNWhere.cpp:264-269), landing in host memory.
The timed region therefore runs from host frames to host results.

--mode kernel: the round-1 line, BASELINE.json configs[1] (1 camera, 512
points, 21x21 window, frames resident in HBM), also reported as `secondary`.

Single GPU:  python bench.py --steps 100 --warmup 5
Multi GPU:   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import ctypes
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Tracker2D frames/sec (all cameras) + achieved HBM GB/s fraction, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
TIMING_EVERY = 8


def level_sizes(w, h, nlev):
    out = []
    for _ in range(nlev):
        out.append((w, h))
        w, h = (w + 1) // 2, (h + 1) // 2
    return out


def algorithmic_bytes(w, h, nlev, npts, c_in=1):
    """B = c_in*S0 + 4*S_pyr - S_{L-1} + 21*N per camera-frame,
    split per kernel: pyramid = c_in*S0 + S_pyr (write) + (S_pyr - S_{L-1})
    (pyrDown reads); LK = 2*S_pyr (I and J pyramids read once) + 21*N."""
    sz = [a * b for a, b in level_sizes(w, h, nlev)]
    s_pyr = sum(sz)
    pyr = c_in * sz[0] + s_pyr + (s_pyr - sz[-1])
    lk = 2 * s_pyr + 21 * npts
    return pyr, lk


def ping_pong(t, period):
    """Frame index of step t in a 0..P-1..0 sequence (keeps boxes in view)."""
    m = t % (2 * (period - 1))
    return m if m < period else 2 * (period - 1) - m


def host_info():
    """nproc, the CPU share this process may use, the CPU model (lscpu)."""
    info = {"nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
    except Exception:  # lscpu missing: platform's best effort
        info["cpu_model"] = platform.processor() or None
    return info


def cpu_threads():
    """The host cores this run may use: the affinity set, capped by OMP_NUM_THREADS
    when the box sets it (the GPU box allots 16 host cores per GPU)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


# ---------------------------------------------------------------------------
# Tracker2D mode (default): configs[2] on every rank
# ---------------------------------------------------------------------------

import numpy as np  # noqa: E402


class CameraFeed:
    """One camera's synthetic video (mcmtt_opticalflow_amd/synth.py): BGR frames
    in pinned host memory and, per frame, the detections (box, head box, 3D
    estimate) with their feature points."""

    def __init__(self, cam, W, H, npts, nboxes, period, t2d, pinned, jpeg=False):
        from mcmtt_opticalflow_amd import synth

        self.scene = synth.make_scene(cam, W, H, npts, nboxes=nboxes)
        self.period = period
        self.jpeg = None
        if jpeg:  # the camera's frames as baseline JPEG files (PIL/libjpeg-turbo, q90, 4:2:0, a restart per MCU row)
            import io

            from PIL import Image

            self.jpeg = []
            for t in range(period):
                b = io.BytesIO()
                Image.fromarray(synth.to_bgr(self.scene.frame(t))[..., ::-1]).save(
                    b, "JPEG", quality=90, subsampling=2, restart_marker_rows=1)
                buf = pinned((len(b.getvalue()),))
                buf[:] = np.frombuffer(b.getvalue(), np.uint8)
                self.jpeg.append(buf)
            self.frames = None
        else:
            self.frames = [pinned((H, W, 3)) for _ in range(period)]
            for t in range(period):
                self.frames[t][...] = synth.to_bgr(self.scene.frame(t))
        self.boxes, self.feats = [], []
        for t in range(period):
            bx = [(float(int(x)), float(int(y)), float(self.scene.box_w), float(self.scene.box_h))
                  for x, y in self.scene.box_at(t)]
            pts = self.scene.points_at(t)
            self.boxes.append(bx)
            self.feats.append([pts[self.scene.pt_box == k] for k in range(nboxes)])
        self.t2d = t2d

    def detections(self, t):
        """Fresh records of frame t (the group writes its outputs into them)."""
        f = ping_pong(t, self.period)
        out = []
        for b, pts in zip(self.boxes[f], self.feats[f]):
            head = (b[0] + b[2] / 4, b[1], b[2] / 2, b[3] / 8)
            loc = ((b[0] + b[2] / 2) * 10.0, (b[1] + b[3]) * 10.0, 0.0)  # a ground-plane stand-in, mm
            out.append(self.t2d.make_detection(b, pts, head=head, location=loc, height=1700.0))
        return out

    def frame(self, t):
        return self.frames[ping_pong(t, self.period)]

    def push(self, group, k, t):
        """Camera k's frame t into the group (async upload of BGR, or JPEG bytes decoded on the device)."""
        if self.jpeg is not None:
            group.push_frame_jpeg(k, self.jpeg[ping_pong(t, self.period)])
        else:
            group.push_frame(k, self.frame(t))


def pinned_allocator():
    import numpy as np
    import torch

    keep = []

    def alloc(shape):
        t = torch.empty(shape, dtype=torch.uint8).pin_memory()
        keep.append(t)
        return t.numpy()

    alloc.keep = keep
    _ = np
    return alloc


def tracker_cpu_baseline(args, n_frames_cap=400):
    """The oracle Tracker2D (oracle/tracker2d_oracle.py CameraTracker + oracle/lk_oracle.c)
    on this host: the same synthetic cameras, detections and points, the
    reference call schedule (every calcOpticalFlowPyrLK rebuilds both pyramids),
    OpenMP over points as OpenCV's parallel_for_. Legs: the allotted host cores,
    1 thread, and the shared-pyramid schedule at the allotted cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle  # cpu_baseline leg only
    import tracker2d_oracle as T2  # cpu_baseline leg only
    from mcmtt_opticalflow_amd import synth

    W, H, C = args.width, args.height, args.cameras
    scenes = [synth.make_scene(c, W, H, args.points, nboxes=args.boxes) for c in range(C)]
    grays = [[oracle.bgr2gray(synth.to_bgr(sc.frame(t))) for t in range(args.period)] for sc in scenes]

    def leg(threads, shared, budget):
        T2.NTHREADS, T2.SHARED_PYRAMIDS = threads, shared
        cams = [T2.CameraTracker(c) for c in range(C)]
        n, t0 = 0, None
        for t in range(n_frames_cap + 2):
            if t == 2:  # the ring holds frames: the steady state starts
                t0 = time.perf_counter()
            f = ping_pong(t, args.period)
            for c, sc in enumerate(scenes):
                bx = [T2.Rect(float(int(x)), float(int(y)), float(sc.box_w), float(sc.box_h)) for x, y in sc.box_at(f)]
                pts = sc.points_at(f)
                feats = [pts[sc.pt_box == k] for k in range(args.boxes)]
                extra = [(T2.Rect(b.x + b.w / 4, b.y, b.w / 2, b.h / 8), ((b.x + b.w / 2) * 10.0, (b.y + b.h) * 10.0, 0.0),
                          1700.0) for b in bx]
                cams[c].run(grays[c][f], bx, feats, t, extra)
                if t >= 2:
                    n += 1
            if t0 is not None and time.perf_counter() - t0 >= budget:
                break
        dt = time.perf_counter() - t0
        T2.NTHREADS, T2.SHARED_PYRAMIDS = 0, False
        return n / dt, n, dt

    threads = cpu_threads()
    v, n, dt = leg(threads, False, args.cpu_budget)
    v1, n1, dt1 = leg(1, False, args.cpu_budget / 2)
    vs, ns, dts = leg(threads, True, args.cpu_budget / 2)
    hi = host_info()
    return {"value": round(v, 4), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} camera-frames ({C} cameras x {n // C} frames, {dt:.1f} s) of the same workload "
                      "(1080p BGR->gray, 8 detections x 64 points, box windows, backward chains + forward + "
                      "matching) through oracle/tracker2d_oracle.py + oracle/lk_oracle.c, OpenMP over points, "
                      "reference call schedule (both pyramids rebuilt in every calcOpticalFlowPyrLK)",
            "single_thread": round(v1, 4), "single_thread_sample": f"{n1} camera-frames, {dt1:.1f} s",
            "shared_pyramid": round(vs, 4), "shared_pyramid_sample": f"{ns} camera-frames, {dts:.1f} s, {threads} threads",
            "cores_note": "threads = the host cores this GPU's job is allotted (the box sets OMP_NUM_THREADS to its "
                          "per-GPU CPU share; nproc counts the whole machine)",
            **hi}


def tracker_main(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    from mcmtt_opticalflow_amd import _lib
    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import tracker2d as t2d

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:  # control plane (barriers, the RCCL id, max-over-ranks) on gloo; data plane on psn_comm (RCCL)
        dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)
    W, H, C = args.width, args.height, args.cameras
    cams = [rank * C + k for k in range(C)]
    L = _lib.load()
    pinned = pinned_allocator()
    feeds = [CameraFeed(c, W, H, args.points, args.boxes, args.period, t2d, pinned, jpeg=args.ingest == "jpeg")
             for c in cams]
    max_obj = 2 * args.boxes
    group = t2d.Group(W, H, cams, device=local_rank, max_objects=max_obj)
    slot_bytes = t2d.result_slot_bytes(max_obj, 1)
    send = pinned((C, slot_bytes))
    exch = pdist.ResultExchange(world, rank, C * slot_bytes, device=local_rank) if world > 1 else None
    T = t2d.load()

    def step(t, dets, next_dets):
        group.launch(t, dets)  # after complete_next(t-1): a confirmation (frame t is in flight)
        for k, fd in enumerate(feeds):  # frame t+1 uploads while frame t runs
            fd.push(group, k, t + 1)
        if next_dets is None:
            group.complete_raw()
        else:  # frame t+1's chains go to the GPU before the host matches frame t
            group.complete_next(t + 1, next_dets, raw=True)
        for k in range(C):  # the hand-off slots (psn_t2d_pack_result) in host memory
            rc = T.psn_t2d_pack_result(ctypes.byref(group.result_struct(k)), send[k].ctypes.data, slot_bytes)
            if rc:
                raise t2d.T2dError(rc, "psn_t2d_pack_result")
        return exch.allgather(send) if exch else send

    def all_dets(t):
        return [fd.detections(t) for fd in feeds]

    for k, fd in enumerate(feeds):
        fd.push(group, k, 0)
    t = 0
    dets_warm = [all_dets(t + i) for i in range(args.warmup)]
    # records built outside the timed region; one more frame: the last timed step launches its chains
    # ahead, as the warm-up's last step did for the first timed frame (the timed region holds exactly
    # `steps` frames' backward chains and forward calls)
    dets_timed = [all_dets(args.warmup + i) for i in range(args.steps + 1)]
    seq = [group.records(d) for d in dets_warm + dets_timed]  # ctypes records, built before timing
    for i in range(args.warmup):
        step(t, seq[i], seq[i + 1] if i + 1 < len(seq) else None)
        t += 1
    lkh = group.lk_handle()
    L.psn_lk_enable_timing(lkh, 16 * args.steps + 64, 1)  # every LK launch (forward + 3 chain steps)
    sampler = SampleCounter(L, lkh)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        j = args.warmup + i
        gathered = step(t, seq[j], seq[j + 1])
        t += 1
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(elapsed)
    ts = {}
    np_, nt, pm, tm = ctypes.c_int(), ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
    L.psn_lk_timing_stats(lkh, ctypes.byref(np_), ctypes.byref(pm), ctypes.byref(nt), ctypes.byref(tm))
    ts = {"n_track": nt.value, "track_ms": tm.value, "n_push": np_.value, "push_ms": pm.value}
    samples = sampler.read()
    # the gathered hand-off of the last frame: every camera's result, index == camID
    objs_last = 0
    if rank == 0:
        rows = np.asarray(gathered).reshape(world * C, slot_bytes)
        for cam in range(world * C):
            r = t2d.unpack_result(rows[cam], max_obj, 1)
            assert r["cam_id"] == cam and r["frame_idx"] == t - 1, (cam, r["cam_id"], r["frame_idx"])
            objs_last += len(r["objects"])
    group.close()
    if exch:
        exch.close()

    fps_all = world * C * args.steps / elapsed
    per_gpu_fps = C * args.steps / elapsed
    pyr_b, lk_b = algorithmic_bytes(W, H, 4, args.points, c_in=3)
    frame_b = pyr_b + lk_b
    cam_frames_rank = C * args.steps
    lk_ms_cf = ts["track_ms"] / cam_frames_rank  # LK kernel time per camera-frame (all launches, HIP events)
    lk_gbps = lk_b / (lk_ms_cf * 1e-3) / 1e9 if lk_ms_cf > 0 else 0.0
    out = None
    if rank == 0:
        pmc = tracker_traffic(args.tracker_pmc_summary, cam_frames_per_set=C)
        out = {
            "metric": METRIC, "value": round(fps_all, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
            "config": {
                "workload": (f"BASELINE.json configs[2] per GPU: {C} cameras x 1920x1080 BGR, {args.boxes} detections/camera "
                             f"(64x160 boxes) x {args.points // args.boxes} points = {args.points} tracked points/camera, "
                             "CPSNWhere_Tracker2D::Run: async H2D ingest from pinned host + BGR->gray + pyramid, "
                             "3-step backward chains (64x64 windows, LocalSearchKLT on device), forward LK (64x160) "
                             "+ matching cost, assignment + tracker update + ResultWithTracker, packed result slots "
                             "in host memory" + (", RCCL all-gather of the slots (psn_comm)" if world > 1 else ""))
                if (W, H, C, args.points, args.boxes) == (1920, 1080, 4, 512, 8) else
                f"Tracker2D Run, {C} cameras/GPU, {W}x{H}, {args.boxes} detections x {args.points // args.boxes} points",
                "cameras": world * C, "cameras_per_gpu": C, "width": W, "height": H, "points_per_camera": args.points,
                "detections_per_camera": args.boxes, "box": [64, 160], "levels": 4,
                "win_backward": [64, 64], "win_forward": [64, 160],
                "ingest": ("baseline JPEG files in host memory (q90 4:2:0, restart per MCU row), decoded on the device"
                           if args.ingest == "jpeg" else "BGR frames in pinned host memory"),
                "parallelism": f"{C} cameras-per-GPU x{world} (camera-sharded, RCCL all-gather of result slots)"},
            "roofline": {
                "kernel": "lk_kernel_bx (every LK launch of a frame-set: forward + 3 chain steps)",
                "bound": "hbm", "limiter": "latency / VALU (ordered float chains of the box-window sums)",
                "achieved": round(lk_gbps, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(lk_gbps / HBM_PEAK_GBPS, 6),
                "traffic": pmc, "traffic_unit": "HBM bytes per camera-frame over all LK launches (PMC)",
                "traffic_source": os.path.relpath(args.tracker_pmc_summary, ROOT) if pmc else None,
                "bytes_per_camera_frame": lk_b,
                "bytes_note": "SURVEY 8(d) LK bytes 2*S_pyr + 21*N per camera-frame over the summed LK launch time",
                "lk_ms_per_camera_frame": round(lk_ms_cf, 5), "lk_launches": ts["n_track"]},
            "frame_level": {"algorithmic_bytes_per_camera_frame": frame_b,
                            "bytes_formula": "SURVEY 8(d) c_in*S0 + 4*S_pyr - S_top + 21*N, c_in = 3 (BGR)",
                            "achieved_GBps_per_gpu": round(frame_b * per_gpu_fps / 1e9, 3),
                            "hbm_fraction": round(frame_b * per_gpu_fps / 1e9 / HBM_PEAK_GBPS, 6)},
            "compute": {"window_samples_per_camera_frame": round(samples / cam_frames_rank) if samples else None,
                        "gsamples_per_s_per_gpu": round(samples / cam_frames_rank * per_gpu_fps / 1e9, 3)
                        if samples else None,
                        "definition": "SURVEY 8(d): sum over points and levels of w*h*(1 + iterations), "
                                      "counted on the device"},
            "frames_per_set_per_s": round(args.steps / elapsed, 2),
            "result_objects_last_frame": objs_last,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = tracker_cpu_baseline(args)
            out["speedup_vs_cpu"] = round(fps_all / out["cpu_baseline"]["value"], 1)
            out["speedup_vs_cpu_shared_pyramid"] = round(fps_all / out["cpu_baseline"]["shared_pyramid"], 1)
        if world == 1 and not args.no_secondary:
            out["secondary"] = kernel_secondary(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


class SampleCounter:
    """Device-side window-sample counter of the LK launches (psn_lk_debug_count_samples)."""

    def __init__(self, L, lkh):
        self.L, self.h = L, lkh
        self.ok = L.psn_lk_debug_count_samples(lkh, 1) == 0

    def read(self):
        if not self.ok:
            return None
        v = ctypes.c_ulonglong()
        rc = self.L.psn_lk_debug_read_samples(self.h, ctypes.byref(v))
        self.L.psn_lk_debug_count_samples(self.h, 0)
        return v.value if rc == 0 else None


def tracker_traffic(path, cam_frames_per_set):
    """PMC HBM bytes per camera-frame over every LK launch of a profiled default run
    (tools/pmc_summary.py output; pyramid_kernel dispatches count camera-frames)."""
    if not path or not os.path.exists(path):
        return None
    ks = json.load(open(path)).get("kernels", {})
    frames = ks.get("pyramid_kernel", {}).get("dispatches", 0)
    lk = [v for k, v in ks.items() if k.startswith("lk_kernel")]
    if not frames or not lk:
        return None
    return int(sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in lk) / frames)


# ---------------------------------------------------------------------------
# Kernel mode: BASELINE.json configs[1] (the round-1 headline, kept as secondary)
# ---------------------------------------------------------------------------

def kernel_cpu_baseline(scene, period, npts, win, max_level, budget_s, max_frames):
    """The oracle (reference call schedule: both pyramids + Scharr rebuilt in
    every calcOpticalFlowPyrLK call) on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only

    threads = cpu_threads()
    frames = [scene.frame(t) for t in range(period)]
    pts = scene.points_at(0)
    oracle.calc_optical_flow_pyr_lk(frames[0], frames[1], pts, win, max_level, nthreads=threads)  # warm
    n = 0
    t0 = time.perf_counter()
    while n < max_frames:
        a, b = frames[ping_pong(n, period)], frames[ping_pong(n + 1, period)]
        pts, _, _ = oracle.calc_optical_flow_pyr_lk(a, b, pts, win, max_level, nthreads=threads)
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} camera-frames of the same workload (1920x1080, {npts} pts, 21x21, 4 levels), "
                      f"oracle/lk_oracle.c with OpenMP over points, {dt:.1f} s", **host_info()}


def kernel_run(args, steps, warmup, world=1, rank=0, local_rank=0):
    """configs[1]-style LK step: frames resident in HBM, C cameras per GPU, 21x21."""
    import numpy as np
    import torch

    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import lk, synth

    device = torch.device("cuda", local_rank)
    C = max(1, args.kcameras)
    cams = [rank * C + k for k in range(C)]
    W, H, N, Lv, win = args.width, args.height, args.kpoints, 4, 21
    R = 4
    scenes = [synth.make_scene(c, W, H, N) for c in cams]
    frames = []
    for sc in scenes:
        f = torch.empty((args.period, H, W), dtype=torch.uint8, device=device)
        for t in range(args.period):
            f[t].copy_(torch.from_numpy(sc.frame(t)))
        frames.append(f)
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    ctx = lk.LKContext(W, H, ring_slots=R * C, max_level_cap=Lv - 1, device=local_rank)
    ctx.set_stream(stream.cuda_stream)
    mode = 2 if C == 1 else 1
    ctx.set_ingest_overlap(mode)
    sb = pdist.slot_bytes(N, C)
    slots = [torch.zeros(sb, dtype=torch.uint8, device=device) for _ in range(2)]
    views = [pdist.slot_views(s, N, C) for s in slots]
    for hdr, nxt, _, _ in views:
        hdr.copy_(torch.tensor([[c, 0, N, 0] for c in cams], dtype=torch.int32).view(hdr.shape))
    views[0][1].copy_(torch.from_numpy(np.concatenate([sc.points_at(0) for sc in scenes])))
    gathered = torch.empty((world, sb), dtype=torch.uint8, device=device)
    params = lk.make_params((win, win), Lv - 1)

    def push(t):
        for k in range(C):
            ctx.push_frame_device(k * R + t % R, frames[k][ping_pong(t, args.period)].data_ptr(), W, 1)

    push(0)
    push(1)
    ctx.sync()
    queries = [[lk.make_query(k * R + (t - 1) % R, k * R + t % R, k * N, N, params) for k in range(C)]
               for t in range(R)]

    def step(t):
        cur, prv = views[t % 2], views[(t - 1) % 2]
        push(t + 1)
        ctx.track_device(queries[t % R], prv[1].data_ptr(), cur[1].data_ptr(), cur[3].data_ptr(), cur[2].data_ptr())
        (cur[0][:, 1] if C > 1 else cur[0][1]).fill_(t)
        if world > 1:
            pdist.allgather_slots(slots[t % 2], world, out=gathered)

    t = 1
    for _ in range(warmup):
        step(t)
        t += 1
    ctx.enable_timing(steps + 1, TIMING_EVERY)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(t)
        t += 1
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    ts = ctx.timing_stats()
    ctx.close()
    torch.cuda.set_stream(torch.cuda.default_stream(device))
    pyr_b, lk_b = algorithmic_bytes(W, H, Lv, N)
    lk_us = 1e3 * ts["track_ms"] / max(ts["n_track"], 1)
    launch_b = C * lk_b + (pyr_b if mode == 2 else 0)
    return {"fps": C * steps / elapsed, "ms_per_step": 1e3 * elapsed / steps, "lk_us": lk_us,
            "launch_bytes": launch_b, "frame_bytes": pyr_b + lk_b, "scene": scenes[0], "elapsed": elapsed,
            "mode": mode}


def kernel_secondary(args):
    r = kernel_run(args, 400, 20)
    ach = r["launch_bytes"] / (r["lk_us"] * 1e-6) / 1e9
    return {"workload": "BASELINE.json configs[1]: 1 camera, 1920x1080 gray resident in HBM, 512 points, 4 levels, "
                        "21x21 window, fused pyramid build + LK + propagation",
            "value": round(r["fps"], 2), "unit": "frames/s", "ms_per_step": round(r["ms_per_step"], 5),
            "roofline": {"kernel": "lk_kernel_st+fused_pyramid", "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 5), "bytes_per_launch": r["launch_bytes"],
                         "avg_launch_us": round(r["lk_us"], 3)}}


def kernel_main(args):
    import torch
    import torch.distributed as dist

    from mcmtt_opticalflow_amd import dist as pdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
        dist.barrier()
    r = kernel_run(args, args.steps, args.warmup, world, rank, local_rank)
    elapsed = pdist.max_over_ranks(r["elapsed"], device)
    C = max(1, args.kcameras)
    fps_all = world * C * args.steps / elapsed
    if rank == 0:
        ach = r["launch_bytes"] / (r["lk_us"] * 1e-6) / 1e9
        traffic = None
        if args.pmc_summary and os.path.exists(args.pmc_summary):
            ks = json.load(open(args.pmc_summary)).get("kernels", {})
            if "lk_kernel_st" in ks:
                traffic = ks["lk_kernel_st"]["hbm_bytes_per_launch"]
        out = {"metric": METRIC, "value": round(fps_all, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 5), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
               "config": {"workload": f"BASELINE.json configs[1] shape: {C} camera(s) per GPU, {args.width}x{args.height} "
                                      f"gray resident in HBM, {args.kpoints} points, 4 levels, 21x21 window",
                          "cameras": world * C, "cameras_per_gpu": C, "parallelism": f"camera-per-GPU x{world}"},
               "roofline": {"kernel": "lk_kernel_st" + ("+fused_pyramid" if r["mode"] == 2 else ""), "bound": "hbm",
                            "limiter": "latency (serial iteration chains)",
                            "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": traffic,
                            "bytes_per_launch": r["launch_bytes"], "avg_launch_us": round(r["lk_us"], 3)},
               "cpu_baseline": None}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = kernel_cpu_baseline(r["scene"], args.period, args.kpoints, (21, 21), 3,
                                                      args.cpu_budget, 2000)
            out["speedup_vs_cpu"] = round(fps_all / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["tracker", "kernel"], default="tracker")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cameras", type=int, default=4, help="tracker mode: cameras per GPU (configs[2]: 4)")
    ap.add_argument("--points", type=int, default=512, help="tracker mode: feature points per camera")
    ap.add_argument("--boxes", type=int, default=8, help="tracker mode: detections per camera")
    ap.add_argument("--ingest", choices=["bgr", "jpeg"], default="bgr",
                    help="tracker mode: frames arrive as BGR arrays (default) or as JPEG files (device decode)")
    ap.add_argument("--kcameras", type=int, default=1, help="kernel mode: cameras per GPU")
    ap.add_argument("--kpoints", type=int, default=512, help="kernel mode: points per camera")
    ap.add_argument("--period", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--tracker-pmc-summary", default=os.path.join(ROOT, "profiles", "r02k_tracker_pmc_summary.json"),
                    help="PMC FETCH/WRITE_SIZE summary of a default (tracker) run, for roofline.traffic")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "r02k_kernel_mode_pmc_summary.json"),
                    help="PMC summary of a kernel-mode run, for roofline.traffic")
    args = ap.parse_args()
    if args.mode == "kernel":
        return kernel_main(args)
    if args.points % args.boxes:
        raise SystemExit("--points must be a multiple of --boxes")
    return tracker_main(args)


if __name__ == "__main__":
    main()
