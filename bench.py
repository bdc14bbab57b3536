#!/usr/bin/env python3
"""Tracker2D LK hot-path benchmark (BASELINE.json metric) on MI355X.

One step = one camera-frame of the per-camera hot path on every rank:
  1. ingest frame t into the camera's device ring + build its 4-level pyramid
     (pyramid_kernel; replaces cvtColor/resize + buildOpticalFlowPyramid,
     PSNWhere_Tracker2D.cpp:257-262, :776-782, :871-877),
  2. pyramidal LK of the camera's 512 tracked points from frame t-1 to t
     (lk_kernel; the calcOpticalFlowPyrLK call), outputs written in place into
     the camera's tracklet slot; the tracked points of t are the inputs of t+1
     (tracklet propagation, no host round trip),
  3. N>1: one RCCL all-gather of the per-camera slots (the hand-off into
     Associator3D, PSNWhere.cpp:264-269).
Workload (BASELINE.json configs[1]): 1 camera per GPU, 1920x1080 gray, 512
points, 4-level pyramid, 21x21 window, default criteria. Inputs are synthetic
(mcmtt_opticalflow_amd/synth.py) and resident in HBM before timing.
--cameras C puts C cameras on every GPU (north_star's "4 x 1080p cameras at
1 GPU" target): their LK queries share ONE launch per frame-set and their
pyramid builds run on the ingest stream beside it.

Single GPU:  python bench.py --steps 200 --warmup 10
Multi GPU:   python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Tracker2D frames/sec (all cameras) + achieved HBM GB/s fraction, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0
TIMING_EVERY = 8  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


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


def render_frames_torch(scene, period, device):
    import numpy as np
    import torch

    from mcmtt_opticalflow_amd import synth

    frames = torch.empty((period, scene.height, scene.width), dtype=torch.uint8, device=device)
    for t in range(period):
        frames[t].copy_(torch.from_numpy(scene.frame(t)))
    return frames


def cpu_baseline(scene, period, npts, win, max_level, budget_s, max_frames):
    """The oracle (reference call schedule: both pyramids + Scharr rebuilt in
    every calcOpticalFlowPyrLK call) on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
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
                      f"oracle/lk_oracle.c with OpenMP over points, {dt:.1f} s"}


def tracker_lk_bytes(w, h, win_w, win_h, npts):
    """Algorithmic bytes of one LK query point over its levels (maxLevel 3, the
    reference's): per level the I window with its Scharr border ((w+3) x (h+3))
    and the J window of one bilinear step ((w+1) x (h+1)), + the point I/O."""
    nlev = 0
    for lev in range(4):
        if (w >> lev) < win_w or (h >> lev) < win_h:
            break
        nlev += 1
    return npts * (max(nlev, 1) * ((win_w + 3) * (win_h + 3) + (win_w + 1) * (win_h + 1)) + 8 + 8 + 1 + 4)


def cpu_tracker_baseline(scene, period, budget_s, max_frames):
    """The oracle Tracker2D restatement (oracle/tracker2d_oracle.py: GridFAST,
    backward chains with LocalSearchKLT, forward LK + matching cost; every
    calcOpticalFlowPyrLK call rebuilds both pyramids, the reference schedule)
    on this host's cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle  # cpu_baseline leg only
    import tracker2d_oracle as T2  # cpu_baseline leg only

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    frames = [scene.frame(t) for t in range(period)]
    ring = [None] * T2.INTERVAL
    prev = []
    n, t0 = 0, None
    for t in range(max_frames + 2):
        if t == 2:
            t0 = time.perf_counter()
        img = frames[ping_pong(t, period)]
        ring = ring[1:] + [img]
        boxes = [T2.Rect(float(np.floor(x)), float(np.floor(y)), float(scene.box_w), float(scene.box_h))
                 for x, y in scene.box_at(ping_pong(t, period))]
        rois = [(int(b.x), int(b.y), int(b.w), int(b.h)) for b in boxes]
        feats, _ = oracle.gridfast_detect(img, rois, seed=t)
        dets = T2.backward_tracking(ring, boxes, feats)
        trackers = [T2.Tracker([b], f) for b, f in prev]
        if ring[-2] is not None:
            T2.forward_tracking(ring, trackers, dets)
        prev = [(d.box, d.sets[0]) for d in dets if d.sets and len(d.sets[0]) >= 4]
        if t >= 2:
            n += 1
            if time.perf_counter() - t0 >= budget_s:
                break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{n} Tracker2D frames of the same synthetic video (oracle/tracker2d_oracle.py + "
                      f"oracle/lk_oracle.c, OpenMP over points; GridFAST restricted to the boxes, cheaper than "
                      f"the reference's full-frame masked detect), {dt:.1f} s"}


def tracker_main(args):
    """--tracker: the Tracker2D flow stage as CPSNWhere_Tracker2D::Run drives it
    (box-derived LK windows, not the 21x21 step of the default run): per frame
    ingest (frames resident in HBM), GridFAST features of every detection,
    3-step backward chains with device LocalSearchKLT, forward LK of every
    tracker + matching cost. --cameras C runs C independent cameras on the GPU,
    one host thread and one flow-stage context (own HIP stream) per camera, so
    their launches overlap (ctypes releases the GIL in every library call)."""
    import ctypes
    import threading

    if args.cameras > 1:
        # every camera's flow stage uses 3 streams (LK, ingest, forward LK); HIP's default of
        # 4 hardware queues would map several cameras' streams onto one queue and serialize them
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(16, 4 * args.cameras))
    import numpy as np
    import torch

    from mcmtt_opticalflow_amd import _lib, synth
    from mcmtt_opticalflow_amd import tracker2d as t2d

    torch.cuda.set_device(0)
    device = torch.device("cuda", 0)
    W, H, B, C = args.width, args.height, args.boxes, max(1, args.cameras)
    L = _lib.load()

    class Camera:
        def __init__(self, cam):
            self.scene = synth.make_scene(cam, W, H, 64 * B, nboxes=B)
            self.frames = render_frames_torch(self.scene, args.period, device)
            self.ft = t2d.FlowTracker(W, H, cam_id=cam)
            self.lkh = self.ft.lk_handle()
            self.prev = []
            self.lk_bytes = 0
            self.features = 0
            self.t = 0

        def step(self, count):
            sc, t = self.scene, self.t
            self.ft.push_frame_device(self.frames[ping_pong(t, args.period)].data_ptr(), W, 1)
            boxes = [(float(np.floor(x)), float(np.floor(y)), float(sc.box_w), float(sc.box_h))
                     for x, y in sc.box_at(ping_pong(t, args.period))]
            dets_in = [t2d.make_detection(b, np.zeros((0, 2), np.float32)) for b in boxes]
            trackers = [t2d.make_tracker([b], f) for b, f in self.prev]
            if args.tracker_split:  # psn_t2d_detect_features, then psn_t2d_track_frame
                dets = self.ft.detect_features(dets_in, seed=t)
                dets_out, _, _ = self.ft.track_frame(dets, trackers)
            else:  # one device pass: GridFAST into the chains, forward beside them
                dets_out, _, _ = self.ft.track_frame_detect(dets_in, trackers, seed=t)
                dets = dets_out
            if count:  # LK points of this frame: backward chain steps (their inputs) + forward
                for d_in, d in zip(dets, dets_out):
                    bw = int(d.box.w)
                    if d.num_boxes >= 1:
                        self.lk_bytes += tracker_lk_bytes(W, H, bw, bw, d_in.num_features)
                    for k in range(1, min(d.num_boxes, 3)):
                        self.lk_bytes += tracker_lk_bytes(W, H, bw, bw, d.set_count[k])
                    self.features += d_in.num_features
                for tr in trackers:
                    self.lk_bytes += tracker_lk_bytes(W, H, int(sc.box_w), int(sc.box_h), tr.num_features)
            self.prev = [(d.box.tuple(), t2d.points(d.sets[0], d.set_count[0])) for d in dets_out
                         if d.valid and d.set_count[0] >= 4]
            self.ft.rotate()
            self.t += 1

    cams = [Camera(c) for c in range(C)]
    torch.cuda.synchronize(device)
    start = threading.Barrier(C + 1)
    done = threading.Barrier(C + 1)
    errors = []

    def run(cam):
        try:
            for _ in range(args.warmup):
                cam.step(False)
            L.psn_lk_enable_timing(cam.lkh, 4 * args.steps + 8, 1)
            start.wait()
            for _ in range(args.steps):
                cam.step(True)
        except Exception as e:  # surfaced after the join
            errors.append(e)
            start.abort()
        finally:
            try:
                done.wait()
            except threading.BrokenBarrierError:
                pass

    threads = [threading.Thread(target=run, args=(c,)) for c in cams]
    for th in threads:
        th.start()
    start.wait()
    t0 = time.perf_counter()
    done.wait()
    elapsed = time.perf_counter() - t0
    for th in threads:
        th.join()
    if errors:
        raise errors[0]
    lk_ms, calls = 0.0, 0
    for cam in cams:
        np_, nt = ctypes.c_int(), ctypes.c_int()
        pm, tm = ctypes.c_double(), ctypes.c_double()
        L.psn_lk_timing_stats(cam.lkh, ctypes.byref(np_), ctypes.byref(pm), ctypes.byref(nt), ctypes.byref(tm))
        lk_ms += tm.value
        calls += nt.value
    lk_bytes = sum(c.lk_bytes for c in cams)
    fps = C * args.steps / elapsed
    achieved = lk_bytes / (lk_ms * 1e-3) / 1e9 if lk_ms > 0 else 0.0
    sc0 = cams[0].scene
    out = {
        "metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
        "config": {"workload": f"Tracker2D mode: {C} camera(s) per GPU, {W}x{H} gray, {B} detections/frame "
                               f"({sc0.box_w}x{sc0.box_h} boxes), GridFAST features (cap 100), 3-step backward "
                               "chains + forward LK with box-derived windows, maxLevel 3, LocalSearchKLT on device",
                   "cameras": C, "cameras_per_gpu": C, "width": W, "height": H, "detections": B,
                   "box": [sc0.box_w, sc0.box_h],
                   "parallelism": f"{C} camera(s) per GPU, one stream each" if C > 1 else "camera-per-GPU x1"},
        "roofline": {"kernel": "lk_kernel_bx (every LK launch of the timed frames)", "bound": "hbm",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": tracker_traffic(args.tracker_pmc_summary),
                     "traffic_unit": "HBM bytes per camera-frame, all lk_kernel_bx launches",
                     "traffic_source": os.path.relpath(args.tracker_pmc_summary, ROOT),
                     "bytes_per_camera_frame": int(lk_bytes / (C * args.steps)),
                     "lk_ms_per_camera_frame": round(lk_ms / (C * args.steps), 4), "lk_calls": calls},
        "features_per_camera_frame": round(sum(c.features for c in cams) / (C * args.steps), 1),
        "cpu_baseline": None,
    }
    for cam in cams:
        cam.ft.close()
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_tracker_baseline(sc0, args.period, args.cpu_budget, 400)
        out["speedup_vs_cpu"] = round(fps / out["cpu_baseline"]["value"], 1)
    print(json.dumps(out), flush=True)



def tracker_traffic(path):
    """PMC HBM bytes per camera-frame of every lk_kernel_bx launch (tools/pmc_summary.py output of a
    --tracker run; one pyramid_kernel launch per camera-frame gives the frame count), or None."""
    if not path or not os.path.exists(path):
        return None
    ks = json.load(open(path)).get("kernels", {})
    frames = ks.get("pyramid_kernel", {}).get("dispatches", 0)
    bx = [v for k, v in ks.items() if k.startswith("lk_kernel_bx")]
    if not frames or not bx:
        return None
    return int(sum(v["hbm_bytes_per_launch"] * v["dispatches"] for v in bx) / frames)

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--points", type=int, default=512)
    ap.add_argument("--levels", type=int, default=4)
    ap.add_argument("--win", type=int, default=21)
    ap.add_argument("--period", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cameras", type=int, default=1, help="cameras per GPU (default 1 = configs[1])")
    ap.add_argument("--sg", action="store_true",
                    help="SG(9, 1) post-filter of every tracked point's trajectory after the LK (configs[4])")
    ap.add_argument("--overlap", choices=["auto", "off", "stream", "fused"], default="auto",
                    help="ingest of frame t+1: serial on the LK stream, on a second stream, or fused "
                         "into the tail of frame t's LK launch (auto: fused for 1 camera per GPU, "
                         "stream for more)")
    ap.add_argument("--tracker-pmc-summary",
                    default=os.path.join(ROOT, "profiles", "r01f_tracker_mode_pmc_summary.json"),
                    help="--tracker: FETCH/WRITE_SIZE summary of a --tracker run for roofline.traffic")
    ap.add_argument("--pmc-summary", default=os.path.join(ROOT, "profiles", "r01f_pmc_summary.json"),
                    help="rocprofv3 FETCH/WRITE_SIZE summary (tools/profile_round.sh) for roofline.traffic")
    ap.add_argument("--tracker", action="store_true",
                    help="Tracker2D mode (box windows, GridFAST, chains; 1 GPU) instead of configs[1]")
    ap.add_argument("--boxes", type=int, default=8, help="--tracker: detections per frame")
    ap.add_argument("--tracker-split", action="store_true",
                    help="--tracker: separate detect_features + track_frame calls (default: track_frame_detect)")
    args = ap.parse_args()
    if args.tracker:
        return tracker_main(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import lk, synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    C = max(1, args.cameras)
    cams = [rank * C + k for k in range(C)]
    W, H, N, L, win = args.width, args.height, args.points, args.levels, args.win
    R = 4  # ring slots per camera, PSN_2D_BACKTRACKING_INTERVAL (PSNWhere_Tracker2D.cpp:16)

    scenes = [synth.make_scene(c, W, H, N) for c in cams]
    scene = scenes[0]
    frames = [render_frames_torch(sc, args.period, device) for sc in scenes]
    # one explicit stream for the library kernels and the torch ops around them
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    # one context holds every local camera's ring: camera k uses slots [k*R, k*R + R)
    ctx = lk.LKContext(W, H, ring_slots=R * C, max_level_cap=L - 1, device=local_rank)
    ctx.set_stream(stream.cuda_stream)
    # frame t+1's pyramid overlaps frame t's LK (fused: built by the LK launch's
    # tail workgroups; stream: on the ingest stream); the frames are resident and
    # complete before timing starts
    overlap = args.overlap if args.overlap != "auto" else ("fused" if C == 1 else "stream")
    mode = {"off": 0, "stream": 1, "fused": 2}[overlap]
    ctx.set_ingest_overlap(mode)

    sb = pdist.slot_bytes(N, C)
    slots = [torch.zeros(sb, dtype=torch.uint8, device=device) for _ in range(2)]
    views = [pdist.slot_views(s, N, C) for s in slots]
    for hdr, nxt, _, _ in views:
        hdr.copy_(torch.tensor([[c, 0, N, 0] for c in cams], dtype=torch.int32).view(hdr.shape))
    views[0][1].copy_(torch.from_numpy(np.concatenate([sc.points_at(0) for sc in scenes])))
    gathered = torch.empty((world, sb), dtype=torch.uint8, device=device)
    params = lk.make_params((win, win), L - 1)

    def push(t):  # frame t of every local camera into its ring
        for k in range(C):
            ctx.push_frame_device(k * R + t % R, frames[k][ping_pong(t, args.period)].data_ptr(), W, 1)

    push(0)
    if mode:
        push(1)
        ctx.sync()
    queries = [[lk.make_query(k * R + (t - 1) % R, k * R + t % R, k * N, N, params) for k in range(C)]
               for t in range(R)]

    sg = None
    if args.sg:  # trajectory post-filter: one SGSmooth Insert per point and frame, same stream
        sg = lk.SGSmoother(C * N, 2, 9, 1, device=local_rank)
        sg.set_stream(stream.cuda_stream)
        sg_ref = torch.empty(C * N, dtype=torch.int32, device=device)
        sg_out = torch.empty((C * N, 9, 2), dtype=torch.float64, device=device)

    def step(t):
        cur, prv = views[t % 2], views[(t - 1) % 2]
        if mode:  # ingest frame t+1 (overlapping this step's LK launch)
            push(t + 1)
        else:  # ingest frame t
            push(t)
        ctx.track_device(queries[t % R], prv[1].data_ptr(), cur[1].data_ptr(), cur[3].data_ptr(),
                         cur[2].data_ptr())
        if sg is not None:  # status as the active mask: lost points are not inserted
            sg.insert_device(cur[1].data_ptr(), 2, cur[3].data_ptr(), sg_ref.data_ptr(), sg_out.data_ptr())
        (cur[0][:, 1] if C > 1 else cur[0][1]).fill_(t)
        if world > 1:
            pdist.allgather_slots(slots[t % 2], world, out=gathered)

    t = 1
    for _ in range(args.warmup):
        step(t)
        t += 1
    # HIP events around every TIMING_EVERY-th LK launch (an event pair costs GPU
    # time, so sampling keeps it from slowing the measured loop)
    ctx.enable_timing(args.steps + 1, TIMING_EVERY)  # syncs the stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(t)
        t += 1
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(elapsed, device)
    ts = ctx.timing_stats()
    tracked = int(views[(t - 1) % 2][3].sum().item())

    pyr_bytes, lk_bytes = algorithmic_bytes(W, H, L, N)
    pyr_us = 1e3 * ts["push_ms"] / max(ts["n_push"], 1) if ts["n_push"] else None
    lk_us = 1e3 * ts["track_ms"] / max(ts["n_track"], 1)
    fps_all = world * C * args.steps / elapsed
    per_gpu_fps = C * args.steps / elapsed
    frame_bytes = pyr_bytes + lk_bytes

    if rank == 0:
        if mode == 2:  # one launch per frame: LK of frame t + pyramid of frame t+1 (+ C-1 separate builds)
            dom = ("lk_kernel_st+fused_pyramid", C * lk_bytes + pyr_bytes, lk_us)
        elif pyr_us is None or lk_us >= pyr_us:
            dom = ("lk_kernel", C * lk_bytes, lk_us)
        else:
            dom = ("pyramid_kernel", pyr_bytes, pyr_us)
        achieved = dom[1] / (dom[2] * 1e-6) / 1e9
        traffic, traffic_src = None, None
        if args.pmc_summary and os.path.exists(args.pmc_summary):
            ks = json.load(open(args.pmc_summary)).get("kernels", {})
            key = "lk_kernel_st" if dom[0].startswith("lk_kernel") and "lk_kernel_st" in ks else dom[0]
            if key in ks:
                traffic = ks[key]["hbm_bytes_per_launch"]
                traffic_src = os.path.relpath(args.pmc_summary, ROOT)
        out = {
            "metric": METRIC,
            "value": round(fps_all, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8+f32",
            "data": "synthetic",
            "config": {
                "workload": (("BASELINE.json configs[1]: 1 camera per GPU"
                              if (C, W, H, N, L, win) == (1, 1920, 1080, 512, 4, 21) else
                              f"{C} camera(s) per GPU" + (" (north_star 4-camera target shape)" if C == 4 else ""))
                             + f", {W}x{H} gray, {N} points, {L}-level pyramid, {win}x{win} window, "
                               "per-frame pyramid build + LK + tracklet propagation"
                             + (", RCCL all-gather of per-camera slots" if world > 1 else "")),
                "cameras": world * C, "cameras_per_gpu": C, "width": W, "height": H, "points_per_camera": N,
                "levels": L, "win": [win, win],
                "parallelism": f"camera-per-GPU x{world}" if C == 1 else f"{C} cameras-per-GPU x{world}",
            },
            "roofline": {
                "kernel": dom[0], "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": dom[1], "avg_launch_us": round(dom[2], 3),
            },
            "kernels_us": {"pyramid_kernel": None if pyr_us is None else round(pyr_us, 3),
                           "lk_kernel": round(lk_us, 3)},
            "ingest_overlap": overlap,
            "sg_post_filter": bool(args.sg),
            "frame_level": {
                "algorithmic_bytes_per_camera_frame": frame_bytes,
                "achieved_GBps_per_gpu": round(frame_bytes * per_gpu_fps / 1e9, 2),
                "hbm_fraction": round(frame_bytes * per_gpu_fps / 1e9 / HBM_PEAK_GBPS, 5),
            },
            "tracked_points_last_frame": tracked,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, args.period, N, (win, win), L - 1, args.cpu_budget, 2000)
            out["speedup_vs_cpu"] = round(fps_all / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if sg is not None:
        sg.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
