#!/usr/bin/env python3
"""Tracker2D benchmark (BASELINE.json metric) on MI355X.

Default line = BASELINE.json configs[2] on every GPU (north_star's target
shape, "4x1080p cameras with 512 tracked points/camera at 1 GPU"): C = 4
cameras per rank, 1920x1080 BGR frames, 8 detections per camera (64x160 boxes,
SURVEY 8(d)) with 64 feature points each (512 per camera; SURVEY 8(d) point
recipe: uniform inside the boxes, seed 3000+cam), box-derived LK windows
(64x64 backward, 64x160 forward), maxLevel 3. Per-GPU work is fixed as N grows
(scaling "weak"), so SCALE's N=1 equals BENCH.

One step = one frame of every camera through CPSNWhere_Tracker2D::Run
(psn_where/PSNWhere_Tracker2D.cpp:251-373) as psn_t2d_group runs it:
  1. upload of frame t+2 of every camera from pinned host memory (copy engine)
     + BGR->gray + pyramid build, overlapping frame t's work (:256-263; two
     frames staged ahead, --stage-ahead);
  2. features of every detection: given (SURVEY 8(d) point recipe) or GridFAST
     on the device (--features gridfast, :735-758);
  3. backward chains of every detection: 3 LK steps (64x64) with LocalSearchKLT
     between them, all cameras in one launch per step (:763-811);
  4. forward LK of every active tracker (64x160) + matching cost (:851-1025);
  5. the reference's Munkres assignment, tracker update, ResultWithTracker
     (:1038-1164, :1231-1257);
  6. every camera's stTrack2DResult packed into its binary slot in host memory;
     N > 1: one RCCL all-gather of the slots over xGMI (psn_comm_allgather, the
     hand-off into Associator3D, PSNWhere.cpp:264-269), landing in host memory.
Frames are pipelined as psn_t2d_group_complete_next allows (frame t+1's
backward chains run while the host does frame t's steps 5-6; same results).
The timed region runs from host frames to host results.

Modes and legs:
  --total-cameras M   strong scaling, SURVEY 8(e): M cameras sharded over the
                      ranks (configs[3]: --total-cameras 8 --points 2048
                      --boxes 32; 8/4/2/1 cameras per GPU at N = 1/2/4/8).
  --features gridfast the whole Run, GridFAST inside the timed region.
  --verify            every frame's gathered result slots (warm-up and timed)
                      checked against the oracle's CameraTracker replay of the
                      same frames, after the timed region.
  --mode kernel       BASELINE.json configs[1] (1 camera, 512 points, 21x21,
                      frames resident in HBM); reported as `secondary`.
  --mode config4      BASELINE.json configs[4]: 8 cameras sharded over the
                      ranks, 3840x2160, 4096 points/camera, 21x21, 5 levels,
                      SG(9, 1) post-filter of every point's trajectory.
  --box-dist pets     per-detection box sizes from a seeded PETS-like
                      distribution (synth.pets_box_sizes): windows of every
                      kernel class in one frame.
  At N = 1 the default line also carries `legs`: configs[3] on one GPU,
  configs[4] on one GPU, the GridFAST Run and the PETS-like mixed-box Run
  (--no-legs skips them).

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (one process per
GPU, RANK/LOCAL_RANK/WORLD_SIZE set before anything touches a GPU); under
torch.distributed.run the ranks come from the environment. --dry-run checks
the launcher and the control plane without a GPU (gloo only).
"""
import argparse
import ctypes
import hashlib
import json
import os
import platform
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Tracker2D frames/sec (all cameras) + achieved HBM GB/s fraction, 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU
# instruction per SIMD every 2 cycles (32 lanes per cycle) at 2.4 GHz
N_SIMD, CLOCK_HZ = 256 * 4, 2.4e9
VALU_PEAK_WAVE_INSTR = N_SIMD * CLOCK_HZ / 2.0
OPS_PER_SAMPLE = 8  # ~8 integer ops per window sample per iteration
DEFAULT_PROFILE = os.path.join(ROOT, "profiles", "r06c_tracker_profile.json")


def progress(msg):
    """A progress line on stderr (long legs stay visibly alive; stdout keeps the one JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


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


def cpu_quota_cores():
    """The CPU quota of this process's cgroup in cores (cgroup v2 cpu.max or v1
    cfs quota), else the affinity set: more OpenMP threads than that only
    time-slice (spinning barriers make such a leg crawl)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(n, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return max(1, min(n, q // p))
    except (OSError, ValueError):
        pass
    return n


def cpu_share_threads():
    """The host cores allotted to this GPU's job: the affinity set, capped by
    OMP_NUM_THREADS when the box sets it (16 per GPU on the GPU box)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


def dist_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def file_sha16(path):
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


# ---------------------------------------------------------------------------
# Launcher: --gpus N without torch.distributed.run
# ---------------------------------------------------------------------------

def launch_ranks(args, argv):
    """Start N rank processes of this script (one per GPU) before anything here
    touches a GPU; rank 0's JSON line is the output. Non-zero if any rank fails."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a failed rank: the others would wait for it forever
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return 1 if rc else 0


def init_control_plane(world):
    """Barriers, the RCCL id and max-over-ranks on gloo; the data plane is psn_comm (RCCL)."""
    import torch.distributed as dist

    if world > 1 and not dist.is_initialized():
        dist.init_process_group("gloo")


def barrier(world):
    import torch.distributed as dist

    if world > 1:
        dist.barrier()


# ---------------------------------------------------------------------------
# Tracker2D workload (default line, configs[2] / configs[3], GridFAST, verify)
# ---------------------------------------------------------------------------

def cameras_of_rank(args, world, rank):
    """Weak (cameras per GPU) or strong (--total-cameras sharded): the camera ids of this rank."""
    if args.total_cameras:
        if args.total_cameras % world:
            raise SystemExit(f"--total-cameras {args.total_cameras} is not a multiple of {world} ranks")
        c = args.total_cameras // world
    else:
        c = args.cameras
    return [rank * c + k for k in range(c)]


class CameraFeed:
    """One camera's synthetic video (mcmtt_opticalflow_amd/synth.py): BGR frames
    (or JPEG files) in pinned host memory and, per frame, the detections (box,
    head box, 3D estimate) with their feature points (given mode)."""

    def __init__(self, cam, args, pinned):
        from mcmtt_opticalflow_amd import synth

        W, H = args.width, args.height
        self.scene = synth.make_scene(cam, W, H, args.points, nboxes=args.boxes, box_dist=args.box_dist)
        self.period = args.period
        self.gridfast = args.features == "gridfast"
        self.jpeg = None
        if args.ingest == "jpeg":  # baseline JPEG files (PIL/libjpeg-turbo, q90, 4:2:0, a restart per MCU row)
            import io

            from PIL import Image

            self.jpeg = []
            for t in range(self.period):
                b = io.BytesIO()
                Image.fromarray(synth.to_bgr(self.scene.frame(t))[..., ::-1]).save(
                    b, "JPEG", quality=90, subsampling=2, restart_marker_rows=1)
                buf = pinned((len(b.getvalue()),))
                buf[:] = np.frombuffer(b.getvalue(), np.uint8)
                self.jpeg.append(buf)
            self.frames = None
        else:
            self.frames = [pinned((H, W, 3)) for _ in range(self.period)]
            for t in range(self.period):
                self.frames[t][...] = synth.to_bgr(self.scene.frame(t))
        self.boxes, self.feats = [], []
        for t in range(self.period):
            self.boxes.append(detection_boxes(self.scene, t))
            pts = self.scene.points_at(t)
            self.feats.append([pts[self.scene.pt_box == k] for k in range(args.boxes)])

    def detections(self, t2d, t):
        """Fresh records of frame t (the group writes its outputs into them)."""
        f = ping_pong(t, self.period)
        out = []
        for b, pts in zip(self.boxes[f], self.feats[f]):
            head, loc, height = detection_extra(b)
            out.append(t2d.make_detection(b, np.zeros((0, 2), np.float32) if self.gridfast else pts, head=head,
                                          location=loc, height=height))
        return out

    def push(self, group, k, t):
        """Camera k's frame t into the group (async upload of BGR, or JPEG bytes decoded on the device)."""
        f = ping_pong(t, self.period)
        if self.jpeg is not None:
            group.push_frame_jpeg(k, self.jpeg[f])
        else:
            group.push_frame(k, self.frames[f])


def uniform_box(width):
    """synth.make_scene's uniform box at a frame width (32x80 at 640x480,
    64x160 at 1080p, 128x320 at 4K)."""
    bw = 32 if width <= 640 else 64 if width <= 1920 else 128
    return bw, int(bw * 2.5)


def detection_boxes(scene, f):
    return [(float(int(x)), float(int(y)), float(scene.box_ws[k]), float(scene.box_hs[k]))
            for k, (x, y) in enumerate(scene.box_at(f))]


def detection_extra(b):
    """Head box (vecPartBoxes.front()), a ground-plane stand-in location (mm) and height."""
    head = (b[0] + b[2] / 4, b[1], b[2] / 2, b[3] / 8)
    loc = ((b[0] + b[2] / 2) * 10.0, (b[1] + b[3]) * 10.0, 0.0)
    return head, loc, 1700.0


def pinned_allocator(kind="hip"):
    """Pinned host buffers (uint8 numpy arrays) from the library's HIP runtime
    (mcmtt_opticalflow_amd/hip.py): hipHostMalloc (default, "hip"; coherent with
    "hip-coherent"), or (diagnostic --host-alloc register) page-aligned numpy
    memory registered with hipHostRegister."""
    from mcmtt_opticalflow_amd import hip

    if kind == "register":
        keep = []
        H = hip.rt()
        H.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]

        def alloc(shape):
            n = int(np.prod(shape))
            raw = np.empty(n + 4096, np.uint8)
            off = (-raw.ctypes.data) % 4096
            a = raw[off:off + n]
            hip.check(H.hipHostRegister(a.ctypes.data, n, 0), "hipHostRegister")
            keep.append(raw)
            return a.reshape(shape)

        alloc.keep = keep
        return alloc
    return hip.PinnedAllocator(coherent=(kind == "hip-coherent"))


class LaunchTimes:
    """Every LK launch of the timed region (HIP events on the stream each was
    launched on), per kernel (psn_lk_timing_launches)."""

    def __init__(self, L, lkh, cap):
        self.L, self.h, self.cap = L, lkh, cap
        L.psn_lk_enable_timing(lkh, cap, 1)

    def read(self):
        from mcmtt_opticalflow_amd import _lib

        per = {}
        for ms, tag in _lib.timing_launches(self.L, self.h, self.cap):
            k = _lib.kernel_of_tag(tag)
            n, tot = per.get(k, (0, 0.0))
            per[k] = (n + 1, tot + ms)
        np_, nt, pm, tm = ctypes.c_int(), ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        self.L.psn_lk_timing_stats(self.h, ctypes.byref(np_), ctypes.byref(pm), ctypes.byref(nt), ctypes.byref(tm))
        return per, {"n_track": nt.value, "track_ms": tm.value}


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


def tracker_run(args, world=1, rank=0, local_rank=0, steps=None, warmup=None):
    """The Tracker2D workload on this rank: warm-up, `steps` timed frames. Returns
    the measurements (rank 0: with the gathered results of every frame when
    args.verify)."""
    from mcmtt_opticalflow_amd import _lib, hip
    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import tracker2d as t2d

    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    warmup = max(warmup, 1)  # the first step launches the frame the next one completes
    hip.set_device(local_rank)
    cams = cameras_of_rank(args, world, rank)
    C = len(cams)
    gridfast = args.features == "gridfast"
    L = _lib.load()
    pinned = pinned_allocator(args.host_alloc)
    feeds = [CameraFeed(c, args, pinned) for c in cams]
    max_obj = 2 * args.boxes
    c_t0 = time.perf_counter()
    group = t2d.Group(args.width, args.height, cams, device=local_rank, max_objects=max_obj)
    create_ms = 1e3 * (time.perf_counter() - c_t0)
    warm = ctypes.c_double()
    warm_ms = (warm.value if hasattr(L, "psn_lk_sdma_warmup_ms") and
               L.psn_lk_sdma_warmup_ms(local_rank, ctypes.byref(warm)) == 0 else None)
    slot_bytes = t2d.result_slot_bytes(max_obj, 1)
    send = pinned((C, slot_bytes))
    # N > 1 always; N = 1 with --exchange (what the RCCL hand-off costs on one rank)
    exch = (pdist.ResultExchange(world, rank, C * slot_bytes, device=local_rank)
            if world > 1 or args.exchange else None)
    T = t2d.load()
    recorded = [] if args.verify else None

    ahead = args.stage_ahead

    parts = [] if args.step_profile else None  # (launch, pushes, complete_next) host ms per step
    # N > 1: frame t's exchange is enqueued at step t and its gathered slots are
    # consumed (the Associator3D hand-off) at step t+1, while frame t+1 runs
    pending = []

    def consume(g):
        if recorded is not None:
            recorded.append(np.array(g, copy=True).reshape(-1))
        return g

    def drain():
        g = None
        while pending:
            g = consume(exch.wait(pending.pop(0)))
        return g

    def step(t, dets, next_dets):
        c0 = time.perf_counter()
        group.launch(t, dets, gridfast=gridfast, seed=t)  # after complete_next(t-1): a confirmation
        c1 = time.perf_counter()
        if not args.push_last:
            for k, fd in enumerate(feeds):  # frame t+ahead uploads (and builds) while frame t runs
                fd.push(group, k, t + ahead)
        c2 = time.perf_counter()
        group.complete_next(t + 1, next_dets, gridfast=gridfast, seed=t + 1, raw=True)
        if args.push_last:  # frame t+1's work is on the GPU before the uploads are issued
            for k, fd in enumerate(feeds):
                fd.push(group, k, t + ahead)
        if parts is not None:
            parts.append((t, round(1e3 * (c1 - c0), 3), round(1e3 * (c2 - c1), 3),
                          round(1e3 * (time.perf_counter() - c2), 3), group.debug_host_times()))
        for k in range(C):  # the hand-off slots (psn_t2d_pack_result) in host memory
            rc = T.psn_t2d_pack_result(ctypes.byref(group.result_struct(k)), send[k].ctypes.data, slot_bytes)
            if rc:
                raise t2d.T2dError(rc, "psn_t2d_pack_result")
        if not exch:
            return consume(send)
        pending.append(exch.start(send))
        return consume(exch.wait(pending.pop(0))) if len(pending) > 1 else None

    def all_dets(t):
        return [fd.detections(t2d, t) for fd in feeds]

    for f in range(ahead):  # frames 0 .. ahead-1 staged before the first launch
        for k, fd in enumerate(feeds):
            fd.push(group, k, f)
    # ctypes records of every frame, built outside the timed region; one more
    # frame than completed: the last step launches its successor ahead, as the
    # warm-up's last step did for the first timed frame
    measure = 0 if args.verify else args.measure_steps
    seq = [group.records(all_dets(t)) for t in range(warmup + steps + measure + 1)]
    t = 0
    wticks = [time.perf_counter()]
    for i in range(warmup):
        step(t, seq[i], seq[i + 1])
        wticks.append(time.perf_counter())
        t += 1
    drain()
    barrier(world)
    hip.synchronize()
    t0 = time.perf_counter()
    ticks = []  # host time after each step (its frame's results are in host memory): no sync added
    for i in range(steps):
        j = warmup + i
        gathered = step(t, seq[j], seq[j + 1])
        ticks.append(time.perf_counter())
        t += 1
        if i == args.diag_sync_at or (args.diag_sync_every and i % args.diag_sync_every == args.diag_sync_every - 1):
            hip.synchronize()  # diagnostic runs only: a device sync inside the timed region
    g_last = drain()  # the last timed frame's hand-off
    gathered = g_last if g_last is not None else gathered
    hip.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = pdist.max_over_ranks(elapsed)
    if parts is not None:
        for p_ in parts:
            if sum(p_[1:4]) > 4.0:
                print(f"step {p_[0]}: launch {p_[1]} ms, pushes {p_[2]} ms, complete_next {p_[3]} ms {p_[4]}",
                      file=sys.stderr)
    # after the timed region (events between the launches would perturb it): per-launch
    # HIP-event durations of every LK launch and the device window-sample count
    lkh = group.lk_handle()
    per_kernel, ts, samples = {}, {"n_track": 0, "track_ms": 0.0}, None
    if measure:
        launches = LaunchTimes(L, lkh, 8 * measure + 64)  # forward + 3 chain steps per frame
        sampler = SampleCounter(L, lkh)
        for i in range(measure):
            j = warmup + steps + i
            gathered = step(t, seq[j], seq[j + 1])
            t += 1
        g_last = drain()
        gathered = g_last if g_last is not None else gathered
        hip.synchronize()
        per_kernel, ts = launches.read()
        samples = sampler.read()
    # feature points of the last completed frame (GridFAST mode: what GridFAST kept)
    arrs, _, nd = seq[warmup + steps + measure - 1]
    pts_last = sum(int(arrs[c][i].num_features) for c in range(C) for i in range(nd[c])) / C
    objs_last = 0
    if rank == 0:  # the gathered hand-off of the last frame: every camera's result, index == camID
        rows = np.asarray(gathered).reshape(-1, slot_bytes)
        for cam in range(rows.shape[0]):
            r = t2d.unpack_result(rows[cam], max_obj, 1)
            assert r["cam_id"] == cam and r["frame_idx"] == t - 1, (cam, r["cam_id"], r["frame_idx"])
            objs_last += len(r["objects"])
    group.close()
    if exch:
        exch.close()
    if hasattr(pinned, "close"):
        pinned.close()
    isolated = None
    if args.isolated and world == 1:
        isolated = isolated_launches(args, C)
    box_sizes = [[[int(fd.scene.box_ws[k]), int(fd.scene.box_hs[k])] for k in range(args.boxes)] for fd in feeds]
    return {"elapsed": elapsed, "steps": steps, "warmup": warmup, "cams_per_rank": C, "world": world,
            "step_ends": [x - t0 for x in ticks],
            "warmup_step_ms": [round(1e3 * (b - a), 3) for a, b in zip(wticks[:-1], wticks[1:])],
            "box_sizes": box_sizes, "isolated": isolated,
            "measure_steps": measure,
            "per_kernel": per_kernel, "ts": ts, "samples": samples, "objs_last": objs_last,
            "points_per_camera": pts_last, "recorded": recorded, "slot_bytes": slot_bytes, "max_obj": max_obj,
            "setup": {"group_create_ms": round(create_ms, 3),
                      "sdma_warmup_ms": None if warm_ms is None else round(warm_ms, 3),
                      "note": "outside the timed region: psn_t2d_group creation, of which the process's first "
                              "psn_lk_create sets up every SDMA engine (psn_lk_sdma_warmup_ms)"}}


def verify_tracker(args, r):
    """Every recorded frame's gathered result slots against the oracle's
    CameraTracker (oracle/tracker2d_oracle.py: the reference schedule, the
    reference's Munkres) replayed over the same frames, detections and points
    (GridFAST mode: the oracle's GridFAST with the same seeds). Outside the
    timed region; checker only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # verify leg only: the checker
    import tracker2d_oracle as T2  # verify leg only: the checker
    from mcmtt_opticalflow_amd import synth
    from mcmtt_opticalflow_amd import tracker2d as t2d

    ncam = r["world"] * r["cams_per_rank"]
    frames = len(r["recorded"])
    T2.NTHREADS, T2.SHARED_PYRAMIDS = cpu_share_threads(), True
    W, H = args.width, args.height
    mism, checked, objects, first = 0, 0, 0, None
    for cam in range(ncam):
        sc = synth.make_scene(cam, W, H, args.points, nboxes=args.boxes, box_dist=args.box_dist)
        ref = T2.CameraTracker(cam_id=cam)
        jpeg = {}
        for t in range(frames):
            f = ping_pong(t, args.period)
            bgr = synth.to_bgr(sc.frame(f))
            if args.ingest == "jpeg":  # the bench's JPEG files, decoded by the oracle
                if f not in jpeg:
                    import io

                    from PIL import Image

                    b = io.BytesIO()
                    Image.fromarray(bgr[..., ::-1]).save(b, "JPEG", quality=90, subsampling=2, restart_marker_rows=1)
                    jpeg[f] = oracle.jpeg_decode_bgr(b.getvalue())
                bgr = jpeg[f]
            gray = oracle.bgr2gray(bgr)
            boxes = detection_boxes(sc, f)
            if args.features == "gridfast":
                rois = []
                for b in boxes:
                    x, y = max(0.0, b[0]), max(0.0, b[1])
                    rois.append((int(x), int(y), int(min(W - x - 1, b[2])), int(min(H - y - 1, b[3]))))
                feats, _ = oracle.gridfast_detect(gray, rois, seed=t)
            else:
                pts = sc.points_at(f)
                feats = [pts[sc.pt_box == k] for k in range(args.boxes)]
            extra = [(T2.Rect(*h), loc, hh) for h, loc, hh in (detection_extra(b) for b in boxes)]
            _, _, exp = ref.run(gray, [T2.Rect(*b) for b in boxes], feats, t, extra)
            row = r["recorded"][t].reshape(-1, r["slot_bytes"])[cam]
            got = t2d.unpack_result(row, r["max_obj"], 1)
            ok = (got["cam_id"], got["frame_idx"], len(got["objects"])) == (exp["cam_id"], exp["frame_idx"],
                                                                           len(exp["objects"]))
            for go, eo in zip(got["objects"], exp["objects"]):
                ok = ok and (go["id"], go["box"], go["head"], go["score"]) == (eo["id"], eo["box"], eo["head"],
                                                                              eo["score"])
                ok = ok and np.array_equal(go["prev"], eo["prev"]) and np.array_equal(go["curr"], eo["curr"])
            checked += 1
            objects += len(exp["objects"])
            if not ok:
                mism += 1
                first = first or {"camera": cam, "frame": t}
    T2.NTHREADS, T2.SHARED_PYRAMIDS = 0, False
    return {"frames": frames, "cameras": ncam, "camera_frames_checked": checked, "objects_checked": objects,
            "mismatches": mism, "first_mismatch": first,
            "compared": "every frame's packed stTrack2DResult (ids, boxes, heads, scores, featurePointsPrev/Curr) "
                        "bit for bit against oracle/tracker2d_oracle.py CameraTracker.run"}


def tracker_cpu_baseline(args, n_frames_cap=400, legs=("share", "single", "all", "shared")):
    """The oracle Tracker2D (oracle/tracker2d_oracle.py CameraTracker + oracle/lk_oracle.c)
    on this host: the same synthetic cameras, detections and points (or, with
    --features gridfast, the oracle's GridFAST per detection with the run's seeds,
    PSNWhere_Tracker2D.cpp:735-757), the reference call schedule (every
    calcOpticalFlowPyrLK rebuilds both pyramids), OpenMP over points and over the
    rows of the full-frame passes. Legs: the cores allotted to this GPU, 1 thread,
    all cores, and the shared-pyramid schedule at the allotted cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only
    import tracker2d_oracle as T2  # cpu_baseline leg only
    from mcmtt_opticalflow_amd import synth

    W, H, C = args.width, args.height, args.cameras
    gridfast = args.features == "gridfast"
    scenes = [synth.make_scene(c, W, H, args.points, nboxes=args.boxes, box_dist=args.box_dist) for c in range(C)]
    grays = [[oracle.bgr2gray(synth.to_bgr(sc.frame(t))) for t in range(args.period)] for sc in scenes]

    def features(gray, boxes, sc, f, t):
        if not gridfast:
            pts = sc.points_at(f)
            return [pts[sc.pt_box == k] for k in range(args.boxes)]
        rois = []  # the detection boxes clipped as the reference clips its masks
        for b in boxes:
            x, y = max(0.0, b[0]), max(0.0, b[1])
            rois.append((int(x), int(y), int(min(W - x - 1, b[2])), int(min(H - y - 1, b[3]))))
        feats, _ = oracle.gridfast_detect(gray, rois, seed=t)
        return feats

    def leg(threads, shared, budget, ncams=C):
        T2.NTHREADS, T2.SHARED_PYRAMIDS = threads, shared
        cams = [T2.CameraTracker(c) for c in range(ncams)]
        n, t0 = 0, None
        progress(f"cpu baseline leg: {threads} threads, shared pyramids {shared}, {ncams} cameras, {budget:.0f} s")
        for t in range(n_frames_cap + 2):
            if t == 2:  # the ring holds frames: the steady state starts
                t0 = time.perf_counter()
            f = ping_pong(t, args.period)
            if t < 4 or t % 10 == 0:
                progress(f"  frame {t}")
            for c, sc in enumerate(scenes[:ncams]):
                boxes = detection_boxes(sc, f)
                feats = features(grays[c][f], boxes, sc, f, t)
                extra = [(T2.Rect(*h), loc, hh) for h, loc, hh in (detection_extra(b) for b in boxes)]
                cams[c].run(grays[c][f], [T2.Rect(*b) for b in boxes], feats, t, extra)
                if t >= 2:
                    n += 1
            if t0 is not None and time.perf_counter() - t0 >= budget:
                break
        dt = time.perf_counter() - t0
        T2.NTHREADS, T2.SHARED_PYRAMIDS = 0, False
        return n / dt, n, dt

    # all cores: every core this process may run on at once (the affinity set,
    # capped by the cgroup's CPU quota), the thread count set explicitly
    share, allc = cpu_share_threads(), cpu_quota_cores()
    v, n, dt = leg(share, False, args.cpu_budget)
    feat_txt = ("GridFAST per detection (oracle/gridfast_oracle.c, the run's seeds)" if gridfast else
                f"{args.points // args.boxes} given points")
    box_txt = "PETS-like box sizes (synth.pets_box_sizes)" if args.box_dist == "pets" else "64x160 boxes"
    out = {"value": round(v, 4), "unit": "frames/s", "cores": share, "kind": "port",
           "sample": f"{n} camera-frames ({C} cameras x {n // C} frames, {dt:.1f} s) of the same workload "
                     f"({W}x{H} BGR->gray, {args.boxes} detections ({box_txt}) x {feat_txt}, box windows, backward "
                     "chains + forward + Munkres matching) through oracle/tracker2d_oracle.py + oracle/lk_oracle.c, "
                     "OpenMP over points and over the rows of every pyramid/border/Scharr pass, reference call "
                     "schedule (both pyramids rebuilt in every calcOpticalFlowPyrLK)"}
    if "single" in legs:
        v1, n1, dt1 = leg(1, False, args.cpu_budget / 2, ncams=1)  # one camera: bounded warm-up
        out.update({"single_thread": round(v1, 4), "single_thread_sample": f"{n1} camera-frames (camera 0), {dt1:.1f} s"})
    if "all" in legs:
        va, na, dta = leg(allc, False, args.cpu_budget / 2)
        out.update({"all_cores": round(va, 4), "all_cores_threads": allc,
                    "all_cores_sample": f"{na} camera-frames, {dta:.1f} s"})
    if "shared" in legs:
        vs, ns, dts = leg(share, True, args.cpu_budget / 2)
        out.update({"shared_pyramid": round(vs, 4),
                    "shared_pyramid_sample": f"{ns} camera-frames, {dts:.1f} s, {share} threads"})
    out.update({"cores_note": "cores = the host cores this GPU's job is allotted (the box sets OMP_NUM_THREADS to its "
                              "per-GPU CPU share); all_cores = every core this process may run on at once (the "
                              f"affinity set of {len(os.sched_getaffinity(0))} CPUs capped by the cgroup CPU quota)",
                **host_info()})
    return out


def load_profile(path):
    """A round profile summary (tools/profile_summary.py): per kernel the rocprofv3
    kernel-trace mean duration, PMC HBM bytes (FETCH/WRITE, corrected per the
    guide's HBM section) and SQ counters per launch, plus the sha of the profiled
    libpsn_lk.so."""
    if not path or not os.path.exists(path):
        return None
    try:
        return json.load(open(path))
    except ValueError:
        return None


def isolated_launches(args, C, reps=20):
    """The frame-set's LK launches alone on the GPU (nothing else in flight):
    C cameras' pyramids (frames 0 -> 1 of each camera's synthetic scene) and one
    query per camera over its `points` given features, with the forward (w x h)
    and the backward (w x w) box windows; per shape the median HIP-event duration
    of `reps` launches. Outside the timed region."""
    from mcmtt_opticalflow_amd import _lib, lk, synth

    L = _lib.load()
    W, H = args.width, args.height
    bw, bh = uniform_box(W)
    out = {}
    scenes = [synth.make_scene(c, W, H, args.points, nboxes=args.boxes) for c in range(C)]
    with lk.LKContext(W, H, ring_slots=2 * C, max_level_cap=3) as ctx:
        for c, sc in enumerate(scenes):
            ctx.push_frame(2 * c, synth.to_bgr(sc.frame(0)))
            ctx.push_frame(2 * c + 1, synth.to_bgr(sc.frame(1)))
        pts = np.concatenate([sc.points_at(0) for sc in scenes])
        for name, win in (("forward", (bw, bh)), ("backward", (bw, bw))):
            qs = [lk.make_query(2 * c, 2 * c + 1, c * args.points, args.points, lk.make_params(win, 3))
                  for c in range(C)]
            for _ in range(3):
                ctx.track(qs, pts)
            L.psn_lk_enable_timing(ctx.handle, reps + 1, 1)
            for _ in range(reps):
                ctx.track(qs, pts)
            ms = np.array([m for m, _ in _lib.timing_launches(L, ctx.handle, reps + 1)])
            tags = {t for _, t in _lib.timing_launches(L, ctx.handle, reps + 1)}
            L.psn_lk_enable_timing(ctx.handle, 0, 1)
            out[name] = {"window": list(win), "mean_us": round(1e3 * float(ms.mean()), 2),
                         "median_us": round(1e3 * float(np.median(ms)), 2),
                         "min_us": round(1e3 * float(ms.min()), 2), "launches": int(ms.size),
                         "kernel": ",".join(sorted(_lib.kernel_of_tag(t) for t in tags))}
    return out


def tracker_roofline(args, r, C, profile):
    """Roofline of the dominant LK kernel (largest share of the timed LK time),
    per launch: SURVEY 8(d) LK bytes per camera-frame (2*S_pyr + 21*N) x the C
    camera-frames one launch processes, over the launch's mean HIP-event duration;
    VALU issue from the profile's SQ_INSTS_VALU per launch over the same duration."""
    from mcmtt_opticalflow_amd import _lib

    _, lk_b = algorithmic_bytes(args.width, args.height, 4, args.points)
    per = r["per_kernel"]
    if not per:
        return None
    launch_b = C * lk_b
    iso = r.get("isolated") or {}
    meas = max(r["measure_steps"], 1)
    # the dominant kernel: the largest cost per frame-set when each launch runs
    # alone on the GPU (isolated mean x launches per step); without isolated
    # timings, the largest in-pipeline time per step
    cand = [(v["mean_us"] * per[v["kernel"]][0] / meas, v) for v in iso.values()
            if v and v.get("mean_us") and v.get("kernel") in per]
    if cand:
        _, dom = max(cand, key=lambda c: c[0])
        name = dom["kernel"]
    else:
        dom = None
        name = max(per.items(), key=lambda kv: kv[1][1])[0]
    n, tot = per[name]
    pipe_ms = tot / n  # wall time of the launch in the running pipeline (overlapping launches)
    # the contract's achieved / frac: the dominant launch's own duration, timed
    # alone on the GPU (HIP events on its stream, mean of the launches), so the
    # kernel's time per step is its cost and not the overlap of several streams;
    # the in-pipeline wall time is reported beside it
    if dom is not None:
        avg_ms, timing = dom["mean_us"] * 1e-3, "isolated"
    else:
        avg_ms, timing = pipe_ms, "in_pipeline"
    fw = dom
    ach = launch_b / (avg_ms * 1e-3) / 1e9
    ms_step = r["elapsed"] / r["steps"] * 1e3
    per_step = {k: v[1] / max(r["measure_steps"], 1) for k, v in per.items()}
    out = {"kernel": name, "bound": "latency",
           "achieved": round(ach, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 6),
           "traffic": None, "bytes_per_launch": launch_b, "avg_launch_us": round(1e3 * avg_ms, 2),
           "timing": timing,
           "launches_per_step": round(n / max(r["measure_steps"], 1), 3),
           "kernel_ms_per_step": round(avg_ms * n / max(r["measure_steps"], 1), 4),
           "kernel_within_step": avg_ms * n / max(r["measure_steps"], 1) <= ms_step,
           "in_pipeline": {"avg_launch_us": round(1e3 * pipe_ms, 2), "launches_timed": n,
                           "achieved": round(launch_b / (pipe_ms * 1e-3) / 1e9, 3),
                           "note": "the launch's wall time inside the running pipeline (HIP events on its stream; "
                                   "consecutive forward launches overlap on two streams and share the CUs with the "
                                   "backward chains), so it exceeds the launch's own cost"},
           "bytes_note": f"SURVEY 8(d) LK bytes 2*S_pyr + 21*N = {lk_b} per camera-frame x {C} camera-frames per "
                         "launch; achieved/peak/frac are the HBM roofline of this kernel (contract fields) over "
                         "avg_launch_us (timing: isolated = the frame-set's launch alone on the GPU)",
           "per_kernel_us": {k: {"launches": v[0], "avg_us": round(1e3 * v[1] / v[0], 2),
                                 "ms_per_step": round(per_step[k], 4)} for k, v in sorted(per.items())}}
    if fw:
        which = [k for k, v in iso.items() if v is fw][0]
        out["isolated"] = {**fw, "call": which, "bytes_per_launch": launch_b,
                           "workload": f"the {which} launch of one frame-set alone on the GPU: {C} cameras x "
                                       f"{args.points} points, {fw['launches']} launches"}
        out["isolated_all"] = iso
        # the same launches under rocprofv3 --kernel-trace (the round profile's
        # `isolated` section: bench.py --mode isolated, this workload)
        pi = ((profile or {}).get("isolated") or {}).get("kernels", {})
        if fw.get("kernel") in pi:
            pki = pi[fw["kernel"]]
            a_p = launch_b / (pki["avg_us"] * 1e-6) / 1e9
            out["isolated"].update({"profile_avg_us": pki["avg_us"], "profile_launches": pki["launches"],
                                    "profile_achieved": round(a_p, 3), "profile_frac": round(a_p / HBM_PEAK_GBPS, 6),
                                    "profile_vs_live": round(pki["avg_us"] / (1e3 * avg_ms), 4)})
    lib_sha = file_sha16(_lib.LIB_PATH)
    if profile:
        pk = profile.get("kernels", {}).get(name, {})
        out["traffic"] = pk.get("hbm_bytes_per_launch")
        out["profile"] = os.path.relpath(args.profile, ROOT)
        out["profile_lib_sha16"] = profile.get("lib_sha16")
        out["lib_sha16"] = lib_sha
        out["profile_matches_binary"] = profile.get("lib_sha16") == lib_sha
        out["profile_avg_launch_us"] = pk.get("avg_us")
        vi = pk.get("SQ_INSTS_VALU")
        if vi:
            issue = vi / (avg_ms * 1e-3)
            v = {"achieved": round(issue / 1e9, 2), "peak": round(VALU_PEAK_WAVE_INSTR / 1e9, 2),
                 "unit": "G wave64-VALU-instructions/s", "frac": round(issue / VALU_PEAK_WAVE_INSTR, 4),
                 "instructions_per_launch": int(vi),
                 "peak_note": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction"}
            # useful lane work of every LK launch of a frame-set vs the lane slots they issued
            lk_vi = sum(kv.get("SQ_INSTS_VALU", 0) * per.get(k, (0, 0))[0]
                        for k, kv in profile.get("kernels", {}).items() if k.startswith("lk_kernel")) / max(r["measure_steps"], 1)
            if r["samples"] and lk_vi:
                useful = r["samples"] / max(r["measure_steps"], 1) * OPS_PER_SAMPLE
                v["useful_lane_frac"] = round(useful / (lk_vi * 64), 4)
                v["useful_note"] = (f"SURVEY 8(d) window samples x {OPS_PER_SAMPLE} ops per frame-set / "
                                    "(SQ_INSTS_VALU of every LK launch per frame-set x 64 lanes)")
            # the whole frame-set: every profiled kernel's VALU instructions x its timed
            # launches per frame-set, over the step time
            ms_step = r["elapsed"] / r["steps"] * 1e3
            frame_vi = sum(kv.get("SQ_INSTS_VALU", 0) * per.get(k, (0, 0))[0]
                           for k, kv in profile.get("kernels", {}).items()) / max(r["measure_steps"], 1)
            if frame_vi:
                v["frame_set_frac"] = round(frame_vi / (VALU_PEAK_WAVE_INSTR * ms_step * 1e-3), 4)
                v["frame_set_note"] = "SQ_INSTS_VALU of every LK launch of a frame-set / issue capacity over ms_per_step"
            for key in ("SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                        "SQ_WAIT_INST_ANY"):
                if key in pk:
                    v[key + "_per_launch"] = int(pk[key])
            if pk.get("SQ_WAVE_CYCLES") and pk.get("SQ_WAIT_INST_ANY"):
                v["wait_frac"] = round(pk["SQ_WAIT_INST_ANY"] / pk["SQ_WAVE_CYCLES"], 4)
            cyc2 = pk.get("SQ_WAVE_CYCLES_sq2") or pk.get("SQ_WAVE_CYCLES")
            if cyc2 and pk.get("SQ_WAIT_ANY"):
                v["SQ_WAIT_ANY_per_launch"] = int(pk["SQ_WAIT_ANY"])
                v["wait_any_frac"] = round(pk["SQ_WAIT_ANY"] / cyc2, 4)
            out["valu"] = v
            # what bounds it, from the counters: VALU issue when either issue fraction
            # nears the peak; the HBM roofline when the PMC traffic rate does; else the
            # workgroups' dependency latency (serial ordered chains, barriers) at the
            # occupancy the registers and LDS allow
            hbm_rate = (out["traffic"] or 0) / (avg_ms * 1e-3) / 1e9
            if max(v["frac"], v.get("frame_set_frac", 0)) >= 0.6:
                out["bound"] = "valu"
            elif hbm_rate >= 0.6 * HBM_PEAK_GBPS:
                out["bound"] = "hbm"
            out["bound_note"] = (f"VALU issue {v['frac']:.0%} of peak over the launch, "
                                 f"{v.get('frame_set_frac', 0):.0%} over the frame-set; PMC HBM "
                                 f"{hbm_rate:.0f} GB/s; below 60 % of either peak the kernel is latency-bound"
                                 + (f"; waves wait {v['wait_any_frac']:.0%} of their cycles (SQ_WAIT_ANY)"
                                    if "wait_any_frac" in v else ""))
    return out


def mixed_roofline(args, line, profile):
    """Roofline of the mixed-box leg's dominant kernel from the round profile's
    `mixed_boxes` section (bench.py --box-dist pets under rocprofv3 --kernel-trace):
    the kernel's BUSY time per frame-set (the union of its launches' intervals:
    launches overlapping on several streams count once, so busy <= the frame-set
    period) against the frame-set's SURVEY 8(d) LK bytes; traffic = PMC HBM bytes
    of its launches per frame-set; wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES."""
    mb = (profile or {}).get("mixed_boxes")
    if not mb or not mb.get("kernels"):
        return None
    name, pk = max(mb["kernels"].items(), key=lambda kv: kv[1]["busy_us"] if kv[0].startswith("lk_kernel") else -1)
    b = mb.get("bench") or {}
    frames = (b.get("steps") or 0) + (b.get("warmup") or 0) + args.measure_steps + 1
    if not frames or not pk.get("busy_us"):
        return None
    C = args.cameras
    _, lk_b = algorithmic_bytes(args.width, args.height, 4, args.points)
    busy_ms = pk["busy_us"] / frames / 1e3
    ach = C * lk_b / (busy_ms * 1e-3) / 1e9
    out = {"kernel": name, "bound": "latency", "achieved": round(ach, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBPS, 6), "bytes_per_frame_set": C * lk_b,
           "busy_ms_per_frame_set": round(busy_ms, 4), "launches_per_frame_set": round(pk["launches"] / frames, 2),
           "avg_launch_us": pk["avg_us"], "profile_ms_per_step": b.get("ms_per_step"),
           "busy_within_step": b.get("ms_per_step") is not None and busy_ms <= b["ms_per_step"],
           "frames_traced": frames, "profile": os.path.relpath(args.profile, ROOT),
           "note": "busy time = union of the kernel's launch intervals in the profiled run, per frame-set; "
                   "bytes = SURVEY 8(d) LK bytes 2*S_pyr + 21*N per camera-frame x cameras"}
    if pk.get("hbm_bytes_per_launch") is not None:
        out["traffic_per_frame_set"] = int(pk["hbm_bytes_per_launch"] * pk["launches"] / frames)
    if pk.get("wait_any_frac") is not None:
        out["wait_any_frac"] = pk["wait_any_frac"]
    if line.get("compute"):
        out["compute"] = line["compute"]
    return out


def segment_rates(r, cams, nseg=5):
    """SURVEY 8(d)'s median of 5: the timed steps cut into five consecutive
    segments by the host clock at each step's end (this rank's view; no sync
    inside the timed region), camera-frames/s per segment and their median.
    `value` stays the whole timed region's rate."""
    ends = r.get("step_ends") or []
    n = len(ends)
    if n < nseg:
        return None
    cuts = [round(k * n / nseg) for k in range(nseg + 1)]
    vals = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        t_a = ends[a - 1] if a > 0 else 0.0
        vals.append(cams * (b - a) / (ends[b - 1] - t_a))
    dts = np.diff(np.concatenate([[0.0], np.asarray(ends)]))
    slow = np.argsort(dts)[::-1][:3]
    return {"n": nseg, "steps_each": [b - a for a, b in zip(cuts[:-1], cuts[1:])],
            "values": [round(v, 2) for v in vals], "median": round(float(np.median(vals)), 2),
            "step_ms_median": round(1e3 * float(np.median(dts)), 4),
            "slowest_steps": [[int(i), round(1e3 * float(dts[i]), 3)] for i in slow],
            "warmup_step_ms": r.get("warmup_step_ms")}


def tracker_line(args, r, world, C, scaling, profile):
    """The JSON line of a Tracker2D run (rank 0)."""
    fps_all = world * C * r["steps"] / r["elapsed"]
    per_gpu_fps = C * r["steps"] / r["elapsed"]
    pyr_b, lk_b = algorithmic_bytes(args.width, args.height, 4, args.points, c_in=3)
    frame_b = pyr_b + lk_b
    cam_frames = C * max(r["measure_steps"], 1)
    cfg3 = (args.total_cameras == 8 and args.points == 2048)
    what = ("BASELINE.json configs[3]" if cfg3 else "BASELINE.json configs[2] per GPU"
            if (args.width, args.height, args.cameras, args.points, args.boxes) == (1920, 1080, 4, 512, 8)
            and not args.total_cameras else "Tracker2D Run")
    pets = args.box_dist == "pets"
    bw, bh = uniform_box(args.width)
    box_txt = ("PETS-like boxes, synth.pets_box_sizes" if pets else f"{bw}x{bh} boxes")
    win_txt = ("box-derived windows (backward w x w, forward w x h, mixed kernel classes)" if pets else
               f"{bw}x{bw} backward, {bw}x{bh} forward windows")
    out = {
        "metric": METRIC, "value": round(fps_all, 2), "unit": "frames/s", "n_gpus": world, "steps": r["steps"],
        "warmup": r["warmup"], "ms_per_step": round(1e3 * r["elapsed"] / r["steps"], 5), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
        "config": {
            "workload": (f"{what}: {world * C} cameras ({C} per GPU) x {args.width}x{args.height} "
                         f"{'JPEG' if args.ingest == 'jpeg' else 'BGR'}, {args.boxes} detections/camera ({box_txt}"
                         f") x " + ("GridFAST features (<= 100 each)" if args.features == "gridfast" else
                                    f"{args.points // args.boxes} points = {args.points} tracked points/camera")
                         + f", CPSNWhere_Tracker2D::Run: async H2D ingest + BGR->gray + pyramid, 3-step backward "
                         f"chains + forward LK ({win_txt}; LocalSearchKLT on device) + matching cost, "
                         "Munkres + tracker update + ResultWithTracker, packed result slots in host memory"
                         + (", RCCL all-gather of the slots (psn_comm)" if world > 1 else "")),
            "cameras": world * C, "cameras_per_gpu": C, "width": args.width, "height": args.height,
            "points_per_camera": args.points if args.features == "given" else round(r["points_per_camera"], 1),
            "features": args.features, "detections_per_camera": args.boxes, "levels": 4 if args.width <= 1920 else "maxLevel 3, truncated per window (buildOpticalFlowPyramid)",
            **({"box_dist": "pets", "boxes_per_camera": r.get("box_sizes")} if pets else
               {"box": [bw, bh], "win_backward": [bw, bw], "win_forward": [bw, bh]}),
            "ingest": ("baseline JPEG files in host memory (q90 4:2:0, restart per MCU row), decoded on the device"
                       if args.ingest == "jpeg" else "BGR frames in pinned host memory"),
            "parallelism": f"camera-sharded x{world} ({C} cameras per GPU), RCCL all-gather of result slots"},
        "roofline": tracker_roofline(args, r, C, profile),
        "frame_level": {"algorithmic_bytes_per_camera_frame": frame_b,
                        "bytes_formula": "SURVEY 8(d) c_in*S0 + 4*S_pyr - S_top + 21*N, c_in = 3 (BGR)",
                        "achieved_GBps_per_gpu": round(frame_b * per_gpu_fps / 1e9, 3),
                        "hbm_fraction": round(frame_b * per_gpu_fps / 1e9 / HBM_PEAK_GBPS, 6),
                        "lk_ms_per_step": round(r["ts"]["track_ms"] / max(r["measure_steps"], 1), 4),
                        "lk_timing_note": "LK launch times from HIP events in the measure_steps frames after the "
                                          "timed region (no events inside it)"},
        "compute": {"window_samples_per_camera_frame": round(r["samples"] / cam_frames) if r["samples"] else None,
                    "gsamples_per_s_per_gpu": round(r["samples"] / cam_frames * per_gpu_fps / 1e9, 3)
                    if r["samples"] else None,
                    "definition": "SURVEY 8(d): sum over points and levels of w*h*(1 + iterations), "
                                  "counted on the device"},
        "frames_per_set_per_s": round(r["steps"] / r["elapsed"], 2),
        "segments": segment_rates(r, world * C),
        "result_objects_last_frame": r["objs_last"],
        "runtime": runtime_record(),
        "setup": r.get("setup"),
        "cpu_baseline": None,
    }
    return out


def runtime_record():
    """The ROCm runtime files this process runs on (psn_lk_runtime_info + /proc/self/maps)."""
    from mcmtt_opticalflow_amd import _lib

    info = _lib.runtime_info()
    return {k: info.get(k) for k in ("libamdhip64", "libhsa-runtime64", "librccl", "libamd_comgr",
                                     "hip_runtime_version", "rccl_version", "built_against_hip", "one_runtime",
                                     "mapped")}


def tracker_main(args):
    world, rank, local_rank = dist_env()
    init_control_plane(world)
    profile = load_profile(args.profile)
    progress(f"rank {rank}: tracker run, {args.warmup} warm-up + {args.steps} timed frames")
    r = tracker_run(args, world, rank, local_rank)
    progress(f"rank {rank}: tracker run done ({r['elapsed']:.3f} s timed)")
    C = r["cams_per_rank"]
    out = None
    if rank == 0:
        out = tracker_line(args, r, world, C, "strong" if args.total_cameras else "weak", profile)
        if args.verify:
            out["verify"] = verify_tracker(args, r)
            out["verify"]["note"] = "the timed loop copied each step's gathered slots (a few KB) for this check"
        if world == 1 and not args.no_cpu_baseline and not args.total_cameras:
            out["cpu_baseline"] = tracker_cpu_baseline(args)
            out["speedup_vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
            out["speedup_vs_cpu_all_cores"] = round(out["value"] / out["cpu_baseline"]["all_cores"], 1)
    if world == 1 and not args.no_legs and not args.total_cameras and not args.verify:
        progress("legs")
        out["legs"] = tracker_legs(args, profile)
    if world == 1 and not args.no_secondary:
        progress("secondary (kernel mode)")
        out["secondary"] = kernel_secondary(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


def run_child(argv, timeout=600):
    """One bench.py line in a fresh process (one rank, this GPU): each leg starts
    from the same process state as the default line -- streams, their hardware
    queues, host and device allocations of earlier legs do not carry over (a
    configs[4] leg after five Tracker2D legs in one process measured 1,199 vs
    2,053 frames/s alone)."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.abspath(__file__)] + argv, capture_output=True, text=True,
                       timeout=timeout, env=env)
    sys.stderr.write(p.stderr[-4000:])
    if p.returncode != 0:
        raise RuntimeError(f"bench leg {argv} failed ({p.returncode})")
    return json.loads(p.stdout.strip().splitlines()[-1])


def child_args(args, **over):
    """argv of a child line: this run's shared options plus the leg's own."""
    base = ["--no-legs", "--no-secondary", "--no-cpu-baseline", "--no-isolated", "--period", str(args.period),
            "--measure-steps", str(args.measure_steps), "--profile", args.profile]
    if args.lib_dir:
        base += ["--lib-dir", args.lib_dir]
    for k, v in over.items():
        base += [f"--{k.replace('_', '-')}", str(v)]
    return base


def tracker_legs(args, profile):
    """Extra single-GPU lines of the default run, each in its own process
    (run_child): configs[3] on one GPU (8 cameras x 2048 points, the
    strong-scaling run's N=1), the GridFAST Run, PETS-like mixed boxes, the
    realistic Run (GridFAST + PETS boxes, with its CPU baseline), configs[4]
    (host and HBM frames), and configs[4] through the whole Tracker2D Run."""
    legs = {}
    steps = str(args.leg_steps)
    l3 = run_child(child_args(args, total_cameras=8, points=2048, boxes=32, steps=steps, warmup=3))
    legs["configs3_1gpu"] = {k: l3[k] for k in ("value", "unit", "ms_per_step", "steps", "config", "compute")}
    legs["configs3_1gpu"]["roofline"] = {k: l3["roofline"].get(k) for k in ("kernel", "achieved", "frac",
                                                                            "avg_launch_us", "per_kernel_us")}
    lg = run_child(child_args(args, features="gridfast", steps=steps, warmup=3))
    legs["gridfast"] = {k: lg[k] for k in ("value", "unit", "ms_per_step", "steps", "config")}
    lm = run_child(child_args(args, box_dist="pets", steps=steps, warmup=3))
    legs["mixed_boxes"] = {k: lm[k] for k in ("value", "unit", "ms_per_step", "steps", "config", "compute")}
    legs["mixed_boxes"]["lk_launches"] = {k: lm["roofline"].get(k) for k in ("kernel", "avg_launch_us", "per_kernel_us")}
    am = argparse.Namespace(**{**vars(args), "box_dist": "pets", "verify": False, "isolated": False})
    legs["mixed_boxes"]["roofline"] = mixed_roofline(am, lm, profile)
    # the reference Run's real per-frame work together (PSNWhere_Tracker2D.cpp:735-757, 776-782,
    # 871-877): GridFAST per detection feeding PETS-sized box windows
    lr = run_child(child_args(args, features="gridfast", box_dist="pets", steps=steps, warmup=3))
    legs["realistic"] = {k: lr[k] for k in ("value", "unit", "ms_per_step", "steps", "config", "compute")}
    legs["realistic"]["lk_launches"] = {k: lr["roofline"].get(k) for k in ("kernel", "avg_launch_us", "per_kernel_us")}
    if not args.no_cpu_baseline:  # the reference's real per-frame work on the host cores (oracle restatement)
        progress("realistic leg: cpu baseline")
        ar = argparse.Namespace(**{**vars(args), "features": "gridfast", "box_dist": "pets"})
        cb = tracker_cpu_baseline(ar, legs=("share", "single"))
        legs["realistic"]["cpu_baseline"] = cb
        legs["realistic"]["speedup_vs_cpu"] = round(lr["value"] / cb["value"], 1)
        legs["realistic"]["speedup_vs_cpu_single_thread"] = round(lr["value"] / cb["single_thread"], 1)
    c4_steps = str(max(args.leg_steps // 2, 10))
    for name, ingest in (("config4", "host"), ("config4_frames_in_hbm", "hbm")):
        l4 = run_child(child_args(args, mode="config4", c4_ingest=ingest, steps=c4_steps, warmup=3))
        legs[name] = {"workload": l4["config"]["workload"], "ingest": ingest,
                      **{k: l4[k] for k in ("value", "unit", "n_gpus", "steps", "ms_per_step", "scaling", "roofline")}}
    # configs[4] through the whole Tracker2D Run: 8 x 4K BGR cameras, 4096 points per camera
    # (64 detections x 64), 128 x 320 boxes: 128 x 128 backward windows (the
    # 16-unit box kernel) and 128 x 320 forward windows (the large-window kernel)
    l4t = run_child(child_args(args, width=3840, height=2160, cameras=8, points=4096, boxes=64,
                               steps=max(args.leg_steps // 8, 5), warmup=2))
    legs["config4_tracker"] = {k: l4t[k] for k in ("value", "unit", "ms_per_step", "steps", "config", "compute")}
    legs["config4_tracker"]["lk_launches"] = {k: l4t["roofline"].get(k) for k in ("kernel", "avg_launch_us",
                                                                                 "per_kernel_us")}
    legs["note"] = "each leg is a bench.py line of its own process (run_child)"
    return legs


# ---------------------------------------------------------------------------
# Kernel modes: configs[1] (secondary) and configs[4] (4K, 5 levels, SG)
# ---------------------------------------------------------------------------

def kernel_cpu_baseline(scene, period, npts, win, max_level, budget_s, max_frames):
    """The oracle (reference call schedule: both pyramids + Scharr rebuilt in
    every calcOpticalFlowPyrLK call) on this host's allotted cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # cpu_baseline leg only

    threads = cpu_share_threads()
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
            "sample": f"{n} camera-frames of the same workload ({scene.width}x{scene.height}, {npts} pts, "
                      f"{win[0]}x{win[1]}, {max_level + 1} levels), oracle/lk_oracle.c with OpenMP, {dt:.1f} s",
            **host_info()}


def kernel_run(args, steps, warmup, world=1, rank=0, local_rank=0, C=1, W=1920, H=1080, N=512, levels=4,
               sg=False, ingest="hbm"):
    """LK step over C cameras per GPU, 21x21, `levels` pyramid levels; frames
    resident in HBM (ingest "hbm": gray, pushed from device memory) or BGR in
    pinned host memory uploaded every frame (ingest "host":
    psn_lk_push_frame_async, copy engines, as the Tracker2D headline does);
    sg: SG(9, 1) Insert of every tracked point's position per frame (status as
    the active mask), on the same stream."""
    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import hip, lk, synth

    hip.set_device(local_rank)
    cams = [rank * C + k for k in range(C)]
    win, R = 21, 4
    scenes = [synth.make_scene(c, W, H, N) for c in cams]
    frames = []
    period = args.period if ingest == "hbm" else min(args.period, 4)  # pinned 4K BGR: 25 MB a frame
    pinned = None
    if ingest == "host":
        pinned = pinned_allocator()
        for sc in scenes:
            fr = []
            for t in range(period):
                b = pinned((H, W, 3))
                b[...] = synth.to_bgr(sc.frame(t))
                fr.append(b)
            frames.append(fr)
    else:  # gray frames resident in HBM (device buffers of the library's runtime)
        for sc in scenes:
            frames.append([hip.DeviceBuffer.from_array(sc.frame(t)) for t in range(period)])
    stream = hip.Stream()
    ctx = lk.LKContext(W, H, ring_slots=R * C, max_level_cap=levels - 1, device=local_rank)
    ctx.set_stream(stream.handle)
    for kv in getattr(args, "lk_variant", None) or []:  # experiments: psn_lk_debug_set_variant
        k, v = kv.split("=")
        ctx.set_variant(k, int(v))
    mode = 2 if C == 1 else 1
    ctx.set_ingest_overlap(mode)
    sb = pdist.slot_bytes(N, C)
    offs = pdist.slot_offsets(N, C)  # header, next_xy, err, status
    hdr0 = np.array([[c, 0, N, 0] for c in cams], np.int32)
    slot_host = np.zeros(sb, np.uint8)
    slot_host[:hdr0.nbytes] = hdr0.view(np.uint8).reshape(-1)
    slot_host[offs[1]:offs[2]] = np.concatenate([sc.points_at(0) for sc in scenes]).astype(np.float32).view(
        np.uint8).reshape(-1)
    slots = [hip.DeviceBuffer.from_array(slot_host) for _ in range(2)]
    gathered = hip.DeviceBuffer(world * sb)
    comm = pdist.init_comm(world, rank, local_rank) if world > 1 else None
    params = lk.make_params((win, win), levels - 1)
    smoother = None
    if sg:
        smoother = lk.SGSmoother(C * N, 2, 9, 1, device=local_rank)
        smoother.set_stream(stream.handle)
        sg_ref = hip.DeviceBuffer(4 * C * N)
        sg_out = hip.DeviceBuffer(8 * C * N * 9 * 2)

    # the harness's per-step host work kept to the calls themselves: frame
    # pointers, query arrays and slot pointers built once
    fptr = [[frames[k][i].addr for i in range(period)] for k in range(C)] if ingest != "host" else None

    def push(t):
        for k in range(C):
            if ingest == "host":
                ctx.push_frame_async(k * R + t % R, frames[k][ping_pong(t, period)])
            else:
                ctx.push_frame_device(k * R + t % R, fptr[k][ping_pong(t, period)], W, 1)

    push(0)
    push(1)
    ctx.sync()
    queries = [lk.query_array([lk.make_query(k * R + (t - 1) % R, k * R + t % R, k * N, N, params) for k in range(C)])
               for t in range(R)]
    ptrs = [tuple(sl.addr + o for o in offs) for sl in slots]  # (header, next, err, status) per parity
    sg_ptrs = (sg_ref.addr, sg_out.addr) if sg else None
    # every step's slot headers (cam, frame, npts, 0), prepared in pinned host
    # memory before the timed region and written by one small copy kernel per
    # step (psn_t2d_upload_device), the frame index of the slot the LK fills
    measure = max(1, min(steps, 50))
    t_end = warmup + steps + measure + 2
    hdr_alloc = pinned_allocator("hip-coherent")
    hdr_pin = hdr_alloc((t_end, C * 16))
    hdr_tab = hdr_pin.view(np.int32).reshape(t_end, C, 4)
    hdr_tab[:] = hdr0[None]
    hdr_tab[:, :, 1] = np.arange(t_end, dtype=np.int32)[:, None]
    L = ctx._L
    L.psn_t2d_upload_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    hstream = hip.Stream() if comm is None else None

    def step(t):
        cur, prv = ptrs[t % 2], ptrs[(t - 1) % 2]
        push(t + 1)
        ctx.track_device(queries[t % R], prv[1], cur[1], cur[3], cur[2])
        if smoother is not None:  # lost points (status 0) are not inserted
            smoother.insert_device(cur[1], 2, cur[3], sg_ptrs[0], sg_ptrs[1])
        # the header bytes are disjoint from what the LK writes: at N = 1 they go on
        # a stream of their own, beside the launch; N > 1 orders them before the gather
        rc = L.psn_t2d_upload_device(cur[0], hdr_pin[t].ctypes.data, 16 * C, (hstream or stream).handle)
        if rc:
            raise RuntimeError(f"psn_t2d_upload_device failed ({rc})")
        if comm is not None:
            pdist.comm_allgather(comm, slots[t % 2].addr, gathered.addr, sb, stream.handle)

    t = 1
    for _ in range(warmup):
        step(t)
        t += 1
    hip.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(t)
        t += 1
    hip.synchronize()
    elapsed = time.perf_counter() - t0
    # launch durations after the timed region (HIP events on the LK stream)
    ctx.enable_timing(measure + 1, 1)
    for _ in range(measure):
        step(t)
        t += 1
    hip.synchronize()
    ts = ctx.timing_stats()
    ctx.close()
    if smoother is not None:
        smoother.close()
    if comm is not None:
        pdist.comm_destroy(comm)
    stream.destroy()
    if hstream is not None:
        hstream.destroy()
    if pinned is not None:
        pinned.close()
    hdr_alloc.close()
    pyr_b, lk_b = algorithmic_bytes(W, H, levels, N)
    lk_us = 1e3 * ts["track_ms"] / max(ts["n_track"], 1)
    launch_b = C * lk_b + (pyr_b if mode == 2 else 0)
    return {"fps": C * steps / elapsed, "ms_per_step": 1e3 * elapsed / steps, "lk_us": lk_us,
            "launch_bytes": launch_b, "frame_bytes": pyr_b + lk_b, "scene": scenes[0], "elapsed": elapsed,
            "mode": mode if ingest == "hbm" else "async-host"}


def kernel_secondary(args):
    """BASELINE.json configs[1] (--mode kernel) as a line of its own process."""
    l1 = run_child(child_args(args, mode="kernel", steps=400, warmup=20, kcameras=max(1, args.kcameras),
                              kpoints=args.kpoints))
    return {"workload": "BASELINE.json configs[1]: 1 camera, 1920x1080 gray resident in HBM, 512 points, 4 levels, "
                        "21x21 window, fused pyramid build + LK + propagation",
            **{k: l1[k] for k in ("value", "unit", "ms_per_step", "roofline")}}


def config4_run(args, world, rank, local_rank, steps, warmup, ingest="host"):
    """BASELINE.json configs[4]: 8 cameras sharded over the ranks (strong), 3840x2160,
    4096 points/camera, 21x21, 5 levels (maxLevel 4), SG(9, 1) post-filter of every
    tracked point's trajectory (CPSNWhere_SGSmooth, PSNWhere_SGSmooth.cpp:198-274).
    ingest "host": BGR frames in pinned host memory uploaded every frame (8 x 24.9 MB
    per frame-set over PCIe); "hbm": gray frames resident in HBM (no upload)."""
    total = 8
    if total % world:
        raise SystemExit(f"configs[4] shards 8 cameras: {world} ranks do not divide them")
    C = total // world
    W, H, N, levels = 3840, 2160, 4096, 5
    r = kernel_run(args, steps, warmup, world, rank, local_rank, C=C, W=W, H=H, N=N, levels=levels, sg=True,
                   ingest=ingest)
    from mcmtt_opticalflow_amd import dist as pdist

    elapsed = pdist.max_over_ranks(r["elapsed"])
    fps_all = total * steps / elapsed
    ach = r["launch_bytes"] / (r["lk_us"] * 1e-6) / 1e9
    src = ("BGR in pinned host memory, uploaded every frame (psn_lk_push_frame_async)" if ingest == "host"
           else "gray resident in HBM (no upload)")
    line = {"workload": f"BASELINE.json configs[4]: {total} cameras ({C} per GPU) x 3840x2160 {src}, "
                        f"{N} points/camera, 21x21, 5 levels, SG(9,1) post-filter of every point trajectory",
            "ingest": ingest,
            "value": round(fps_all, 2), "unit": "frames/s", "n_gpus": world, "steps": steps,
            "ms_per_step": round(1e3 * elapsed / steps, 5), "scaling": "strong",
            "roofline": {"kernel": "lk_kernel_st (all cameras in one launch) + sg_insert_kernel", "bound": "latency",
                         "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach / HBM_PEAK_GBPS, 5), "bytes_per_launch": r["launch_bytes"],
                         "avg_launch_us": round(r["lk_us"], 3)}}
    return {"line": line, "fps": fps_all, "elapsed": elapsed}


def kernel_main(args):
    world, rank, local_rank = dist_env()
    # control plane (barriers, the RCCL id, the timing max) on gloo; the slots'
    # all-gather is the library's RCCL communicator (psn_comm)
    init_control_plane(world)
    if args.mode == "config4":
        res = config4_run(args, world, rank, local_rank, args.steps, args.warmup, ingest=args.c4_ingest)
        if rank == 0:
            line = res["line"]
            out = {"metric": METRIC, "value": line["value"], "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                   "warmup": args.warmup, "ms_per_step": line["ms_per_step"], "higher_is_better": True,
                   "scaling": "strong", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
                   "config": {"workload": line["workload"], "cameras": 8, "cameras_per_gpu": 8 // world},
                   "roofline": line["roofline"], "cpu_baseline": None}
            print(json.dumps(out), flush=True)
        if world > 1:
            import torch.distributed as dist

            dist.destroy_process_group()
        return
    C = max(1, args.kcameras)
    r = kernel_run(args, args.steps, args.warmup, world, rank, local_rank, C=C, N=args.kpoints)
    from mcmtt_opticalflow_amd import dist as pdist

    elapsed = pdist.max_over_ranks(r["elapsed"])
    fps_all = world * C * args.steps / elapsed
    if rank == 0:
        ach = r["launch_bytes"] / (r["lk_us"] * 1e-6) / 1e9
        out = {"metric": METRIC, "value": round(fps_all, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 5), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "u8+f32", "data": "synthetic",
               "config": {"workload": f"BASELINE.json configs[1] shape: {C} camera(s) per GPU, 1920x1080 "
                                      f"gray resident in HBM, {args.kpoints} points, 4 levels, 21x21 window",
                          "cameras": world * C, "cameras_per_gpu": C, "parallelism": f"camera-per-GPU x{world}"},
               "roofline": {"kernel": "lk_kernel_st" + ("+fused_pyramid" if r["mode"] == 2 else ""), "bound": "latency",
                            "achieved": round(ach, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBPS, 5), "traffic": None,
                            "bytes_per_launch": r["launch_bytes"], "avg_launch_us": round(r["lk_us"], 3)},
               "cpu_baseline": None}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = kernel_cpu_baseline(r["scene"], args.period, args.kpoints, (21, 21), 3,
                                                      args.cpu_budget, 2000)
            out["speedup_vs_cpu"] = round(fps_all / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# Dry run: the launcher and the control plane without a GPU
# ---------------------------------------------------------------------------

def dry_main(args):
    """No GPU work: every rank joins the gloo control plane, shards the cameras as the
    real run would, times an empty loop with the barrier + max-over-ranks protocol;
    rank 0 prints the line's shape (n_gpus, cameras per rank, scaling)."""
    world, rank, _ = dist_env()
    init_control_plane(world)
    import torch.distributed as dist

    from mcmtt_opticalflow_amd import dist as pdist

    cams = cameras_of_rank(args, world, rank)
    barrier(world)
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))
    barrier(world)
    elapsed = pdist.max_over_ranks(time.perf_counter() - t0)
    all_cams = [None] * world
    if world > 1:
        dist.all_gather_object(all_cams, cams)
    else:
        all_cams = [cams]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": None, "dry_run": True,
                          "scaling": "strong" if args.total_cameras else "weak",
                          "cameras_by_rank": all_cams, "elapsed_max_over_ranks": round(elapsed, 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mode", choices=["tracker", "kernel", "config4", "isolated"], default="tracker")
    ap.add_argument("--lk-variant", action="append", metavar="KEY=VALUE",
                    help="kernel-variant override of --mode kernel/config4 (A/B experiments; _lib.VARIANTS keys)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cameras", type=int, default=4, help="tracker mode: cameras per GPU (configs[2]: 4)")
    ap.add_argument("--total-cameras", type=int, default=0,
                    help="strong scaling: this many cameras sharded over the ranks (configs[3]: 8)")
    ap.add_argument("--points", type=int, default=512, help="tracker mode: feature points per camera")
    ap.add_argument("--boxes", type=int, default=8, help="tracker mode: detections per camera")
    ap.add_argument("--features", choices=["given", "gridfast"], default="given",
                    help="tracker mode: points given (SURVEY 8(d) recipe) or GridFAST on the device")
    ap.add_argument("--box-dist", choices=["uniform", "pets"], default="uniform",
                    help="tracker mode: every detection 64x160 (SURVEY 8(d), default) or per-detection sizes from "
                         "a seeded PETS-like distribution scaled to the frame (synth.pets_box_sizes)")
    ap.add_argument("--ingest", choices=["bgr", "jpeg"], default="bgr",
                    help="tracker mode: frames arrive as BGR arrays (default) or as JPEG files (device decode)")
    ap.add_argument("--stage-ahead", type=int, choices=[1, 2], default=2,
                    help="tracker mode: frames uploaded ahead of the running one (2: frame t+2 uploads and builds "
                         "while frame t runs; 1: frame t+1 only)")
    ap.add_argument("--verify", action="store_true", help="check every frame's results against the oracle")
    ap.add_argument("--kcameras", type=int, default=1, help="kernel mode: cameras per GPU")
    ap.add_argument("--kpoints", type=int, default=512, help="kernel mode: points per camera")
    ap.add_argument("--period", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--leg-steps", type=int, default=40)
    ap.add_argument("--measure-steps", type=int, default=20,
                    help="frames after the timed region with per-launch HIP-event timing (roofline)")
    ap.add_argument("--diag-sync-at", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--diag-sync-every", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--host-alloc", choices=["hip", "hip-coherent", "register"], default="hip",
                    help=argparse.SUPPRESS)
    ap.add_argument("--exchange", action="store_true",
                    help="tracker mode, N = 1: run the RCCL result exchange (psn_comm, one rank) every frame as N > 1 "
                         "does")
    ap.add_argument("--push-last", action="store_true",
                    help="tracker mode: push frame t+ahead after complete_next(t+1) instead of before it")
    ap.add_argument("--step-profile", action="store_true", help="tracker mode: host ms of each slow step to stderr")
    ap.add_argument("--no-isolated", dest="isolated", action="store_false",
                    help="skip the isolated-launch timing of the frame-set's LK launches (roofline.isolated)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--no-legs", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--lib-dir", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--runtime", choices=["rocm", "torch"], default="rocm", help=argparse.SUPPRESS)
    ap.add_argument("--c4-ingest", choices=["host", "hbm"], default="host",
                    help="--mode config4: BGR frames uploaded from pinned host memory every frame, or gray frames "
                         "resident in HBM")
    ap.add_argument("--profile", default=DEFAULT_PROFILE,
                    help="round profile summary (tools/profile_summary.py) for roofline.traffic / valu")
    args = ap.parse_args(argv)
    if args.points % args.boxes:
        raise SystemExit("--points must be a multiple of --boxes")
    return args


import numpy as np  # noqa: E402


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    if args.dry_run:
        return dry_main(args)
    # the product library before anything imports torch (the gloo control
    # plane): one HIP/HSA/RCCL runtime in this process, ROCm's (psn_runtime.cpp)
    from mcmtt_opticalflow_amd import _lib

    if args.runtime == "torch":  # diagnostic: torch first, so the library binds torch's bundled ROCm runtime
        import torch  # noqa: F401
    if args.lib_dir:  # A/B experiments: another build of both libraries (tools/gpu_ab.sh)
        from mcmtt_opticalflow_amd import tracker2d

        _lib.LIB_PATH = os.path.abspath(os.path.join(args.lib_dir, "libpsn_lk.so"))
        tracker2d.LIB_PATH = os.path.abspath(os.path.join(args.lib_dir, "libpsn_tracker2d.so"))
    _lib.load()
    if args.mode == "isolated":  # the profile pass of roofline.isolated (tools/profile_round.sh)
        print(json.dumps({"isolated": isolated_launches(args, args.cameras)}), flush=True)
        return None
    if args.mode in ("kernel", "config4"):
        return kernel_main(args)
    return tracker_main(args)


if __name__ == "__main__":
    main()
