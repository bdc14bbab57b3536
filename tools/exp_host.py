#!/usr/bin/env python3
"""Host-overhead experiment: is the bench step GPU-bound or launch-bound?

Runs the bench's per-frame step (push + LK, propagated points) with variants
and reports, per step, the wall time with a final sync and the host time spent
enqueueing. Usage: python tools/exp_host.py [--steps 400]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    args = ap.parse_args()
    import torch

    from mcmtt_opticalflow_amd import dist as pdist
    from mcmtt_opticalflow_amd import lk, synth

    dev = torch.device("cuda", 0)
    W, H, N, L, R, P = 1920, 1080, 512, 4, 4, 10
    sc = synth.make_scene(0, W, H, N)
    frames = torch.stack([torch.from_numpy(sc.frame(t)) for t in range(P)]).to(dev)
    res = {}
    for name, overlap, timing, fill in [("fused", 2, True, True), ("fused_no_fill", 2, True, False),
                                        ("fused_no_timing_no_fill", 2, False, False),
                                        ("stream_no_timing_no_fill", 1, False, False),
                                        ("off_no_timing_no_fill", 0, False, False)]:
        stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(stream)
        ctx = lk.LKContext(W, H, R, L - 1)
        ctx.set_stream(stream.cuda_stream)
        ctx.set_ingest_overlap(overlap)
        sb = pdist.slot_bytes(N)
        slots = [torch.zeros(sb, dtype=torch.uint8, device=dev) for _ in range(2)]
        views = [pdist.slot_views(s, N) for s in slots]
        views[0][1].copy_(torch.from_numpy(sc.points_at(0)))
        params = lk.make_params((21, 21), L - 1)
        ctx.push_frame_device(0, frames[0].data_ptr(), W, 1)
        if overlap == 2:
            ctx.push_frame_device(1, frames[1].data_ptr(), W, 1)
            ctx.sync()
        qs = [lk.make_query((t - 1) % R, t % R, 0, N, params) for t in range(R)]

        def step(t):
            cur, prv = views[t % 2], views[(t - 1) % 2]
            if overlap == 2:
                ctx.push_frame_device((t + 1) % R, frames[(t + 1) % P].data_ptr(), W, 1)
            else:
                ctx.push_frame_device(t % R, frames[t % P].data_ptr(), W, 1)
            ctx.track_device([qs[t % R]], prv[1].data_ptr(), cur[1].data_ptr(), cur[3].data_ptr(), cur[2].data_ptr())
            if fill:
                cur[0][1].fill_(t)

        t = 1
        for _ in range(20):
            step(t)
            t += 1
        if timing:
            ctx.enable_timing(args.steps + 1, 1)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(t)
            t += 1
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        res[name] = {"us_per_step": round(1e6 * (t2 - t0) / args.steps, 2),
                     "host_enqueue_us_per_step": round(1e6 * (t1 - t0) / args.steps, 2)}
        if timing:
            ts = ctx.timing_stats()
            res[name]["lk_us"] = round(1e3 * ts["track_ms"] / max(ts["n_track"], 1), 2)
            res[name]["pyr_us"] = round(1e3 * ts["push_ms"] / max(ts["n_push"], 1), 2)
        ctx.close()
    # bare call costs
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
