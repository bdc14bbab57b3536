"""Host-side duration of hipMemcpyAsync (pinned H2D 6 MB / D2H 256 KB) when the
copy's stream first waits for an event of another stream that is still
running, vs a stream with running kernels of its own: the Tracker2D bench saw
7-8 ms host stalls in some of these copies."""
import time

import torch

dev = torch.device("cuda", 0)
src = torch.empty(6 << 20, dtype=torch.uint8).pin_memory()
dst = torch.empty(6 << 20, dtype=torch.uint8, device=dev)
hres = torch.empty(256 << 10, dtype=torch.uint8).pin_memory()
dres = torch.empty(256 << 10, dtype=torch.uint8, device=dev)
A, B = torch.cuda.Stream(), torch.cuda.Stream()
busy = torch.empty(8192, 8192, device=dev)


def timed(fn):
    t = time.perf_counter()
    fn()
    return round(1e3 * (time.perf_counter() - t), 3)


def work(st, n):
    with torch.cuda.stream(st):
        for _ in range(n):
            busy @ busy


for _ in range(2):
    work(A, 1)
torch.cuda.synchronize()
for label in ("h2d after cross-stream wait", "h2d behind own kernels", "d2h after cross-stream wait",
              "d2h behind own kernels"):
    out = []
    for rep in range(4):
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        if "cross" in label:
            work(A, 8)
            ev = torch.cuda.Event()
            ev.record(A)
            B.wait_event(ev)
        else:
            work(B, 8)
        with torch.cuda.stream(B):
            if label.startswith("h2d"):
                ms = timed(lambda: dst.copy_(src, non_blocking=True))
            else:
                ms = timed(lambda: hres.copy_(dres, non_blocking=True))
        launched = round(1e3 * (time.perf_counter() - g0), 3)
        torch.cuda.synchronize()
        out.append((ms, launched, round(1e3 * (time.perf_counter() - g0), 3)))
    print(f"{label:30s} (copy call ms, enqueue ms, total ms)", out, flush=True)
