#!/usr/bin/env python3
"""VGPR liveness of one kernel in a gfx950 assembly listing (analysis only).

Builds the basic blocks of the function, runs a backward liveness fixpoint over
architectural VGPRs and prints the points of highest pressure with the source
lines (.loc, build with -gline-tables-only) where the live registers were last
defined -- which values the allocator has to hold at the peak.

  hipcc ... --cuda-device-only -S -gline-tables-only -o k.s psn_lk_kernels.hip
  python tools/vgpr_live.py k.s _ZN3psn12lk_kernel_bxILi10EEEvNS_12LkLaunchArgsE
"""
import re
import sys
from collections import Counter, defaultdict

VR = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
NO_DEF = ("ds_write", "ds_store", "global_store", "buffer_store", "scratch_store", "flat_store", "s_", "v_cmpx",
          "exp ", "global_atomic_add_f32 ", "ds_add_u32", "ds_bpermute_nodef")
ACC = ("v_fmac", "v_mac", "v_dot2c", "v_writelane", "v_pk_fmac", "v_cndmask_nodef")


def regs(text):
    out = set()
    for m in VR.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(lines):
    insts = []  # (op, defs, uses, loc, label_or_None, targets, falls)
    loc = (0, 0)
    for l in lines:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (int(m.group(1)), int(m.group(2)))
            continue
        code = l.split(";")[0].rstrip()
        if not code.strip():
            continue
        if re.match(r"^\.?[A-Za-z_0-9$.]+:$", code.strip()):
            insts.append(("LABEL", set(), set(), loc, code.strip()[:-1], [], True))
            continue
        if code.strip().startswith("."):
            continue
        parts = code.strip().split(None, 1)
        op = parts[0]
        args = parts[1] if len(parts) > 1 else ""
        ops = [a.strip() for a in args.split(",")]
        defs, uses = set(), set()
        if op.startswith(NO_DEF) or op.startswith("v_cmp_") and "vcc" in ops[0] or op.startswith("v_readlane") \
                or op.startswith("v_readfirstlane"):
            uses = regs(args)
        else:
            defs = regs(ops[0]) if ops else set()
            for o in ops[1:]:
                uses |= regs(o)
            if op.startswith(ACC):
                uses |= defs
        targets = []
        falls = True
        if op.startswith("s_branch"):
            targets = [args.strip()]
            falls = False
        elif op.startswith("s_cbranch"):
            targets = [args.strip()]
        elif op.startswith(("s_endpgm", "s_setpc")):
            falls = False
        insts.append((op, defs, uses, loc, None, targets, falls))
    return insts


def main():
    path, fn = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    insts = parse(lines[st + 1:en])
    label_at = {ins[4]: i for i, ins in enumerate(insts) if ins[0] == "LABEL"}
    n = len(insts)
    succ = [[] for _ in range(n)]
    for i, ins in enumerate(insts):
        for t in ins[5]:
            if t in label_at:
                succ[i].append(label_at[t])
        if ins[6] and i + 1 < n:
            succ[i].append(i + 1)
    live_in = [set() for _ in range(n)]
    changed = True
    while changed:
        changed = False
        for i in range(n - 1, -1, -1):
            out = set()
            for s in succ[i]:
                out |= live_in[s]
            new = (out - insts[i][1]) | insts[i][2]
            if new != live_in[i]:
                live_in[i] = new
                changed = True
    # last def site of each register along the listing (approximate provenance)
    peak = sorted(range(n), key=lambda i: -len(live_in[i]))[:1][0]
    print(f"instructions {n}, peak live VGPRs {len(live_in[peak])} at listing index {peak} (loc {insts[peak][3]})")
    hist = Counter()
    for i in range(n):
        hist[len(live_in[i]) // 10 * 10] += 1
    print("pressure histogram:", dict(sorted(hist.items())))
    by_loc = defaultdict(int)
    for i in range(n):
        if len(live_in[i]) >= len(live_in[peak]) - 5:
            by_loc[insts[i][3]] += 1
    print("source lines of the near-peak points:", sorted(by_loc.items())[:40])
    # provenance: nearest preceding def of each live register
    prov = Counter()
    for r in sorted(live_in[peak]):
        j = peak - 1
        while j >= 0 and r not in insts[j][1]:
            j -= 1
        prov[insts[j][3] if j >= 0 else (-1, -1)] += 1
    print("defining source lines of the peak's live registers:", sorted(prov.items()))
    mx = defaultdict(int)
    for i in range(n):
        mx[insts[i][3]] = max(mx[insts[i][3]], len(live_in[i]))
    top = sorted(mx.items(), key=lambda kv: -kv[1])[:60]
    print("highest pressure per source line:", top)


if __name__ == "__main__":
    main()
