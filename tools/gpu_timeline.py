#!/usr/bin/env python3
"""GPU timeline of a rocprofv3 run (--kernel-trace [--memory-copy-trace], csv): busy time of
the steady-state batches.

The window is the last `steps` batches, delimited by the launches of the parse kernel (one per
batch).  Reported: wall time per batch, the union of kernel time (GPU busy), the union of copy
time, kernels + copies together, and the top kernels by time inside the window.

    python tools/gpu_timeline.py <rocprof out dir> [--steps N] [--anchor k_parse_lines]
"""
import argparse
import collections
import csv
import glob
import os
import re


def _rows(d, pat):
    out = []
    for p in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def _union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def short(n):
    n = re.sub(r"rocprim::ROCPRIM_\w+::", "rocprim::", n).replace("(anonymous namespace)::", "")
    m = re.search(r"wrapped_(\w+?)_config", n)
    if "trampoline_kernel" in n and m:
        return "rocprim::" + m.group(1)
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--anchor", default="k_parse_lines")
    a = ap.parse_args()
    ks = _rows(a.dir, "*kernel_trace.csv")
    cs = _rows(a.dir, "*memory_copy_trace.csv")
    kern = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in ks]
    qcol = next((c for c in ("Stream_Id", "Queue_Id") if ks and c in ks[0]), None)
    kq = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get(qcol, "?")) for r in ks] if qcol else []
    cop = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy")) for r in cs]
    anchors = sorted(s for s, _e, n in kern if a.anchor in n)
    if len(anchors) < a.steps + 1:
        raise SystemExit(f"only {len(anchors)} {a.anchor} launches")
    t0, t1 = anchors[-a.steps - 1], anchors[-1]
    n = a.steps
    kin = [(max(s, t0), min(e, t1), nm) for s, e, nm in kern if e > t0 and s < t1]
    cin = [(max(s, t0), min(e, t1), d) for s, e, d in cop if e > t0 and s < t1]
    wall = t1 - t0
    kb = _union([(s, e) for s, e, _ in kin])
    cb = _union([(s, e) for s, e, _ in cin])
    ab = _union([(s, e) for s, e, _ in kin] + [(s, e) for s, e, _ in cin])
    print(f"window: {n} batches, {wall / 1e6 / n:.3f} ms/batch")
    print(f"kernels busy (union): {kb / 1e6 / n:.3f} ms/batch ({100.0 * kb / wall:.1f} %)")
    print(f"copies busy (union):  {cb / 1e6 / n:.3f} ms/batch ({100.0 * cb / wall:.1f} %)")
    print(f"GPU busy (kernels + copies, union): {ab / 1e6 / n:.3f} ms/batch ({100.0 * ab / wall:.1f} %)")
    print(f"kernel launches per batch: {len(kin) / n:.1f}, copies per batch: {len(cin) / n:.1f}")
    if kq:  # busy time per stream / hardware queue: which one is saturated
        byq = collections.defaultdict(list)
        for s_, e_, q in kq:
            if e_ > t0 and s_ < t1:
                byq[q].append((max(s_, t0), min(e_, t1)))
        print(f"\n| {qcol} | kernels/batch | busy ms/batch | busy % |\n|---|---|---|---|")
        for q, iv in sorted(byq.items(), key=lambda x: -_union(x[1])):
            u = _union(iv)
            print(f"| {q} | {len(iv) / n:.1f} | {u / 1e6 / n:.3f} | {100.0 * u / wall:.1f} |")
    by = collections.defaultdict(lambda: [0, 0])
    for s, e, nm in kin:
        by[short(nm)][0] += e - s
        by[short(nm)][1] += 1
    for s, e, d in cin:
        by["[copy " + d + "]"][0] += e - s
        by["[copy " + d + "]"][1] += 1
    print("\n| kernel | calls/batch | us/batch |\n|---|---|---|")
    for k, (t, c) in sorted(by.items(), key=lambda x: -x[1][0])[:40]:
        print(f"| {k} | {c / n:.1f} | {t / 1e3 / n:.1f} |")
    if qcol:  # the runtime's own kernels (hipMemsetAsync fills, hipMemcpyAsync blits) per stream
        rt = collections.defaultdict(lambda: [0, 0])
        for r in ks:
            s_, e_ = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if not (e_ > t0 and s_ < t1):
                continue
            nm = r["Kernel_Name"]
            kind = "fill" if "fillBuffer" in nm else ("blit" if "copyBuffer" in nm or "copyImage" in nm else None)
            if kind:
                rt[(kind, r.get(qcol, "?"))][0] += 1
                rt[(kind, r.get(qcol, "?"))][1] += e_ - s_
        print(f"\n| runtime kernel | {qcol} | per batch | us/batch |\n|---|---|---|---|")
        for (kind, q), (c, t) in sorted(rt.items()):
            print(f"| {kind} | {q} | {c / n:.1f} | {t / 1e3 / n:.1f} |")
        for kind in ("fill", "blit"):
            c = sum(v[0] for (k, _q), v in rt.items() if k == kind)
            print(f"{kind}s per batch (all streams): {c / n:.1f}")


if __name__ == "__main__":
    main()
