#!/usr/bin/env python3
"""Summarise bench.py --rank-report directories (one rankR.json per rank) as markdown: per rank
the lines it processed, its communicator size, the node-wide counters it saw, and the per-step
time distribution (p50 / p90 / p99 / max and a coarse histogram) with the time spent in the
per-batch lock-step clock collective.

    python tools/rank_summary.py <report dir> [<report dir> ...] > profiles/r4_ranks/README.md
"""
import glob
import json
import os
import sys


def pct(v, p):
    v = sorted(v)
    return v[min(len(v) - 1, (p * len(v)) // 100)] if v else float("nan")


def hist(v, edges=(0.5, 1, 1.5, 2, 3, 5, 10, 1e9)):
    out, lo = [], 0.0
    for e in edges:
        n = sum(1 for x in v if lo <= x < e)
        out.append(f"{'<' if lo == 0 else ''}{e if e < 1e9 else '>' + str(edges[-2])}: {n}")
        lo = e
    return ", ".join(out)


def main(dirs):
    for d in dirs:
        reps = [json.load(open(p)) for p in sorted(glob.glob(os.path.join(d, "rank*.json")))]
        if not reps:
            continue
        print(f"## {os.path.basename(os.path.normpath(d))}: {len(reps)} ranks, collective `{reps[0]['coll']}`\n")
        print("| rank | device | comm ranks | lines (timed) | node ranks / lines seen | step ms p50 | p90 | p99 | max "
              "| lock-step ms/step | lock-step max ms |")
        print("|---|---|---|---|---|---|---|---|---|---|---|")
        for r in reps:
            s = r["step_ms"]
            nm = r.get("node_metrics") or [0, 0, 0]
            print(f"| {r['rank']} | {r['device']} | {r['comm_ranks']} | {r['lines_timed']:,} | {nm[0]:.0f} / {nm[2]:,.0f} "
                  f"| {pct(s, 50):.3f} | {pct(s, 90):.3f} | {pct(s, 99):.3f} | {max(s):.3f} "
                  f"| {r['lockstep_ms_per_step']:.3f} | {r['lockstep_max_ms']:.3f} |")
        print("\nPer-step time histogram (ms), per rank:\n")
        for r in reps:
            print(f"- rank {r['rank']}: {hist(r['step_ms'])}")
        print()


if __name__ == "__main__":
    main(sys.argv[1:])
