"""Per-lane busy time per step from a bench.py --trace Chrome trace (timed batches only).

    python tools/trace_summary.py gpurun_out/trace.json [first_batch]
"""
import collections
import json
import sys


def main(path, first=7):
    t = json.load(open(path))
    ev = t["traceEvents"] if isinstance(t, dict) else t
    xs = [e for e in ev if e.get("ph") == "X" and e.get("args", {}).get("batch", 0) >= first]
    nb = len({e["args"]["batch"] for e in xs}) or 1
    agg = collections.defaultdict(float)
    for e in xs:
        agg[(e["tid"], e["name"])] += e["dur"]
    for (tid, name), d in sorted(agg.items()):
        print(f"tid {tid} {name:24s} {d / 1000 / nb:8.3f} ms/batch")
    span = (max(e["ts"] + e["dur"] for e in xs) - min(e["ts"] for e in xs)) / 1000
    print(f"batches {nb}  wall {span:.2f} ms  ({span / nb:.3f} ms/batch)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 7)
