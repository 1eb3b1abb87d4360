"""One line per bench / torchrun log under a gpurun_out directory: lines/s, ms/step, p50/p99 step,
lock-step ms/step (rank reports when present).

    python tools/rank_brief.py gpurun_out/r6d
"""
import glob
import json
import os
import sys


def main(root):
    for log in sorted(glob.glob(os.path.join(root, "*.log"))):
        for line in open(log, errors="replace"):
            if not line.startswith('{"metric"'):
                continue
            d = json.loads(line)
            extra = {k: d[k] for k in ("step_ms_p50", "step_ms_p99", "drain_ms", "p50_ingest_to_alert_ms") if k in d}
            rep = os.path.join(root, os.path.basename(log)[:-4])
            lock = []
            for rj in sorted(glob.glob(os.path.join(rep, "rank*.json"))):
                r = json.load(open(rj))
                lock.append((r.get("lockstep_ms_per_step"), r.get("lockstep_max_ms")))
            print(f"{os.path.basename(log):24s} {d['value'] / 1e6:8.1f} M  {d.get('ms_per_step', float('nan')):.3f} ms  {extra}"
                  + (f"  lockstep(ms/step,max)={[(round(a, 3), round(b, 2)) for a, b in lock]}" if lock else ""))


if __name__ == "__main__":
    main(sys.argv[1])
