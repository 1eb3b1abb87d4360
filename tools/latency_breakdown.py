"""Where p50 ingest->alert goes: the per-batch chain from a bench.py --trace Chrome trace.

The headline's second metric (bench.py `p50_ingest_to_alert_ms`) is the time from a
batch's arrival (its parse launch, tid 0 "parse" start) to the moment its rollover's alert
candidates are on the host (tid 1 "rollover wait" end, engine.cpp finish_rollover_body).  Every
stage of that chain is a trace span; this lists, averaged over the timed batches, each span's start
and end relative to the batch's arrival, in chain order, plus the p50 of the end-to-end time.
Spans recorded once per batch are matched to batches by their order of occurrence.

    python tools/latency_breakdown.py gpurun_out/r6f/trace_13.json [skip_batches] > profiles/.../latency.md
"""
import collections
import json
import sys

THREADS = {0: "ingest", 1: "stats", 2: "join detail", 3: "ahead lane", 4: "output lane"}


def main(path, skip=10):
    t = json.load(open(path))
    ev = t["traceEvents"] if isinstance(t, dict) else t
    xs = sorted((e for e in ev if e.get("ph") == "X"), key=lambda e: e["ts"])
    by = collections.defaultdict(list)
    for e in xs:
        by[(e["tid"], e["name"])].append(e)
    parse = by[(0, "parse")]
    wait = by[(1, "rollover wait")]
    n = min(len(parse), len(wait))
    rows = []
    lat = []
    for k in range(skip, n):
        t0 = parse[k]["ts"]
        lat.append((wait[k]["ts"] + wait[k]["dur"] - t0) / 1000.0)
    for (tid, name), es in by.items():
        if len(es) < n:
            continue  # not once per batch (several per batch, or only some batches)
        st = [(es[k]["ts"] - parse[k]["ts"]) / 1000.0 for k in range(skip, n)]
        en = [(es[k]["ts"] + es[k]["dur"] - parse[k]["ts"]) / 1000.0 for k in range(skip, n)]
        if not st:
            continue
        rows.append((sum(st) / len(st), sum(en) / len(en), tid, name))
    rows.sort()
    lat.sort()
    print(f"# ingest -> alert chain ({len(lat)} batches, {path.split('/')[-1]})\n")
    print(f"p50 ingest->alert {lat[len(lat) // 2]:.3f} ms (min {lat[0]:.3f}, max {lat[-1]:.3f})\n")
    print("| span | thread | starts at ms | ends at ms | ms |")
    print("|---|---|---|---|---|")
    for s, e, tid, name in rows:
        if s > lat[-1] + 1.0:
            continue  # the next batch's work
        print(f"| {name} | {THREADS.get(tid, tid)} | {s:.3f} | {e:.3f} | {e - s:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
