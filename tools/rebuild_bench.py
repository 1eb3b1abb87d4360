#!/usr/bin/env python3
"""Isolated timing of the join's key-table rebuild (devjoin.hip apm_dj_rebuild_selftest): the
in-place cluster compaction against the reinsert into a zeroed copy, one kernel alone on the GPU,
at table sizes around the headline's 2M slots and its steady-state load.

    python -m tools.rebuild_bench <out dir>      (gpu.sh task py:tools.rebuild_bench)
"""
import json
import os
import sys


def main(out_dir):
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    rows = []
    for cap in (1 << 20, 1 << 21, 1 << 22):
        for copy in (False, True):
            N.dj_rebuild_selftest(cap, 0.55, 0.2, 1, copy)  # (code object load)
            runs = [N.dj_rebuild_selftest(cap, 0.55, 0.2, 2 + i, copy) for i in range(5)]
            r = dict(runs[0])
            r["us"] = min(x["us"] for x in runs)
            r.update(cap=cap, form="reinsert (+ memset of the copy, not timed)" if copy else "in place",
                     ok=all(x["found"] == x["want_live"] == x["live"] and x["dead_left"] == 0 for x in runs))
            rows.append(r)
            print(json.dumps(r), flush=True)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "rebuild_bench.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/rebuild_bench")
