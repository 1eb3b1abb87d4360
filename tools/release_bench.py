#!/usr/bin/env python3
"""Isolated timing of the release kernels on one GPU (txcopy.hip apm_release_bench): the wire
gather (k_gather_lines) and the GPU COPY encoder (k_txcopy_len + scan + k_txcopy_write) over a
rollover's worth of released tx lines in shuffled ring order, each alone on its stream -- the
per-kernel numbers a concurrent bench trace cannot give (there every kernel shares the CUs with
the parse and join streams).

    python -m tools.release_bench <out dir>      (gpu.sh task py:tools.release_bench)
"""
import json
import os
import sys


def main(out_dir):
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    rows = []
    for n in (20000, 60000, 200000, 1000000):
        r = N.release_bench(n, 20, 1)
        r["gather_GBps"] = r["wire_bytes"] / r["gather_us"] / 1e3
        r["txcopy_GBps_out"] = r["copy_bytes"] / r["txcopy_us"] / 1e3
        r["txcopy_write_GBps_out"] = r["copy_bytes"] / r["txcopy_write_us"] / 1e3
        rows.append(r)
        print(json.dumps(r), flush=True)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "release_bench.json"), "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/release_bench")
