"""rocprofv3 --pmc passes (tools/gpu_check.sh `pmc` step) -> one markdown table per kernel.

Each pass directory holds `run_counter_collection.csv` with one row per (dispatch, counter).
Counters are summed over the dispatches of a kernel and joined across passes by kernel name;
durations come from the first pass's kernel trace.  Derived:
  * HBM GB/s  = (FETCH_SIZE + WRITE_SIZE) [KB] / kernel time (L2 <-> memory traffic);
  * VALU/wave = SQ_INSTS_VALU / SQ_WAVES;
  * LDS conflict = SQ_LDS_BANK_CONFLICT cycles per LDS instruction;
  * L2 hit %  = TCC_HIT / (TCC_HIT + TCC_MISS).

    python tools/pmc_summary.py gpurun_out profiles/pmc_kernels.md [title]
"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import short  # noqa: E402


def _rows(pattern):
    for p in sorted(glob.glob(pattern, recursive=True)):
        with open(p) as fh:
            yield from csv.DictReader(fh)


def collect(root):
    ctr = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    for d in sorted(glob.glob(os.path.join(root, "pmc*"))):
        if not os.path.isdir(d):
            continue
        for r in _rows(os.path.join(d, "**", "*counter_collection.csv")):
            k = short(r.get("Kernel_Name", "?"))
            ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if dur:
            continue
        for r in _rows(os.path.join(d, "**", "*kernel_trace.csv")):
            k = short(r.get("Kernel_Name", "?"))
            dur[k] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
    return ctr, dur


def main(root, dst, title="rocprofv3 hardware counters"):
    ctr, dur = collect(root)
    names = sorted(ctr, key=lambda k: -dur.get(k, 0.0))
    cols = sorted({c for k in ctr for c in ctr[k]})
    with open(dst, "w") as f:
        f.write(f"# {title}\n\n")
        f.write("Counters summed over every dispatch of the kernel in the profiled run; derived columns as in "
                "`tools/pmc_summary.py`.\n\n")
        f.write("| kernel | time ms | HBM GB/s | VALU/wave | LDS conflict cyc/inst | L2 hit % |\n")
        f.write("|---|---|---|---|---|---|\n")
        for k in names:
            c = ctr[k]
            t = dur.get(k, 0.0)
            by = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
            gbs = f"{by / t / 1e9:.0f}" if t > 0 and by > 0 else "-"
            vpw = f"{c['SQ_INSTS_VALU'] / c['SQ_WAVES']:.0f}" if c.get("SQ_WAVES") else "-"
            lds = f"{c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.2f}" if c.get("SQ_INSTS_LDS") else "-"
            h = c.get("TCC_HIT_sum", c.get("TCC_HIT", 0.0))
            m = c.get("TCC_MISS_sum", c.get("TCC_MISS", 0.0))
            hit = f"{100.0 * h / (h + m):.0f}" if h + m > 0 else "-"
            f.write(f"| {k} | {t * 1e3:.3f} | {gbs} | {vpw} | {lds} | {hit} |\n")
        f.write("\n## Raw counters\n\n| kernel | " + " | ".join(cols) + " |\n|---|" + "---|" * len(cols) + "\n")
        for k in names:
            f.write(f"| {k} | " + " | ".join(f"{ctr[k].get(c, 0.0):.0f}" for c in cols) + " |\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
