"""Roofline table of the engine's kernels from rocprofv3 --pmc passes (tools/gpu.sh `pmc:` tasks).

Every pass collects its counters with the dispatches serialised, so a kernel's duration in the
pass's own kernel trace is its isolated time.  Counters and durations are summed over every
dispatch of the profiled bench run (10 timed + 3 warmup + the pre-history batches) and joined across
passes by kernel name.  Per kernel:

  * HBM GB/s      = (FETCH_SIZE + WRITE_SIZE) [KiB] x 1024 / time   (L2 <-> HBM/MALL traffic)
  * % HBM         = of the 6.3 TB/s a streaming copy reaches on MI355X (8 TB/s spec,
                    MI355X_MICROARCH.md "HBM [CDNA4]")
  * f64 MFMA TF/s = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 / time (the counter counts MFMA f64 flops / 512)
  * MFMA busy %   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs)
  * VALU/wave, LDS conflict cycles per LDS instruction, L2 hit %
  * bound         = HBM (>= 50 % of 6.3 TB/s), MFMA (busy >= 50 %), launch (< 8 us per dispatch),
                    else latency (neither pipe near its roof: dependent loads, atomics, divergence)

    python tools/roofline.py gpurun_out/r6f profiles/r6_f/roofline.md [top N]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import collect  # noqa: E402

HBM_ACHIEVABLE = 6.3e12   # B/s, float4 copy (MI355X_MICROARCH.md)
HBM_SPEC = 8.0e12
F64_MFMA_PEAK = 78.6e12   # FLOP/s, MI355X FP64 matrix (spec sheet)
SIMDS = 256 * 4


def calls_of(root):
    import csv
    import glob
    from prof_summary import short
    n = {}
    for d in sorted(glob.glob(os.path.join(root, "pmc*"))):
        for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(p)):
                k = short(r.get("Kernel_Name", "?"))
                n[k] = n.get(k, 0) + 1
        if n:
            return n
    return n


def main(root, dst, top="16"):
    ctr, dur = collect(root)
    calls = calls_of(root)
    names = sorted(dur, key=lambda k: -dur[k])[: int(top)]
    rows = []
    for k in names:
        c = ctr.get(k, {})
        t = dur[k]
        by = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
        gbs = by / t if t > 0 else 0.0
        flops = c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512.0
        tfs = flops / t if t > 0 else 0.0
        act = c.get("GRBM_GUI_ACTIVE", 0.0)
        busy = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (act * SIMDS) if act else 0.0
        vpw = c["SQ_INSTS_VALU"] / c["SQ_WAVES"] if c.get("SQ_WAVES") else 0.0
        lds = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_INSTS_LDS"] if c.get("SQ_INSTS_LDS") else 0.0
        h = c.get("TCC_HIT_sum", c.get("TCC_HIT", 0.0))
        m = c.get("TCC_MISS_sum", c.get("TCC_MISS", 0.0))
        hit = 100.0 * h / (h + m) if h + m else 0.0
        n = calls.get(k, 0)
        per = t / n * 1e6 if n else 0.0
        if gbs >= 0.5 * HBM_ACHIEVABLE:
            bound = "HBM"
        elif busy >= 50.0:
            bound = "MFMA"
        elif n and per < 8.0:
            bound = "launch"
        else:
            bound = "latency"
        rows.append((k, n, t * 1e3, per, by / 1e6, gbs / 1e9, 100.0 * gbs / HBM_ACHIEVABLE, tfs / 1e12,
                     100.0 * tfs / F64_MFMA_PEAK, busy, vpw, lds, hit, bound))
    with open(dst, "w") as f:
        f.write("# Roofline: isolated kernel time vs MI355X HBM and f64 MFMA roofs\n\n")
        f.write(__doc__.split("\n\n")[1] + "\n\n")
        f.write("| kernel | calls | ms | us/call | HBM MB | GB/s | % of 6.3 TB/s | f64 MFMA TF/s | % of 78.6 TF/s "
                "| MFMA busy % | VALU/wave | LDS confl/inst | L2 hit % | bound |\n")
        f.write("|---|" + "---|" * 14 + "\n")
        for r in rows:
            f.write(f"| {r[0]} | {r[1]} | {r[2]:.3f} | {r[3]:.1f} | {r[4]:.1f} | {r[5]:.0f} | {r[6]:.1f} | {r[7]:.3f} | "
                    f"{r[8]:.2f} | {r[9]:.2f} | {r[10]:.0f} | {r[11]:.2f} | {r[12]:.0f} | {r[13]} |\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
