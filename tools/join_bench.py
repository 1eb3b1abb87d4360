"""CPU microbenchmark of the host join workers (csrc/runtime/join.cpp).

Events come from ops/parse_ref.py (the Python model of the parse kernels) over the native
synthetic generator's output for one JVM, so this runs without a GPU.  Usage:
    python tools/join_bench.py [--batches 6] [--tx-rate 250]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from apmbackend_amd import _native
from apmbackend_amd.ops.parse_ref import parse_batch, tz_table
from apmbackend_amd.utils.timeparse import TzOffset


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--tx-rate", type=float, default=250.0)
    ap.add_argument("--ejb", type=int, default=6000)
    ap.add_argument("--providers", type=int, default=4000)
    a = ap.parse_args()
    N = _native.load()
    UTC = TzOffset("UTC")
    gen = N.SynthGen({"servers": 1, "ejb_services": a.ejb, "provider_services": a.providers,
                      "tx_per_sec_per_server": a.tx_rate, "seed": 3})
    h = N.JoinHarness({"tz_table": tz_table(UTC)})
    files = gen.files()
    for path, kind, server in files:
        h.add_file(path, kind, server)
    start = 1578391200000
    fo = {}
    tot_t = tot_ev = tot_tx = 0
    for b in range(a.batches):
        data, chunks = gen.generate(start + (b + 1) * 10000, 4)
        bch = [(files[f][1], data[lo:hi]) for f, lo, hi in chunks]
        cf = [f for f, _, _ in chunks]
        ev, n_lines, wm, buf = parse_batch(bch, UTC, fo, cf)
        t0 = time.perf_counter()
        out = h.process(ev.tobytes(), buf, cf, float(start + b * 10000))
        dt = time.perf_counter() - t0
        if b > 0:
            tot_t += dt
            tot_ev += len(ev)
            tot_tx += len(out)
        print(f"batch {b}: lines={n_lines} events={len(ev)} tx={len(out)} join+py={dt*1e3:.2f} ms")
    print(f"steady: {tot_t / max(tot_ev, 1) * 1e9:.0f} ns/event, {tot_t / max(tot_tx, 1) * 1e9:.0f} ns/tx "
          f"(includes Python list conversion)")


if __name__ == "__main__":
    main()
