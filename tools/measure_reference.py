"""Measure the reference implementation's throughput on CPU (BASELINE config 1) and record it in
profiles/reference_cpu_baseline.json, which bench.py uses for ``vs_baseline``.

The corpus comes from the same native synthetic generator as bench.py (one JVM, 100 services,
the bench's per-JVM transaction rate, 10 s batches with the engine's watermark clock); the
reference's stage code runs unmodified in one node process (tools/reference_pipeline.js).

Usage: python tools/measure_reference.py [--batches 60] [--services 100] [--out profiles/...]
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def write_corpus(path, batches, servers, ejb, providers, rate, seed=1):
    from apmbackend_amd import _native
    from apmbackend_amd.utils.timeparse import TzOffset, leading_line_ts
    N = _native.load(build_if_missing=False)
    gen = N.SynthGen({"servers": servers, "ejb_services": ejb, "provider_services": providers,
                      "tx_per_sec_per_server": rate, "seed": seed})
    files = gen.files()
    start = 1578391200000
    tz = TzOffset("UTC")
    wm = 0.0
    n_lines = 0
    with open(path, "w") as f:
        for b in range(batches):
            data, chunks = gen.generate(start + (b + 1) * 10000, 4)
            f.write(f"#B {wm:.0f}\n")
            for fid, lo, hi in chunks:
                f.write(f"#F {files[fid][0]}\n")
                txt = data[lo:hi].decode("utf-8")
                f.write(txt)
                for ln in txt.split("\n"):
                    if ln:
                        n_lines += 1
                        v = leading_line_ts(ln, tz)
                        if v is not None and v > wm:
                            wm = v
    return n_lines


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--servers", type=int, default=1)
    ap.add_argument("--ejb", type=int, default=60)
    ap.add_argument("--providers", type=int, default=40)
    ap.add_argument("--tx-rate", type=float, default=250.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "reference_cpu_baseline.json"))
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        corpus = os.path.join(td, "corpus.txt")
        t0 = time.time()
        n = write_corpus(corpus, a.batches, a.servers, a.ejb, a.providers, a.tx_rate)
        print(f"corpus: {n} lines in {time.time() - t0:.1f}s", file=sys.stderr)
        env = dict(os.environ, TZ="UTC")
        r = subprocess.run(["node", os.path.join(ROOT, "tools", "reference_pipeline.js"), corpus,
                            os.path.join(ROOT, "config", "apm_config.json"), "2"],
                           capture_output=True, text=True, env=env, timeout=3600)
        if r.returncode != 0:
            print(r.stderr, file=sys.stderr)
            sys.exit(r.returncode)
        res = json.loads(r.stdout.strip().splitlines()[-1])
    out = {
        "metric": "log-lines/sec z-scored (whole node)",
        "value": round(res["lines_per_s"], 1),
        "unit": "lines/s",
        "what": "reference stage code (parse->stats->zscore->alerts) unmodified, one node process, "
                "queues replaced by direct calls (upper bound on the deployed 5-process + RabbitMQ form)",
        "config": {"jvms": a.servers, "services": a.ejb + a.providers, "tx_per_s_per_jvm": a.tx_rate,
                   "batches": a.batches, "batch_seconds": 10},
        "host_cpu": cpu_model(),
        "raw": res,
        "measured_at": time.strftime("%Y-%m-%dT%H:%M:%S"),
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
