"""Host-join profiler: dumps one JVM's synthetic batches (bench shape) as parse events and
replays them through tests/native/join_replay.cpp built at -O3 (optionally with
-DAPM_JOIN_PROF for per-event-kind cycle counts).  CPU only.

    python tools/join_prof.py [--batches 6] [--prof]
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from apmbackend_amd import _native  # noqa: E402
from apmbackend_amd.ops.parse_ref import parse_batch, tz_table  # noqa: E402
from apmbackend_amd.utils.timeparse import TzOffset  # noqa: E402

CSRC = os.path.join(ROOT, "apmbackend_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--tx-rate", type=float, default=250.0)
    ap.add_argument("--ejb", type=int, default=6000)
    ap.add_argument("--providers", type=int, default=4000)
    ap.add_argument("--prof", action="store_true", help="per-event-kind rdtsc cycle counts")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--hip", action="store_true", help="link the HIP runtime (JOIN_REPLAY_PINNED=1 replays from pinned memory)")
    a = ap.parse_args()
    N = _native.load()
    UTC = TzOffset("UTC")
    gen = N.SynthGen({"servers": 1, "ejb_services": a.ejb, "provider_services": a.providers,
                      "tx_per_sec_per_server": a.tx_rate, "seed": 3})
    files = gen.files()
    d = a.dir or tempfile.mkdtemp(prefix="joinprof_")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "files.txt"), "w") as f:
        for path, kind, server in files:
            f.write(f"{path}\t{kind}\tsrv{server}\n")
    start = 1578391200000
    fo = {}
    for b in range(a.batches):
        data, chunks = gen.generate(start + (b + 1) * 10000, 4)
        bch = [(files[fi][1], data[lo:hi]) for fi, lo, hi in chunks]
        cf = [fi for fi, _, _ in chunks]
        ev, _, _, buf = parse_batch(bch, UTC, fo, cf)
        pre = os.path.join(d, f"batch_{b}")
        with open(pre + ".meta", "w") as f:
            f.write(f"{float(start + b * 10000)!r}\n" + "".join(f"{c}\n" for c in cf))
        with open(pre + ".events", "wb") as f:
            f.write(ev.tobytes())
        with open(pre + ".bytes", "wb") as f:
            f.write(bytes(buf))
    exe = os.path.join(d, "join_replay")
    cmd = ["hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "-I", CSRC,
           os.path.join(ROOT, "tests", "native", "join_replay.cpp"), os.path.join(CSRC, "runtime", "join.cpp"),
           "-o", exe] + (["-DAPM_JOIN_PROF"] if a.prof else []) + (["-DJOIN_REPLAY_HIP"] if a.hip else [])
    subprocess.run(cmd, check=True)
    r = subprocess.run([exe, d, str(a.batches)], env=dict(os.environ, JOIN_REPLAY_QUIET="1"),
                       capture_output=True, text=True)
    sys.stderr.write(r.stderr)
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
