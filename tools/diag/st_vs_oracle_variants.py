"""st vs the CPU oracle at 48 JVMs under config variants (which stage breaks past ~40 JVMs)."""
import collections
import copy
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_engine_gpu as T  # noqa: E402
from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402

VARIANTS = {
    "base": {},
    "host_join": {"joinOnDevice": False},
    "cells16": {"bucketCellCapacity": 16},
    "cells64_spill1M": {"bucketCellCapacity": 64, "bucketOverflowCapacity": 1 << 20},
    "spill1M": {"bucketOverflowCapacity": 1 << 20},
    "maxSeries64k": {"maxSeries": 1 << 16},
}
servers = int(sys.argv[1]) if len(sys.argv) > 1 else 48
lines, bl = T.synth_batches(10, duration=120, servers=servers)
P = PipelineOracle(copy.deepcopy(T.small_cfg("exact")), T.UTC)
P.run_batches(bl)
for name, g in VARIANTS.items():
    C = T.small_cfg("exact")
    C["gpu"].update(g)
    eng = APMEngine(C, keep_text=True)
    st, tx = [], []
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        st += eng.take("st")
        tx += eng.take("transactions")
    bad = set(st) ^ set(P.stats)
    m = eng.metrics()
    print(f"{name}: st differing {len(bad)} of {len(P.stats)}; tx == oracle: {sorted(tx) == sorted(P.tx_out)}; "
          f"metrics: " + ", ".join(f"{k}={m[k]}" for k in m if any(w in k for w in ("spill", "overflow", "drop", "lost"))),
          flush=True)
