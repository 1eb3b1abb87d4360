"""st stream of the GPU engine vs the CPU oracle as the number of JVMs grows (exact mode)."""
import collections
import copy
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_engine_gpu as T  # noqa: E402
from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402

for servers in [int(x) for x in sys.argv[1:]]:
    lines, bl = T.synth_batches(10, duration=120, servers=servers)
    P = PipelineOracle(copy.deepcopy(T.small_cfg("exact")), T.UTC)
    P.run_batches(bl)
    eng = APMEngine(T.small_cfg("exact"), keep_text=True)
    st = []
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        st += eng.take("st")
    bad = set(st) ^ set(P.stats)
    print(f"servers={servers}: st {len(st)} vs oracle {len(P.stats)}; differing {len(bad)}; series {eng.eng.n_series()}",
          sorted(collections.Counter(l.split('|')[2] for l in bad).items())[:6], flush=True)
