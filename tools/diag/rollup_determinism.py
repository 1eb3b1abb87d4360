"""Runs the K14 70-JVM rollup input twice through fresh engines and diffs the st / sx / fs streams
(run-to-run determinism check; a tolerance check of this input failed on 2 of 5 GPU runs)."""
import sys
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_engine_gpu as T  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.runtime.jmx import SyntheticJmx  # noqa: E402
from apmbackend_amd.utils.records import JmxEntry  # noqa: E402


def run():
    lines, bl = T.synth_batches(10, duration=200, servers=70)
    eng = APMEngine(T.small_cfg("exact"), keep_text=True)
    jx = JmxEntry.from_stats(T.START, "jvm00", SyntheticJmx(5).payload("jvm00")).to_csv()
    out = {k: [] for k in ("st", "sx", "fs", "transactions")}
    for i, (now, chunks) in enumerate(bl):
        eng.process_lines(chunks, now)
        if i == 3:
            eng.set_server_context(jx, vm_load=1.5)
        for k in out:
            out[k] += eng.take(k)
    return out


runs = [run() for _ in range(3)]
import copy  # noqa: E402
from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
P = PipelineOracle(copy.deepcopy(T.small_cfg("exact")), T.UTC)
P.run_batches(T.synth_batches(10, duration=200, servers=70)[1])
for r in range(len(runs)):
    bad = [l for l in set(runs[r]["st"]) ^ set(P.stats)]
    import collections
    print(f"st run{r} vs oracle: {len(bad)} differing lines;",
          sorted(collections.Counter(l.split("|")[1] for l in bad).items())[:8])
for k in runs[0]:
    for r in range(1, len(runs)):
        a, b = runs[0][k], runs[r][k]
        same = a == b
        print(f"{k}: run0 vs run{r}: {'identical' if same else 'DIFFER'} ({len(a)} vs {len(b)} lines)")
        if not same:
            sa, sb = set(a), set(b)
            print("   only in run0:", sorted(sa - sb)[:5])
            print("   only in run%d:" % r, sorted(sb - sa)[:5])
            print("   same multiset:", sorted(a) == sorted(b))
            import collections
            c = collections.Counter(l.split("|")[1] for l in sa ^ sb)
            print("   differing lines per ts:", sorted(c.items())[:12])
