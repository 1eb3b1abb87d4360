"""Reference resume-file exporter / importer (runtime/resume_compat.py) on the GPU engine:
the exported documents hold exactly the state the reference's own stages hold after the same
input (checked against the oracle's data structures), and export -> import -> export is the
identity."""
import collections
import copy
import json
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.runtime import resume_compat as rc  # noqa: E402
from test_engine_gpu import UTC, small_cfg, synth_batches  # noqa: E402


def norm_stats(doc):
    d = json.loads(json.dumps(doc))
    for so in d["servers"].values():
        for sv in so["services"].values():
            for k in sv["buckets"]:
                sv["buckets"][k] = sorted(sv["buckets"][k])
    d["minHeap"]["content"] = sorted(json.dumps(o, sort_keys=True) for o in d["minHeap"]["content"])
    return d


def same_num(a, b):
    if a is None or b is None:
        return a is None and b is None
    return a == b or (math.isnan(a) and math.isnan(b))


def test_export_matches_reference_state_and_roundtrips():
    lines, bl = synth_batches(7, duration=700)
    C = small_cfg("exact")
    eng = APMEngine(C, keep_text=True)
    P = PipelineOracle(copy.deepcopy(C), UTC)
    for now, chunks in bl:
        eng.process_lines(chunks, now)
    P.run_batches(bl)
    stats, zscore, alerts = rc.export_reference_resume(eng)

    # ---- stats: buckets, latest label, pending heap == StatParser state
    assert int(stats["latestBucket"]) == P.st.latest
    for srv, svcs in P.st.servers.items():
        for svc, buckets in svcs.items():
            got = stats["servers"][srv]["services"][svc]["buckets"]
            assert {int(k): sorted(v) for k, v in got.items()} == {k: sorted(v) for k, v in buckets.items() if v}
    heap = sorted((tx.endTs, tx.logId, tx.service) for tx in P.st.heap.content)
    exp = sorted((o["endTs"], o["logId"], o["service"]) for o in stats["minHeap"]["content"])
    assert exp == heap and len(exp) > 0

    # ---- z-score: the per-series LAG lists (exact mode: bit-identical values)
    n_checked = 0
    for srv, svcs in P.zs.servers.items():
        for svc, lags in svcs.items():
            node = zscore["servers"][srv]["services"][svc]["lags"]
            for lag, o in lags.items():
                for k in rc.STAT_LISTS:
                    want = [None if (v is None or (isinstance(v, float) and math.isnan(v))) else v for v in o[k]]
                    got = node[str(lag)][k]
                    assert len(got) == len(want)
                    assert all(same_num(a, b) for a, b in zip(got, want)), (srv, svc, lag, k)
                    n_checked += 1
    assert n_checked > 10

    # ---- roundtrip through a fresh engine
    eng2 = APMEngine(C, keep_text=True)
    info = rc.import_reference_resume(eng2, stats, zscore, alerts)
    assert info["series"] == len(eng.eng.export_series())
    s2, z2, a2 = rc.export_reference_resume(eng2)
    assert norm_stats(s2) == norm_stats(stats)
    assert json.dumps(z2) == json.dumps(zscore)
    assert dict(a2["alerts"]) == dict(alerts["alerts"]) and len(alerts["alerts"]) > 0


def test_import_then_continue_produces_stats_rows():
    """An imported engine keeps emitting st/fs rows for every resumed series at the next
    rollover, in the resumed emission order."""
    lines, bl = synth_batches(8, duration=600)
    C = small_cfg("exact")
    eng = APMEngine(C, keep_text=True)
    cut = len(bl) // 2
    for now, chunks in bl[:cut]:
        eng.process_lines(chunks, now)
    eng.take("st")
    stats, zscore, alerts = rc.export_reference_resume(eng)
    eng2 = APMEngine(C, keep_text=True)
    rc.import_reference_resume(eng2, stats, zscore, alerts)
    for now, chunks in bl[cut:cut + 4]:
        eng2.process_lines(chunks, now)
    st = eng2.take("st")
    assert st, "no st rows after import"
    first_ts = st[0].split("|")[1]
    first_round = [l.split("|")[2:4] for l in st if l.split("|")[1] == first_ts]
    want = [list(k) for k in eng.eng.export_series()]
    assert first_round[:len(want)] == want[:len(first_round)]
