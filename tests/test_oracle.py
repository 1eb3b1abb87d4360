"""The CPU oracle against (a) SURVEY Appendix B golden values and (b) the reference's own JS
(executed under node through tests/js/ref_harness.js, byte-for-byte comparison)."""
import copy
import json
import math

import pytest

from apmbackend_amd.models.oracle import (AlertsOracle, JsBinaryHeap, ParseOracle, PipelineOracle,
                                          StatsOracle, ZScoreOracle, calc_percentile, js_average,
                                          js_stddev, percentile_ranks, process_zscore_stats)
from apmbackend_amd.utils.config import default_config
from apmbackend_amd.utils.records import FullStatEntry, StatEntry, TxEntry, entry_from_csv
from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks
from apmbackend_amd.utils.timeparse import TzOffset
from conftest import requires_reference

UTC = TzOffset("UTC")


def test_percentile_golden():
    gold = {1: (10, 10), 2: (20, 20), 3: (30, 30), 4: (30, 40), 5: (45, 50), 10: (85, 100),
            20: (150, 190), 31: (245, 305)}
    for n, (p75, p95) in gold.items():
        arr = [10 * (i + 1) for i in range(n)]
        assert calc_percentile(arr, 75) == p75
        assert calc_percentile(arr, 95) == p95
        for p, want in ((75, p75), (95, p95)):
            lo, hi = percentile_ranks(n, p)
            assert (arr[lo] + arr[hi]) / 2 == want


def test_average_stddev_golden():
    assert js_average([1, None, 3, float("nan")]) == 2
    assert js_stddev([5, 5, 5]) == pytest.approx(math.sqrt(5), rel=0, abs=0)
    assert js_stddev([1, 2, 3, 4]) == math.sqrt(2.5)
    assert js_stddev([0, 0]) is None
    assert js_average([]) is None


def test_process_zscore_golden():
    prev = [100 + (i % 5) for i in range(360)]
    r = process_zscore_stats(360, 20, 0.1, 500, prev)
    assert r == (0.1 * 500 + (1 - 0.1) * 104, 102, -99.99009876724153, 303.99009876724153, 1)
    r2 = process_zscore_stats(360, 20, 0.1, 300, prev)
    assert r2[4] == 0 and r2[0] == 300


def test_zscore_process_data_golden():
    cfg = default_config(replay=True)
    cfg["streamCalcZScore"]["defaults"] = [{"LAG": 3, "THRESHOLD": 2, "INFLUENCE": 0.5}]
    out = []
    z = ZScoreOracle(cfg, out.append)
    vals = [(100, 110, 120), (100, 110, 120), (100, 110, 120), (400, 500, 600), (None, None, None),
            (100, 110, 120)]
    for i, (a, b, c) in enumerate(vals):
        st = StatEntry.make(1000 * i, "srv", "svc", 1.0, a, b, c)
        z.consume(st.to_csv())
    avg_fields = [l.split("|")[6] for l in out]
    assert avg_fields[0] == "100.0:undefined:undefined:undefined:0"
    assert avg_fields[3] == "400.0:100.0:80.0:120.0:1"
    # stored value after the signal = 0.5*400 + 0.5*100 = 250 -> mean 150, sigma sqrt(150)
    assert out[3].split("|")[7] == "500.0:110.0:89.0:131.0:1.0"
    assert avg_fields[4] == "undefined:150.0:125.5:174.5:0"
    assert avg_fields[5] == "100.0:175.0:148.5:201.5:-1"


def test_override_aliasing_emulation():
    cfg = default_config(replay=True)
    z = ZScoreOracle(cfg, lambda l: None, emulate_aliasing=True)
    z.settings("S:getLateFeeWaiver")
    assert [d["THRESHOLD"] for d in cfg["streamCalcZScore"]["defaults"]] == [25.0, 25.0]
    cfg2 = default_config(replay=True)
    z2 = ZScoreOracle(cfg2, lambda l: None, emulate_aliasing=False)
    z2.settings("S:getLateFeeWaiver")
    assert [d["THRESHOLD"] for d in cfg2["streamCalcZScore"]["defaults"]] == [20.0, 15.0]


def test_alert_leaky_counter_golden():
    cfg = default_config(replay=True)
    a = AlertsOracle(cfg)
    fs = FullStatEntry.make(0, "srv", "S:x", 5, "360", 900, 100, 50, 150, 1, 900, 100, 50, 150, 1,
                            900, 100, 50, 150, 1)
    first = None
    for i in range(50):
        fs.timestamp = 1000 * i
        if a.process(entry_from_csv(fs.to_csv())) is not None and first is None:
            first = i + 1
    assert first == 45
    assert a.recent[("srv", "S:x", "360")] == 50


def test_stats_golden():
    st, db = [], []
    s = StatsOracle(st.append, db.append)
    base = 1578412800000
    for i in range(50):
        tx = TxEntry.make("srvA", "S:svc", "L", "1", base + i * 10000, base + i * 10000 + 5, i + 1, "Y")
        s.consume(tx.to_csv())
    # the 50th tx (bucket +49) triggers the rollover whose window is buckets +13..+43
    assert st[-1] == "st|1578413220000|srvA|S:svc|6.20|29.0|37.5|43.5"
    assert len(db) == 42  # endTs <= edge (bucket +42) released, in endTs order
    assert db == sorted(db, key=lambda l: int(l.split("|")[7]))
    assert StatsOracle.bucket_label(1578412801959) == 157841280


def test_binary_heap_order():
    h = JsBinaryHeap(lambda x: x[0])
    for i, v in enumerate([5, 3, 3, 9, 1, 3, 7]):
        h.push((v, i))
    out = h.pop_all_le(5)
    assert [x[0] for x in out] == [1, 3, 3, 3, 5]


def _synth(seed=1, duration=300, servers=2, anomalies=()):
    cfg = SynthConfig(servers=servers, duration_s=duration, tx_per_sec_per_server=3, seed=seed,
                      ejb_services=4, provider_services=3, anomalies=anomalies)
    lines = Generator(cfg).generate()
    return cfg, with_watermarks(batches(lines, cfg.start_ms, 5.0), UTC)


@requires_reference
@pytest.mark.parametrize("seed", [1, 2])
def test_parse_matches_reference_js(seed):
    import refjs
    _, bl = _synth(seed)
    out = []
    po = ParseOracle(lambda q, l: out.append([q, l]), tz=UTC)
    for now, chunks in bl:
        po.begin_batch(now)
        for fp, ls in chunks:
            for ln in ls:
                po.read_line(fp, ln)
    js = refjs.parse(bl)
    assert js["errors"] == []
    assert po.counters["need_expired"] > 0  # expiry path exercised
    assert out == js["records"]


@requires_reference
def test_stats_zscore_alerts_match_reference_js():
    import refjs
    start = 1578391200000
    an = [Anomaly("jvm00", "getSvc0001", start + 400_000, start + 1500_000, 30.0)]
    _, bl = _synth(1, duration=1500, anomalies=an)
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                         {"LAG": 30, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    C["streamCalcZScore"]["overrides"]["services"]["S:getSvc0002"] = {"6": {"THRESHOLD": 4.0, "INFLUENCE": 0.25}}
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 10
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 3
    C["streamProcessAlerts"]["perServiceAlertCooldownInMinutes"] = 2
    C["gpu"]["emulateOverrideAliasing"] = True
    ct = json.dumps(C)
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    js = refjs.stats(P.tx_out)
    assert js["st"] == P.stats
    assert js["db"] == P.tx_db
    assert refjs.zscore(ct, P.stats) == P.fs
    al = refjs.alerts(ct, P.fs, "entry")
    assert al == P.al and len(al) > 0


@requires_reference
def test_util_methods_match_reference_js():
    import random
    import refjs
    rng = random.Random(3)
    arrs = [sorted(rng.randint(1, 1000) for _ in range(rng.randint(1, 60))) for _ in range(40)]
    req_p = [[a, p] for a in arrs for p in (0, 25, 50, 75, 90, 95, 99, 100)]
    lists = [[rng.choice([None, rng.uniform(0, 500)]) for _ in range(rng.randint(0, 20))] for _ in range(30)]
    res = refjs.util(percentile=req_p, average=lists, stddev=lists)
    assert res["percentile"] == [calc_percentile(a, p) for a, p in req_p]
    for l, v in zip(lists, res["average"]):
        assert js_average(l) == v
    for l, v in zip(lists, res["stddev"]):
        mine = js_stddev(l)
        assert (mine is None and v is None) or mine == v


@requires_reference
def test_stats_nan_elapsed_matches_reference_js():
    """A tx whose elapsed is not a number (e.g. a CT exit line carrying 'time') is pushed as
    parseInt -> NaN: it counts toward tpm, poisons the average and lands wherever the JS
    binaryInsert's NaN comparisons put it, so later percentiles depend on arrival order
    (stream_calc_stats.js:131,172-184, util_methods.js:57-106)."""
    import random
    import refjs
    _, bl = _synth(2, duration=900)
    P = PipelineOracle(default_config(replay=True), UTC)
    P.run_batches(bl)
    rng = random.Random(11)
    lines = []
    for ln in P.tx_out:
        f = ln.split("|")
        if f[0] == "tx" and rng.random() < 0.02:
            f[7] = rng.choice(["time", "NaN", "", "abc"])
        lines.append("|".join(f))
    js = refjs.stats(lines)
    out_st, out_db = [], []
    so = StatsOracle(out_st.append, out_db.append)
    for ln in lines:
        so.consume(ln)
    assert any(l.split("|")[5] == "undefined" and l.split("|")[4] != "0.00" for l in js["st"])
    assert js["st"] == out_st
    assert js["db"] == out_db


def test_js_average_float_view_path_is_the_same_left_to_right_sum():
    """oracle.js_average's numpy path (histories offering float_view(), used at LAG 8640 in the
    bench-scale GPU test) performs the same sequential double additions as the Python loop."""
    import random

    import numpy as np
    from apmbackend_amd.models.oracle import js_average, js_stddev

    class View(list):
        def float_view(self):
            return np.array([np.nan if v is None else v for v in self], dtype=np.float64)

    rng = random.Random(3)
    for n in (1, 7, 360, 8640):
        vals = [rng.choice([None, float("nan")]) if rng.random() < 0.05 else rng.lognormvariate(5, 1.5)
                for _ in range(n)]
        assert js_average(View(vals)) == js_average(vals)
        assert js_stddev(View(vals)) == js_stddev(vals)
    assert js_average(View([None, float("nan")])) is None


@requires_reference
def test_config_reload_oracle_matches_reference_js():
    """The oracle's reload (thresholds, a LAG added / removed / re-added, alert gates) against the
    reference's own watcher callbacks run on the same st / fs streams: updateAllServiceSettings +
    removeStaleLagData (stream_calc_z_score.js:362-382) and the per-entry ALERTSCONFIG reads."""
    import refjs
    start = 1578391200000
    an = [Anomaly("jvm00", "getSvc0001", start + 400_000, start + 1500_000, 30.0)]
    _, bl = _synth(1, duration=1500, anomalies=an)
    C0 = default_config(replay=True)
    C0["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                          {"LAG": 30, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    C0["streamCalcZScore"]["overrides"]["services"]["S:getSvc0002"] = {"6": {"THRESHOLD": 4.0, "INFLUENCE": 0.25}}
    C0["streamProcessAlerts"].update({"rollingAlertWindowSizeInIntervals": 10,
                                      "requiredNumberBadIntervalsInAlertWindowToTrigger": 3,
                                      "perServiceAlertCooldownInMinutes": 2})
    C0["gpu"]["emulateOverrideAliasing"] = True
    C1 = copy.deepcopy(C0)
    C1["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 2.5, "INFLUENCE": 0.5},
                                          {"LAG": 12, "THRESHOLD": 2.0, "INFLUENCE": 0.2}]
    C1["streamCalcZScore"]["overrides"]["services"]["S:getSvc0002"] = {"12": {"THRESHOLD": 3.5}}
    C1["streamProcessAlerts"].update({"hardMinMsAlertThreshold": 150, "alertOnBothOnly": False,
                                      "rollingAlertWindowSizeInIntervals": 8,
                                      "requiredNumberBadIntervalsInAlertWindowToTrigger": 2,
                                      "suppressedServices": ["S:getSvc0003"]})
    C2 = copy.deepcopy(C1)
    C2["streamCalcZScore"]["defaults"].append({"LAG": 30, "THRESHOLD": 1.5, "INFLUENCE": 0.0})
    C2["streamProcessAlerts"].update({"suppressedLags": [12], "perServiceAlertCooldownInMinutes": 1,
                                      "hardMaxMsAlertThreshold": 5000, "suppressedServices": []})
    k1, k2 = len(bl) * 2 // 5, len(bl) * 7 // 10
    P = PipelineOracle(copy.deepcopy(C0), UTC)
    P.run_batches(bl[:k1])
    at_st1, at_fs1 = len(P.stats), len(P.fs)
    P.reload(copy.deepcopy(C1))
    P.run_batches(bl[k1:k2])
    at_st2, at_fs2 = len(P.stats), len(P.fs)
    P.reload(copy.deepcopy(C2))
    P.run_batches(bl[k2:])
    assert {l.split("|")[4] for l in P.fs[at_fs2:]} == {"6", "12", "30"}
    assert "30" not in {l.split("|")[4] for l in P.fs[at_fs1:at_fs2]}
    fs = refjs.zscore(json.dumps(C0), P.stats, reloads=[(at_st1, json.dumps(C1)), (at_st2, json.dumps(C2))])
    assert fs == P.fs
    al = refjs.alerts(json.dumps(C0), P.fs, "entry", reloads=[(at_fs1, json.dumps(C1)), (at_fs2, json.dumps(C2))])
    assert al == P.al and len(al) > 0
