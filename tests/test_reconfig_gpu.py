"""Live reconfiguration: a config reload mid-stream changes z-score thresholds, alert gates and
the LAG set, and the engine's st / fs / al streams stay equal to the oracle that applies the same
reload between the same two batches (stream_calc_z_score.js:152-193,362-382 updateAllServiceSettings
+ removeStaleLagData; stream_process_alerts.js:335-471 gates read per fs entry)."""
import collections
import copy
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_engine_gpu import UTC, small_cfg, synth_batches  # noqa: E402

from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402

pytestmark = pytest.mark.gpu


def _reloads():
    C0 = small_cfg("exact")
    C1 = copy.deepcopy(C0)
    zc, ac = C1["streamCalcZScore"], C1["streamProcessAlerts"]
    # thresholds, a new LAG (12: empty history) and a removed one (30: history dropped)
    zc["defaults"] = [{"LAG": 6, "THRESHOLD": 2.5, "INFLUENCE": 0.5}, {"LAG": 12, "THRESHOLD": 2.0, "INFLUENCE": 0.2}]
    zc["overrides"]["services"]["S:getSvc0002"] = {"12": {"THRESHOLD": 3.5}}
    # alert gates
    ac.update({"hardMinMsAlertThreshold": 150, "alertOnBothOnly": False, "rollingAlertWindowSizeInIntervals": 8,
               "requiredNumberBadIntervalsInAlertWindowToTrigger": 2, "suppressedServices": ["S:getSvc0003"]})
    C2 = copy.deepcopy(C1)
    zc, ac = C2["streamCalcZScore"], C2["streamProcessAlerts"]
    # LAG 30 comes back (empty history, its alert counters resume), LAG 12 suppressed, cooldown 1 min
    zc["defaults"].append({"LAG": 30, "THRESHOLD": 1.5, "INFLUENCE": 0.0})
    ac.update({"suppressedLags": [12], "perServiceAlertCooldownInMinutes": 1, "hardMaxMsAlertThreshold": 5000,
               "suppressedServices": []})
    return C0, C1, C2


def test_reload_thresholds_gates_and_lag_set_mid_stream():
    _lines, bl = synth_batches(1)
    C0, C1, C2 = _reloads()
    k1, k2 = 100, 170
    P = PipelineOracle(copy.deepcopy(C0), UTC)
    P.run_batches(bl[:k1])
    P.reload(copy.deepcopy(C1))
    P.run_batches(bl[k1:k2])
    P.reload(copy.deepcopy(C2))
    P.run_batches(bl[k2:])
    assert len(P.al) > 0

    eng = APMEngine(copy.deepcopy(C0), keep_text=True)
    out = collections.defaultdict(list)
    for i, (now, chunks) in enumerate(bl):
        if i == k1:
            assert eng.reload(copy.deepcopy(C1), gen=1) == []  # nothing here needs a restart
        if i == k2:
            eng.reload(copy.deepcopy(C2), gen=2)
        eng.process_lines(chunks, now)
        for k in ("st", "fs", "al"):
            out[k] += eng.take(k)
    info = eng.eng.reconfig_info()
    assert info["applied"] == 2 and info["applied_gen"] == 2 and info["lag_set_changes"] == 2
    assert eng.eng.lag_values() == [6, 12, 30]
    assert out["st"] == P.stats
    lags = lambda fs: collections.Counter(l.split("|")[4] for l in fs)
    assert lags(out["fs"]) == lags(P.fs) and set(lags(P.fs)) == {"6", "12", "30"}
    assert out["fs"] == P.fs
    assert out["al"] == P.al


def test_reload_stats_window_interval_and_many_lags():
    """The stats settings apply live too (stream_calc_stats.js:228-261 getParseSettings re-read on
    every change, used at the next rollover): the window shrinks 30 -> 20 with a 4-interval buffer
    and a 15 s intervalLengthInSeconds (TPM divisor :186), then grows to 31 (it fills in from the
    buckets removeOldBuckets kept), with 5 and then 6 LAGs (more than the old 4-LAG cap;
    stream_calc_z_score.js:216 iterates any number).  st / fs / al equal the oracle applying the
    same reloads between the same batches."""
    _lines, bl = synth_batches(2)
    C0 = small_cfg("exact")
    C0["streamCalcZScore"]["defaults"] = [{"LAG": l, "THRESHOLD": t, "INFLUENCE": i} for l, t, i in
                                          ((3, 3.0, 0.5), (6, 3.0, 0.5), (12, 2.5, 0.2), (20, 2.0, 0.0),
                                           (30, 2.0, 0.0))]
    C1 = copy.deepcopy(C0)
    C1["streamCalcStats"].update({"windowSizeInIntervals": 20, "bufferSizeInIntervals": 4,
                                  "intervalLengthInSeconds": 15})
    C2 = copy.deepcopy(C1)
    C2["streamCalcStats"].update({"windowSizeInIntervals": 31, "bufferSizeInIntervals": 6,
                                  "intervalLengthInSeconds": 10})
    C2["streamCalcZScore"]["defaults"].append({"LAG": 45, "THRESHOLD": 1.5, "INFLUENCE": 0.1})
    k1, k2 = 90, 160
    P = PipelineOracle(copy.deepcopy(C0), UTC)
    P.run_batches(bl[:k1])
    P.reload(copy.deepcopy(C1))
    P.run_batches(bl[k1:k2])
    P.reload(copy.deepcopy(C2))
    P.run_batches(bl[k2:])
    eng = APMEngine(copy.deepcopy(C0), keep_text=True)
    out = collections.defaultdict(list)
    for i, (now, chunks) in enumerate(bl):
        if i == k1:
            assert eng.reload(copy.deepcopy(C1), gen=1) == []
        if i == k2:
            assert eng.reload(copy.deepcopy(C2), gen=2) == []
        eng.process_lines(chunks, now)
        for k in ("st", "fs", "al"):
            out[k] += eng.take(k)
    info = eng.eng.reconfig_info()
    assert info["applied"] == 2 and info["window_changes"] == 2 and info["lag_set_changes"] == 1
    assert eng.eng.lag_values() == [3, 6, 12, 20, 30, 45]
    assert out["st"] == P.stats and len(P.stats) > 1000
    assert out["fs"] == P.fs
    assert {l.split("|")[4] for l in P.fs} == {"3", "6", "12", "20", "30", "45"}
    assert out["al"] == P.al


def test_reload_warns_about_restart_keys():
    C0 = small_cfg("exact")
    eng = APMEngine(copy.deepcopy(C0), keep_text=True)
    C1 = copy.deepcopy(C0)
    C1["gpu"]["maxSeries"] = 8192
    C1["streamCalcStats"]["windowSizeInIntervals"] = 20  # (live since round 5)
    restart = eng.reload(C1, gen=1)
    assert "max_series" in restart and "window" not in restart


def _stream(eng, bl, reloads=None, start=0, stop=None):
    out = collections.defaultdict(list)
    for i, (now, chunks) in enumerate(bl[start:stop], start):
        if reloads and i in reloads:
            assert eng.reload(copy.deepcopy(reloads[i][0]), gen=reloads[i][1]) == []
        eng.process_lines(chunks, now)
        for k in ("st", "fs", "al"):
            out[k] += eng.take(k)
    return out


def test_reload_to_long_windows_and_ten_lags():
    """Any windowSizeInIntervals / bufferSizeInIntervals and any number of LAG defaults
    (stream_calc_stats.js:172,186,228-261; stream_calc_z_score.js:216): a reload to a 60-interval
    window grows the bucket ring (40 -> 67 slots, live buckets keep their samples), a second one
    to a 90-interval window puts every series' K8 on the block pass (more window buckets than a
    wave has lanes) and brings the LAG set to 10.  st / fs / al equal the oracle applying the same
    reloads between the same batches."""
    _lines, bl = synth_batches(4, duration=2400)
    C0 = small_cfg("exact")
    C1 = copy.deepcopy(C0)
    C1["streamCalcStats"].update({"windowSizeInIntervals": 60, "bufferSizeInIntervals": 6})
    C2 = copy.deepcopy(C1)
    C2["streamCalcStats"].update({"windowSizeInIntervals": 90, "bufferSizeInIntervals": 8})
    C2["streamCalcZScore"]["defaults"] = [{"LAG": l, "THRESHOLD": 2.0 + 0.1 * i, "INFLUENCE": 0.1 * (i % 3)}
                                          for i, l in enumerate((3, 6, 9, 12, 18, 24, 30, 36, 48, 60))]
    k1, k2 = 150, 300
    P = PipelineOracle(copy.deepcopy(C0), UTC)
    P.run_batches(bl[:k1])
    P.reload(copy.deepcopy(C1))
    P.run_batches(bl[k1:k2])
    P.reload(copy.deepcopy(C2))
    P.run_batches(bl[k2:])
    eng = APMEngine(copy.deepcopy(C0), keep_text=True)
    assert eng.eng.reconfig_info()["ring_slots"] == 40
    out = _stream(eng, bl, {k1: (C1, 1), k2: (C2, 2)})
    info = eng.eng.reconfig_info()
    assert info["applied"] == 2 and info["window_changes"] == 2 and info["lag_set_changes"] == 1
    assert info["ring_slots"] == 99 and info["ring_grows"] == 2
    assert len(eng.eng.lag_values()) == 10
    assert out["st"] == P.stats and len(P.stats) > 1000
    assert out["fs"] == P.fs
    assert len({l.split("|")[4] for l in P.fs}) == 10
    assert out["al"] == P.al


def test_long_window_checkpoint_restores_into_another_ring_size(tmp_path):
    """A 70-interval window engine whose ring was configured at 128 slots (gpu.bucketRingSlots)
    saves a checkpoint; a fresh engine with the automatic ring (window + buffer + 1 = 77 slots)
    restores it -- every saved bucket lands in slot b % 77 -- and continues: st / fs / al equal an
    uninterrupted oracle run."""
    _lines, bl = synth_batches(5, duration=1800)
    C = small_cfg("exact")
    C["streamCalcStats"].update({"windowSizeInIntervals": 70, "bufferSizeInIntervals": 6})
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    cut = 200
    Cbig = copy.deepcopy(C)
    Cbig["gpu"]["bucketRingSlots"] = 128
    eng = APMEngine(copy.deepcopy(Cbig), keep_text=True)
    assert eng.eng.reconfig_info()["ring_slots"] == 128
    out = _stream(eng, bl, stop=cut)
    ck = str(tmp_path / "long.ckpt")
    assert eng.save_state(ck) > 0
    del eng
    eng2 = APMEngine(copy.deepcopy(C), keep_text=True)
    assert eng2.eng.reconfig_info()["ring_slots"] == 77
    eng2.load_state(ck)
    more = _stream(eng2, bl, start=cut)
    for k in ("st", "fs", "al"):
        out[k] += more[k]
    assert out["st"] == P.stats and len(P.stats) > 500
    assert out["fs"] == P.fs
    assert out["al"] == P.al
