"""Multi-rank native engines on ONE GPU: the node's collectives (lock-step clocks, fleet moments,
node-wide alert candidates) run over an in-process group (``LocalCollGroup``) instead of RCCL,
so a 2- or 4-rank node is checked against the single-process reference without 2-4 GPUs.

Each rank owns a shard of the JVM hosts (parallel.dist.shard_servers) and runs its own engine
on its own host thread, exactly as the per-GPU processes of a node do.  The union of the ranks'
st / fs streams must equal the single-stream oracle per series, and the al stream must equal the
oracle's with the DEFAULT 15-minute per-service cooldown -- two JVMs on different ranks degrade
on the same service, and only the first candidate in the reference's emission order may alert.
"""
import collections
import copy
import threading

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU containers
    pytest.skip("no GPU", allow_module_level=True)

from apmbackend_amd import _native  # noqa: E402
from apmbackend_amd.models.oracle import PipelineOracle  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.parallel.dist import shard_servers  # noqa: E402
from apmbackend_amd.parallel.fleet import FleetBaseline  # noqa: E402
from apmbackend_amd.utils.config import default_config  # noqa: E402
from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks  # noqa: E402
from apmbackend_amd.utils.timeparse import TzOffset  # noqa: E402

UTC = TzOffset("UTC")
START = 1578391200000


def node_cfg():
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                         {"LAG": 30, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 5
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 2
    # perServiceAlertCooldownInMinutes: the default (15)
    C["gpu"].update({"zscoreMeanMode": "exact", "timezone": "UTC", "maxSeries": 4096, "batchBytes": 4 << 20,
                     "maxLinesPerBatch": 1 << 16, "bucketCellCapacity": 8, "bucketOverflowCapacity": 1 << 16})
    return C


def corpus():
    an = [Anomaly("jvm01", "getSvc0001", START + 100_000, START + 900_000, 30.0),
          Anomaly("jvm02", "getSvc0001", START + 100_000, START + 900_000, 30.0),
          Anomaly("jvm03", "getSvc0002", START + 150_000, START + 900_000, 30.0),
          Anomaly("jvm04", "getSvc0002", START + 200_000, START + 900_000, 30.0),
          Anomaly("jvm02", "getSvc0003", START + 600_000, START + 900_000, 40.0)]
    sc = SynthConfig(servers=4, duration_s=1000, tx_per_sec_per_server=3, seed=21, ejb_services=3,
                     provider_services=2, anomalies=an)
    lines = Generator(sc).generate()
    return lines, with_watermarks(batches(lines, sc.start_ms, 5.0), UTC)


def server_of(fp):
    return fp.split("/")[2]


def per_series(stream):
    d = collections.defaultdict(list)
    for l in stream:
        f = l.split("|")
        d[(f[2], f[3])].append(l)
    return d


def run_node(world, bl, servers):
    """`world` engines, one host thread each, joined by an in-process collective group."""
    group = _native.load().LocalCollGroup(world, 120000.0)
    shards = shard_servers(servers, world)
    engs, outs, errs = [], [], []
    for r in range(world):
        eng = APMEngine(copy.deepcopy(node_cfg()), keep_text=True)
        # register this rank's files up front, in the global layout order
        for _now, chunks in bl:
            for fp, _ls in chunks:
                if server_of(fp) in shards[r]:
                    eng.add_file(fp)
        engs.append(eng)
        outs.append(collections.defaultdict(list))
    fleets = [None] * world

    def rank_main(r):
        try:
            fleets[r] = FleetBaseline(engs[r], world, r, max_services=64, local_group=group, servers=servers)
            for now, chunks in bl:
                engs[r].process_lines([(fp, ls) for fp, ls in chunks if server_of(fp) in shards[r]], now)
                for k in ("st", "fs", "al", "fb"):
                    outs[r][k] += engs[r].take(k)
            fleets[r].drain_alerts()
            for k in ("st", "fs", "al", "fb"):
                outs[r][k] += engs[r].take(k)
        except Exception as e:  # pragma: no cover - reported below
            errs.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not errs, errs
    assert all(not t.is_alive() for t in th)
    return engs, outs


@pytest.mark.parametrize("world", [1, 2, 4])
def test_local_group_node_matches_single_process(world):
    lines, bl = corpus()
    servers = sorted({server_of(fp) for fp in lines})
    P = PipelineOracle(copy.deepcopy(node_cfg()), UTC)
    P.run_batches(bl)
    engs, outs = run_node(world, bl, servers)
    for name, want in (("st", P.stats), ("fs", P.fs)):
        got = collections.defaultdict(list)
        for o in outs:
            for k, v in per_series(o[name]).items():
                got[k] += v
        assert got == per_series(want), name
    al = sorted(l for o in outs for l in o["al"])
    assert al == sorted(P.al)
    svcs = collections.Counter(l.split("|")[4] for l in P.al)
    assert {"S:getSvc0001", "S:getSvc0002"} <= set(svcs)
    ms = [e.metrics() for e in engs]
    assert sum(m["alerts"] for m in ms) == len(P.al)
    if world > 1:
        # candidates were raised on more ranks than alerted: the cooldown was decided node-wide
        assert sum(m["alert_candidates"] for m in ms) > len(P.al)
    # node-wide counters (all-reduce SUM at each interval edge): same vector on every rank,
    # field 0 counts the ranks, the line count is the node's as of the last edge
    nms = [e.eng.node_metrics() for e in engs]
    assert nms[0] and all(nm == nms[0] for nm in nms)
    nm = nms[0]
    assert nm[0] == world
    assert 0 < nm[2] <= sum(m["lines"] for m in ms)
    assert nm[1] >= world  # every rank counted its batches


def _fleet_by_name(eng):
    import numpy as np
    names = eng.eng.fleet_slot_names()
    m = np.frombuffer(eng.eng.fleet_merged(), dtype=np.float64).reshape(64, 2, 3, 3)
    return {n: m[i] for i, n in enumerate(names)}, m[len(names):]


@pytest.mark.parametrize("world", [2, 4])
def test_fleet_registry_merges_services_node_wide(world):
    """Ranks intern services in different orders; the moments matrix is indexed by node-wide
    slots (hash + name all-gathered in the lock-step round, assigned in rank order), so the
    merged per-service baselines of a 2/4-rank node equal the 1-rank ones service by service,
    every rank holds the same table, and the ranks emit the interval's fb rows in disjoint slices."""
    import numpy as np
    lines, bl = corpus()
    servers = sorted({server_of(fp) for fp in lines})
    e1, o1 = run_node(1, bl, servers)
    ref, _ = _fleet_by_name(e1[0])
    engs, outs = run_node(world, bl, servers)
    tables = [_fleet_by_name(e) for e in engs]
    names0 = engs[0].eng.fleet_slot_names()
    for e, (t, rest) in zip(engs, tables):
        assert e.eng.fleet_slot_names() == names0  # same registry on every rank
        assert not rest.any()  # nothing outside the registered slots
    got = tables[0][0]
    assert set(got) == set(ref) and len(ref) >= 5
    for name in ref:
        np.testing.assert_allclose(got[name], ref[name], rtol=1e-12, atol=1e-9)
    # fb rows: every rank formats and emits its own slice of the node-wide slots (the merged
    # moments are on every rank), one row per (service, LAG) with a baseline, every interval
    # after warm-up; the slices are disjoint and together are the 1-rank stream, row for row
    fb = [l for o in outs for l in o["fb"]]
    assert fb and all(l.startswith("fb|") for l in fb)
    assert sum(1 for o in outs if o["fb"]) == world  # the formatting is split, not rank 0's alone
    key = lambda l: (l.split("|")[1], l.split("|")[2], l.split("|")[3])
    for o in outs:
        assert len(set(map(key, o["fb"]))) == len(o["fb"])
    ref_fb = o1[0]["fb"]
    assert sorted(map(key, fb)) == sorted(map(key, ref_fb))
    # values: fp64 sums in another order, printed to 1 dp.  The std is sqrt(E[x^2] - mean^2): a
    # std on a .x5 tie (two series 0.1 apart: common with 1-dp means) prints either way, so rows
    # agree field by field to one printed digit
    def vals(l):
        f = l.split("|")
        return [float(f[4])] + [float(v) for part in f[5:8] for v in part.split(":")]
    ref_by_key = {key(l): vals(l) for l in ref_fb}
    for l in fb:
        np.testing.assert_allclose(vals(l), ref_by_key[key(l)], rtol=0, atol=0.1001, err_msg=l)
    same = len(set(fb) & set(ref_fb))
    assert same >= len(ref_fb) * 9 // 10, (same, len(ref_fb))
    assert sum(e.eng.fleet_info()["fb_rows"] for e in engs) == len(fb)


# ---------------------------------------------------------------- multi-PROCESS node (TCP transport)
import json  # noqa: E402
import os  # noqa: E402
import socket  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")
sys.path.insert(0, FIX)
import node_rank  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_env(rank, world, port):
    env = dict(os.environ)
    env.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               PYTHONUNBUFFERED="1")
    return env


def _process_outputs(out, world):
    outs = []
    for r in range(world):
        d = {}
        for k in node_rank.KINDS:
            with open(os.path.join(out, f"rank{r}.{k}")) as f:
                d[k] = [l for l in f.read().split("\n") if l]
        outs.append(d)
    return outs


def _assert_node_equals_oracle(outs, P):
    for name, want in (("st", P.stats), ("fs", P.fs)):
        got = collections.defaultdict(list)
        for o in outs:
            for k, v in per_series(o[name]).items():
                got[k] += v
        assert got == per_series(want), name
    assert sorted(l for o in outs for l in o["al"]) == sorted(P.al)


def _oracle():
    lines, bl = node_rank.corpus()
    P = PipelineOracle(copy.deepcopy(node_rank.node_cfg()), UTC)
    P.run_batches(bl)
    assert {"S:getSvc0001", "S:getSvc0002"} <= {l.split("|")[4] for l in P.al}
    return P


@pytest.mark.parametrize("world", [2, 4])
def test_process_node_over_host_transport_matches_single_process(tmp_path, world):
    """`world` OS processes, one native engine each on the shared GPU, node-wide exchanges over the
    TCP host transport (HostCollective): the per-series st / fs streams and the alerts (default
    15-minute node-wide cooldown) equal the single-stream oracle -- the multi-process node of
    BASELINE config 3, executed instead of simulated by threads."""
    P = _oracle()
    out = str(tmp_path / "node")
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.join(FIX, "node_rank.py"), out, "--ckpt-every", "0",
                               "--idle", "0"], env=_rank_env(r, world, port), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT) for r in range(world)]
    try:
        logs = [p.communicate(timeout=400)[0].decode() for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), logs
    _assert_node_equals_oracle(_process_outputs(out, world), P)
    done = [json.load(open(os.path.join(out, f"done.rank{r}"))) for r in range(world)]
    assert sum(d["alerts"] for d in done) == len(P.al)
    assert sum(d["alert_candidates"] for d in done) > len(P.al)  # the cooldown was decided node-wide
    nm = done[0]["node_metrics"]
    assert nm[0] == world and all(d["node_metrics"][0] == world for d in done)


def test_peer_process_death_aborts_the_group_and_supervisor_resumes_from_checkpoints(tmp_path):
    """A rank process dies mid-run (fault injection: os._exit after batch 110).  The survivor's
    next collective fails at once (peer gone), it aborts and exits non-zero; the supervisor
    (apm_manager.js:303-356 semantics, rank group restarted as a whole) restarts the group, every
    rank resumes from the newest checkpoint the whole group has (batch 80), and the node's output
    is exactly the uninterrupted one."""
    from apmbackend_amd.runtime import supervisor as sup
    from apmbackend_amd.runtime.notifier import Mailer
    from apmbackend_amd.utils.config import default_config
    P = _oracle()
    out = str(tmp_path / "node")
    C = default_config(replay=True)
    C["logDir"] = str(tmp_path / "logs")
    C["appDirectory"] = FIX
    C["apmConfigFilePath"] = None
    C["applicationManager"].update({
        "moduleSettings": [{"name": "node", "relativePath": "node_rank.py", "ranks": 2, "passConfig": False,
                            "args": [out, "--ckpt-every", "40", "--kill", "1:110"], "masterPort": _free_port(),
                            "elasticDegrade": False}],
        "stateDir": str(tmp_path / "state"), "restartDelaySeconds": 0.5, "crashLoopWindowSeconds": 0.0,
        "inspectionFrequencySeconds": 3600, "alertCollectionIntervalInSeconds": 3600,
        "diskSpaceGBAvailableThreshold": 0, "diskSpacePercentageUsedThreshold": 101})
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda *a: None)
    s.start_all()
    mod = s.modules[0]
    try:
        t_end = time.time() + 600
        log0 = ""
        log_path = os.path.join(C["logDir"], "node.rank0.start.log")
        t_print = time.time()
        while time.time() < t_end and not all(os.path.exists(os.path.join(out, f"done.rank{r}")) for r in range(2)):
            time.sleep(1.0)  # slow polling: the survivor notices the dead peer on its own first
            if time.time() - t_print > 15:
                t_print = time.time()
                print(f"[peer-death test] restarts {[p.restarts for p in mod.procs]} "
                      f"alerts {len(s.alert_buffer)}", flush=True)
            # (a restart truncates the start log, as the reference's openSync(.., 'w') does: keep
            # the first generation's before the supervisor restarts it)
            if not log0 and os.path.exists(log_path):
                txt = open(log_path).read()
                if "host collective" in txt:
                    log0 = txt
            s.check_children()
        assert all(os.path.exists(os.path.join(out, f"done.rank{r}")) for r in range(2)), "group did not finish"
        assert os.path.exists(os.path.join(out, "killed"))
        assert all(p.restarts >= 1 for p in mod.procs)  # the group restarted as a whole
        assert "peer process gone" in log0, log0[-2000:]
        assert any("exited: code:17" in a for a in s.alert_buffer), s.alert_buffer
        # the survivor aborted its collectives and exited PEER_FAILURE_EXIT (not blamed)
        assert any("node.rank0" in a and "code:75" in a for a in s.alert_buffer), s.alert_buffer
        done = [json.load(open(os.path.join(out, f"done.rank{r}"))) for r in range(2)]
        assert [d["start"] for d in done] == [80, 80]
    finally:
        open(os.path.join(out, "stop"), "w").close()
        s.stop_all()
    _assert_node_equals_oracle(_process_outputs(out, 2), P)


def _dump_logs(log_dir, tail=4000):
    """The rank processes' logs (the supervisor's per-module files), printed on a failure."""
    import glob as _glob
    for p in sorted(_glob.glob(os.path.join(log_dir, "*"))):
        try:
            with open(p, errors="replace") as f:
                text = f.read()
        except OSError:
            continue
        print(f"===== {p} ({len(text)} bytes)\n{text[-tail:]}", flush=True)


def _all_outputs(out):
    """Every output file of every world (w<world>.rank<r>.* after a re-shard) as one node."""
    import glob as _glob
    outs = []
    for p in sorted(_glob.glob(os.path.join(out, "*rank*.st"))):
        base = p[:-3]
        d = {}
        for k in node_rank.KINDS:
            with open(f"{base}.{k}") as f:
                d[k] = [l for l in f.read().split("\n") if l]
        outs.append(d)
    return outs


@pytest.mark.timeout(600)
def test_elastic_degrade_keeps_state_across_the_world_change(tmp_path):
    """4 rank processes (host transport, one GPU); the rank on GPU 1 keeps dying
    after batch 110, so the supervisor retires GPU 1 and restarts the group with 2 ranks.  Each new
    rank merges the 4-rank checkpoints of batch 100 for the servers it now owns -- series windows,
    z-score rings, alert counters, join caches, parked records, pending lines (merge.cpp) -- and
    continues.  The node's st / fs / al over every file equal the uninterrupted single-stream
    oracle (no series restarts its history, no transaction in flight is lost)."""
    from apmbackend_amd.runtime import supervisor as sup
    from apmbackend_amd.runtime.notifier import Mailer
    from apmbackend_amd.utils.config import default_config
    P = _oracle()
    out = str(tmp_path / "node")
    C = default_config(replay=True)
    C["logDir"] = str(tmp_path / "logs")
    C["appDirectory"] = FIX
    C["apmConfigFilePath"] = None
    C["applicationManager"].update({
        "moduleSettings": [{"name": "node", "relativePath": "node_rank.py", "ranks": 4, "passConfig": False,
                            "args": [out, "--ckpt-every", "20", "--kill-world", "4:1:110", "--first-world", "4"],
                            "masterPort": _free_port(), "elasticDegrade": True, "elasticMaxFailures": 2,
                            "elasticWindowSeconds": 3600}],
        "stateDir": str(tmp_path / "state"), "restartDelaySeconds": 0.5, "crashLoopWindowSeconds": 0.0,
        "groupAbortGraceSeconds": 20, "inspectionFrequencySeconds": 3600, "alertCollectionIntervalInSeconds": 3600,
        "diskSpaceGBAvailableThreshold": 0, "diskSpacePercentageUsedThreshold": 101})
    notes = []
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda g, text, tags: notes.append(text))
    s.start_all()
    mod = s.modules[0]
    try:
        t_end = time.time() + 420
        t_print = time.time()
        while time.time() < t_end and not (mod.ranks == 2 and all(
                os.path.exists(os.path.join(out, f"done.rank{r}")) for r in range(2))):
            time.sleep(0.5)
            if time.time() - t_print > 15:
                t_print = time.time()
                print(f"[degrade test] world {mod.ranks} generation {mod.generation} restarts "
                      f"{[p.restarts for p in mod.procs]}", flush=True)
            s.check_children()
            if mod.ranks < 2:  # degraded past the expected world: the new ranks kept failing
                break
        if not (mod.ranks == 2 and mod.bad_devices == {1}):
            _dump_logs(C["logDir"])
        assert mod.ranks == 2 and mod.bad_devices == {1}, (mod.ranks, mod.bad_devices, s.alert_buffer)
        assert any("degraded from 4 to 2 GPUs" in n for n in notes), notes
        done = [json.load(open(os.path.join(out, f"done.rank{r}"))) for r in range(2)]
        assert [d["start"] for d in done] == [100, 100]
        logs = [open(os.path.join(C["logDir"], f"node.rank{r}.start.log")).read() for r in range(2)]
        assert all("world 4 -> 2: merged the first world's batch-100 checkpoints" in l for l in logs), logs
    finally:
        open(os.path.join(out, "stop"), "w").close()
        s.stop_all()
    _assert_node_equals_oracle(_all_outputs(out), P)
