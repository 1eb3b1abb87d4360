"""Ingest service plumbing on CPU (the oracle engine stands in for the GPU engine):
tail files -> engine -> DB insert stage / AMQP db_insert queue / e-mail notifier."""
import copy
import json
import os
import time

import pytest

from apmbackend_amd.models.oracle import PipelineOracle
from apmbackend_amd.runtime import sinks
from apmbackend_amd.runtime.amqp_broker import Broker
from apmbackend_amd.runtime.service import IngestService
from apmbackend_amd.utils.config import default_config
from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches
from apmbackend_amd.utils.timeparse import TzOffset, leading_line_ts

UTC = TzOffset("UTC")
START = 1578391200000


class ListWriter(sinks.Writer):
    def __init__(self):
        self.rows = {}

    def write(self, table, columns, rows):
        self.rows.setdefault(table, []).extend(rows)


def srv_of(p):
    return p.split("/")[-2]


def make_env(tmp_path, mode="inproc", servers=2, duration=400):
    an = [Anomaly("jvm00", "getSvc0001", START + 60_000, START + 350_000, 40.0)]
    sc = SynthConfig(servers=servers, duration_s=duration, tx_per_sec_per_server=3, seed=4, ejb_services=3,
                     provider_services=2, anomalies=an)
    lines = Generator(sc).generate()
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5}]
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 5
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 2
    C["streamProcessAlerts"]["alertCollectionIntervalInSeconds"] = 1
    C["logDir"] = str(tmp_path / "logs")
    C["apmConfigFilePath"] = None
    C["streamParseTransactions"]["tailPauseFileFullPath"] = str(tmp_path / "PAUSE")
    C["streamParseTransactions"]["tailOffsetFileFullPath"] = str(tmp_path / "offsets.json")
    C["streamInsertDb"]["bufferResumeFileFullPath"] = str(tmp_path / "ins.resume")
    C["gpu"].update({"timezone": "UTC", "outputMode": mode, "tailFromStart": True})
    # files on disk: <tmp>/logs_in/<server>/<basename>
    mapping = {}
    for fp in lines:
        server = fp.split("/")[2]
        d = tmp_path / "in" / server
        d.mkdir(parents=True, exist_ok=True)
        mapping[fp] = str(d / os.path.basename(fp))
        open(mapping[fp], "w").close()
    return C, lines, mapping, sc


def feed_in_steps(svc, lines, mapping, sc, oracle=None):
    """Append one 5 s slice of every file, then run one service step (= one tailer poll)."""
    bl = batches(lines, sc.start_ms, 5.0)
    file_order = [p for p, _ in sorted(svc.file_ids.items(), key=lambda kv: kv[1])]
    rev = {v: k for k, v in mapping.items()}
    wm = 0.0
    for chunks in bl:
        for fp, ls in chunks:
            with open(mapping[fp], "a") as f:
                f.write("\n".join(ls) + "\n")
        svc.step()
        svc._housekeeping()
        if oracle is not None:  # same batch: files in tailer order, watermark clock
            by = dict(chunks)
            oracle.parse.begin_batch(wm)
            for p in file_order:
                for ln in by.get(rev[p], []):
                    oracle.parse.read_line(p, ln)
                    v = leading_line_ts(ln, UTC)
                    if v is not None and v > wm:
                        wm = v


def test_service_inproc_matches_oracle(tmp_path):
    C, lines, mapping, sc = make_env(tmp_path)
    svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=1,
                        server_of_path=srv_of)
    w = ListWriter()
    svc.inserter.writer = w
    P = PipelineOracle(copy.deepcopy(C), UTC, server_fn=srv_of)
    feed_in_steps(svc, lines, mapping, sc, P)
    svc.shutdown()
    want = sinks.copy_encode_lines(P.tx_db + P.audit_db + P.fs + P.al)
    assert sorted(w.rows["tx"]) == sorted(want["tx"]) and len(want["tx"]) > 100
    assert w.rows["stats"] == want["fs"]
    assert w.rows.get("alerts", []) == want["al"] and len(want["al"]) > 0
    assert svc.notifier.emails >= 1 or svc.notifier.buffer
    offs = json.load(open(tmp_path / "offsets.json"))
    assert sorted(offs) == sorted(mapping.values())
    assert all(v[0] == os.path.getsize(k) for k, v in offs.items())
    logs = os.listdir(tmp_path / "logs")
    assert any(l.startswith("apm_engine.log.") for l in logs)


def test_pause_file_holds_the_tails(tmp_path):
    C, lines, mapping, sc = make_env(tmp_path, duration=60)
    svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=1,
                        server_of_path=srv_of)
    for chunks in batches(lines, sc.start_ms, 5.0):
        for fp, ls in chunks:
            with open(mapping[fp], "a") as f:
                f.write("\n".join(ls) + "\n")
    (tmp_path / "PAUSE").write_text("")
    assert svc.step() == 0
    os.remove(tmp_path / "PAUSE")
    assert svc.step() > 0
    svc.shutdown()


def test_service_sharding_by_server(tmp_path):
    C, lines, mapping, sc = make_env(tmp_path, servers=4, duration=30)
    files = sorted(mapping.values())
    per_rank = [IngestService(C, engine="cpu-oracle", files=files, rank=r, world=2, server_of_path=srv_of).files
                for r in range(2)]
    assert sorted(per_rank[0] + per_rank[1]) == files
    assert not ({srv_of(f) for f in per_rank[0]} & {srv_of(f) for f in per_rank[1]})


def test_service_amqp_mode_publishes_db_insert(tmp_path):
    b = Broker(port=0).start()
    try:
        C, lines, mapping, sc = make_env(tmp_path, mode="amqp", duration=200)
        C["amqpConnectionString"] = b.url
        C["gpu"]["bridgeQueues"] = ["transactions"]
        svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=1,
                            server_of_path=srv_of)
        feed_in_steps(svc, lines, mapping, sc)
        svc.shutdown()
        st = b.stats()
        assert st["db_insert"]["messages"] > 0 and st["transactions"]["messages"] > 0
        n_tx = st["transactions"]["messages"]
        m = svc.native.metrics()
        assert n_tx + 0 <= m["tx"]
    finally:
        b.stop()


def test_request_gc_and_reload(tmp_path):
    C, lines, mapping, sc = make_env(tmp_path, duration=30)
    svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=1,
                        server_of_path=srv_of)
    assert "garbage collection" in svc.request_gc()
    C2 = copy.deepcopy(C)
    C2["streamInsertDb"]["dbInsertBufferLimit"] = 7
    svc.reload(C2)
    assert svc.inserter.limit == 7
    svc.shutdown()


def test_fault_injection_drop_and_duplicate(tmp_path):
    C, lines, mapping, sc = make_env(tmp_path, duration=120)
    C["gpu"]["faultInjection"] = {"dropBatchEvery": 5, "duplicateBatchEvery": 7}
    svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=1,
                        server_of_path=srv_of)
    feed_in_steps(svc, lines, mapping, sc)
    n = len(batches(lines, sc.start_ms, 5.0))
    assert svc.faults == {"dropped": n // 5, "duplicated": len([i for i in range(1, n + 1) if i % 7 == 0 and i % 5])}
    assert svc.native.batches == n - n // 5 + svc.faults["duplicated"]
    svc.shutdown()


def test_fault_injection_exit(tmp_path):
    import subprocess
    import sys
    code = (
        "import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
        "from test_service import *\n"
        "import pathlib\n"
        "tmp = pathlib.Path(%r)\n"
        "C, lines, mapping, sc = make_env(tmp, duration=60)\n"
        "C['gpu']['faultInjection'] = {'exitAtBatch': 3, 'exitCode': 17}\n"
        "svc = IngestService(C, engine='cpu-oracle', files=sorted(mapping.values()), rank=0, world=1, "
        "server_of_path=srv_of)\n"
        "feed_in_steps(svc, lines, mapping, sc)\n"
    ) % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.dirname(os.path.abspath(__file__)),
         str(tmp_path))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=120)
    assert r.returncode == 17, r.stderr.decode()[-2000:]


def test_latency_percentiles_nearest_rank():
    from apmbackend_amd.runtime.service import _percentiles
    assert _percentiles([], (50, 99)) == ["-", "-"]
    xs = [float(i) for i in range(1, 101)]
    assert _percentiles(xs, (50, 90, 99)) == ["50.0", "90.0", "99.0"]
    assert _percentiles([7.0], (50, 99)) == ["7.0", "7.0"]


def test_resharded_restart_resumes_tails_from_previous_world(tmp_path):
    """Elastic degrade 2 -> 1 ranks: the surviving rank's checkpoint metadata no longer matches
    its shard, so it starts fresh but resumes every tail it now owns from the newest offset any
    old rank recorded (no data gap, no replay)."""
    from apmbackend_amd.parallel.dist import shard_servers
    from apmbackend_amd.runtime.service import write_json_atomic
    C, lines, mapping, sc = make_env(tmp_path, servers=4, duration=30)
    files = sorted(mapping.values())
    for f in files:  # some bytes to resume into
        with open(f, "w") as fh:
            fh.write("x" * 1000 + "\n")
    ck = tmp_path / "ckpt"
    ck.mkdir()
    servers = sorted({srv_of(f) for f in files})
    shards = shard_servers(servers, 2)
    now = time.time()
    for r in range(2):
        mine = [f for f in files if srv_of(f) in shards[r]]
        offs = {f: [100 + 10 * r + i, os.stat(f).st_ino] for i, f in enumerate(mine)}
        offs[files[0]] = [7, os.stat(files[0]).st_ino]  # stale duplicate entry in both tail files
        write_json_atomic(str(ck / f"tail.rank{r}.json"), offs)
        os.utime(ck / f"tail.rank{r}.json", (now - 100 + r, now - 100 + r))
        write_json_atomic(str(ck / f"meta.rank{r}.json"), {"world": 2, "rank": r, "servers": sorted(shards[r]),
                                                           "ts": now - 100})
    svc = IngestService(C, engine="cpu-oracle", files=files, rank=0, world=1, server_of_path=srv_of)
    svc.ckpt_dir = str(ck)
    assert not svc._checkpoint_is_mine()
    svc._restore_offsets_resharded()
    out = tmp_path / "resumed.json"
    svc.tailer.save_offsets(str(out))
    got = json.load(open(out))
    for r in range(2):
        for i, f in enumerate(f for f in files if srv_of(f) in shards[r]):
            if f != files[0]:
                assert got[f][0] == 100 + 10 * r + i, f
    assert got[files[0]][0] == 7  # the newest tail file's value (rank 1's, written last)
    svc.shutdown()


def test_checkpoint_ownership_rules(tmp_path):
    from apmbackend_amd.runtime.service import write_json_atomic
    C, lines, mapping, sc = make_env(tmp_path, servers=2, duration=30)
    files = sorted(mapping.values())
    ck = tmp_path / "ckpt"
    ck.mkdir()
    svc = IngestService(C, engine="cpu-oracle", files=files, rank=0, world=1, server_of_path=srv_of)
    svc.ckpt_dir = str(ck)
    assert svc._checkpoint_is_mine()  # no metadata: a checkpoint from before metadata existed
    now = time.time()
    write_json_atomic(str(ck / "meta.rank0.json"), {"world": 1, "servers": svc.my_servers, "ts": now})
    assert svc._checkpoint_is_mine()
    # same shard, but far older than another rank's checkpoint: a survivor of an older world
    write_json_atomic(str(ck / "meta.rank0.json"), {"world": 1, "servers": svc.my_servers, "ts": now - 10000})
    write_json_atomic(str(ck / "meta.rank3.json"), {"world": 4, "servers": [], "ts": now})
    assert not svc._checkpoint_is_mine()
    write_json_atomic(str(ck / "meta.rank0.json"), {"world": 2, "servers": svc.my_servers, "ts": now})
    assert not svc._checkpoint_is_mine()
    svc.shutdown()


def test_paused_lockstep_rank_still_joins_the_collective():
    """under downstream backpressure a lock-step rank holds its tails but still calls
    process_batch (with an empty batch) once per poll, so the ranks' collective sequences stay
    aligned; a rank without lock-step just skips the poll."""
    from apmbackend_amd.runtime.service import IngestService

    class Prod:
        paused = True

    class Tail:
        polled = 0

        def poll(self):
            Tail.polled += 1
            return b"x\n", [(0, 0, 2)]

    class Eng:
        calls = []

        def process_batch(self, buf, chunks, now):
            Eng.calls.append((buf, list(chunks)))

        def take_bytes(self, k):
            return b""

    for lockstep in (True, False):
        Eng.calls, Tail.polled = [], 0
        svc = IngestService.__new__(IngestService)
        svc.qm, svc.producers = object(), {"db": Prod()}
        svc.fleet = object() if lockstep else None
        svc.readahead, svc.tailer, svc.native, svc.input_mode = False, Tail(), Eng(), "logs"
        svc.polls, svc.batches, svc.fault, svc.rank, svc.outputs = 0, 0, {}, 0, []
        svc.inserter, svc.notifier = None, None
        svc.step()
        assert Tail.polled == 0
        assert Eng.calls == ([(b"", [])] if lockstep else [])


def test_sink_snapshot_pruning_follows_commits(tmp_path):
    """a sink snapshot is retired only once a LATER checkpoint committed.  Checkpoint
    #2's write fails in the writer thread (the chain manifest still names #1); starting #3 must not
    delete #1's pending file, which a crash before #3 commits would restore from."""
    class FakeEngine:
        def __init__(self):
            self.done, self.busy = 0, False

        def checkpoint_info(self):
            return {"busy": self.busy, "done": self.done}

    svc = IngestService.__new__(IngestService)
    svc.ckpt_dir, svc.rank, svc.n_checkpoints = str(tmp_path), 0, 0
    svc._sink_incarnation, svc._sink_committed, svc._ck_started = 0xabc, None, None
    svc.eng = FakeEngine()

    def start(ok):  # what checkpoint() does around one native async checkpoint
        svc._note_checkpoint_outcome()
        done_before = svc.eng.done
        name = svc._sink_snapshot_name()
        open(os.path.join(svc.ckpt_dir, name), "wb").close()
        svc._ck_started = (name, done_before)
        svc.eng.busy = True
        svc._prune_sink_snapshots(name)
        svc.n_checkpoints += 1
        svc.eng.done += 1 if ok else 0  # the writer thread finishes (or fails) it
        svc.eng.busy = False
        return name

    n1 = start(True)
    n2 = start(False)   # #2's write fails: manifest still names #1
    assert set(os.listdir(tmp_path)) == {n1, n2}
    n3 = start(True)    # starting #3: #1 is still the committed restore point
    assert n1 in os.listdir(tmp_path) and n3 in os.listdir(tmp_path)
    assert n2 not in os.listdir(tmp_path)  # never named by a committed checkpoint
    n4 = start(True)    # #3 committed: #1 may go now
    assert set(os.listdir(tmp_path)) == {n3, n4}
    assert svc._sink_committed == n3


def _fake_ckpt(path, batch):
    """A checkpoint file reduced to what checkpoint_batches reads: the binio header and SEC_CLOCK
    (watermark, batch_no) -- binio.h / checkpoint.cpp."""
    import struct
    ver = 9  # binio.h kCkptVersion
    with open(path, "wb") as f:
        f.write(b"APMCKPT\0" + struct.pack("<I", ver))
        f.write(struct.pack("<IQ", 4, 16) + struct.pack("<dQ", 1.0e12, batch))
        f.write(struct.pack("<I", 0xE0F))


def _manifest(path, names):
    with open(path, "w") as f:
        f.write("APMCHAIN 1\n" + "".join(n + "\n" for n in names))


def test_node_restore_batch_is_common_to_every_rank_and_survives_a_lost_base(tmp_path):
    """rank 1 died while the node wrote the aligned base at batch 130.  Rank 0 then
    holds only the new base in its current chain -- its old chain (100, 110, 120) is kept as the
    previous chain -- and rank 1 still has 100, 110, 120.  Every rank resumes (and a re-shard merges)
    at 120, the newest batch both hold, each from the chain that has it."""
    C, lines, mapping, sc = make_env(tmp_path, servers=2, duration=30)
    ck = tmp_path / "ckpt"
    ck.mkdir()
    for r in (0, 1):
        for b in (100, 110, 120):
            _fake_ckpt(ck / f"engine.rank{r}.{'b' if b == 100 else 'i'}{b}.ckpt", b)
    _fake_ckpt(ck / "engine.rank0.b130.ckpt", 130)
    old = ["engine.rank0.b100.ckpt", "engine.rank0.i110.ckpt", "engine.rank0.i120.ckpt"]
    _manifest(ck / "engine.rank0.ckpt", ["engine.rank0.b130.ckpt"])
    _manifest(ck / "engine.rank0.prev.ckpt", old)
    _manifest(ck / "engine.rank1.ckpt", [n.replace("rank0", "rank1") for n in old])
    svc = IngestService(C, engine="cpu-oracle", files=sorted(mapping.values()), rank=0, world=2,
                        server_of_path=srv_of)
    svc.ckpt_dir = str(ck)
    try:
        assert sorted(svc._chain_batches(0)) == [100, 110, 120, 130]
        at, where = svc._node_common_batch([0, 1])
        assert at == 120
        assert where == {0: str(ck / "engine.rank0.prev.ckpt"), 1: str(ck / "engine.rank1.ckpt")}
        # rank 1 never got past 110: 110 is the node's batch
        _manifest(ck / "engine.rank1.ckpt", [n.replace("rank0", "rank1") for n in old[:2]])
        assert svc._node_common_batch([0, 1])[0] == 110
        os.remove(ck / "engine.rank1.ckpt")
        assert svc._node_common_batch([0, 1]) == (0, {})
    finally:
        svc.shutdown()
