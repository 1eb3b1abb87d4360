"""Ingest service with the native GPU engine: equals the CPU oracle service, and a
checkpoint / restart in the middle of the stream changes nothing."""
import copy
import os

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

from apmbackend_amd.runtime.service import IngestService  # noqa: E402
from apmbackend_amd.utils.synth import batches  # noqa: E402
from test_service import ListWriter, feed_in_steps, make_env, srv_of  # noqa: E402


def gpu_cfg(C):
    C["gpu"].update({"zscoreMeanMode": "exact", "maxSeries": 4096, "batchBytes": 4 << 20,
                     "maxLinesPerBatch": 1 << 16, "bucketCellCapacity": 8, "bucketOverflowCapacity": 1 << 16,
                     "emulateOverrideAliasing": True, "tailReadAhead": False})
    return C


def run(svc, lines, mapping, sc, lo=0, hi=None):
    bl = batches(lines, sc.start_ms, 5.0)[lo:hi]
    for chunks in bl:
        for fp, ls in chunks:
            with open(mapping[fp], "a") as f:
                f.write("\n".join(ls) + "\n")
        svc.step()
        svc._housekeeping()


def test_native_service_matches_cpu_oracle_service(tmp_path):
    outs = []
    for engine in ("native", "cpu-oracle"):
        d = tmp_path / engine
        d.mkdir()
        C, lines, mapping, sc = make_env(d)
        gpu_cfg(C)
        svc = IngestService(C, engine=engine, files=sorted(mapping.values()), rank=0, world=1, server_of_path=srv_of)
        w = ListWriter()
        svc.inserter.writer = w
        run(svc, lines, mapping, sc)
        svc.shutdown()
        outs.append(w.rows)
    nat, cpu = outs
    assert nat["stats"] == cpu["stats"] and len(nat["stats"]) > 0
    assert nat.get("alerts") == cpu.get("alerts")
    assert sorted(nat["tx"]) == sorted(cpu["tx"])


def test_service_checkpoint_restart_is_seamless(tmp_path):
    res = []
    for restart in (False, True):
        d = tmp_path / ("restart" if restart else "straight")
        d.mkdir()
        C, lines, mapping, sc = make_env(d)
        gpu_cfg(C)
        C["gpu"]["checkpointDir"] = str(d / "ckpt")
        C["gpu"]["checkpointEverySeconds"] = 1e9
        nb = len(batches(lines, sc.start_ms, 5.0))
        files = sorted(mapping.values())
        w = ListWriter()
        svc = IngestService(C, engine="native", files=files, rank=0, world=1, server_of_path=srv_of)
        svc.inserter.writer = w
        if restart:
            run(svc, lines, mapping, sc, 0, nb // 2)
            svc.shutdown()  # flush + checkpoint + offsets
            del svc
            svc = IngestService(C, engine="native", files=files, rank=0, world=1, server_of_path=srv_of)
            svc.inserter.writer = w
            run(svc, lines, mapping, sc, nb // 2, None)
        else:
            run(svc, lines, mapping, sc)
        svc.shutdown()
        assert os.path.exists(d / "ckpt" / "engine.rank0.ckpt")
        res.append(w.rows)
    a, b = res
    assert a["stats"] == b["stats"] and len(a["stats"]) > 0
    assert sorted(a["tx"]) == sorted(b["tx"])
    assert a.get("alerts") == b.get("alerts")


def test_readahead_service_processes_every_line(tmp_path):
    """Production path: tailer read-ahead into pinned slots + engine prefetch of the next batch,
    with the files appended while the read-ahead thread runs.  Every byte is consumed and
    committed, and the outputs equal the CPU oracle fed the very batches the tailer formed (the
    reference's cross-file join depends on how the files interleave, so batches are replayed
    rather than assumed: tests/test_tailer.py covers the batching itself)."""
    import time as _time
    from apmbackend_amd.models.oracle import PipelineOracle
    from apmbackend_amd.runtime import sinks
    from apmbackend_amd.utils.synth import with_watermarks
    from apmbackend_amd.utils.timeparse import TzOffset
    C, lines, mapping, sc = make_env(tmp_path)
    gpu_cfg(C)
    C["gpu"]["tailReadAhead"] = True
    C["gpu"]["tailIdleMs"] = 5.0
    svc = IngestService(copy.deepcopy(C), engine="native", files=sorted(mapping.values()), rank=0, world=1,
                        server_of_path=srv_of)
    svc.batch_log = []
    w = ListWriter()
    svc.inserter.writer = w
    for chunks in batches(lines, sc.start_ms, 5.0):
        for fp, ls in chunks:
            with open(mapping[fp], "a") as f:
                f.write("\n".join(ls) + "\n")
        svc.step()
    total = sum(os.path.getsize(f) for f in mapping.values())
    deadline = _time.time() + 60
    while _time.time() < deadline:
        svc.step()
        svc._idle(0.01)
        if sum(o[1] for o in svc.tailer.offsets()) == total and svc._held is None:
            break
    assert sum(o[1] for o in svc.tailer.offsets()) == total
    path_of = {i: p for p, i in svc.file_ids.items()}
    svc.shutdown()
    assert svc.perf["prefetched"] > 0 and len(svc.batch_log) > 3
    bl = [[(path_of[fid], data[lo:hi].decode().rstrip("\n").split("\n")) for fid, lo, hi in ch]
          for data, ch in svc.batch_log]
    P = PipelineOracle(copy.deepcopy(C), TzOffset("UTC"), server_fn=srv_of)
    P.run_batches(with_watermarks(bl, TzOffset("UTC")))
    want = sinks.copy_encode_lines(P.tx_db + P.audit_db + P.fs + P.al)
    assert sorted(w.rows["tx"]) == sorted(want["tx"]) and len(want["tx"]) > 100
    assert w.rows["stats"] == want["fs"] and len(want["fs"]) > 0
    assert w.rows.get("alerts", []) == want["al"]


def test_transactions_queue_roundtrip_with_reference_stages(tmp_path):
    """Mixed deployment: a reference parser stage publishes tx lines (entries.js TxEntry CSV,
    one message per line) to `transactions`; the GPU engine (inputMode transactions) takes over
    stats / z-score / alerts and publishes fs to `z_score` -- what stream_process_alerts.js
    consumes -- and tx / fs / al to db_insert, persistent and publisher-confirmed."""
    import time as _time
    from apmbackend_amd.models.oracle import PipelineOracle
    from apmbackend_amd.runtime.amqp_broker import Broker
    from apmbackend_amd.runtime.queue import QueueManager
    from apmbackend_amd.utils.synth import with_watermarks
    from apmbackend_amd.utils.timeparse import TzOffset
    C, lines, mapping, sc = make_env(tmp_path)
    gpu_cfg(C)
    P = PipelineOracle(copy.deepcopy(C), TzOffset("UTC"))
    P.run_batches(with_watermarks(batches(lines, sc.start_ms, 5.0), TzOffset("UTC")))
    assert P.tx_out and P.fs and P.al
    b = Broker(port=0).start()
    try:
        C["amqpConnectionString"] = b.url
        C["gpu"].update({"outputMode": "amqp", "inputMode": "transactions", "bridgeQueues": ["z_score"]})
        svc = IngestService(C, engine="native", files=[], rank=0, world=1, server_of_path=srv_of)
        ref = QueueManager(b.url)  # the reference parser's producer side
        prod = ref.get_queue("transactions", "p")
        for i in range(0, len(P.tx_out), 37):
            prod.write_lines(P.tx_out[i:i + 37])
            _time.sleep(0.01)
            svc.step()
        deadline = _time.time() + 60
        while svc.native.metrics()["tx"] < len(P.tx_out) and _time.time() < deadline:
            svc.step()
            _time.sleep(0.02)
        svc.native.flush()
        svc._drain_outputs()
        assert svc.native.metrics()["tx"] == len(P.tx_out), (svc.native.metrics()["tx"], len(P.tx_out), {
            k: (getattr(p, "paused", None), p.buffer_count()) for k, p in svc.producers.items()}, b.stats())
        assert svc.qm.wait_confirms(10.0)
        got_z, got_db = [], []
        zc = amqp_collect(b.url, "z_score", got_z)
        dc = amqp_collect(b.url, "db_insert", got_db)
        assert wait_until(lambda: len(got_z) >= len(P.fs))
        assert got_z == P.fs
        assert wait_until(lambda: sum(1 for l in got_db if l.startswith("al|")) >= len(P.al)
                          and sum(1 for l in got_db if l.startswith("fs|")) >= len(P.fs))
        assert [l for l in got_db if l.startswith("al|")] == P.al
        assert [l for l in got_db if l.startswith("fs|")] == P.fs
        zc.close()
        dc.close()
        svc.shutdown()
        ref.shutdown()
    finally:
        b.stop()


def wait_until(pred, timeout=20.0):
    import time as _time
    t0 = _time.time()
    while _time.time() - t0 < timeout:
        if pred():
            return True
        _time.sleep(0.05)
    return pred()


def amqp_collect(url, queue, out):
    from apmbackend_amd.runtime.amqp import Connection
    c = Connection(url)
    c.queue_declare(queue)
    c.consume(queue, lambda m: (out.append(m.body.decode()), c.ack(m.delivery_tag)))
    return c


def _spool_rows(d):
    import collections
    import glob as g
    rows = collections.defaultdict(collections.Counter)
    for p in g.glob(os.path.join(d, "*.copy")):
        table = os.path.basename(p).split(".")[0].rsplit("_lane", 1)[0]
        with open(p) as f:
            rows[table].update(l for l in f.read().split("\n") if l)
    return rows


def test_native_sink_checkpoint_snapshots_keep_every_row_once(tmp_path):
    """VERDICT r3 #5 on the GPU service path: the native COPY sink (GPU-encoded fs / db rows,
    2 writer lanes) with a checkpoint at every poll -- each one captures the sink's unacknowledged
    flushes by reference and the engine's checkpoint writer persists them before the manifest
    names it.  The spool holds exactly the rows of a run without checkpoints, and the named
    snapshot files exist and parse."""
    from apmbackend_amd.runtime import sinks
    res = []
    for ck in (False, True):
        d = tmp_path / ("ck" if ck else "plain")
        d.mkdir()
        C, lines, mapping, sc = make_env(d)
        gpu_cfg(C)
        C["streamInsertDb"].update({"sink": "spool", "copySinkDir": str(d / "spool"), "writerLanes": 2,
                                    "copySinkRotateBytes": 1 << 40})
        if ck:
            C["gpu"]["checkpointDir"] = str(d / "ckpt")
            C["gpu"]["checkpointEverySeconds"] = 0
        svc = IngestService(C, engine="native", files=sorted(mapping.values()), rank=0, world=1, server_of_path=srv_of)
        assert svc.inserter.core is not None
        run(svc, lines, mapping, sc)
        if ck:
            assert svc.n_checkpoints >= 3
            svc.eng.checkpoint_wait()
            extra = open(os.path.join(d, "ckpt", "engine.rank0.ckpt"), "rb").read()
            assert extra.startswith(b"APMCHAIN")
            snaps = [p for p in os.listdir(d / "ckpt") if p.startswith("sink_pending.")]
            assert snaps
            for p in snaps:
                sinks.read_sink_snapshot(str(d / "ckpt" / p), 0)
        svc.shutdown()
        res.append(_spool_rows(str(d / "spool")))
    a, b = res
    assert set(a) == set(b) and sum(len(c) for c in a.values()) > 0
    for t in a:
        assert a[t] == b[t], t
