"""DB insert stage (runtime/sinks.py) against the reference's stream_insert_db.js behaviour."""
import os
import time
import datetime as dt
import json

import pytest

from apmbackend_amd.runtime import sinks
from apmbackend_amd.utils.config import default_config

TX = "tx|jvm01|S:getFoo|[L1]|12345|1578391200000|1578391200250|250|Y"
FS = ("fs|1578391200000|jvm01|S:getFoo|360|1.20|250.0:240.1:200.0:280.2:1|300.0:undefined:undefined:"
      "undefined:0.0|400.0:390.0:380.0:400.0:-1.0")
AL = ("al|1578391201000|1578391200000|jvm01|S:getFoo|average exceeded hard ms threshold|"
      + FS.replace("|", "&"))
JX = "jx|1578391200000|jvm01|1|2|3|100|200|300|10|20|30|0.5|1000|50|20|5|6|7"


class ListWriter(sinks.Writer):
    def __init__(self, fail=0):
        self.calls = []
        self.fail = fail

    def write(self, table, columns, rows):
        if self.fail:
            self.fail -= 1
            raise RuntimeError("db down")
        self.calls.append((table, list(columns), list(rows)))


class Clock:
    t = 0.0

    def __call__(self):
        return self.t


def cfg(limit=3, wait_ms=5000, resume=None):
    C = default_config(replay=True)
    C["streamInsertDb"]["dbInsertBufferLimit"] = limit
    C["streamInsertDb"]["dbMaxTimeBetweenInsertsMs"] = wait_ms
    C["streamInsertDb"]["bufferResumeFileFullPath"] = resume
    return C


def test_copy_rows_for_every_type():
    rows = sinks.copy_encode_lines([TX, FS, AL, JX, "st|1|a|b|0.00|1.0|2.0|3.0", "garbage"])
    tx = rows["tx"][0].rstrip("\n").split("\t")
    assert tx == ["2020-01-07 10:00:00.250+00", "2020-01-07 10:00:00.000+00", "jvm01", "S:getFoo", "[L1]",
                  "12345", "250", "Y"]
    fs = rows["fs"][0].rstrip("\n").split("\t")
    assert fs[:5] == ["2020-01-07 10:00:00.000+00", "jvm01", "S:getFoo", "1.2", "360"]
    stats = json.loads(fs[5])
    assert stats["average"] == 250 and stats["averagesignal"] == 1 and stats["per75avg"] is None
    assert stats["per95signal"] == -1
    assert '"per75signal":0' in fs[5]  # JS number text, not 0.0
    al = rows["al"][0].rstrip("\n").split("\t")
    assert al[0] == "2020-01-07 10:00:00.000+00" and al[1] == "2020-01-07 10:00:01.000+00"
    assert json.loads(al[5])["server"] == "jvm01"
    jx = rows["jx"][0].rstrip("\n").split("\t")
    assert len(jx) == 18 and jx[11] == "0.5"
    assert rows["tx"] and not any("st|" in r for r in sum(rows.values(), []))


def test_copy_escaping_and_nulls():
    line = "tx|jv\\m|S:a\tb|x|NaN|NaN|1578391200250|NaN|N"
    row = sinks.copy_encode_lines([line])["tx"][0]
    f = row.rstrip("\n").split("\t")
    assert f[1] == "\\N" and f[2] == "jv\\\\m" and f[5] == "\\N" and f[6] == "\\N"
    assert "S:a\\tb" in row


def test_buffer_limit_flushes_before_append():
    w = ListWriter()
    ins = sinks.DBInserter(cfg(limit=3), writer=w, clock=Clock())
    for _ in range(7):
        ins.consume_line(TX)
    # 4th row flushes 3, 7th row flushes 3 more, 1 left buffered
    assert [len(c[2]) for c in w.calls] == [3, 3]
    assert len(ins.buffers["tx"]) == 1
    assert w.calls[0][0] == "tx" and w.calls[0][1][0] == "endts"


def test_timeout_flush_and_failure_rebuffers_at_front():
    clk = Clock()
    w = ListWriter(fail=1)
    ins = sinks.DBInserter(cfg(limit=1000, wait_ms=5000), writer=w, clock=clk)
    ins.consume_line(AL)
    clk.t = 4.9
    assert ins.tick() == 0 and not w.calls
    clk.t = 5.0
    assert ins.tick() == 0 and ins.failures == 1  # writer failed: row kept
    assert len(ins.buffers["al"]) == 1
    ins.consume_line(AL.replace("jvm01", "jvm02"))
    clk.t = 10.1
    assert ins.tick() == 2
    rows = w.calls[0][2]
    assert "jvm01" in rows[0] and "jvm02" in rows[1]  # failed batch stays first
    assert ins.stats.total_rows == 2
    assert "DBRecordsIns: 2" in ins.stats.line()


def test_resume_file_roundtrip(tmp_path):
    path = str(tmp_path / "buf.resume")
    w = ListWriter(fail=100)
    ins = sinks.DBInserter(cfg(resume=path), writer=w, clock=Clock())
    for ln in (TX, FS, AL, JX):
        ins.consume_line(ln)
    ins.close()  # flush fails -> everything persisted
    doc = json.load(open(path))
    assert doc["dataType"] == "Map" and [t for t, _ in doc["value"]] == ["tx", "fs", "al", "jx"]
    assert doc["value"][0][1][0]["endts"] == "2020-01-07T10:00:00.250Z"
    w2 = ListWriter()
    ins2 = sinks.DBInserter(cfg(resume=path), writer=w2, clock=Clock())
    assert sum(len(b) for b in ins2.buffers.values()) == 4
    assert isinstance(ins2.buffers["tx"][0]["endts"], dt.datetime)
    ins2.flush_all()
    assert sorted(c[0] for c in w2.calls) == ["alerts", "jmx", "stats", "tx"]


def test_spool_writer(tmp_path):
    w = sinks.CopySpoolWriter(str(tmp_path))
    ins = sinks.DBInserter(cfg(limit=2), writer=w, clock=Clock())
    for _ in range(5):
        ins.consume_line(TX)
    ins.flush_all()
    w.close()
    data = open(tmp_path / "tx.copy").read().splitlines()
    assert len(data) == 5
    assert open(tmp_path / "tx.columns").read().strip().split(",")[0] == "endts"


def _oracle_stream():
    import copy
    from apmbackend_amd.models.oracle import PipelineOracle
    from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks
    from apmbackend_amd.utils.timeparse import TzOffset
    UTC = TzOffset("UTC")
    start = 1578391200000
    an = [Anomaly("jvm00", "getSvc0001", start + 100_000, start + 700_000, 30.0)]
    sc = SynthConfig(servers=2, duration_s=800, tx_per_sec_per_server=3, seed=11, ejb_services=3,
                     provider_services=2, anomalies=an)
    lines = Generator(sc).generate()
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5}]
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 5
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 2
    C["gpu"]["timezone"] = "UTC"
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(with_watermarks(batches(lines, start, 5.0), UTC))
    return P.tx_db + P.audit_db + P.fs + P.al


def test_native_copy_encoder_matches_python():
    from apmbackend_amd import _native
    N = _native.load()
    stream = _oracle_stream()
    jx = [JX, "jx|1578391260000|jvm02|1|x|3|100|200|300|10|20|30|abc|1000|50|20|5|6"]
    weird = ["tx|a\\b|S:x\ty|[L9]|0x1F|  12|1578391200250|NaN|Y", "tx|short", "fs|1578391200000|s|v|8640|Infinity|"
             "1e3:-0:undefined:2.5e-7:-1|1:2:3:4:1.0|5:6:7:8:0.0", "al|1|2|s|v|c|fs&1578391200000&s&v&6&0.00&u:u:u:u:0"]
    lines = stream + jx + weird
    assert any(l.startswith("al|") for l in stream) and any(l.startswith("fs|") for l in stream)
    want = sinks.copy_encode_lines(lines)
    got = N.copy_encode(("\n".join(lines) + "\n").encode())
    for t in sinks.TYPES:
        blob, cnt = got[t]
        assert cnt == len(want[t]), t
        assert blob.decode() == "".join(want[t]), t


def test_inserter_native_and_python_paths_agree(tmp_path):
    stream = _oracle_stream()
    outs = []
    for native in (True, False):
        C = cfg(limit=500)
        C["streamInsertDb"]["nativeCopyEncoder"] = native
        w = ListWriter()
        ins = sinks.DBInserter(C, writer=w, clock=Clock())
        ins.consume_bytes(("\n".join(stream) + "\n").encode())
        ins.flush_all()
        outs.append(sorted((c[0], tuple(c[2])) for c in w.calls))
    assert outs[0] == outs[1] and len(outs[0]) >= 3


# ----------------------------------------------------------------------------- native DbSink

def _wire_lines(n=40):
    from apmbackend_amd.utils.records import StatEntry, TxEntry
    out = []
    for i in range(n):
        out.append(TxEntry("srv", f"S:svc{i % 3}", f"LOG{i}", "1234", 1578391200000 + i, 1578391200100 + i,
                           str(100 + i), "Y").to_csv())
        out.append(f"fs|{1578391200000 + i}|srv|S:svc{i % 3}|12.50|6|100.0:99.5:90.1:110.2:0|"
                   f"120.0:119.0:100.0:130.0:1|150.0:149.0:140.0:160.0:0")
    out.append("junk line")
    return out


def _native_ok():
    N = sinks._native()
    return N is not None and hasattr(N, "DbSink")


@pytest.mark.skipif(not _native_ok(), reason="native extension not built")
def test_native_sink_spool_matches_python_encoder(tmp_path):
    lines = _wire_lines()
    C = cfg(limit=7)
    C["streamInsertDb"].update({"sink": "spool", "copySinkDir": str(tmp_path / "spool")})
    ins = sinks.DBInserter(C, clock=Clock())
    assert ins.core is not None
    assert ins.consume_bytes(("\n".join(lines) + "\n").encode()) == len(lines) - 1
    ins.close()
    want = sinks.copy_encode_lines(lines)
    for t in ("tx", "fs"):
        table = C["streamInsertDb"][sinks.COLUMNS[t][0]]
        got = open(tmp_path / "spool" / f"{table}.copy").read()
        assert got == "".join(want[t])
        assert open(tmp_path / "spool" / f"{table}.columns").read().strip() == ", ".join(sinks.COLUMNS[t][1])
    assert ins.stats.total_rows == len(lines) - 1


@pytest.mark.skipif(not _native_ok(), reason="native extension not built")
def test_native_sink_limit_and_timer_semantics():
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    s = N.DbSink(3, 50.0, ["t_tx", "t_fs", "t_al", "t_jx", "t_fb"], ["a", "b", "c", "d", "e"], "null", [], 0, 1)
    tx = [l for l in _wire_lines() if l.startswith("tx|")][:7]
    s.consume(("\n".join(tx) + "\n").encode())
    s.drain()
    st = s.stats()
    # flushed before the 4th and 7th rows were appended: 2 flushes x 3 rows, 1 row buffered
    assert st["flushes"] == 2 and st["rows"] == 6 and st["buffered"] == 1
    assert s.tick() == 0  # deadline not reached yet
    time.sleep(0.08)
    assert s.tick() == 1
    s.drain()
    assert s.stats()["rows"] == 7 and s.stats()["buffered"] == 0
    assert s.close() == [b"", b"", b"", b"", b""]


@pytest.mark.skipif(not _native_ok(), reason="native extension not built")
def test_native_sink_persistent_psql_copy_and_rebuffer(tmp_path, monkeypatch):
    """One long-lived psql process, one acknowledged COPY per flush; a failed COPY puts its rows
    back at the front of the buffer and they go out with the next flush once the table works."""
    import sys
    out = tmp_path / "pg"
    out.mkdir()
    monkeypatch.setenv("FAKE_PSQL_OUT", str(out))
    monkeypatch.setenv("FAKE_PSQL_FAIL", "apm_stats")
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    fake = [sys.executable, os.path.join(os.path.dirname(__file__), "fixtures", "fake_psql.py")]
    s = N.DbSink(1000, 1e9, ["apm_tx", "apm_stats", "apm_alerts", "apm_jmx", "apm_fleet_stats"], ["a", "b", "c", "d", "e"],
                 "psql", fake, 0, 2)
    lines = _wire_lines(10)
    s.consume(("\n".join(lines) + "\n").encode())
    s.flush_all()
    s.drain()
    st = s.stats()
    assert st["rows"] == 10 and st["failures"] == 1 and st["buffered"] == 10  # fs rows re-buffered
    assert "apm_stats" in st["last_error"]
    want = sinks.copy_encode_lines(lines)
    assert open(out / "apm_tx.rows").read() == "".join(want["tx"])
    monkeypatch.setenv("FAKE_PSQL_FAIL", "")  # the running psql keeps failing that table...
    left = s.close()
    assert left[1].count(b"\n") == 10  # ...so close() hands the rows back (resume file)
    assert left[0] == b""


def test_copy_rows_parse_back_for_the_resume_file():
    lines = _wire_lines(6)
    enc = sinks.copy_encode_lines(lines)
    for t in ("tx", "fs"):
        for row in enc[t]:
            assert sinks.copy_row(t, sinks.pg_row_from_copy(t, row)) == row


def test_fleet_rows_encode_natively_like_python():
    from apmbackend_amd.utils.records import entry_from_csv
    lines = ["fb|1578391200000|S:getFoo|6|8|123.4:5.6|130.0:7.0|undefined:undefined",
             "fb|1578391210000|Provider:cb-util-001|360|3|0.5:0.0|1.2:0.3|9.9:1.0"]
    assert entry_from_csv(lines[0]).to_csv() == lines[0]
    want = sinks.copy_encode_lines(lines)
    nat = sinks.copy_encode_native(lines)
    if nat is not None:
        assert nat["fb"][0].decode() == "".join(want["fb"]) and nat["fb"][1] == 2
    assert want["fb"][0].startswith("2020-01-07 10:00:00.000+00\tS:getFoo\t6\t8\t{\"averagemean\":123.4,")
    assert '"per95mean":null' in want["fb"][0]


@pytest.mark.skipif(not _native_ok(), reason="native extension not built")
@pytest.mark.parametrize("limit,pre", [(1000, 0), (1000, 437), (1000, 1000), (7, 3), (1, 0)])
def test_native_sink_parallel_cut_equals_serial(tmp_path, limit, pre):
    """A rollover's COPY rows (> 4 MB) are cut at the flush limit and copied by several threads;
    the flushes (rows each, order, bytes) and the buffered remainder must be those of the serial
    path, which the same rows fed in small pieces take -- whatever the buffer held before."""
    import random
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    rng = random.Random(limit * 1000 + pre)
    rows = [("r%07d\t" % i) + "x" * rng.randint(5, 400) + "\n" for i in range(50000)]  # > 8 MB: parallel spool writes too
    head, body = "".join(rows[:pre]), "".join(rows[pre:])
    assert len(body) > 4 << 20
    results = []
    for mode in ("one-shot", "pieces"):
        d = tmp_path / mode
        s = N.DbSink(limit, 1e9, ["t_tx", "t_fs", "t_al", "t_jx", "t_fb"], ["a", "b", "c", "d", "e"], "spool",
                     [str(d)], 1 << 62, 2)
        if head:
            s.consume_encoded(1, head.encode())
        if mode == "one-shot":
            assert s.consume_encoded(1, body.encode()) == len(rows) - pre
        else:
            b = body.encode()
            pos = 0
            while pos < len(b):  # < 4 MB pieces at row boundaries: the serial path
                end = b.find(b"\n", min(len(b) - 1, pos + (1 << 20))) + 1
                s.consume_encoded(1, b[pos:end])
                pos = end
        s.drain()
        st = s.stats()
        s.flush_all()
        s.drain()
        results.append((st["flushes"], st["rows"], st["buffered"], open(d / "t_fs.copy").read()))
    assert results[0] == results[1]
    assert results[0][3] == head + body
    assert results[0][1] == (len(rows) - results[0][2])


@pytest.mark.skipif(not _native_ok(), reason="native extension not built")
@pytest.mark.parametrize("limit,pre,size", [(1000, 0, 50000), (1000, 437, 50000), (7, 3, 3000), (1000, 10, 300)])
def test_native_sink_row_offset_cut_equals_scan(tmp_path, limit, pre, size):
    """The engine hands its fs COPY rows with K12's row offsets (write_rows_held): the sink cuts
    its flushes from the offsets (empty rows skipped) instead of scanning the text.  Flushes,
    rows and bytes must equal the scanning path's, small and large blobs alike."""
    import random
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    rng = random.Random(limit + pre + size)
    rows = [("r%07d\t" % i) + "x" * rng.randint(5, 400) + "\n" for i in range(size)]
    head, body = "".join(rows[:pre]), "".join(rows[pre:])
    off = [0]
    for r in rows[pre:]:
        while rng.random() < 0.2:  # inactive (series, LAG) cells: zero-length rows
            off.append(off[-1])
        off.append(off[-1] + len(r))
    results = []
    for mode in ("scan", "offsets"):
        d = tmp_path / mode
        s = N.DbSink(limit, 1e9, ["t_tx", "t_fs", "t_al", "t_jx", "t_fb"], ["a", "b", "c", "d", "e"], "spool",
                     [str(d)], 1 << 62, 2)
        if head:
            s.consume_encoded(1, head.encode())
        if mode == "scan":
            assert s.consume_encoded(1, body.encode()) == len(rows) - pre
        else:
            assert s.consume_encoded_rows(1, body.encode(), off) == len(rows) - pre
        s.drain()
        st = s.stats()
        s.flush_all()
        s.drain()
        results.append((st["flushes"], st["rows"], st["buffered"], open(d / "t_fs.copy").read()))
    assert results[0] == results[1]
    assert results[0][3] == head + body


@pytest.mark.parametrize("lanes", [2, 4])
def test_native_sink_writer_lanes_write_every_row_once_in_lane_order(tmp_path, lanes):
    """Writer lanes (dbsink.cpp): flushes go round-robin (blocks of 16) to `lanes` independent
    writers, each with its own spool file per table.  Every row lands exactly once, the
    `<table>.columns` file is shared, and each lane's file holds its rows in submission order
    (a subsequence of the input).  Serial mixed-type input (wire lines) and a parallel-cut COPY blob
    both go through the lanes."""
    import glob
    import random
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    rng = random.Random(lanes)
    d = tmp_path / "spool"
    s = N.DbSink(7, 1e9, ["t_tx", "t_fs", "t_al", "t_jx", "t_fb"], ["a", "b", "c", "d", "e"], "spool",
                 [str(d)], 1 << 62, 2, lanes)
    rows = [("r%07d\t" % i) + "y" * rng.randint(5, 300) + "\n" for i in range(40000)]
    blob = "".join(rows)
    assert len(blob) > 4 << 20  # parallel cut path
    assert s.consume_encoded(1, blob.encode()) == len(rows)
    small = [("s%05d\t" % i) + "z\n" for i in range(500)]
    for i in range(0, len(small), 13):
        s.consume_encoded(1, "".join(small[i:i + 13]).encode())
    s.flush_all()
    s.drain()
    st = s.stats()
    s.close()
    assert st["lanes"] == lanes and st["failures"] == 0 and st["rows"] == len(rows) + len(small)
    files = sorted(glob.glob(str(d / "t_fs*.copy")))
    assert len(files) == lanes, files
    order = {r: i for i, r in enumerate(rows + small)}
    seen = []
    for f in files:
        got = open(f).read().splitlines(keepends=True)
        idx = [order[r] for r in got]
        assert idx == sorted(idx), f"{f}: rows out of submission order"
        seen += got
    assert sorted(seen) == sorted(rows + small)
    assert open(d / "t_fs.columns").read() == "b\n"
    assert not glob.glob(str(d / "*.tmp"))


def test_native_sink_psql_writer_lanes_use_one_connection_each(tmp_path, monkeypatch):
    """`lanes` = 3: three long-lived psql connections, each acknowledging its own COPYs; every
    row is committed once."""
    import sys
    out = tmp_path / "pg"
    out.mkdir()
    monkeypatch.setenv("FAKE_PSQL_OUT", str(out))
    monkeypatch.setenv("FAKE_PSQL_FAIL", "")
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    fake = [sys.executable, os.path.join(os.path.dirname(__file__), "fixtures", "fake_psql.py")]
    s = N.DbSink(5, 1e9, ["apm_tx", "apm_stats", "apm_alerts", "apm_jmx", "apm_fleet_stats"], ["a", "b", "c", "d", "e"],
                 "psql", fake, 0, 2, 3)
    lines = [l for l in _wire_lines(400) if l.startswith("tx|")]
    assert len(lines) >= 160  # >= 32 flushes of 5: all three lanes get work
    s.consume(("\n".join(lines) + "\n").encode())
    s.flush_all()
    s.drain()
    st = s.stats()
    s.close()
    assert st["failures"] == 0 and st["rows"] == len(lines) and st["lanes"] == 3
    want = sinks.copy_encode_lines(lines)["tx"]
    assert sorted(open(out / "apm_tx.rows").read().splitlines(keepends=True)) == sorted(want)
    assert len(set(open(out / "connections").read().split())) == 3


def test_native_sink_psql_unacknowledged_copy_is_not_retried(tmp_path, monkeypatch):
    """a COPY whose acknowledgement never arrives may have committed (the whole
    COPY and its terminator were sent).  Re-buffering it duplicated its rows in the DB; now the
    flush is reported as 'outcome unknown' (doubtful_rows), not retried, and the timeout is
    streamInsertDb.psqlAckTimeoutSeconds."""
    import sys
    out = tmp_path / "pg"
    out.mkdir()
    monkeypatch.setenv("FAKE_PSQL_OUT", str(out))
    monkeypatch.setenv("FAKE_PSQL_HANG", "apm_stats")
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    fake = [sys.executable, os.path.join(os.path.dirname(__file__), "fixtures", "fake_psql.py")]
    s = N.DbSink(1000, 1e9, ["apm_tx", "apm_stats", "apm_alerts", "apm_jmx", "apm_fleet_stats"], ["a", "b", "c", "d", "e"],
                 "psql", fake, 0, 2, 1, 500.0)
    lines = _wire_lines(10)
    s.consume(("\n".join(lines) + "\n").encode())
    s.flush_all()
    s.drain()
    st = s.stats()
    assert st["doubtful_rows"] == 10 and st["doubtful_flushes"] == 1
    assert st["buffered"] == 0  # not re-buffered: no duplicate on the next flush
    assert "outcome unknown" in st["last_error"]
    want = sinks.copy_encode_lines(lines)
    assert open(out / "apm_stats.rows").read() == "".join(want["fs"])  # committed exactly once
    s.close()


@pytest.mark.parametrize("mode", ["copy", "capture"])
def test_sink_snapshot_watermark_restores_unwritten_rows_once(tmp_path, monkeypatch, mode):
    """checkpoints snapshot the sink's unacknowledged flushes instead of draining
    it.  Flushes the writer acknowledged after the snapshot are skipped on restore (the ack file's
    watermark), flushes it never wrote are submitted again -- every row lands exactly once."""
    import sys
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    tables = ["apm_tx", "apm_stats", "apm_alerts", "apm_jmx", "apm_fleet_stats"]
    fake = [sys.executable, os.path.join(os.path.dirname(__file__), "fixtures", "fake_psql.py")]
    out = tmp_path / "pg"
    out.mkdir()
    monkeypatch.setenv("FAKE_PSQL_OUT", str(out))
    monkeypatch.setenv("FAKE_PSQL_FAIL", "apm_stats")  # the stats table is down: fs flushes fail
    ack = str(tmp_path / "sink.ack")
    s = N.DbSink(1000, 1e9, tables, ["a", "b", "c", "d", "e"], "psql", fake, 0, 2)
    s.set_ack_file(ack, 7)
    lines = _wire_lines(10)
    s.consume(("\n".join(lines) + "\n").encode())
    s.flush_all()
    s.drain()
    snap = str(tmp_path / "pending.bin")
    if mode == "copy":
        acked_before, jobs = s.snapshot_pending()  # (no drain: the fs rows are back in their buffer)
        assert sum(j[3] for j in jobs) == 10 and {j[1] for j in jobs} == {1}
        sinks.write_sink_snapshot(snap, jobs)
        n_jobs = len(jobs)
    else:
        # the checkpoint writer's form: references taken now, written (and released) later
        h = s.snapshot_capture()
        assert h.rows == 10 and h.jobs >= 1
        h.write(snap)
        n_jobs = h.jobs
    s.close()  # "crash": the fs rows were never written
    acked = sinks.read_sink_ack(ack, 7)
    assert acked >= 0 and sinks.read_sink_ack(ack, 8) == -1  # another incarnation: unknown
    n, todo = sinks.read_sink_snapshot(snap, acked)
    assert n == n_jobs and sum(j[3] for j in todo) == 10
    monkeypatch.setenv("FAKE_PSQL_FAIL", "")  # the restarted service: table back
    s2 = N.DbSink(1000, 1e9, tables, ["a", "b", "c", "d", "e"], "psql", fake, 0, 2)
    for _seq, ti, enc, rows, data in todo:
        if enc:
            s2.add_encoded(ti, data, rows)
        else:
            s2.consume(data)
    s2.flush_all()
    s2.drain()
    s2.close()
    want = sinks.copy_encode_lines(lines)
    assert open(out / "apm_tx.rows").read() == "".join(want["tx"])
    assert open(out / "apm_stats.rows").read() == "".join(want["fs"])


@pytest.mark.parametrize("mode", ["copy", "capture"])
def test_sink_snapshot_of_acknowledged_flushes_restores_nothing(tmp_path, mode):
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    tables = ["apm_tx", "apm_stats", "apm_alerts", "apm_jmx", "apm_fleet_stats"]
    ack = str(tmp_path / "sink.ack")
    s = N.DbSink(3, 1e9, tables, ["a", "b", "c", "d", "e"], "spool", [str(tmp_path / "spool")], 1 << 30, 2, 2)
    s.set_ack_file(ack, 11)
    lines = _wire_lines(40)
    s.consume(("\n".join(lines) + "\n").encode())
    if mode == "copy":
        _acked, jobs = s.snapshot_pending()  # taken while the lanes may still be writing
        sinks.write_sink_snapshot(str(tmp_path / "p.bin"), jobs)
    else:
        h = s.snapshot_capture()  # the lanes keep writing (and acknowledging) meanwhile
        s.drain()
        h.write(str(tmp_path / "p.bin"))  # written flushes released only now
    s.drain()  # everything gets written and acknowledged
    s.close()
    _n, todo = sinks.read_sink_snapshot(str(tmp_path / "p.bin"), sinks.read_sink_ack(ack, 11))
    assert todo == []
