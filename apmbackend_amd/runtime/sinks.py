"""DB insert stage: buffered Postgres loading of the ``db_insert`` stream (reference
``stream_insert_db.js:1-402``, ``dbstats.js:1-45``, row mappers ``entries.js:23-42,120-151,
218-240,310-331``).

Behaviour kept from the reference:

* one buffer per record type (``tx``, ``fs``, ``al``, ``jx``); a record is converted to its row
  object on arrival (``toPostgresObject``);
* a buffer is flushed when it already holds ``dbInsertBufferLimit`` rows *before* the new row is
  appended (so a flush carries at most ``limit`` rows, :341-345), or when
  ``dbMaxTimeBetweenInsertsMs`` passed since the first row entered an empty buffer (:333-339);
* a failed flush puts the rows back at the *front* of the buffer (:310-320) and is retried by the
  next flush;
* on shutdown every buffer is flushed and whatever is left is written to
  ``bufferResumeFileFullPath`` in the reference's Map JSON format (util_methods.js:189-219);
* ``DBStats`` logs rows inserted / total ms / ms per row every ``statLogIntervalInSeconds``.

Changed on purpose:

* rows are loaded with ``COPY ... FROM STDIN`` text format instead of multi-row ``INSERT``
  (K13).  The encoder is native for the high-volume streams (``_apm_native.copy_encode``);
  this module holds the Python definition it is tested against;
* writers: ``psql`` pipe when a ``psql`` binary and DB settings exist, else a COPY spool
  directory (``copySinkDir``; load later with ``\\copy``), or a null writer;
* the resume file is actually re-loaded (the reference resets it, :176-180 -- Q19).
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import math
import os
import shutil
import subprocess
import threading
import time
from collections import deque
from typing import Any, Callable, Deque, Dict, Iterable, List, Optional, Sequence, Tuple

from ..utils.jsfmt import js_str
from ..utils.records import entry_from_csv

log = logging.getLogger("apm.insert_db")

# ColumnSets of stream_insert_db.js:149-160 (type -> config key of the table, columns)
COLUMNS: Dict[str, Tuple[str, List[str]]] = {
    "tx": ("dbTxTable", ["endts", "startts", "server", "service", "logid", "acctnum", "elapsed", "toplevel"]),
    "fs": ("dbStatTable", ["timestamp", "server", "service", "tpm", "lag", "stats"]),
    "al": ("dbAlertTable", ["entrytimestamp", "alerttimestamp", "server", "service", "cause", "entry"]),
    "jx": ("dbJmxTable", ["timestamp", "server", "dsinusenodes", "dsactivenodes", "dsavailablenodes", "heapused",
                          "heapcommitted", "heapmax", "metaused", "metacommitted", "metamax", "sysload", "classcnt",
                          "threadcnt", "daemonthreadcnt", "beanpoolavailablecnt", "beanpoolcurrentsize",
                          "beanpoolmaxsize"]),
    # fleet-merged per-service baselines (fb records, rank 0): not part of the reference schema
    "fb": ("dbFleetTable", ["timestamp", "service", "lag", "nseries", "stats"]),
}
TYPES = ("tx", "fs", "al", "jx", "fb")


# --------------------------------------------------------------------------- COPY text encoding

def _js_json(v: Any) -> str:
    """JSON.stringify-compatible value text (numbers in JS String() form, dates ISO)."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
            return "null"
        return js_str(v)
    if isinstance(v, _dt.datetime):
        return json.dumps(_iso_js(v))
    if isinstance(v, dict):
        return "{" + ",".join(json.dumps(str(k)) + ":" + _js_json(x) for k, x in v.items()) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_js_json(x) for x in v) + "]"
    return json.dumps(str(v), ensure_ascii=False)


def _iso_js(d: _dt.datetime) -> str:
    """Date.prototype.toISOString(): 2020-01-07T10:00:00.000Z"""
    d = d.astimezone(_dt.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%S.") + f"{d.microsecond // 1000:03d}Z"


def _pg_ts(d: _dt.datetime) -> str:
    d = d.astimezone(_dt.timezone.utc)
    return d.strftime("%Y-%m-%d %H:%M:%S.") + f"{d.microsecond // 1000:03d}+00"


def _copy_escape(s: str) -> str:
    return (s.replace("\\", "\\\\").replace("\t", "\\t").replace("\n", "\\n").replace("\r", "\\r"))


def copy_field(v: Any) -> str:
    if v is None:
        return "\\N"
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return "\\N"
    if isinstance(v, _dt.datetime):
        return _pg_ts(v)
    if isinstance(v, (dict, list)):
        return _copy_escape(_js_json(v))
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return js_str(v)
    return _copy_escape(str(v))


def copy_row(rtype: str, row: Dict[str, Any]) -> str:
    return "\t".join(copy_field(row.get(c)) for c in COLUMNS[rtype][1]) + "\n"


def _copy_unescape(s: str) -> Optional[str]:
    if s == "\\N":
        return None
    out, i = [], 0
    while i < len(s):
        ch = s[i]
        if ch == "\\" and i + 1 < len(s):
            nx = s[i + 1]
            out.append({"t": "\t", "n": "\n", "r": "\r"}.get(nx, nx))
            i += 2
        else:
            out.append(ch)
            i += 1
    return "".join(out)


def pg_row_from_copy(rtype: str, row: str) -> Dict[str, Any]:
    """A COPY text row (copy_row / the GPU's fs COPY rows) back to its row object -- for the
    resume file when rows are still buffered at shutdown."""
    cols = COLUMNS[rtype][1]
    vals = [_copy_unescape(f) for f in row.rstrip("\n").split("\t")]
    out: Dict[str, Any] = {}
    for c, v in zip(cols, vals):
        if v is None:
            out[c] = None
        elif c in _TS_COLS:
            out[c] = _dt.datetime.strptime(v[:-3], "%Y-%m-%d %H:%M:%S.%f").replace(tzinfo=_dt.timezone.utc)
        elif c in ("stats", "entry"):
            out[c] = json.loads(v)
        elif c in ("tpm", "elapsed", "acctnum", "nseries") or rtype == "jx" and c not in ("server",):
            f = float(v)
            out[c] = int(f) if f.is_integer() and "." not in v and "e" not in v else f
        else:
            out[c] = v
    return out


def pg_row_from_line(line: str) -> Optional[Tuple[str, Dict[str, Any]]]:
    """consumeMsg (:355-376): CSV -> entry -> toPostgresObject, for tx/fs/al/jx only."""
    e = entry_from_csv(line)
    if e is None or e.type not in COLUMNS:
        return None
    return e.type, e.to_pg_row()


def as_bool_cfg(v) -> bool:
    return v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on")


def _native():
    try:
        from .. import _native as nat
        return nat.load(build_if_missing=False)
    except Exception:  # pragma: no cover - no compiled extension: Python path
        return None


def copy_encode_native(lines: Sequence[str]) -> Optional[Dict[str, Tuple[bytes, int]]]:
    """``_apm_native.copy_encode`` over newline-joined wire lines (None if not built)."""
    N = _native()
    if N is None:
        return None
    return N.copy_encode(("\n".join(lines) + "\n").encode("utf-8"))


def copy_encode_lines(lines: Iterable[str]) -> Dict[str, List[str]]:
    """Python definition of the native ``copy_encode``: wire lines -> COPY rows per type."""
    out: Dict[str, List[str]] = {t: [] for t in TYPES}
    for ln in lines:
        if not ln:
            continue
        r = pg_row_from_line(ln)
        if r is not None:
            out[r[0]].append(copy_row(*r))
    return out


# --------------------------------------------------------------------------- stats

class DBStats:
    """dbstats.js: rows inserted and insert time, logged and reset every interval."""

    def __init__(self, interval_s: float = 60.0):
        self.interval = interval_s
        self.rows = 0
        self.ms = 0.0
        self.total_rows = 0
        self._lock = threading.Lock()

    def add(self, rows: int, ms: float):
        with self._lock:
            self.rows += rows
            self.ms += ms
            self.total_rows += rows

    def line(self) -> str:
        avg = (self.ms / self.rows) if self.rows else float("nan")
        return (f"DBRecordsIns: {self.rows} - TotalInsTime: {self.ms:.1f} ms - "
                f"AvgDBInsTimePerRec: {avg:.3f} ms")

    def log_and_reset(self, logger=log) -> str:
        with self._lock:
            s = self.line()
            self.rows = 0
            self.ms = 0.0
        logger.info(s)
        return s


# --------------------------------------------------------------------------- writers

class Writer:
    """Loads COPY text rows into one table.  ``write`` raises on failure (rows are re-buffered)."""

    def write(self, table: str, columns: Sequence[str], rows: Sequence[str]) -> None:  # pragma: no cover
        raise NotImplementedError

    def close(self) -> None:
        pass


class NullWriter(Writer):
    def __init__(self):
        self.rows = 0

    def write(self, table, columns, rows):
        self.rows += len(rows)


class CopySpoolWriter(Writer):
    """Appends COPY text to ``<dir>/<table>.copy`` (one file per table, rotated by size).

    Load with: ``\\copy <table> (<columns>) FROM '<file>'`` -- a ``<table>.columns`` file next
    to the data holds the column list."""

    def __init__(self, directory: str, rotate_bytes: int = 1 << 30):
        self.dir = directory
        self.rotate = rotate_bytes
        os.makedirs(directory, exist_ok=True)
        self._fh: Dict[str, Any] = {}

    def _file(self, table: str, columns: Sequence[str]):
        fh = self._fh.get(table)
        path = os.path.join(self.dir, f"{table}.copy")
        if fh is not None and fh.tell() >= self.rotate:
            fh.close()
            os.replace(path, os.path.join(self.dir, f"{table}.{int(time.time() * 1000)}.copy"))
            fh = None
        if fh is None:
            with open(os.path.join(self.dir, f"{table}.columns"), "w") as c:
                c.write(",".join(columns) + "\n")
            fh = open(path, "a", encoding="utf-8")
            self._fh[table] = fh
        return fh

    def write(self, table, columns, rows):
        fh = self._file(table, columns)
        fh.write("".join(rows))
        fh.flush()

    def close(self):
        for fh in self._fh.values():
            fh.close()
        self._fh.clear()


class PsqlWriter(Writer):
    """``COPY table (cols) FROM STDIN`` through the psql client (libpq)."""

    def __init__(self, user: str, host: str, database: str, psql: Optional[str] = None):
        self.psql = psql or shutil.which("psql")
        if not self.psql:
            raise RuntimeError("psql not found")
        self.args = [self.psql, "-X", "-q", "-v", "ON_ERROR_STOP=1", "-U", user, "-h", host, "-d", database]

    def write(self, table, columns, rows):
        cmd = self.args + ["-c", f"COPY {table} ({', '.join(columns)}) FROM STDIN"]
        r = subprocess.run(cmd, input="".join(rows).encode("utf-8"), capture_output=True, timeout=120)
        if r.returncode != 0:
            raise RuntimeError(r.stderr.decode(errors="replace").strip())


def native_writer_spec(ins_cfg: Dict[str, Any]) -> Optional[Tuple[str, List[str]]]:
    """(writer kind, args) of the native DbSink for this configuration, mirroring make_writer."""
    mode = ins_cfg.get("sink", "auto")
    if mode == "null":
        return "null", []
    psql = ins_cfg.get("psqlPath") or shutil.which("psql")
    if mode in ("auto", "psql") and psql and ins_cfg.get("dbHost"):
        return "psql", [psql, "-X", "-q", "-v", "ON_ERROR_STOP=0", "-U", ins_cfg.get("dbUser", ""),
                        "-h", ins_cfg["dbHost"], "-d", ins_cfg.get("dbDatabase", ""), "-f", "-"]
    if mode == "psql":
        raise RuntimeError("sink=psql requested but no psql client is installed")
    return "spool", [ins_cfg.get("copySinkDir", "/tmp/apm/copy")]


def make_writer(ins_cfg: Dict[str, Any]) -> Writer:
    mode = ins_cfg.get("sink", "auto")
    if mode == "null":
        return NullWriter()
    if mode in ("auto", "psql") and shutil.which("psql") and ins_cfg.get("dbHost"):
        return PsqlWriter(ins_cfg.get("dbUser", ""), ins_cfg["dbHost"], ins_cfg.get("dbDatabase", ""))
    if mode == "psql":
        raise RuntimeError("sink=psql requested but no psql client is installed")
    return CopySpoolWriter(ins_cfg.get("copySinkDir", "/tmp/apm/copy"))


# --------------------------------------------------------------------------- resume format

def save_resume(path: str, buffers: Dict[str, Deque[Dict[str, Any]]]):
    """util_methods.saveToResumeFile with the Map replacer: {"dataType":"Map","value":[...]}
    (atomic: tmp + rename)."""
    # the reference's four buffers always; the fleet buffer (our addition) only when it holds rows
    doc = {"dataType": "Map", "value": [[t, [_json_row(r) for r in rows]] for t, rows in buffers.items()
                                        if t != "fb" or rows]}
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(tmp, "w") as f:
        json.dump(doc, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def _json_row(r: Any) -> Any:
    if isinstance(r, dict):
        return {k: _json_row(v) for k, v in r.items()}
    if isinstance(r, _dt.datetime):
        return _iso_js(r)
    return r


_TS_COLS = {"endts", "startts", "timestamp", "entrytimestamp", "alerttimestamp"}


def load_resume(path: str) -> Dict[str, List[Dict[str, Any]]]:
    """Reverse of save_resume; accepts the reference's own resume files too."""
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        doc = json.load(f)
    if not (isinstance(doc, dict) and doc.get("dataType") == "Map"):
        return {}
    out = {}
    for t, rows in doc["value"]:
        conv = []
        for r in rows:
            rr = dict(r)
            for k in _TS_COLS & set(rr):
                if isinstance(rr[k], str):
                    rr[k] = _dt.datetime.fromisoformat(rr[k].replace("Z", "+00:00"))
            conv.append(rr)
        out[t] = conv
    return out


# --------------------------------------------------------------------------- inserter

# ---- checkpointed sink snapshots (service.checkpoint / _restore_sink)
def write_sink_snapshot(path: str, jobs) -> None:
    """The sink's unacknowledged flushes [(seq, type index, encoded, rows, bytes)], fsync'd and
    renamed into place (it must be durable before the checkpoint naming it is published)."""
    import struct
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(struct.pack("<8sQ", b"APMSINK1", len(jobs)))
        for seq, ti, enc, rows, data in jobs:
            f.write(struct.pack("<QIBqQ", int(seq), int(ti), 1 if enc else 0, int(rows), len(data)))
            f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def read_sink_ack(path: str, incarnation: int) -> int:
    """The acknowledged watermark the sink of `incarnation` left in its ack file, or -1 when the
    file is missing or belongs to another incarnation (then nothing is known to be written)."""
    import struct
    try:
        with open(path, "rb") as f:
            inc, acked = struct.unpack("<QQ", f.read(16))
    except (OSError, struct.error):
        return -1
    return int(acked) if inc == int(incarnation) else -1


def read_sink_snapshot(path: str, acked: int):
    """(flushes in the snapshot, [the ones at or above `acked`])."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    magic, n = struct.unpack_from("<8sQ", data, 0)
    if magic != b"APMSINK1":
        raise RuntimeError(f"{path}: not a sink snapshot")
    off, jobs = 16, []
    hdr = struct.calcsize("<QIBqQ")
    for _ in range(n):
        seq, ti, enc, rows, ln = struct.unpack_from("<QIBqQ", data, off)
        off += hdr
        if seq >= acked:
            jobs.append((seq, ti, bool(enc), rows, data[off:off + ln]))
        off += ln
    return n, jobs


class DBInserter:
    """The consumer side of ``db_insert`` (one per node, or one per rank).

    With the configured writers (spool / psql / null) the buffering, COPY encoding and loading
    run in the native ``DbSink`` (csrc/runtime/dbsink.cpp: per-type buffers, encoder thread pool,
    one ordered writer thread, a persistent psql process); the Python path below serves custom
    ``Writer`` objects (tests, embedding) and is the reference definition of the semantics."""

    def __init__(self, cfg: Dict[str, Any], writer: Optional[Writer] = None,
                 clock: Callable[[], float] = time.monotonic, stats: Optional[DBStats] = None):
        ic = cfg["streamInsertDb"]
        self.cfg = cfg
        self._limit = int(ic.get("dbInsertBufferLimit", 1000))
        self._max_wait_s = float(ic.get("dbMaxTimeBetweenInsertsMs", 5000)) / 1000.0
        self.tables = {t: ic.get(key, "apm_fleet_stats" if t == "fb" else t) for t, (key, _cols) in COLUMNS.items()}
        self.clock = clock
        self.stats = stats or DBStats(float(cfg.get("statLogIntervalInSeconds", 60)))
        self.buffers: Dict[str, Deque[Dict[str, Any]]] = {t: deque() for t in TYPES}
        self.deadline: Dict[str, Optional[float]] = {t: None for t in TYPES}
        self.failures = 0
        self._stats_synced = 0.0  # monotonic time of the last interval-counter read (tick)
        self.native = bool(ic.get("nativeCopyEncoder", True))
        self.resume_path = ic.get("bufferResumeFileFullPath")
        self.core = None
        self.gpu_fs_copy = as_bool_cfg(ic.get("gpuFsCopyRows", True))
        # released db rows (the transactions table) encoded on the GPU (engine.set_db_copy)
        self.gpu_tx_copy = as_bool_cfg(ic.get("gpuTxCopyRows", True))
        self._writer: Optional[Writer] = writer
        if writer is None:
            N = _native() if as_bool_cfg(ic.get("nativeSink", True)) else None
            if N is not None and hasattr(N, "DbSink"):
                kind, args = native_writer_spec(ic)
                self.core = N.DbSink(self._limit, self._max_wait_s * 1000.0, [self.tables[t] for t in TYPES],
                                     [", ".join(COLUMNS[t][1]) for t in TYPES], kind, args,
                                     int(ic.get("copySinkRotateBytes", 1 << 30)), int(ic.get("encoderThreads", 2)),
                                     int(ic.get("writerLanes", 1)),
                                     float(ic.get("psqlAckTimeoutSeconds", 120)) * 1000.0)
            else:
                self._writer = make_writer(ic)
        if self.resume_path:
            for t, rows in load_resume(self.resume_path).items():
                if t in self.buffers and rows:
                    if self.core is not None:
                        self.core.add_encoded(TYPES.index(t), "".join(copy_row(t, r) for r in rows).encode("utf-8"),
                                              len(rows))
                    else:
                        self.buffers[t].extend(rows)
                        self.deadline[t] = self.clock() + self.max_wait_s

    # -- configuration (hot reload) and writer injection
    @property
    def limit(self) -> int:
        return self._limit

    @limit.setter
    def limit(self, v: int):
        self._limit = int(v)
        if self.core is not None:
            self.core.set_limit(self._limit, self._max_wait_s * 1000.0)

    @property
    def max_wait_s(self) -> float:
        return self._max_wait_s

    @max_wait_s.setter
    def max_wait_s(self, v: float):
        self._max_wait_s = float(v)
        if self.core is not None:
            self.core.set_limit(self._limit, self._max_wait_s * 1000.0)

    @property
    def writer(self) -> Optional[Writer]:
        return self._writer

    def attach_engine(self, native_engine, kinds: Sequence[str]) -> bool:
        """Let the engine's output lane hand ``kinds`` straight to the native sink (no Python,
        no extra copy).  Returns False on the Python path."""
        if self.core is None:
            return False
        N = _native()
        fs_copy = self.gpu_fs_copy and ("fs" in kinds or "fb" in kinds)
        if fs_copy:
            # K12 (fs) and the fleet formatter (fb) write COPY text on the GPU; the sink stores it as is
            native_engine.set_fs_copy(True)
        db_copy = (self.gpu_tx_copy and "db" in kinds and hasattr(native_engine, "set_db_copy")
                   and native_engine.set_db_copy(True))
        for k in kinds:
            if k in ("fs", "fb") and fs_copy:
                N.attach_sink(native_engine, k, self.core, TYPES.index(k))
            elif k == "db" and db_copy:
                N.attach_sink(native_engine, k, self.core, TYPES.index("tx"))
            else:
                N.attach_sink(native_engine, k, self.core)
        self._attached = (native_engine, list(kinds), fs_copy, db_copy)
        return True

    def _detach(self):
        att = getattr(self, "_attached", None)
        if att:
            N = _native()
            for k in att[1]:
                N.detach_sink(att[0], k)
            if att[2]:
                att[0].set_fs_copy(False)
            if att[3]:
                att[0].set_db_copy(False)
            self._attached = None

    @writer.setter
    def writer(self, w: Writer):
        """Injecting a Python writer switches to the Python path (anything the native sink still
        buffers is handed over first)."""
        self._detach()
        if self.core is not None:
            left = self.core.close()
            enc = [self.core.is_encoded(i) for i in range(len(TYPES))]  # (the leftovers' format)
            self.core = None
            for t, blob, e in zip(TYPES, left, enc):
                for ln in blob.decode("utf-8").split("\n"):
                    if ln:
                        self._add(t, pg_row_from_copy(t, ln) if e else ln)
        self._writer = w

    # -- ingest: buffers hold wire lines (encoded in bulk at flush) or row dicts (resumed)
    def _add(self, rtype: str, item):
        buf = self.buffers[rtype]
        if not buf:
            self.deadline[rtype] = self.clock() + self.max_wait_s
        if len(buf) >= self.limit:
            self.flush(rtype)
        buf.append(item)

    def add_row(self, rtype: str, row: Dict[str, Any]):
        self._add(rtype, row)

    def consume_line(self, line: str) -> bool:
        if self.core is not None:
            return self.core.consume((line + "\n").encode("utf-8")) > 0
        t = line[:3]
        if len(line) < 3 or t[2] != "|" or t[:2] not in self.buffers:
            if line:
                log.info("Not a tx, fs, al, or jx: %s", line)
            return False
        self._add(t[:2], line)
        return True

    def consume_bytes(self, blob: bytes) -> int:
        if self.core is not None:
            return self.core.consume(blob)
        n = 0
        for ln in blob.decode("utf-8").split("\n"):
            if ln:
                n += self.consume_line(ln)
        return n

    def _encode(self, rtype: str, batch: List[Any]) -> List[str]:
        rows: List[str] = []
        i = 0
        while i < len(batch):
            if isinstance(batch[i], dict):
                rows.append(copy_row(rtype, batch[i]))
                i += 1
                continue
            j = i
            while j < len(batch) and isinstance(batch[j], str):
                j += 1
            nat = copy_encode_native(batch[i:j]) if self.native else None
            if nat is not None:
                blob, cnt = nat[rtype]
                rows.extend(ln + "\n" for ln in blob.decode("utf-8").split("\n")[:cnt])
            else:
                rows.extend(copy_encode_lines(batch[i:j])[rtype])
            i = j
        return rows

    # -- flushing
    def flush(self, rtype: str) -> int:
        buf = self.buffers[rtype]
        if not buf:
            return 0
        batch = list(buf)
        buf.clear()
        t0 = time.perf_counter()
        try:
            self.writer.write(self.tables[rtype], COLUMNS[rtype][1], self._encode(rtype, batch))
        except Exception as e:  # rows go back to the front, retried on the next flush (:310-320)
            self.failures += 1
            log.error("Error during insert attempt: %s", e)
            buf.extendleft(reversed(batch))
            return 0
        self.stats.add(len(batch), (time.perf_counter() - t0) * 1000.0)
        return len(batch)

    def tick(self) -> int:
        """Timer half of the reference's setTimeout per buffer."""
        if self.core is not None:
            # the interval counters are for the stat lines: read them at most every 50 ms (each
            # read takes the sink's lock, contended by its writer lanes while a backlog drains)
            t = time.monotonic()
            if t - self._stats_synced >= 0.05:
                self._stats_synced = t
                self._sync_stats()
            return self.core.tick()
        now = self.clock()
        n = 0
        for t in TYPES:
            d = self.deadline[t]
            if d is not None and now >= d:
                self.deadline[t] = None
                n += self.flush(t)
                if self.buffers[t]:
                    self.deadline[t] = now + self.max_wait_s
        return n

    def flush_all(self) -> int:
        if self.core is not None:
            before = self.core.stats()["rows"]
            self.core.flush_all()
            self.core.drain()
            self._sync_stats()
            return self.core.stats()["rows"] - before
        return sum(self.flush(t) for t in TYPES)

    # -- checkpoint support (service.checkpoint): the acknowledged watermark instead of a drain
    def set_ack_file(self, path: str, incarnation: int):
        if self.core is not None:
            self.core.set_ack_file(path, int(incarnation))

    def snapshot_pending(self):
        """(acked watermark, [(seq, type index, encoded, rows, bytes)]) of every row consumed
        but not yet written -- taken without waiting for a writer (native sink)."""
        if self.core is not None:
            acked, jobs = self.core.snapshot_pending()
            return int(acked), [tuple(j) for j in jobs]
        # the Python path (custom writers) has no acknowledgement watermark: it writes its buffers
        # out synchronously instead, so nothing is pending
        self.flush_all()
        return 0, []

    def resubmit(self, jobs) -> int:
        """Queue flushes taken from a checkpoint's snapshot again (restore after a crash)."""
        n = 0
        for _seq, ti, encoded, rows, data in jobs:
            t = TYPES[int(ti)]
            if self.core is not None:
                if encoded:
                    self.core.add_encoded(int(ti), data, int(rows))
                else:
                    self.core.consume(data)
            else:
                for ln in data.decode("utf-8").split("\n"):
                    if ln:
                        self._add(t, pg_row_from_copy(t, ln) if encoded else ln)
            n += int(rows)
        return n

    def _sync_stats(self):
        rows, ms = self.core.take_interval()
        if rows or ms:
            self.stats.add(rows, ms)
        self.failures = self.core.stats()["failures"]

    def sink_stats(self) -> Dict[str, Any]:
        return dict(self.core.stats()) if self.core is not None else {"rows": self.stats.total_rows,
                                                                      "failures": self.failures}

    def close(self):
        self._detach()
        if self.core is not None:
            left = self.core.close()
            enc = [self.core.is_encoded(i) for i in range(len(TYPES))]  # (the leftovers' format)
            self._sync_stats()
            self.core = None
            for t, blob, e in zip(TYPES, left, enc):
                self.buffers[t].extend((pg_row_from_copy(t, ln) if e else ln)
                                       for ln in blob.decode("utf-8").split("\n") if ln)
        else:
            self.flush_all()
        if self.resume_path:
            rows = {t: [r if isinstance(r, dict) else pg_row_from_line(r)[1] for r in b] for t, b in self.buffers.items()}
            save_resume(self.resume_path, rows)
        if self._writer is not None:
            self._writer.close()
