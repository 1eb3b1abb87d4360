"""The per-GPU ingest service: tail -> engine -> sinks, the runnable form of the reference's five
stage processes (stream_parse_transactions.js, stream_calc_stats.js, stream_calc_z_score.js,
stream_process_alerts.js feeding stream_insert_db.js).

One process per GPU (``torchrun`` / the supervisor set RANK, WORLD_SIZE, LOCAL_RANK):

* **files** -- ``glob(appLogDirMaskPrefix/<maskSuffix>)`` (stream_parse_transactions.js:816-825),
  server = the host path component; the JVM hosts are sharded over ranks
  (parallel/dist.shard_servers) so every join and every series is rank-local;
* **tailing** -- the native Tailer (pause-file contract of perl_tail.pl:36-41, persisted
  offsets, rotation);
* **engine** -- APMEngine (GPU) -- or, only when asked for, the CPU oracle adapter used by tests;
* **outputs** -- ``gpu.outputMode``: ``inproc`` feeds the DB insert stage in this process
  (runtime/sinks.DBInserter, COPY); ``amqp`` publishes the reference's queue contract
  (``db_insert`` gets tx/fs/al like stream_process_alerts.js:618 forwards them; optional
  ``bridgeQueues`` also mirror ``transactions``/``stats``/``z_score``) through runtime/queue.py;
  alert lines also go to the e-mail notifier (runtime/notifier.py);
* **checkpoint** -- every ``gpu.checkpointEverySeconds`` and on SIGTERM/SIGINT: the binary
  engine checkpoint + tail offsets, written atomically; restored at start-up (the reference's
  resume files, SURVEY §5.4, but covering the parser too);
* **hot reload** -- ConfigWatcher: thresholds/overrides re-applied to live series, logger
  re-pointed, notifier and sink limits updated; restart-only keys warn;
* **control** -- SIGUSR1 = ``requestGC`` (util_methods.js:463-467): Python gc + malloc_trim +
  memory report; fleet baseline exchange over RCCL when WORLD_SIZE > 1.
"""
from __future__ import annotations

import ctypes
import gc
import glob
import json
import logging
import math
import os
import signal
import sys
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from ..models.oracle import file_kind, server_of
from ..models.pipeline import DB_OUTPUTS, KIND_CODE, OUT_KINDS, APMEngine
from ..parallel.dist import dist_env, shard_servers
from ..utils.config import ConfigWatcher, as_bool, read_apm_config
from . import logger as apmlog
from .notifier import AlertNotifier
from .sinks import DBInserter


# Exit status of a rank that stops because a PEER rank failed (its collectives aborted): the
# supervisor does not count it against this rank's GPU (runtime/supervisor.py).
PEER_FAILURE_EXIT = 75


def is_peer_failure(e: BaseException) -> bool:
    m = str(e)
    return ("peer process gone" in m or "peer rank dead" in m or "communicator was aborted" in m
            or ("collective" in m and "failed" in m and "peer" in m))


def _native_mod():
    """The native extension if it is built (the sink snapshot path needs it), else None."""
    try:
        from .. import _native
        return _native.load(build_if_missing=False)
    except Exception:  # noqa: BLE001 - CPU containers without the .so
        return None

log = logging.getLogger("apm.service")

RESTART_KEYS = ["apmConfigFilePath", "amqpConnectionString", "streamParseTransactions.appLogDirMaskPrefix",
                "streamParseTransactions.maskSuffixes", "streamCalcStats.intervalLengthInSeconds",
                "streamCalcStats.windowSizeInIntervals", "streamCalcStats.bufferSizeInIntervals",
                "gpu.maxSeries", "gpu.ringDtype", "gpu.zscoreMeanMode", "gpu.outputMode"]


def read_json(path: str) -> Dict[str, Any]:
    with open(path) as f:
        return json.load(f)


def write_json_atomic(path: str, obj: Any):
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "w") as f:
        json.dump(obj, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)


def discover_files(cfg: Dict[str, Any]) -> List[str]:
    pc = cfg["streamParseTransactions"]
    prefix = pc.get("appLogDirMaskPrefix", "")
    out = []
    for suf in pc.get("maskSuffixes", []):
        out += glob.glob(os.path.join(prefix, suf))
    return sorted(set(out))


_STAGE_KEYS = ("t_parse_ms", "t_join_ms", "t_stats_ms", "t_out_ms")


def _percentiles(xs, qs):
    """Nearest-rank percentiles of xs ('-' when empty), formatted with 1 decimal."""
    if not xs:
        return ["-"] * len(qs)
    v = sorted(xs)
    return ["%.1f" % v[min(len(v) - 1, max(0, math.ceil(q / 100.0 * len(v)) - 1))] for q in qs]


class IngestService:
    def __init__(self, cfg: Optional[Dict[str, Any]] = None, config_path: Optional[str] = None,
                 engine: str = "native", files: Optional[Sequence[str]] = None, rank: Optional[int] = None,
                 world: Optional[int] = None, clock: Callable[[], float] = time.time, install_signals: bool = False,
                 server_of_path: Callable[[str], str] = server_of, trace_path: Optional[str] = None):
        self.cfg = cfg if cfg is not None else read_apm_config(config_path, first_run=True)
        self.trace_path = trace_path or self.cfg.get("gpu", {}).get("tracePath") or None
        g = self.cfg.setdefault("gpu", {})
        r, w, local = dist_env()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.local_rank = local
        self.clock = clock
        self.server_of = server_of_path
        apmlog.set_global_logger(self.cfg.get("logDir"), self._log_prefix(), colorize=True)
        self.mode = g.get("outputMode", "inproc")
        self.bridge = list(g.get("bridgeQueues", []))
        # inputMode "transactions": a reference parser stage (stream_parse_transactions.js) keeps
        # tailing and publishing `transactions`; this engine consumes them and takes over stats,
        # z-score, alerts and the DB hand-off (mixed deployment / staged cut-over)
        self.input_mode = g.get("inputMode", "logs")
        if self.input_mode == "transactions":
            if engine != "native":
                raise ValueError("inputMode=transactions needs the native engine")
            g["joinOnDevice"] = False  # tx arrive joined: the host stats path takes them

        # ---- files -> this rank's shard
        all_files = list(files) if files is not None else discover_files(self.cfg)
        servers = sorted({self.server_of(f) for f in all_files})
        self.all_servers = servers
        mine = set(shard_servers(servers, self.world)[self.rank]) if servers else set()
        self.my_servers = sorted(mine)
        self.files = [f for f in all_files if self.server_of(f) in mine]
        log.info("rank %d/%d: %d of %d files, servers %s", self.rank, self.world, len(self.files), len(all_files),
                 sorted(mine))

        # ---- engine
        outs = set(DB_OUTPUTS)
        if as_bool(g.get("serverRollup", False)):  # K14 per-JVM rollup fused with JMX gauges
            outs.add("sx")
        if self.world > 1 and engine == "native" and as_bool(g.get("fleetBaseline", True)) \
                and as_bool(g.get("fleetBaselineRows", True)):
            outs.add("fb")  # fleet-merged per-service baselines (rank 0 emits them)
        if self.mode == "amqp":
            outs |= {"transactions" if "transactions" in self.bridge else "", "st" if "stats" in self.bridge else ""}
            outs.discard("")
        self.outputs = [k for k in OUT_KINDS if k in outs]
        self.outs_set = set(self.outputs)
        if self.mode == "amqp" and "z_score" in self.bridge:
            self.outputs = [k for k in OUT_KINDS if k in set(self.outputs) | {"fs"}]
        if engine == "native":
            self.eng = APMEngine(self.cfg, device=self.local_rank, outputs=self.outputs)
            self.native = self.eng.eng
            if self.trace_path:
                self.native.set_trace(True)
        elif engine == "cpu-oracle":
            from ..models.cpu_engine import CpuOracleEngine
            self.eng = None
            self.native = CpuOracleEngine(self.cfg)
        else:
            raise ValueError(f"unknown engine {engine!r}")

        # ---- checkpoint restore (before files are registered: load_state re-registers them)
        self.ckpt_dir = g.get("checkpointDir")
        self.n_checkpoints = 0
        # sink snapshot named by the last checkpoint known to be committed (in the chain
        # manifest), and (name, writer completions before it) of the last one started
        self._sink_committed: Optional[str] = None
        self._ck_started: Optional[Tuple[str, int]] = None
        self.ckpt_every = float(g.get("checkpointEverySeconds",
                                      self.cfg["streamCalcStats"].get("resumeFileSaveFrequencyInSeconds", 60)))
        self.resharded = False
        self._ckpt_epoch: Optional[int] = None
        self._merge_sinks: List[Tuple[int, Dict[str, Any]]] = []
        self.reshard_info: Optional[Dict[str, Any]] = None
        self._ckpt_extra = b""
        restored = self._restore() if (self.ckpt_dir and engine == "native") else False
        if not restored:
            if engine == "native" and as_bool(g.get("importReferenceResume", False)):
                self._import_reference(mine)
            for f in self.files:
                self.native.add_file(f, KIND_CODE[file_kind(f)], self.server_of(f))
        self.file_ids = {p: i for i, (p, _k, _s) in enumerate(self.native.files())}

        # ---- tailer
        from .. import _native
        N = _native.load(build_if_missing=False)
        pc = self.cfg["streamParseTransactions"]
        self.pause_file = pc.get("tailPauseFileFullPath", "")
        self.batch_bytes = int(g.get("batchBytes", 32 << 20))
        self.tailer = N.Tailer(self.pause_file, self.batch_bytes, int(g.get("tailReadThreads", 3)))
        from_start = as_bool(g.get("tailFromStart", False))
        # batches are laid out grouped by the engine's server order: the engine's canonical
        # (zero-copy) batch layout
        srv_order: Dict[str, int] = {}
        if hasattr(self.native, "servers"):
            srv_order = {name: i for i, name in enumerate(self.native.servers())}
        for p, fid in sorted(self.file_ids.items(), key=lambda kv: kv[1]):
            grp = srv_order.setdefault(self.server_of(p), len(srv_order))
            self.tailer.add(p, fid, from_start, grp)
        self.offsets_path = pc.get("tailOffsetFileFullPath")
        if self.offsets_path:
            os.makedirs(os.path.dirname(os.path.abspath(self.offsets_path)), exist_ok=True)
        if restored:
            self._restore_offsets()
        elif self.resharded:
            self._restore_offsets_resharded()
        # read-ahead into pinned slots (native engine): the tailer fills the next slot while the
        # engine works on the current one, and the engine prefetches (H2D + parse) the batch after
        self.readahead = engine == "native" and as_bool(g.get("tailReadAhead", True)) and self.input_mode == "logs"
        self._slots: List[int] = []
        self._held = None  # batch taken from the read-ahead ring and handed to the engine as prefetch
        self._stopping = False
        self.perf = {"wait_s": 0.0, "engine_s": 0.0, "outputs_s": 0.0, "batches": 0, "bytes": 0, "prefetched": 0,
                     "ckpt_s": 0.0, "ckpt_flush_s": 0.0, "ckpt_sink_snapshot_s": 0.0,
                     "hk_ticks_s": 0.0, "hk_watch_s": 0.0, "hk_ckpt_s": 0.0, "hk_stats_s": 0.0,
                     "next_s": 0.0, "commit_s": 0.0,
                     "hk_jmx_s": 0.0, "hk_sink_s": 0.0}
        self.batch_log = None  # a list to record every read-ahead batch (bytes, chunks) in (tests)
        self._drain_every_s = float(g.get("outputDrainMs", 250.0)) / 1000.0
        self._last_drain = 0.0
        if self.readahead:
            self._slot_bytes = self.batch_bytes
            self._slots = [N.alloc_pinned(self._slot_bytes + 256) for _ in range(int(g.get("tailReadAheadSlots", 3)))]
            self.tailer.start(self._slots, self._slot_bytes, float(g.get("tailIdleMs", 50.0)))

        # ---- outputs
        self.inserter: Optional[DBInserter] = None
        self.qm = None
        self.producers: Dict[str, Any] = {}
        if self.mode == "inproc":
            self.inserter = DBInserter(self.cfg)
            self._sink_incarnation = int.from_bytes(os.urandom(8), "little") >> 1
            self.sink_pending_rows = 0
            if self.ckpt_dir:
                os.makedirs(self.ckpt_dir, exist_ok=True)
                if restored:
                    self._restore_sink()  # (reads the previous incarnation's ack file first)
                    for r, meta in self._merge_sinks:  # re-shard: the old ranks' pending rows
                        self._restore_sink(meta, r)
                self.inserter.set_ack_file(self._sink_ack_path(), self._sink_incarnation)
            if engine == "native":
                # db / audit / fs go engine output lane -> native sink directly; al stays on the
                # Python side (the e-mail notifier reads it too)
                self.inserter.attach_engine(self.native, [k for k in self.outputs
                                                          if (k in DB_OUTPUTS and k != "al") or k == "fb"])
        elif self.mode == "amqp":
            from .queue import QueueManager
            self.qm = QueueManager(self.cfg["amqpConnectionString"], self.cfg.get("statLogIntervalInSeconds", 60),
                                   confirms=as_bool(g.get("publisherConfirms", True)),
                                   persistent=as_bool(g.get("persistentMessages", True)))
            self.producers["db"] = self.qm.get_queue(self.cfg.get("dbInsertQueue", "db_insert"), "p")
            qmap = {"transactions": self.cfg["streamParseTransactions"].get("outQueue", "transactions"),
                    "stats": self.cfg["streamCalcStats"].get("outQueue", "stats"),
                    "z_score": self.cfg["streamCalcZScore"].get("outQueue", "z_score")}
            for q in self.bridge:
                if q in qmap:
                    self.producers[q] = self.qm.get_queue(qmap[q], "p")
            if "fb" in self.outs_set:  # not a db_insert record type of the reference: own queue
                self.producers["fleet"] = self.qm.get_queue(g.get("fleetQueue", "fleet_baseline"), "p")
            self.qm.on("pause", lambda: log.info("queue backpressure: pausing ingest"))
        elif self.mode != "none":
            raise ValueError(f"unknown gpu.outputMode {self.mode!r}")
        self.notifier = AlertNotifier(self.cfg, clock=clock) if self.rank == 0 or self.world == 1 else None
        if self.notifier is not None:  # the alerts module's startup probe (stream_process_alerts.js:597)
            import threading
            threading.Thread(target=self.notifier.send_test_email, name="apm-test-email", daemon=True).start()

        # ---- input queue (inputMode transactions)
        self.in_qm = None
        self._in_lines: List[bytes] = []
        if self.input_mode == "transactions":
            import threading
            from .queue import QueueManager as _QM
            self._in_lock = threading.Lock()
            self.in_qm = self.qm if self.qm is not None else _QM(self.cfg["amqpConnectionString"],
                                                                 self.cfg.get("statLogIntervalInSeconds", 60))
            inq = self.cfg["streamCalcStats"].get("inQueue", "transactions")
            self.in_queue = self.in_qm.get_queue(inq, "c", self._on_tx_message)
            self.in_queue.start_consume()

        # ---- fleet exchange
        self.fleet = None
        # (gpu.fleetSingleRank: the exchange also at world 1 -- the same per-rank work as each rank
        # of a node, as the headline bench runs it)
        if (self.world > 1 or as_bool(g.get("fleetSingleRank", False))) and engine == "native" \
                and as_bool(g.get("fleetBaseline", True)):
            from ..parallel.fleet import FleetBaseline
            self.fleet = FleetBaseline(self.eng, self.world, self.rank, servers=self.all_servers)

        # ---- in-process JMX poller (config 4: JMX gauges fused into the per-JVM rollup)
        self.jmx = None
        if as_bool(g.get("fuseJmx", False)) and self.cfg.get("pullJvmStats", {}).get("jvmHosts"):
            from .jmx import JvmStatsPoller, SyntheticJmx, run_cli
            runner = SyntheticJmx().runner if as_bool(g.get("syntheticJmx", False)) else run_cli
            self.jmx = JvmStatsPoller(self.cfg, self._on_jx, runner=runner, clock=clock)

        self.watcher = ConfigWatcher(self.cfg, self.reload, RESTART_KEYS) if self.cfg.get("apmConfigFilePath") else None
        self._config_paused = self._consume_paused(self.cfg)
        self._stop = False
        self._gc_requested = False
        self.batches = 0
        self.polls = 0
        # fault injection: {"rank", "dropBatchEvery", "duplicateBatchEvery",
        # "exitAtBatch", "exitCode"} -- exercises restarts, checkpoint resume and data loss paths
        self.fault = dict(g.get("faultInjection") or {})
        self.faults = {"dropped": 0, "duplicated": 0}
        self.last_ckpt = clock()
        self.last_stat = clock()
        self._m0 = self._metrics()
        self._m0_prev = dict(self._m0)
        if install_signals:
            signal.signal(signal.SIGTERM, self._on_signal)
            signal.signal(signal.SIGINT, self._on_signal)
            signal.signal(signal.SIGUSR1, lambda *a: setattr(self, "_gc_requested", True))

    # ------------------------------------------------------------------ helpers
    def _log_prefix(self) -> str:
        base = self.cfg.get("gpu", {}).get("logFilePrefix", "apm_engine")
        return f"{base}.rank{self.rank}" if self.world > 1 else base

    def _ckpt_paths(self):
        return (os.path.join(self.ckpt_dir, f"engine.rank{self.rank}.ckpt"),
                os.path.join(self.ckpt_dir, f"tail.rank{self.rank}.json"))

    def _meta_path(self, rank: Optional[int] = None) -> str:
        return os.path.join(self.ckpt_dir, f"meta.rank{self.rank if rank is None else rank}.json")

    def _checkpoint_is_mine(self) -> bool:
        """A rank's checkpoint is reused only if it was written for the same world size and
        server shard, and is not stale relative to the other ranks' (a rank of an older, larger
        world whose files survived a degrade).  Checkpoints without metadata predate it: mine."""
        mp = self._meta_path()
        if not os.path.exists(mp):
            return True
        meta = read_json(mp)
        if meta.get("world") != self.world or sorted(meta.get("servers", [])) != self.my_servers:
            log.warning("checkpoint of rank %d was written for world %s (servers %s); this rank now owns %s "
                        "in world %d: re-sharded start", self.rank, meta.get("world"), meta.get("servers"),
                        self.my_servers, self.world)
            return False
        newest = max((read_json(q).get("ts", 0.0) for q in glob.glob(os.path.join(self.ckpt_dir, "meta.rank*.json"))),
                     default=0.0)
        if newest - float(meta.get("ts", 0.0)) > 2 * self.ckpt_every + 60:
            log.warning("checkpoint of rank %d is %.0f s older than the newest rank checkpoint: re-sharded start",
                        self.rank, newest - float(meta.get("ts", 0.0)))
            return False
        return True

    def _chain_batches(self, rank: int) -> Dict[int, str]:
        """batch -> chain manifest of rank `rank` that holds a checkpoint at that batch, over its
        current and its previous chain (engine.rank<r>.ckpt / .prev.ckpt, checkpoint.cpp
        finish_chain)."""
        N = _native_mod()
        out: Dict[int, str] = {}
        for name in (f"engine.rank{rank}.prev.ckpt", f"engine.rank{rank}.ckpt"):
            p = os.path.join(self.ckpt_dir, name)
            if not os.path.exists(p):
                continue
            try:
                for b, f in N.checkpoint_batches(p):
                    if os.path.exists(f):
                        out[int(b)] = p
            except Exception as e:  # an unreadable chain: that rank offers no batch from it
                log.warning("checkpoint chain %s unreadable: %s", p, e)
        return out

    def _node_common_batch(self, ranks) -> Tuple[int, Dict[int, str]]:
        """The newest batch every one of `ranks` holds a checkpoint at (lock-step ranks checkpoint
        at the same batches), and per rank the manifest holding it; (0, {}) when there is none.
        Computed from the files alone, so every rank of the node arrives at the same batch."""
        per = {r: self._chain_batches(r) for r in ranks}
        common = set.intersection(*(set(v) for v in per.values())) if per else set()
        if not common:
            return 0, {}
        b = max(common)
        return b, {r: per[r][b] for r in ranks}

    def _load_at(self, manifest: str, batch: int) -> bytes:
        """load_state of `manifest`'s chain prefix that ends at `batch` (a truncated manifest next
        to the original: the files are shared)."""
        N = _native_mod()
        files = [f for b, f in N.checkpoint_batches(manifest)]
        bs = [int(b) for b, f in N.checkpoint_batches(manifest)]
        if bs and bs[-1] == batch:
            return self.eng.load_state(manifest)
        k = bs.index(batch)
        keep = [os.path.basename(x) for x in files[:k + 1]]
        tmp = os.path.join(self.ckpt_dir, f".restore.rank{self.rank}.{os.getpid()}.ckpt")
        with open(tmp, "w") as f:
            f.write("APMCHAIN 1\n" + "".join(x + "\n" for x in keep))
        try:
            extra = self.eng.load_state(tmp)
        except Exception:
            os.remove(tmp)
            raise
        # the timeline continues from `batch`: this rank's checkpoints after it are void (their
        # batch numbers will be reused) -- the prefix becomes the current chain, the rest goes
        cur = os.path.join(self.ckpt_dir, f"engine.rank{self.rank}.ckpt")
        prev = os.path.join(self.ckpt_dir, f"engine.rank{self.rank}.prev.ckpt")
        void = [os.path.basename(x) for x in files[k + 1:]]
        if os.path.abspath(manifest) == os.path.abspath(prev) and os.path.exists(cur):
            void += [os.path.basename(f) for _b, f in N.checkpoint_batches(cur)]
            os.remove(prev)
        os.replace(tmp, cur)
        for name in set(void) - set(keep):
            try:
                os.remove(os.path.join(self.ckpt_dir, name))
            except OSError:
                pass
        log.warning("rank %d resumed at batch %d, the newest batch every rank holds: its %d later checkpoint "
                    "file(s) were dropped", self.rank, batch, len(set(void) - set(keep)))
        return extra

    def _restore(self) -> bool:
        ck, _ = self._ckpt_paths()
        if not os.path.exists(ck) and not glob.glob(os.path.join(self.ckpt_dir, "tail.rank*.json")):
            return False
        if not os.path.exists(ck) or not self._checkpoint_is_mine():
            # world size changed (elastic degrade / grow): this rank's state is merged from the
            # previous world's checkpoints of the servers it now owns (merge.cpp); only when they
            # are missing / unreadable does the shard start fresh, with tails resumed from
            # whichever rank owned each file last (_restore_offsets_resharded)
            try:
                if self._restore_merged():
                    return True
            except Exception as e:
                log.error("re-shard merge failed (%s): this shard starts with fresh engine state", e)
            self.resharded = True
            return False
        try:
            # lock-step ranks resume at the newest batch EVERY rank holds (a rank that died while
            # the others checkpointed has an older newest file): same batch, same clocks everywhere
            at, where = (0, {})
            if self.world > 1:
                at, where = self._node_common_batch(range(self.world))
            if at and where.get(self.rank):
                self._ckpt_extra = self._load_at(where[self.rank], at)
                log.info("resumed engine state from %s at batch %d (newest batch of every rank)", where[self.rank], at)
            else:
                self._ckpt_extra = self.eng.load_state(ck)
                log.info("resumed engine state from %s", ck)
            known = {p for p, _k, _s in self.native.files()}
            for f in self.files:  # files that appeared since the checkpoint
                if f not in known:
                    self.native.add_file(f, KIND_CODE[file_kind(f)], self.server_of(f))
            return True
        except Exception as e:
            if "unsupported version" not in str(e):
                log.error("checkpoint %s could not be loaded (%s); refusing to start (move it aside to "
                          "start fresh)", ck, e)
                raise
            # written by an older / newer build (incompatible section layout): keep it for
            # inspection and start this shard fresh instead of crash-looping under the supervisor
            stamp = time.strftime("%Y%m%d%H%M%S")
            moved = []
            for f in [ck] + glob.glob(ck[:-len(".ckpt")] + ".*.ckpt" if ck.endswith(".ckpt") else ck + ".*"):
                if os.path.exists(f):
                    os.replace(f, f"{f}.incompatible-{stamp}")
                    moved.append(os.path.basename(f))
            log.warning("checkpoint %s has an incompatible format version (%s): moved %s aside, starting this "
                        "shard with fresh engine state", ck, e, ", ".join(moved))
            return False

    def _restore_merged(self) -> bool:
        """Elastic re-shard: the previous world's rank checkpoints that hold any of this rank's
        servers are merged at their newest common batch into this rank's starting state -- window
        buckets, z-score rings and moments, alert counters, join caches and parked records, pending
        release lines of exactly these servers (the reference resumes every per-series history
        from its resume files, stream_calc_stats.js:54-87, stream_calc_z_score.js:37-64,
        stream_process_alerts.js:111-142).  Tail offsets come from the same checkpoints."""
        g = self.cfg.get("gpu", {})
        if not as_bool(g.get("reshardMerge", True)):
            return False
        metas = []
        for p in glob.glob(os.path.join(self.ckpt_dir, "meta.rank*.json")):
            try:
                m = read_json(p)
                m["_rank"] = int(os.path.basename(p)[len("meta.rank"):-len(".json")])
                metas.append(m)
            except (OSError, ValueError):
                continue
        prev = [m for m in metas if m.get("world") != self.world]
        if not prev:
            return False
        old_world = max(prev, key=lambda m: float(m.get("ts", 0.0)))["world"]
        old = {m["_rank"]: m for m in prev if m.get("world") == old_world}
        mine = set(self.my_servers)
        inputs = [r for r in sorted(old) if mine & set(old[r].get("servers", []))]
        held = set().union(*(set(old[r].get("servers", [])) for r in inputs)) if inputs else set()
        if not inputs or len(old) != old_world:
            log.warning("re-shard: %d of %d rank checkpoints of world %s found; servers %s start fresh",
                        len(old), old_world, old_world, sorted(mine))
            return False
        paths = [os.path.join(self.ckpt_dir, f"engine.rank{r}.ckpt") for r in inputs]
        missing = [p for p in paths if not os.path.exists(p)]
        if missing:
            log.warning("re-shard: checkpoints %s missing: this shard starts fresh", missing)
            return False
        N = _native_mod()
        # one restore batch for the whole node: the newest batch EVERY old rank holds (not only the
        # inputs of this rank -- two new ranks must start from the same batch, clocks and bucket
        # slots), taken from each old rank's current or previous chain
        at, where = self._node_common_batch(sorted(old))
        if not at:
            log.warning("re-shard: the old ranks' checkpoints share no batch: servers %s start fresh", sorted(mine))
            return False
        paths = [where[r] for r in inputs]
        out = os.path.join(self.ckpt_dir, f"engine.rank{self.rank}.resharded.{os.getpid()}.ckpt")
        t0 = time.perf_counter()
        info = N.merge_checkpoints(paths, sorted(mine), out, b"", at)
        try:
            self.eng.load_state(out)
        finally:
            try:
                os.remove(out)
            except OSError:
                pass
        tails: Dict[str, Any] = {}
        for r, ex in zip(inputs, info["extras"]):
            try:
                doc = json.loads(bytes(ex).decode("utf-8")) if ex else {}
            except (ValueError, UnicodeDecodeError):
                doc = {}
            for path, v in (doc.get("tail") or {}).items():
                if self.server_of(path) in mine:
                    tails[path] = v
            # an old rank's unacknowledged DB rows are re-submitted once: by the new owner of its
            # first server
            srv0 = sorted(old[r].get("servers", []))[:1]
            if doc.get("sink") and srv0 and srv0[0] in mine:
                self._merge_sinks.append((r, doc["sink"]))
        self._ckpt_extra = json.dumps({"tail": tails}).encode("utf-8")
        known = {p for p, _k, _s in self.native.files()}
        for f in self.files:
            if f not in known:
                self.native.add_file(f, KIND_CODE[file_kind(f)], self.server_of(f))
        self.reshard_info = {k: info[k] for k in ("batch_no", "series", "keys", "need", "pending", "raw", "files",
                                                 "servers")}
        self.reshard_info.update({"from_world": old_world, "from_ranks": inputs,
                                  "seconds": round(time.perf_counter() - t0, 3)})
        log.warning("re-sharded start: world %s -> %d, rank %d merged ranks %s at batch %d: %d series, %d join "
                    "keys, %d parked records, %d pending lines (servers %s; %s held by the inputs)", old_world,
                    self.world, self.rank, inputs, info["batch_no"], info["series"], info["keys"], info["need"],
                    info["pending"], sorted(mine), "all" if mine <= held else sorted(mine & held))
        return True

    # ------------------------------------------------------------------ sink watermark
    def _sink_ack_path(self) -> str:
        return os.path.join(self.ckpt_dir, f"sink.rank{self.rank}.ack")

    def _snapshot_sink(self) -> Optional[Dict[str, Any]]:
        """The DB sink's unacknowledged flushes -> <ckdir>/sink_pending.rank<r>.<n>.bin (fsync +
        rename before the engine checkpoint that names it is published)."""
        from .sinks import write_sink_snapshot
        acked, jobs = self.inserter.snapshot_pending()
        name = self._sink_snapshot_name()
        write_sink_snapshot(os.path.join(self.ckpt_dir, name), jobs)
        self._prune_sink_snapshots(name)
        self.sink_pending_rows = sum(int(j[3]) for j in jobs)
        return {"incarnation": self._sink_incarnation, "acked": acked, "pending": name, "jobs": len(jobs),
                "rows": self.sink_pending_rows}

    def _note_checkpoint_outcome(self):
        """The checkpoint started last has finished (the writer is idle): if the writer completed
        it, its sink snapshot is now the one the chain manifest names.  A failed write leaves the
        manifest -- and the snapshot it names -- at the checkpoint before."""
        if self._ck_started is None or self.eng is None:
            return
        ci = getattr(self.eng, "checkpoint_info", None)
        info = ci() if ci is not None else {}
        if info.get("busy"):
            return
        name, done_before = self._ck_started
        if int(info.get("done", done_before + 1)) > done_before:
            self._sink_committed = name
        else:
            log.warning("checkpoint with sink snapshot %s was not committed: keeping %s", name,
                        self._sink_committed)
        self._ck_started = None

    def _prune_sink_snapshots(self, keep: str):
        """Removes this rank's sink snapshots except `keep` (the checkpoint being written) and the
        one the committed checkpoint names (a restore before `keep` commits needs it).  Pruning
        follows commits, not starts: a checkpoint whose write failed never retires its
        predecessor's snapshot (checkpoint() notes the previous one's outcome first)."""
        keep_set = {keep, self._sink_committed}
        for old in glob.glob(os.path.join(self.ckpt_dir, f"sink_pending.rank{self.rank}.*.bin")):
            if os.path.basename(old) in keep_set:
                continue
            try:
                os.remove(old)
            except OSError:
                pass

    def _sink_snapshot_name(self) -> str:
        return f"sink_pending.rank{self.rank}.{self._sink_incarnation:x}.{self.n_checkpoints + 1}.bin"

    def _restore_sink(self, meta: Optional[Dict[str, Any]] = None, ack_rank: Optional[int] = None):
        """After a restore: re-submit the checkpoint's pending flushes that the sink did not
        acknowledge before the process ended (its ack file; a different incarnation in the file --
        an interrupted earlier restore -- means nothing is known: everything is re-submitted, at
        least once)."""
        from .sinks import read_sink_ack, read_sink_snapshot
        if meta is None:
            try:
                meta = json.loads(self._ckpt_extra.decode("utf-8")).get("sink") if self._ckpt_extra else None
            except (ValueError, AttributeError):
                meta = None
        if not meta:
            return 0
        if ack_rank is None:
            self._sink_committed = meta["pending"]  # named by the restored chain: kept until a newer commit
        path = os.path.join(self.ckpt_dir, meta["pending"])
        if not os.path.exists(path):
            log.warning("checkpoint names sink snapshot %s, which is missing: its rows are lost", path)
            return 0
        ack = self._sink_ack_path() if ack_rank is None else os.path.join(self.ckpt_dir, f"sink.rank{ack_rank}.ack")
        acked_now = read_sink_ack(ack, int(meta["incarnation"]))
        n, jobs = read_sink_snapshot(path, acked_now)
        rows = self.inserter.resubmit(jobs)
        log.info("sink: re-submitted %d flushes (%d rows) of the checkpoint's %d unacknowledged ones", len(jobs),
                 rows, n)
        return rows

    def _import_reference(self, servers):
        """Cut-over from a running reference deployment: seed stats buckets, the release heap,
        the z-score histories and alert cooldowns from its JSON resume files."""
        from .resume_compat import import_reference_resume, read_docs
        paths = [self.cfg["streamCalcStats"].get("resumeFileFullPath"),
                 self.cfg["streamCalcZScore"].get("resumeFileFullPath"),
                 self.cfg["streamProcessAlerts"].get("alertsResumeFileFullPath")]
        stats, zscore, alerts = read_docs(paths)
        if not (stats or zscore or alerts):
            return
        info = import_reference_resume(self.eng, stats, zscore, alerts, servers=set(servers))
        log.info("imported reference resume files: %s", info)

    def _restore_offsets(self):
        # the offsets stored inside the engine checkpoint belong to exactly that state (one
        # atomic file); the separate tail file is only a fallback for older checkpoints
        offs = None
        if self._ckpt_extra:
            try:
                offs = json.loads(self._ckpt_extra.decode("utf-8")).get("tail")
            except (ValueError, UnicodeDecodeError):
                offs = None
        if offs is None:
            _, tp = self._ckpt_paths()
            if not os.path.exists(tp):
                return
            with open(tp) as f:
                offs = json.load(f)
        for path, (off, ino) in offs.items():
            self.tailer.set_offset(path, int(off), int(ino))

    def _restore_offsets_resharded(self):
        """Tail offsets after a world-size change: for every file this rank now owns, the offset
        from the most recently written tail file of any old rank that held it."""
        best: Dict[str, Any] = {}
        for tp in glob.glob(os.path.join(self.ckpt_dir, "tail.rank*.json")):
            try:
                mt = os.path.getmtime(tp)
                offs = read_json(tp)
            except (OSError, ValueError):
                continue
            for path, v in offs.items():
                if path in self.file_ids and (path not in best or mt > best[path][0]):
                    best[path] = (mt, v)
        for path, (_mt, (off, ino)) in best.items():
            self.tailer.set_offset(path, int(off), int(ino))
        log.info("re-sharded start: resumed %d of %d tails from the previous world's offsets", len(best),
                 len(self.file_ids))

    def checkpoint(self, wait: bool = False):
        """Incremental asynchronous checkpoint: the engine snapshots its state (dirty ring rows
        D2D into HBM staging) and a writer thread persists it; the tail offsets of exactly that
        state travel inside the engine file (one fsync + atomic rename covers both)."""
        if not self.ckpt_dir or self.eng is None:
            return None
        if self._held is not None:
            return None  # a prefetched batch is in the engine: the next step processes it first
        ci = getattr(self.eng, "checkpoint_info", None)
        if ci is not None and ci().get("busy"):
            # the previous checkpoint is still being written: try again at the next interval
            # (draining the pipeline and the sink first only to be told "busy" cost a full drain
            # per batch while a base checkpoint was written)
            self.last_ckpt = self.clock()
            return None
        os.makedirs(self.ckpt_dir, exist_ok=True)
        ck, tp = self._ckpt_paths()
        t0 = time.perf_counter()
        # the previous checkpoint is finished here (the writer is idle): learn whether it
        # committed before any snapshot is pruned, and count the completions before this one
        self._note_checkpoint_outcome()
        done_before = int(ci().get("done", 0)) if ci is not None else 0
        # undelivered output goes out first so the checkpoint and the sinks agree
        self._drain_outputs()
        sink_meta = None
        sink_snap = None  # (native sink: written by the engine's checkpoint writer, see below)
        if self.inserter is not None and self.mode == "inproc":
            # The engine's output lane feeds the native sink directly.  Every row of the batches this
            # checkpoint covers is handed over (flush: the engine pipeline, not the database), then
            # the rows the DB has not acknowledged yet are snapshotted into the checkpoint instead
            # of being waited for: ingest never waits for the DB writer, and a restore submits
            # exactly the flushes the sink's acknowledged watermark (its ack file) does not cover
            # (stream_insert_db.js persists its buffers on exit for the same reason, :222-244).
            tf = time.perf_counter()
            self.native.flush()
            ts = time.perf_counter()
            N = _native_mod()
            core = getattr(self.inserter, "core", None)
            if core is not None and hasattr(core, "snapshot_capture") and hasattr(self.eng, "eng") \
                    and N is not None and hasattr(N, "checkpoint_async_sink"):
                # references to the unacknowledged flushes now (microseconds under the sink
                # lock); the engine's checkpoint writer thread writes + fsyncs them after the
                # checkpoint file and before the manifest names it -- ingest does not wait
                sink_snap = core.snapshot_capture()
                name = self._sink_snapshot_name()
                self.sink_pending_rows = int(sink_snap.rows)
                sink_meta = {"incarnation": self._sink_incarnation, "acked": int(sink_snap.acked), "pending": name,
                             "jobs": int(sink_snap.jobs), "rows": self.sink_pending_rows}
            else:
                sink_meta = self._snapshot_sink()
            self.perf["ckpt_flush_s"] = self.perf.get("ckpt_flush_s", 0.0) + ts - tf
            self.perf["ckpt_sink_snapshot_s"] = self.perf.get("ckpt_sink_snapshot_s", 0.0) + time.perf_counter() - ts
        if self.qm is not None and not self.qm.wait_confirms(float(self.cfg["gpu"].get("confirmTimeoutSeconds", 60))):
            # offsets may only advance past data the broker has taken responsibility for
            log.warning("checkpoint postponed: the broker has not confirmed every publish yet")
            return None
        extra = json.dumps({"tail": json.loads(self.tailer.offsets_json()), "world": self.world,
                            "rank": self.rank, "servers": self.my_servers, "sink": sink_meta}).encode("utf-8")
        prefix = ck[:-len(".ckpt")]
        if sink_snap is not None:
            seq = _native_mod().checkpoint_async_sink(self.eng.eng, prefix, extra, False, sink_snap,
                                                      os.path.join(self.ckpt_dir, sink_meta["pending"]))
            del sink_snap  # (a skipped checkpoint releases the references here)
        else:
            seq = self.eng.checkpoint_async(prefix, extra)
        if seq < 0:
            log.warning("checkpoint skipped: the previous one is still being written")
            return None
        if sink_meta is not None:
            self._ck_started = (sink_meta["pending"], done_before)
            self._prune_sink_snapshots(sink_meta["pending"])
        self.n_checkpoints += 1
        self.perf["ckpt_s"] = self.perf.get("ckpt_s", 0.0) + time.perf_counter() - t0
        if wait:
            self.eng.checkpoint_wait()
        self.tailer.save_offsets(tp)
        write_json_atomic(self._meta_path(), {"world": self.world, "rank": self.rank, "servers": self.my_servers,
                                              "ts": time.time()})
        if self.offsets_path:
            self.tailer.save_offsets(self.offsets_path)
        info = self.eng.checkpoint_info()
        log.info("checkpoint %s #%d (%s): ingest stall %.1f ms (call %.0f ms)%s", ck, seq,
                 "base" if info["last_base"] else "increment", info["last_stall_ms"],
                 (time.perf_counter() - t0) * 1e3,
                 f", written {info['last_bytes'] / 1e6:.1f} MB" if wait else "")
        self.last_ckpt = self.clock()
        return ck

    def _metrics(self, drain: bool = True) -> Dict[str, Any]:
        try:
            m = self.native.metrics(drain=drain)
        except TypeError:  # engines without the non-draining form (CPU oracle)
            m = self.native.metrics()
        return m if isinstance(m, dict) else {}

    def _on_signal(self, signum, frame):
        log.info("Caught signal %d", signum)
        self._stop = True

    def stop(self):
        self._stop = True

    # ------------------------------------------------------------------ config reload
    @staticmethod
    def _consume_paused(cfg: Dict[str, Any]) -> bool:
        """consumeQueue false on a fused stage (stats / z-score / alerts) stops consumption, as
        the reference's watchers do (stream_calc_stats.js:251-258 and its twins): the fused engine
        holds its input instead -- tails keep their offsets, the backlog is processed in order once
        consumption resumes (lock-step ranks keep polling with empty batches)."""
        return not all(bool((cfg.get(sec) or {}).get("consumeQueue", True))
                       for sec in ("streamCalcStats", "streamCalcZScore", "streamProcessAlerts"))

    def reload(self, cfg: Dict[str, Any]):
        self.cfg = cfg
        apmlog.set_global_logger(cfg.get("logDir"), self._log_prefix())
        paused = self._consume_paused(cfg)
        if paused != self._config_paused:
            log.info("%s consume from watcher!", "Stopping" if paused else "Starting")
            self._config_paused = paused
        if self.eng is not None:
            self.eng.reload(cfg)
        if self.notifier:
            self.notifier.reload(cfg)
        if self.inserter:
            ic = cfg["streamInsertDb"]
            self.inserter.limit = int(ic.get("dbInsertBufferLimit", self.inserter.limit))
            self.inserter.max_wait_s = float(ic.get("dbMaxTimeBetweenInsertsMs", 5000)) / 1000.0
        log.info("configuration reloaded")

    # ------------------------------------------------------------------ outputs
    def _drain_outputs(self) -> Dict[str, int]:
        counts = {}
        for k in self.outputs:
            blob = self.native.take_bytes(k)
            if not blob:
                continue
            counts[k] = blob.count(b"\n")
            if k == "al" and self.notifier:
                self.notifier.add_lines(blob.decode("utf-8").split("\n"))
            if self.inserter is not None and (k in DB_OUTPUTS or k == "fb"):
                self.inserter.consume_bytes(blob)
            elif self.qm is not None:
                if k == "fb":
                    prod = self.producers.get("fleet")
                elif k in DB_OUTPUTS:
                    prod = self.producers["db"]
                elif k == "transactions":
                    prod = self.producers.get("transactions")
                else:
                    prod = self.producers.get("stats")
                if prod is not None:
                    prod.write_lines(ln for ln in blob.decode("utf-8").split("\n") if ln)
                if k == "fs" and "z_score" in self.producers:  # the z-score stage's output queue
                    self.producers["z_score"].write_lines(ln for ln in blob.decode("utf-8").split("\n") if ln)
        return counts

    def _on_jx(self, line: str):
        """A JMX record: to the DB like pull_jvm_stats.js does, and into the engine's gauges."""
        if self.eng is not None:
            try:
                load = os.getloadavg()[0]
            except OSError:
                load = float("nan")
            self.eng.set_server_context(line, load)
        if self.inserter is not None:
            self.inserter.consume_line(line)
        elif self.qm is not None:
            self.producers["db"].write_line(line)

    def _housekeeping(self):
        now = self.clock()
        pf = self.perf
        t0 = time.perf_counter()
        if self.jmx is not None:
            self.jmx.tick()
        ta = time.perf_counter()
        if self.inserter is not None:
            self.inserter.tick()
        tb = time.perf_counter()
        if self.notifier is not None:
            self.notifier.tick()
        t1 = time.perf_counter()
        pf["hk_jmx_s"] = pf.get("hk_jmx_s", 0.0) + ta - t0
        pf["hk_sink_s"] = pf.get("hk_sink_s", 0.0) + tb - ta
        if self.watcher is not None:
            try:
                self.watcher.check_once()
            except Exception as e:  # a broken config must not stop ingest
                log.error("config reload failed: %s", e)
        if self._gc_requested and self._held is None:  # (a held prefetch: the next poll does not prefetch)
            self._gc_requested = False
            self.request_gc()
        t2 = time.perf_counter()
        if self._ckpt_due():
            self.checkpoint()
            if self._lockstep_ckpt():  # (advanced on every rank alike, written or skipped)
                self._ckpt_epoch = int(self.native.batch_no()) // self._ckpt_every_batches()
        t3 = time.perf_counter()
        interval = float(self.cfg.get("statLogIntervalInSeconds", 60))
        if now - self.last_stat >= interval:
            self.log_stats(now - self.last_stat)
            self.last_stat = now
        t4 = time.perf_counter()
        # where the drain loop's housekeeping goes (service_bench reports these)
        for k, v in (("hk_ticks_s", t1 - t0), ("hk_watch_s", t2 - t1), ("hk_ckpt_s", t3 - t2), ("hk_stats_s", t4 - t3)):
            pf[k] = pf.get(k, 0.0) + v

    def log_stats(self, dt_s: float):
        """Per statLogIntervalInSeconds: throughput, per-stage ms per batch, the ingest->alert
        latency distribution of the interval's rollovers, HBM in use.  The counters are
        read without draining the pipeline (a batch behind at most): a stat line never stalls ingest."""
        m = self._metrics(drain=False)
        d = {k: m.get(k, 0) - self._m0.get(k, 0) for k in ("lines", "tx", "alerts", "rollovers", "batches")}
        self._m0 = m
        log.info("ENGINE lines/s: %.0f - tx/s: %.0f - rollovers: %d - alerts: %d - batches: %d - series: %s",
                 d["lines"] / max(dt_s, 1e-9), d["tx"] / max(dt_s, 1e-9), d["rollovers"], d["alerts"], d["batches"],
                 self.native.n_series() if hasattr(self.native, "n_series") else "?")
        prev = getattr(self, "_m0_prev", {})
        stages = {k: m.get(k, 0.0) - prev.get(k, 0.0) for k in _STAGE_KEYS}
        nb = max(d["batches"], 1)
        lat = list(m.get("rollover_latency_ms", []))[len(prev.get("rollover_latency_ms", [])):]
        self._m0_prev = m
        pct = _percentiles(lat, (50, 90, 99))
        hbm = self.native.device_bytes() if hasattr(self.native, "device_bytes") else 0
        log.info("ENGINE ms/batch parse %.2f join %.2f stats %.2f out %.2f - ingest->alert ms p50 %s p90 %s p99 %s "
                 "- HBM %.2f GB - fleet rounds %s",
                 *(stages[k] / nb for k in _STAGE_KEYS), *pct, hbm / 1e9,
                 self.native.fleet_rounds() if hasattr(self.native, "fleet_rounds") else "-")
        # capacity overflows: window samples past the spill area (gpu.bucketOverflowCapacity) or
        # series past gpu.maxSeries make that interval's statistics wrong -- say so every interval
        lost = {k: int(m.get(k, 0)) for k in ("spill_dropped", "series_overflow_tx", "tx_dropped")}
        j = m.get("join", {})
        lost.update({f"join_{k}": int(j.get(k, 0)) for k in ("partial_overflow", "need_overflow", "table_full",
                                                           "pool_exhausted")})
        if any(lost.values()):
            log.warning("ENGINE capacity exceeded (totals): %s -- raise gpu.maxSeries (the other structures grow)",
                     ", ".join(f"{k}={v}" for k, v in lost.items()))
        # CACHE_STATS (stream_parse_transactions.js:329-335): live entries of the join caches
        cs = self.native.cache_stats(drain=False) if hasattr(self.native, "cache_stats") else {}
        if cs:
            log.info("CACHE_STATS acctCache: %d - recordCache: %d (%d open partials) - needNumRecordCache: %d "
                     "- key table %d / %d slots (load %.3f)", cs["acct"], cs["record"], cs["partials"], cs["need"],
                     cs["occupied"], cs["slots"], cs["occupied"] / max(cs["slots"], 1))
        grows = {"spill": int(m.get("spill_grows", 0)),
                 **{k: int(j.get(k + "_grows", 0)) for k in ("table", "arena", "pool")}}
        if grows != getattr(self, "_grows_prev", grows):
            log.info("ENGINE capacity grown (totals): %s", ", ".join(f"{k}={v}" for k, v in grows.items()))
        self._grows_prev = grows
        nm = list(self.native.node_metrics()) if hasattr(self.native, "node_metrics") else []
        if nm and nm[0] > 1 and getattr(self, "rank", 0) == 0:
            prev_nm = getattr(self, "_nm_prev", None) or [0.0] * len(nm)
            self._nm_prev = nm
            log.info("NODE ranks: %d - lines: %d (+%d) - tx: %d - alerts: %d - series: %d", nm[0], nm[2],
                     nm[2] - prev_nm[2], nm[5], nm[10], nm[11])
        if self.inserter is not None:
            self.inserter.stats.log_and_reset()
        if self.qm is not None:
            log.info(self.qm.stats.line())

    def request_gc(self) -> str:
        """requestGC (util_methods.js:398-417): collect Python garbage and hand freed heap back to
        the OS, and -- the engine's share of a process is mostly HBM -- give the grow-only device
        structures back (join key table / need arena shrunk to their live entries, spill lists,
        checkpoint scratch), at this batch boundary."""
        hbm = ""
        trim = getattr(self.native, "trim_device_memory", None)
        if trim is not None and self._held is None:
            before, after = trim()
            hbm = f" hbm={before / 2**30:.3f} GB -> {after / 2**30:.3f} GB"
        gc.collect()
        try:
            ctypes.CDLL("libc.so.6").malloc_trim(0)
        except OSError:
            pass
        rss = 0
        try:
            with open("/proc/self/statm") as f:
                rss = int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")
        except OSError:
            pass
        msg = f"Running garbage collection! rss={rss / 2**20:.1f} MB{hbm}"
        log.info(msg)
        return msg

    # ------------------------------------------------------------------ main loop
    def step(self) -> int:
        """One poll: read new complete lines from every file and run them through the engine."""
        # Lock-step ranks (native engine, world > 1): every process_batch runs the node-wide
        # clock all-reduce, so every rank must call it once per poll -- with an empty batch when
        # its tails have nothing new or downstream is paused -- or the collective sequences diverge.
        lockstep = self.fleet is not None
        paused = self.qm is not None and any(getattr(p, "paused", False) for p in self.producers.values())
        paused = paused or self._config_paused
        if self.input_mode == "transactions":
            return 0 if paused and not lockstep else self._step_tx(lockstep, paused)
        if self.readahead:
            return self._step_readahead(lockstep, paused)
        if paused:
            # downstream backpressure: hold the tails (pause-file semantics)
            if not lockstep:
                return 0
            buf, chunks = b"", []
        else:
            buf, chunks = self.tailer.poll()
        if not chunks and not lockstep:
            return 0
        self.polls += 1
        fi = self.fault
        if fi and fi.get("rank", self.rank) == self.rank:
            if fi.get("exitAtBatch") and self.polls == int(fi["exitAtBatch"]):
                log.error("fault injection: exiting at batch %d", self.polls)
                os._exit(int(fi.get("exitCode", 13)))
            if chunks and fi.get("dropBatchEvery") and self.polls % int(fi["dropBatchEvery"]) == 0:
                log.warning("fault injection: dropping batch %d (%d bytes)", self.polls, len(buf))
                self.faults["dropped"] += 1
                if not lockstep:
                    return len(buf)
                buf, chunks = b"", []  # the rank still takes part in this poll's collectives
        self.native.process_batch(buf, chunks, -1.0)
        self.batches += 1
        if fi and fi.get("rank", self.rank) == self.rank and fi.get("duplicateBatchEvery") \
                and chunks and self.polls % int(fi["duplicateBatchEvery"]) == 0:
            if lockstep:  # a second process_batch on one rank only would desynchronise the ranks
                log.warning("fault injection: duplicateBatchEvery is ignored for lock-step ranks")
            else:
                log.warning("fault injection: replaying batch %d", self.polls)
                self.faults["duplicated"] += 1
                self.native.process_batch(buf, chunks, -1.0)
        self._drain_outputs()
        return len(buf)

    def _on_tx_message(self, body: bytes):
        with self._in_lock:
            self._in_lines.append(body)

    def _step_tx(self, lockstep: bool, paused: bool = False) -> int:
        lines = []
        if not paused:  # (paused lock-step ranks still take part in the poll's collectives)
            with self._in_lock:
                lines, self._in_lines = self._in_lines, []
        if not lines and not lockstep:
            return 0
        blob = b"\n".join(ln.rstrip(b"\n") for ln in lines) + (b"\n" if lines else b"")
        self.native.process_tx_lines(blob, -1.0)
        self.polls += 1
        self.batches += 1
        self._drain_outputs()
        return len(blob)

    def _lockstep_ckpt(self) -> bool:
        """Lock-step ranks checkpoint at the same batches (every gpu.checkpointEveryBatches): any
        batch every rank has a checkpoint for is a consistent node state -- what a same-world
        restart resumes from and a re-shard merges (merge.cpp needs one common batch)."""
        return self.fleet is not None and self.world > 1

    def _ckpt_every_batches(self) -> int:
        g = self.cfg.get("gpu", {})
        k = int(g.get("checkpointEveryBatches", 0) or 0)
        if k <= 0:
            k = 1 if self.ckpt_every <= 0 else max(1, int(round(self.ckpt_every / float(g.get("pollSeconds", 1.0)))))
        return k

    def _ckpt_due(self, ahead: int = 0) -> bool:
        if not self.ckpt_dir or self.eng is None:
            return False
        if self._lockstep_ckpt():
            k = self._ckpt_every_batches()
            b = int(self.native.batch_no()) + ahead
            if self._ckpt_epoch is None:
                self._ckpt_epoch = (b - ahead) // k
            return b // k > self._ckpt_epoch
        return self.clock() - self.last_ckpt >= self.ckpt_every

    def _step_readahead(self, lockstep: bool, paused: bool) -> int:
        """step() over the tailer's read-ahead ring: batches arrive in pinned slots, the batch
        after the current one (if already read) is handed to the engine as its prefetch."""
        pf = self.perf
        t0 = time.perf_counter()
        cur = self._held
        self._held = None
        if cur is None and not paused:
            cur = self.tailer.next(0.0)
        t1 = time.perf_counter()
        pf["wait_s"] += t1 - t0
        if cur is None and not lockstep:
            return 0
        self.polls += 1
        fi = self.fault
        mine = bool(fi) and fi.get("rank", self.rank) == self.rank
        if mine and fi.get("exitAtBatch") and self.polls == int(fi["exitAtBatch"]):
            log.error("fault injection: exiting at batch %d", self.polls)
            os._exit(int(fi.get("exitCode", 13)))
        if cur is None:  # lock-step poll with nothing to read (or paused downstream)
            self.native.process_batch(b"", [], -1.0)
            self.batches += 1
            self._drain_outputs()
            return 0
        slot, ptr, n, chunks, bid = cur
        if mine and fi.get("dropBatchEvery") and self.polls % int(fi["dropBatchEvery"]) == 0:
            log.warning("fault injection: dropping batch %d (%d bytes)", self.polls, n)
            self.faults["dropped"] += 1
            self.tailer.release(slot)
            self.tailer.commit(bid)
            if lockstep:
                self.native.process_batch(b"", [], -1.0)
                self.batches += 1
            return n
        dup = mine and fi.get("duplicateBatchEvery") and self.polls % int(fi["duplicateBatchEvery"]) == 0
        nxt = None
        if not paused and not dup and not self._ckpt_due(ahead=1) and not self._stopping and not self._gc_requested:
            nxt = self.tailer.next(0.0)
        if self.batch_log is not None:
            import ctypes
            self.batch_log.append((ctypes.string_at(ptr, n), list(chunks)))
        t2 = time.perf_counter()
        pf["next_s"] = pf.get("next_s", 0.0) + t2 - t1
        if nxt is not None:
            self.native.process_batch_ptr(ptr, n, chunks, -1.0, nxt[1], nxt[2], nxt[3])
        else:
            self.native.process_batch_ptr(ptr, n, chunks, -1.0)
        t3 = time.perf_counter()
        pf["engine_s"] += t3 - t2
        pf["batches"] += 1
        pf["bytes"] += n
        pf["prefetched"] += nxt is not None
        self.batches += 1
        if dup:
            if lockstep:
                log.warning("fault injection: duplicateBatchEvery is ignored for lock-step ranks")
            else:
                log.warning("fault injection: replaying batch %d", self.polls)
                self.faults["duplicated"] += 1
                self.native.process_batch_ptr(ptr, n, chunks, -1.0)
        self.tailer.release(slot)
        self.tailer.commit(bid)
        self._held = nxt
        t4 = time.perf_counter()
        pf["commit_s"] = pf.get("commit_s", 0.0) + t4 - t3
        # take_bytes waits for the engine's in-flight stats stage: with the DB streams going
        # straight to the native sink, the remaining Python-side streams (al -> notifier) are
        # collected every outputDrainMs instead of once per batch, so batches stay pipelined
        if self._drain_every_s <= 0 or t4 - self._last_drain >= self._drain_every_s:
            self._drain_outputs()
            self._last_drain = time.perf_counter()
        pf["outputs_s"] += time.perf_counter() - t4
        return n

    def _idle(self, idle_sleep_s: float):
        if self.readahead and self._drain_every_s > 0:
            self._drain_outputs()
            self._last_drain = time.perf_counter()
        if self.readahead:
            if self._held is None:
                self._held = self.tailer.next(idle_sleep_s * 1000.0)
        else:
            self.tailer.wait(idle_sleep_s * 1000.0)

    def run(self, max_batches: Optional[int] = None, idle_sleep_s: float = 0.5,
            until: Optional[Callable[[], bool]] = None):
        log.info("ingest loop starting (mode=%s)", self.mode)
        # startup garbage collected once, and the long-lived startup objects (config, file tables,
        # engine wrappers) moved out of the collector's generations: a full collection inside the
        # loop then walks only what the loop itself allocates (the bench saw one ~7 ms step in
        # four 20-step runs from a collection over its setup objects, profiles/r6_w)
        gc.collect()
        gc.freeze()
        try:
            while not self._stop:
                n = self.step()
                self._housekeeping()
                if max_batches is not None and self.batches >= max_batches:
                    break
                if until is not None and until():
                    break
                if n == 0:
                    self._idle(idle_sleep_s)
        except BaseException as e:
            # HIP error, capacity throw, collective abort, ...: leave the engine's state behind
            # before the non-zero exit (the reference's node-oom-heapdump, apm_manager.js:12-18)
            if not isinstance(e, (KeyboardInterrupt, SystemExit)):
                self.fatal_dump(e)
            raise
        self.shutdown()

    def fatal_dump(self, exc: BaseException) -> Optional[str]:
        """Write the engine's host-side state (clocks, batch ids, counters, capacities, fill levels)
        with the failure reason into ``<checkpointDir or logDir>/engine.rank<r>.fatal.<ts>.dump``
        (checkpoint file format, one section; ``read_state_dump`` parses it)."""
        if self.eng is None or not hasattr(self.native, "dump_state"):
            return None
        d = self.ckpt_dir or self.cfg.get("logDir") or "."
        return write_fatal_dump(self.native, d, self.rank, exc)

    def shutdown(self):
        log.info("shutting down")
        if self.trace_path and self.eng is not None:
            try:
                self.eng.dump_trace(self.trace_path if self.world == 1 else f"{self.trace_path}.rank{self.rank}",
                                    pid=self.rank)
                log.info("stage trace written to %s", self.trace_path)
            except Exception as e:  # pragma: no cover
                log.warning("stage trace not written: %s", e)
        if self.fleet is not None and not self._stop:
            # coordinated end (same batch count on every rank): decide the queued node-wide
            # alert candidates -- a collective, so not on a signal-driven (per-rank) stop
            self.fleet.drain_alerts()
        self._stopping = True
        while self._held is not None:  # a prefetched batch is processed before the final checkpoint
            self.step()
        self.native.flush()
        self._drain_outputs()
        if self.readahead:
            self.tailer.stop()
        if self.ckpt_dir and self.eng is not None:
            self.eng.checkpoint_wait()
            self.checkpoint(wait=True)
        if self.offsets_path:
            self.tailer.save_offsets(self.offsets_path)
        for p in self._slots:
            from .. import _native
            _native.load(build_if_missing=False).free_pinned(p)
        self._slots = []
        if self.inserter is not None:
            self.inserter.close()
        if self.notifier is not None:
            self.notifier.tick()
        if self.qm is not None:
            self.qm.wait_confirms(float(self.cfg["gpu"].get("confirmTimeoutSeconds", 60)))
            self.qm.shutdown()
        if self.in_qm is not None and self.in_qm is not self.qm:
            self.in_qm.shutdown()


def write_fatal_dump(native, directory: str, rank: int, exc: BaseException) -> Optional[str]:
    """Engine state dump on a fatal error; never raises (the original error is what matters)."""
    try:
        os.makedirs(directory, exist_ok=True)
        path = os.path.join(directory, f"engine.rank{rank}.fatal.{time.strftime('%Y%m%d%H%M%S')}.dump")
        native.dump_state(path, f"{type(exc).__name__}: {exc}")
        log.error("fatal: %s -- engine state dumped to %s", exc, path)
        return path
    except Exception as e2:  # pragma: no cover - best effort
        log.error("fatal: %s -- state dump failed: %s", exc, e2)
        return None


def read_state_dump(path: str) -> Dict[str, Any]:
    """Parse a fatal dump (binio framing: magic, version, {tag, length, payload}..., end)."""
    import struct
    with open(path, "rb") as f:
        data = f.read()
    if data[:8] != b"APMCKPT\0":
        raise ValueError("not an engine checkpoint / dump file")
    import numpy as np
    off = 12
    state = None
    while off + 4 <= len(data):
        tag = struct.unpack_from("<I", data, off)[0]
        if tag == 0xE0F:
            break
        ln = struct.unpack_from("<Q", data, off + 4)[0]
        body = data[off + 12: off + 12 + ln]
        if tag == 100:
            n1 = struct.unpack_from("<Q", body, 0)[0]
            reason = body[8:8 + n1].decode()
            n2 = struct.unpack_from("<Q", body, 8 + n1)[0]
            state = json.loads(body[16 + n1:16 + n1 + n2].decode())
            state["reason"] = reason
        elif tag == 101 and state is not None:
            state["series"] = _read_series_dump(body, np)
        off += 12 + ln
    if state is None:
        raise ValueError("no dump section")
    return state


def _read_series_dump(body: bytes, np) -> Dict[str, Any]:
    """SEC_DUMP_SERIES (checkpoint.cpp write_series_dump): names, window stats of the last
    rollover, and per LAG the history length, alert counter, z-score bounds / signals, moments."""
    import struct
    pos = [0]

    def u64():
        v = struct.unpack_from("<Q", body, pos[0])[0]
        pos[0] += 8
        return v

    def text():
        n = u64()
        v = body[pos[0]:pos[0] + n].decode()
        pos[0] += n
        return v

    def vec(dt):
        n = u64()
        a = np.frombuffer(body, dtype=dt, count=n, offset=pos[0]).copy()
        pos[0] += n * np.dtype(dt).itemsize
        return a

    hdr = json.loads(text())
    n = hdr["n"]
    out: Dict[str, Any] = dict(hdr)
    out["server"] = [text() for _ in range(u64())]
    out["service"] = [text() for _ in range(u64())]
    out["window"] = vec("<f8").reshape(n, 6)  # tpm, avg, p75, p95, n, active
    out["per_lag"] = {}
    for lag in hdr["lags"]:
        out["per_lag"][lag] = {"len": vec("<i4"), "counter": vec("<i4"),
                               "z": vec("<f8").reshape(n, 4, 3),  # mean / lb / ub / signal x (avg, p75, p95)
                               "sum": vec("<f8").reshape(3, n) if n else np.zeros((3, 0)),
                               "cnt": vec("<i4").reshape(3, n) if n else np.zeros((3, 0), np.int32)}
    return out


def main(argv=None):  # pragma: no cover - process entry point
    import argparse
    ap = argparse.ArgumentParser(description="apmbackend_amd ingest service (one process per GPU)")
    ap.add_argument("--config", default=None)
    ap.add_argument("--engine", default="native", choices=["native", "cpu-oracle"])
    ap.add_argument("--max-batches", type=int, default=None)
    # per-module profiling hooks (the reference starts every module with --inspect=<port>,
    # apm_manager.js:263-267): a Chrome trace of the engine's stages written at shutdown; the
    # engine's roctx ranges (apm.parse / apm.join / ...) are always emitted for rocprofv3
    # --marker-trace
    ap.add_argument("--trace", default=None, help="write a Chrome trace of the pipeline stages here at shutdown")
    a = ap.parse_args(argv)
    env_world = dist_env()[1]
    if env_world > 1 and str(read_apm_config(a.config, first_run=True).get("gpu", {}).get(
            "collectiveBackend", "rccl")) != "host":
        from ..parallel.dist import init_distributed
        init_distributed()
    svc = IngestService(config_path=a.config, engine=a.engine, install_signals=True,
                        trace_path=a.trace)
    try:
        svc.run(max_batches=a.max_batches)
    except RuntimeError as e:
        if is_peer_failure(e):
            # a peer rank died or hung: this rank is healthy -- say so in the exit status, so the
            # supervisor's elastic degrade blames the rank that failed first, not its survivors
            log.error("collective peer failure: %s", e)
            sys.exit(PEER_FAILURE_EXIT)
        raise


if __name__ == "__main__":  # pragma: no cover
    main()
