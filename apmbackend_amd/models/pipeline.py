"""The flagship model: the fused MI355X APM pipeline.

``APMEngine`` maps the reference configuration (``config/apm_config.json`` sections
``streamParseTransactions`` .. ``streamProcessAlerts`` + the new ``gpu`` section) onto the native
``_apm_native.Engine`` and exposes a batch API:

    eng = APMEngine(cfg)
    eng.process([(path, bytes), ...])          # one ingest batch (whole lines per file)
    eng.take("fs"), eng.take("al"), ...        # reference wire-format records (keep_text=True)

One engine == one GPU == one process; the multi-GPU runner (``parallel.dist``) shards JVM hosts
across ranks.
"""
from __future__ import annotations

import logging
import math
import os
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple, Union

from .. import _native
from ..models.oracle import file_kind, server_of
from ..ops.parse_ref import tz_table
from ..utils.timeparse import TzOffset

log = logging.getLogger("apm.pipeline")

KIND_CODE = {"SOAP": 0, "SERVER": 1, "APP": 2}

# Output streams (engine.h OutKind); the bit index is the position in this tuple.
OUT_KINDS = ("transactions", "audit_db", "db", "st", "fs", "al", "sx", "fb")
# What the reference persists (db_insert queue): released + audit tx, fs, al.  `transactions`
# and `st` are internal hand-offs that only the AMQP bridge needs.
DB_OUTPUTS = ("audit_db", "db", "fs", "al")
MAX_LAGS = 16  # apm_types.h MAX_LAGS: LAG capacity per engine (each LAG is an HBM ring; see there)


def output_mask(kinds) -> int:
    m = 0
    for k in kinds:
        m |= 1 << OUT_KINDS.index(k)
    return m


def engine_config(cfg: Dict[str, Any], device: int = 0, keep_text: bool = False, outputs=None,
                  **kw) -> Dict[str, Any]:
    """Engine settings from the reference config keys + the `gpu` section.  keep_text=True
    materialises every stream; `outputs` (iterable of OUT_KINDS) selects explicitly."""
    g = cfg.get("gpu", {})
    zc = cfg["streamCalcZScore"]
    ac = cfg["streamProcessAlerts"]
    sc = cfg["streamCalcStats"]
    lags = sorted(((int(d["LAG"]), float(d["THRESHOLD"]), float(d["INFLUENCE"])) for d in zc["defaults"]),
                  key=lambda x: x[0])
    if len(lags) > MAX_LAGS:
        raise ValueError(f"at most {MAX_LAGS} LAG settings are supported per engine")
    suppressed_lags = {int(x) for x in ac.get("suppressedLags", [])}
    ring = {"float64": 8, "float32": 4, "bfloat16": 2, "bf16": 2}.get(g.get("ringDtype", "float64"), 8)
    tz = TzOffset(g.get("timezone", "local"))
    d = {
        "device": device,
        "max_series": int(g.get("maxSeries", 1 << 17)),
        "cell_cap": int(g.get("bucketCellCapacity", 16)),
        "spill_cap": int(g.get("bucketOverflowCapacity", 1 << 22)) // 40 or 1,
        "max_batch_bytes": int(g.get("batchBytes", 32 << 20)) * 2,
        # (below 2^21: the device join packs its per-event selection counts into 21-bit fields)
        "max_lines": min(int(g.get("maxLinesPerBatch", 1 << 20)) * 2, (1 << 21) - 1),
        # host-join tx staging per batch (grows by doubling when a batch needs more)
        "max_tx_per_batch": int(g.get("maxTxPerBatch", int(g.get("maxLinesPerBatch", 1 << 20)) * 2)),
        "ring_bytes": ring,
        "exact_mean": 1 if g.get("zscoreMeanMode", "rolling") == "exact" else 0,
        "sigma_stddev": 1 if g.get("zscoreSigma", "sqrt_mean") == "stddev" else 0,
        "resync_k": int(g.get("exactRecomputeEveryIntervals", 360)),
        "resync_mfma": bool(g.get("resyncOnMatrixCores", False)),
        "emulate_aliasing": 1 if g.get("emulateOverrideAliasing", False) else 0,
        "lags": lags,
        "lag_suppressed": [1 if l[0] in suppressed_lags else 0 for l in lags],
        "alert_window": int(ac["rollingAlertWindowSizeInIntervals"]),
        "alert_threshold": int(ac["requiredNumberBadIntervalsInAlertWindowToTrigger"]),
        "hard_min_ms": float(ac["hardMinMsAlertThreshold"]),
        "hard_min_tpm": float(ac["hardMinTpmAlertThreshold"]),
        "hard_max_ms": float(ac["hardMaxMsAlertThreshold"]),
        "both_only": 1 if ac.get("alertOnBothOnly") else 0,
        "cooldown_ms": float(ac["perServiceAlertCooldownInMinutes"]) * 60000.0,
        "cooldown_by_service": 1 if g.get("cooldownKey", "service") == "service" else 0,
        "alert_clock_entry": 1 if g.get("alertClock", "entry") == "entry" else 0,
        "interval_len": int(sc["intervalLengthInSeconds"]),
        "window": int(sc["windowSizeInIntervals"]),
        # bucket ring slots (0: window + buffer + 1, at least 40); a reload to a longer window grows it
        "nslot": int(g.get("bucketRingSlots", 0)),
        # HBM staging of a base checkpoint's ring rows; a larger ring streams (checkpoint.cpp)
        "ck_stage_bytes": int(float(g.get("checkpointStageMB", 2048)) * (1 << 20)),
        "buffer": int(sc["bufferSizeInIntervals"]),
        "record_ttl_ms": float(g.get("recordTtlSeconds", 120)) * 1000.0,
        "acct_ttl_ms": float(g.get("acctTtlSeconds", 120)) * 1000.0,
        "need_ttl_ms": float(g.get("needTtlSeconds", 30)) * 1000.0,
        "tz_table": tz_table(tz),
        "join_threads": int(g.get("joinThreads", 0)),
        "pin_threads": bool(g.get("pinThreads", False)),
        "coll_timeout_ms": float(g.get("collectiveTimeoutSeconds", 300)) * 1000.0,
        "coll_init_timeout_ms": float(g.get("collectiveInitTimeoutSeconds", 120)) * 1000.0,
        # lock-step ranks decide the alert cooldown node-wide (one alert per service per node)
        "node_cooldown": 1 if g.get("nodeCooldown", True) else 0,
        # K4/K6 join on the GPU (devjoin.hip); false = host join workers (join.cpp)
        "device_join": 1 if g.get("joinOnDevice", True) else 0,
        "join_table_bits": max(10, (int(g.get("joinTableSlots", 1 << 21)) - 1).bit_length()),
        "need_arena": int(g.get("needArenaEntries", 1 << 18)),
        "join_chain_blocks": int(g.get("joinChainBlocks", 0)),
        # the ring holds every tx line not yet released (~70 s of tx text); small test engines
        # keep it proportional to their batch size
        "tx_ring_bytes": min(int(g.get("txTextRingMB", 4096)), max(256, (128 * int(g.get("batchBytes", 32 << 20))) >> 20)) << 20,
        "max_raw_services": max(int(g.get("maxRawServices", 1 << 18)), 2 * int(g.get("maxSeries", 1 << 17))),
        "outputs": output_mask(OUT_KINDS if keep_text else (outputs or ())),
    }
    # intervalLengthInSeconds only scales the TPM divisor: the bucket label is endTs without its
    # last 4 digits whatever the interval (stream_calc_stats.js:89-96, :186), as here
    w, b = d["window"], d["buffer"]
    if not (w >= 1 and b >= 0 and d["interval_len"] >= 1):
        raise ValueError(f"stats window: windowSizeInIntervals >= 1, bufferSizeInIntervals >= 0, "
                         f"intervalLengthInSeconds >= 1 (got {w} / {b} / {d['interval_len']})")
    d.update(kw)
    return d


def service_overrides(cfg: Dict[str, Any]) -> Dict[str, Dict[str, Any]]:
    """Per-service override table: z-score THRESHOLD/INFLUENCE per LAG, alert hard max, suppression."""
    zc = cfg["streamCalcZScore"]
    ac = cfg["streamProcessAlerts"]
    lags = sorted(int(d["LAG"]) for d in zc["defaults"])
    out: Dict[str, Dict[str, Any]] = {}
    for svc, per_lag in ((zc.get("overrides") or {}).get("services") or {}).items():
        o = out.setdefault(svc, {"thr": [None] * len(lags), "infl": [None] * len(lags)})
        for lag_key, vals in per_lag.items():
            try:
                li = lags.index(int(float(lag_key)))
            except ValueError:
                continue
            if "THRESHOLD" in vals:
                o["thr"][li] = float(vals["THRESHOLD"])
            if "INFLUENCE" in vals:
                o["infl"][li] = float(vals["INFLUENCE"])
    for svc, vals in ((ac.get("overrides") or {}).get("services") or {}).items():
        o = out.setdefault(svc, {"thr": [None] * len(lags), "infl": [None] * len(lags)})
        hm = vals.get("hardMaxMsAlertThreshold")
        if hm:
            o["hard_max"] = float(hm)
    for svc in ac.get("suppressedServices", []) or []:
        o = out.setdefault(svc, {"thr": [None] * len(lags), "infl": [None] * len(lags)})
        o["suppressed"] = True
    return out


_last_gen = [0]


def _reload_generation(cfg: Dict[str, Any]) -> int:
    """Reload generation: the config file's mtime in ms (identical on every rank of a node, so
    the ranks agree on which reload they apply), else a local counter."""
    path = cfg.get("apmConfigFilePath")
    g = 0
    if path and os.path.exists(path):
        g = os.stat(path).st_mtime_ns // 1_000_000
    if g <= 0:
        g = _last_gen[0] + 1
    _last_gen[0] = max(_last_gen[0], g)
    return g


class APMEngine:
    def __init__(self, cfg: Dict[str, Any], device: int = 0, keep_text: bool = False, outputs=None, **kw):
        self.cfg = cfg
        self.N = _native.load()
        self.ecfg = engine_config(cfg, device, keep_text, outputs, **kw)
        self.eng = self.N.Engine(self.ecfg)
        self.file_ids: Dict[str, int] = {}
        self.apply_overrides(cfg)

    def apply_overrides(self, cfg: Dict[str, Any]):
        self.eng.clear_overrides()
        for svc, o in service_overrides(cfg).items():
            self.eng.set_override(svc, o)

    # engine settings a reload applies live (reconfig.cpp); any other change needs a restart
    LIVE_KEYS = ("lags", "lag_suppressed", "alert_window", "alert_threshold", "hard_min_ms", "hard_min_tpm",
                 "hard_max_ms", "both_only", "cooldown_ms", "interval_len", "window", "buffer")

    def reload(self, cfg: Dict[str, Any], gen: Optional[int] = None) -> List[str]:
        """Config hot reload (the reference's watchAPMConfig callbacks): z-score defaults and
        per-service overrides re-applied to every series, LAGs added (empty history) or removed
        (removeStaleLagData), every alert gate replaced -- staged now, applied by the engine at the
        next batch boundary (the same boundary on every lock-step rank).  Returns the engine
        settings that changed but need a restart (they are not applied)."""
        new = engine_config(cfg, self.ecfg["device"], outputs=())
        restart = sorted(k for k in new if k not in self.LIVE_KEYS and k not in ("outputs", "tz_table")
                         and new[k] != self.ecfg.get(k))
        if restart:
            log.warning("config reload: %s changed but need a restart (not applied)", ", ".join(restart))
        if gen is None:
            gen = _reload_generation(cfg)
        self.eng.stage_reconfig(new, service_overrides(cfg), int(gen))
        for k in self.LIVE_KEYS:
            self.ecfg[k] = new[k]
        self.cfg = cfg
        return restart

    def add_file(self, path: str, kind: Optional[str] = None, server: Optional[str] = None) -> int:
        if path in self.file_ids:
            return self.file_ids[path]
        k = KIND_CODE[kind or file_kind(path)]
        fid = self.eng.add_file(path, k, server or server_of(path))
        self.file_ids[path] = fid
        return fid

    def process(self, chunks: Sequence[Tuple[Union[str, int], bytes]], now: Optional[float] = None):
        parts, table = [], []
        off = 0
        for f, data in chunks:
            if not data:
                continue
            if not data.endswith(b"\n"):
                data = data + b"\n"
            fid = f if isinstance(f, int) else self.add_file(f)
            parts.append(data)
            table.append((fid, off, off + len(data)))
            off += len(data)
        buf = b"".join(parts)
        self.eng.process_batch(buf, table, -1.0 if now is None else float(now))

    def process_lines(self, chunks: Sequence[Tuple[str, List[str]]], now: Optional[float] = None):
        self.process([(fp, ("\n".join(ls) + "\n").encode("utf-8")) for fp, ls in chunks if ls], now)

    def take(self, kind: str) -> List[str]:
        return self.eng.take(kind)

    def save_state(self, path: str, extra: bytes = b"") -> int:
        """Binary checkpoint of the whole pipeline (engine + join caches + pending output);
        ``extra`` is stored with it (one atomic file)."""
        return self.eng.save_state(path, extra)

    def checkpoint_async(self, prefix: str, extra: bytes = b"", force_base: bool = False) -> int:
        """Incremental asynchronous checkpoint (``<prefix>.ckpt`` chain manifest): returns its
        sequence number, or -1 if the previous one is still being written."""
        return self.eng.checkpoint_async(prefix, extra, force_base)

    def checkpoint_wait(self) -> int:
        return self.eng.checkpoint_wait()

    def checkpoint_info(self) -> dict:
        return self.eng.checkpoint_info()

    def load_state(self, path: str) -> bytes:
        """Resume from save_state() / checkpoint_async() output; this engine must be fresh (no
        files, no batches).  Returns the ``extra`` blob stored with the state."""
        extra = self.eng.load_state(path)
        self.file_ids = {p: i for i, (p, _k, _s) in enumerate(self.eng.files())}
        return extra

    def take_bytes(self, kind: str) -> bytes:
        return self.eng.take_bytes(kind)

    def dump_trace(self, path: str, pid: int = 0) -> int:
        """Write the recorded stage intervals (set_trace(True) first) as a Chrome trace."""
        import json
        ev = self.eng.take_trace()
        names = {0: "ingest (parse + join)", 1: "stats thread", 2: "device join phases", 3: "next-batch lane", 4: "output lane"}
        out = [{"name": "thread_name", "ph": "M", "pid": pid, "tid": t, "args": {"name": n}} for t, n in names.items()]
        for name, t0, t1, tid, batch in ev:
            out.append({"name": name, "ph": "X", "ts": t0 * 1000.0, "dur": max(0.0, (t1 - t0) * 1000.0), "pid": pid,
                        "tid": tid, "args": {"batch": batch}})
        with open(path, "w") as f:
            json.dump({"traceEvents": out, "displayTimeUnit": "ms"}, f)
        return len(ev)

    def set_server_context(self, jx_line: str, vm_load: float = 0.0) -> bool:
        """Feed a JMX ``jx`` record (pull_jvm_stats) into the per-JVM gauge table fused by K14."""
        from ..utils.records import entry_from_csv
        e = entry_from_csv(jx_line)
        if e is None or e.type != "jx":
            return False
        vals = [float("nan") if v is None else float(v) for v in e.values]
        return self.eng.set_server_context(e.server, float(e.timestamp), vals, float(vm_load))

    NODE_METRICS = ("ranks", "batches", "lines", "events", "bytes", "tx", "tx_db", "released", "rollovers",
                    "alert_candidates", "alerts", "series")

    def node_metrics(self) -> Dict[str, float]:
        """Node-wide sums of the per-rank counters as of the last interval edge (one RCCL
        all-reduce per interval on the collective stream); empty before the first edge or when
        no fleet exchange is configured."""
        return dict(zip(self.NODE_METRICS, self.eng.node_metrics()))

    def metrics(self) -> Dict[str, Any]:
        m = self.eng.metrics()
        m.update({"join": self.eng.join_counters(), "series": self.eng.n_series(),
                  "device_bytes": self.eng.device_bytes()})
        return m
