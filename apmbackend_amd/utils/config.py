"""APM config loader, compatible with the reference ``config/apm_config.json``.

Behaviour parity (reference ``util_methods.js:253-348``):

* ``json_strip`` removes ``[^:]//.*`` (global), *including the character before* ``//``
  (quirk Q20: ``"a": 1,// c`` loses its comma, ``amqp://h`` survives).
* ``read_apm_config`` returns ``None`` on a JSON error (caller keeps the previous config),
  and adds ``apmConfigFilePath``.
* ``ConfigWatcher`` polls the file (md5 + size, 500 ms debounce, like ``watchAPMConfig``),
  logs a warning for every changed key in ``restart_required`` and invokes the callback.

New keys live under a ``gpu`` section (see ``GPU_DEFAULTS``); unknown keys there are
reported, never silently ignored.
"""
from __future__ import annotations

import copy
import hashlib
import json
import logging
import os
import re
import threading
import time
from typing import Any, Callable, Dict, Iterable, List, Optional

log = logging.getLogger("apm.config")

_STRIP_RE = re.compile(r"[^:]//(.*)")

DEFAULT_CONFIG_PATH = os.path.join(
    os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
    "config", "apm_config.json")

# New section: everything the MI355X engine needs that the reference did not have.
GPU_DEFAULTS: Dict[str, Any] = {
    "device": 0,                      # local device index (rank's LOCAL_RANK overrides)
    "maxSeries": 1 << 17,             # (server, service) series capacity per GPU
    "maxServices": 1 << 16,           # distinct service-name capacity
    "maxServers": 1024,
    "bucketCellCapacity": 16,         # samples per (series, 10 s bucket) kept inline
    "bucketRingSlots": 0,             # bucket ring slots (0 = window + buffer + 1, at least 40; grows on reload)
    "bucketOverflowCapacity": 1 << 22,  # spill area for hot series
    "batchBytes": 32 << 20,           # bytes of raw log per ingest batch
    "maxLinesPerBatch": 1 << 20,
    "ringDtype": "float64",          # z-score history ring: float64 | float32 | bfloat16
    "pinThreads": False,             # pin join workers / stats / output lanes to GPU-local cores
    "zscoreMeanMode": "rolling",      # rolling (O(1) compensated) | exact (sequential, JS-bit-exact)
    "zscoreSigma": "sqrt_mean",       # sqrt_mean (reference quirk Q1) | stddev (true sigma)
    "exactRecomputeEveryIntervals": 360,
    "emulateOverrideAliasing": False,  # quirk Q4 (per-service overrides leak into defaults)
    "alertClock": "wall",             # wall (reference: stream_process_alerts.js:437,449-467) | entry (log time: replay)
    "cooldownKey": "service",         # service (reference Q7) | series
    "recordTtlSeconds": 120,          # recordCache stdTTL (stream_parse_transactions.js:215)
    "acctTtlSeconds": 120,            # acctCache stdTTL (:213)
    "needTtlSeconds": 30,             # needNumRecordCache stdTTL (:218)
    "timezone": "local",              # tz for 'YYYY-MM-DD HH:MM:SS,mmm' timestamps
    "fleetBaseline": True,            # RCCL all-reduce of per-service moments + lock-step clocks
    "joinThreads": 0,                 # host join worker threads (0 = auto; joinOnDevice false)
    "joinOnDevice": True,             # K4/K6 join + tx encoding on the GPU (false: host join workers)
    "joinTableSlots": 1 << 21,        # GPU join key table (logId keys, 128 B per slot) -- grows
    "needArenaEntries": 1 << 18,      # GPU needNumRecordCache entries (512 B each) -- grows
    "joinChainBlocks": 0,             # GPU join overflow chains (256 B blocks; 0 = auto) -- grows
    "txTextRingMB": 4096,             # HBM ring holding pending (unreleased) tx lines
    "maxRawServices": 1 << 18,        # distinct (server, raw service name) pairs
    "collectiveTimeoutSeconds": 300,  # RCCL watchdog: abort + exit when a collective hangs this long
    "collectiveInitTimeoutSeconds": 120,  # RCCL communicator init deadline (a peer that never joins -> clear error)
    "collectiveBackend": "rccl",      # node-wide exchanges: rccl (xGMI) or host (TCP via rank 0, ranks sharing a GPU)
    "checkpointDir": "",              # binary engine checkpoints (+ tail offsets) per rank
    "checkpointEverySeconds": 60,
    "checkpointStageMB": 2048,        # HBM staging of a checkpoint's z-score ring rows (larger bases stream)
    "importReferenceResume": False,   # seed a fresh engine from the reference's JSON resume files
    "outputMode": "inproc",           # inproc (DB insert stage in-process) | amqp (queue bridge) | none
    "bridgeQueues": [],               # amqp mode: also mirror "transactions" / "stats"
    "tailFromStart": False,           # File::Tail starts at EOF; true reads existing content
    "serverRollup": False,            # K14 "sx" stream: per-JVM rollup fused with JMX / VM gauges
    "fuseJmx": False,                 # JMX poller inside the engine process feeding K14
    "syntheticJmx": False,            # use the synthetic WildFly CLI (tests / benchmarks)
    "logFilePrefix": "apm_engine",
    "faultInjection": {},             # {"rank", "dropBatchEvery", "duplicateBatchEvery", "exitAtBatch"}
}

_BOOL_STRINGS = {"true": True, "false": False, "1": True, "0": False, "yes": True, "no": False}


def json_strip(txt: str) -> str:
    """The reference JSONstrip (util_methods.js:265-268), including its quirk."""
    return _STRIP_RE.sub("", txt)


def parse_config_text(txt: str) -> Dict[str, Any]:
    return json.loads(json_strip(txt))


def read_apm_config(path: Optional[str] = None, first_run: bool = False) -> Optional[Dict[str, Any]]:
    path = os.path.abspath(path or os.environ.get("APM_CONFIG", DEFAULT_CONFIG_PATH))
    if not os.path.exists(path):
        raise FileNotFoundError(f"APM config file does not exist: {path}")
    with open(path, "r", encoding="utf-8") as fh:
        content = fh.read()
    try:
        cfg = parse_config_text(content)
    except json.JSONDecodeError as e:
        log.error("Could not parse JSON content from APM config file %s: %s", path, e)
        return None
    cfg["apmConfigFilePath"] = path
    cfg.setdefault("gpu", {})
    unknown = set(cfg["gpu"]) - set(GPU_DEFAULTS)
    for k in sorted(unknown):
        log.warning("unknown key gpu.%s in %s (ignored)", k, path)
    merged = dict(GPU_DEFAULTS)
    merged.update({k: v for k, v in cfg["gpu"].items() if k in GPU_DEFAULTS})
    cfg["gpu"] = merged
    return cfg


def resolve(path: str, obj: Any, sep: str = ".") -> Any:
    """``resolve`` from util_methods.js:248-251."""
    cur = obj
    for p in path.split(sep):
        if cur is None:
            return None
        if isinstance(cur, dict):
            cur = cur.get(p)
        else:
            return None
    return cur


def as_bool(v: Any) -> bool:
    """Fix for quirk Q8: ``"false"`` disables (the reference treated any string as true)."""
    if isinstance(v, str):
        return _BOOL_STRINGS.get(v.strip().lower(), bool(v))
    return bool(v)


def default_config(replay: bool = False) -> Dict[str, Any]:
    """The shipped config.  ``replay=True`` switches the alert clock to log time
    (``gpu.alertClock = "entry"``): alert timestamps and cooldowns then depend only on the input,
    which is what replays, benchmarks and oracle comparisons need.  The shipped default is the
    reference's wall clock."""
    cfg = read_apm_config(DEFAULT_CONFIG_PATH)
    assert cfg is not None
    if replay:
        cfg["gpu"]["alertClock"] = "entry"
    return cfg


def overrides_for(cfg: Dict[str, Any], section: str) -> Dict[str, Any]:
    return ((cfg.get(section) or {}).get("overrides") or {}).get("services") or {}


class ConfigWatcher:
    """Poll-based equivalent of ``watchAPMConfig`` (md5 + size + 500 ms debounce)."""

    def __init__(self, cfg: Dict[str, Any], callback: Callable[[Dict[str, Any]], None],
                 restart_required: Iterable[str] = (), poll_s: float = 0.5):
        self.cfg = cfg
        self.path = cfg["apmConfigFilePath"]
        self.callback = callback
        self.restart_required = list(restart_required)
        self.poll_s = poll_s
        self._prev = self._digest()
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def _digest(self):
        try:
            with open(self.path, "rb") as fh:
                b = fh.read()
            return hashlib.md5(b).hexdigest(), len(b)
        except OSError:
            return None

    def check_once(self) -> bool:
        cur = self._digest()
        if cur is None or cur == self._prev:
            return False
        time.sleep(0.5 if self.poll_s >= 0.5 else 0)  # let the file settle (debounce)
        cur = self._digest()
        self._prev = cur
        new = read_apm_config(self.path)
        if new is None:
            log.warning("config JSON could not be processed; keeping the previous config")
            return False
        for var in self.restart_required:
            old_v, new_v = resolve(var, self.cfg), resolve(var, new)
            if json.dumps(old_v, sort_keys=True) != json.dumps(new_v, sort_keys=True):
                log.warning("%s was changed on settings reload, but this will not take effect "
                            "without a restart.", var)
        self.cfg = new
        self.callback(new)
        return True

    def _run(self):
        while not self._stop.wait(self.poll_s):
            try:
                self.check_once()
            except Exception as e:  # pragma: no cover - defensive
                log.error("config watcher error: %s", e)

    def start(self) -> "ConfigWatcher":
        self._th = threading.Thread(target=self._run, name="apm-config-watch", daemon=True)
        self._th.start()
        return self

    def stop(self):
        self._stop.set()


def zscore_lag_settings(cfg: Dict[str, Any], service: str,
                        emulate_aliasing: bool = False) -> List[Dict[str, Any]]:
    """Per-service z-score settings (stream_calc_z_score.js:106-132).

    With ``emulate_aliasing`` the reference bug Q4 is reproduced: the override is written
    into ``cfg['streamCalcZScore']['defaults']`` itself, so it leaks to later services.
    Q5 (an override of 0 is ignored because it is falsy) is kept in both modes only when
    emulating; otherwise an explicit 0 is honoured.
    """
    zc = cfg["streamCalcZScore"]
    defaults = zc["defaults"]
    settings = defaults if emulate_aliasing else copy.deepcopy(defaults)
    ovr = ((zc.get("overrides") or {}).get("services") or {}).get(service)
    if ovr:
        for idx, el in enumerate(settings):
            for lag, vals in ovr.items():
                if str(el["LAG"]) == str(lag) or _num_eq(el["LAG"], lag):
                    if emulate_aliasing:
                        if vals.get("THRESHOLD"):
                            settings[idx]["THRESHOLD"] = vals["THRESHOLD"]
                        if vals.get("INFLUENCE"):
                            settings[idx]["INFLUENCE"] = vals["INFLUENCE"]
                    else:
                        if vals.get("THRESHOLD") is not None:
                            settings[idx]["THRESHOLD"] = vals["THRESHOLD"]
                        if vals.get("INFLUENCE") is not None:
                            settings[idx]["INFLUENCE"] = vals["INFLUENCE"]
    return settings


def _num_eq(a, b) -> bool:
    try:
        return float(a) == float(b)
    except (TypeError, ValueError):
        return False
