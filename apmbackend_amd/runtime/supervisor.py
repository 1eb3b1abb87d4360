"""Supervisor tree: the ``apm_manager.js`` equivalent (reference :1-649).

* **modules** -- ``applicationManager.moduleSettings``; each entry starts one process (or, for
  ``"ranks"``, one process per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set: the
  torchrun-style launch of the per-GPU engine).  stdout/stderr go to
  ``<logDir>/<name>.start.log`` (Module.startProcess :329-356); children run in their own
  session so the supervisor's signals do not reach them.
* **stale processes** -- instead of killing every process whose command line matches a script
  name (Module.killExistingPIDs :274-295), each module records its PID in
  ``<stateDir>/<name>.pid``; a stale PID is terminated only if its /proc cmdline still carries the
  module's ``--apm-module=<name>`` marker.
* **restart** -- on exit: Grafana annotation + manager alert, restart after
  ``restartDelaySeconds`` (1 s), or ``crashLoopDelaySeconds`` (60 s) when it died less than
  ``crashLoopWindowSeconds`` (5 s) after starting (childExitCB :303-327).  A rank group restarts as
  a whole: RCCL communicators cannot lose a member, so the surviving ranks, given
  ``groupAbortGraceSeconds`` (5 s) to abort on their own (exit codes reported), are stopped first.
  **Elastic degrade**: a GPU whose rank keeps failing (``elasticMaxFailures`` within
  ``elasticWindowSeconds``) is retired and the group restarts at the next smaller world size
  (8 -> 4 -> 2 -> 1 by default), re-sharding the JVM hosts; see ``_elastic_degrade``.
* **monitoring** every ``inspectionFrequencySeconds`` aligned to the clock
  (monitorResourcesRecurs :514-530): liveness (kill(pid, 0)), per-module PSS/swap (native
  /proc/<pid>/smaps_rollup reader, the pid_stats.py equivalent) and HBM per process (KFD sysfs)
  against the module / global thresholds -> alert + ``requestGC`` (SIGUSR1) to the child
  (inspectModules :475-512); disk space of the app mount (inspectDiskSpace :397-427); queue depth
  when running with a broker (inspectQueues :429-453).
* **alerts** -- buffered ``"<date> ::: text"`` lines mailed every
  ``alertCollectionIntervalInSeconds`` with backoff up to ``maxCollectionIntervalInSeconds``
  (the reference compares against the undefined ``minCollectionIntervalInSeconds`` and so never
  backs off: quirk fixed);
* **log retention** -- every 12 h delete logs older than ``appLogRetentionDays``.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import shlex
import signal
import subprocess
import sys
import time
from typing import Any, Callable, Dict, List, Optional

from ..utils.config import ConfigWatcher, as_bool, read_apm_config
from . import logger as apmlog
from .notifier import Mailer, post_annotation

# exit status of a rank that stopped because a peer rank failed (runtime/service.py)
PEER_FAILURE_EXIT = 75
HUNG_RANK = -1000  # blame code of a rank still running after every peer aborted on it (never an exit code)

log = logging.getLogger("apm.manager")


def log_date(t: float) -> str:
    return _dt.datetime.fromtimestamp(t).strftime("%Y-%m-%d %H:%M:%S")


def pid_exists(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def proc_cmdline(pid: int) -> str:
    try:
        with open(f"/proc/{pid}/cmdline", "rb") as f:
            return f.read().replace(b"\0", b" ").decode(errors="replace")
    except OSError:
        return ""


def pid_mem_swap_mb(pid: int):
    """(PSS MiB, SwapPss MiB) -- the pid_stats.py -q -m numbers (native reader)."""
    try:
        from .. import _native
        pss, swap = _native.load(build_if_missing=False).pid_pss_swap(int(pid))
        if pss < 0:
            return None, None
        return pss / 2**20, max(swap, 0) / 2**20
    except Exception:
        from ..cli.pid_stats import pss_swap_bytes
        pss, swap = pss_swap_bytes(pid)
        return (None, None) if pss is None else (pss / 2**20, swap / 2**20)


def pid_vram_mb(pid: int) -> float:
    """HBM allocated by a process, from the KFD sysfs (sum over GPUs), 0 if unknown."""
    d = f"/sys/class/kfd/kfd/proc/{pid}"
    total = 0
    try:
        for name in os.listdir(d):
            if name.startswith("vram_"):
                with open(os.path.join(d, name)) as f:
                    total += int(f.read().strip() or 0)
    except OSError:
        return 0.0
    return total / 2**20


def disk_usage(path: str):
    st = os.statvfs(path)
    size = st.f_blocks * st.f_frsize / 2**30
    avail = st.f_bavail * st.f_frsize / 2**30
    used = (st.f_blocks - st.f_bfree) * st.f_frsize / 2**30
    pct = 100.0 * used / (used + avail) if used + avail else 0.0
    return size, used, avail, pct


class Proc:
    def __init__(self, name: str, argv: List[str], env: Dict[str, str], log_path: str, pid_path: str):
        self.name = name
        self.argv = argv
        self.env = env
        self.log_path = log_path
        self.pid_path = pid_path
        self.popen: Optional[subprocess.Popen] = None
        self.last_start = 0.0
        self.restart_at: Optional[float] = None
        self.restarts = 0

    @property
    def pid(self) -> Optional[int]:
        return self.popen.pid if self.popen else None

    def marker(self) -> str:
        return f"--apm-module={self.name}"

    def start(self, now: float):
        os.makedirs(os.path.dirname(self.log_path) or ".", exist_ok=True)
        out = open(self.log_path, "w")
        env = dict(os.environ)
        env.update(self.env)
        self.popen = subprocess.Popen(self.argv + [self.marker()], stdin=subprocess.DEVNULL, stdout=out,
                                      stderr=subprocess.STDOUT, env=env, start_new_session=True)
        out.close()
        self.last_start = now
        self.restart_at = None
        os.makedirs(os.path.dirname(self.pid_path) or ".", exist_ok=True)
        with open(self.pid_path, "w") as f:
            f.write(str(self.popen.pid))
        log.info("Child process started via PID: %d (%s)", self.popen.pid, self.name)

    def kill_stale(self):
        """killExistingPIDs: only the PID this module recorded, and only if it is still ours."""
        try:
            with open(self.pid_path) as f:
                pid = int(f.read().strip())
        except (OSError, ValueError):
            return None
        if pid_exists(pid) and self.marker() in proc_cmdline(pid):
            log.warning("Killing PID: %d (stale %s)", pid, self.name)
            try:
                os.kill(pid, signal.SIGTERM)
            except OSError:
                pass
            return pid
        return None

    def stop(self, timeout: float = 10.0):
        if self.popen and self.popen.poll() is None:
            self.popen.terminate()
            try:
                self.popen.wait(timeout)
            except subprocess.TimeoutExpired:
                self.popen.kill()
                self.popen.wait(5)

    def poll(self) -> Optional[int]:
        return self.popen.poll() if self.popen else None


class Module:
    """One moduleSettings entry: a single process or a group of GPU ranks."""

    def __init__(self, setting: Dict[str, Any], mcfg: Dict[str, Any], cfg: Dict[str, Any], state_dir: str,
                 config_path: Optional[str]):
        self.s = setting
        self.name = setting.get("name") or os.path.basename(setting.get("relativePath", "module")).split(".")[0]
        if "module" in setting:
            base = [sys.executable, "-m", setting["module"]]
        else:
            base = [sys.executable, os.path.join(cfg.get("appDirectory", "."), setting["relativePath"])]
        argv = base + list(mcfg.get("sharedOpts", [])) + list(setting.get("args", []))
        if config_path and setting.get("passConfig", True):
            argv += ["--config", config_path]
        ranks = setting.get("ranks", 0)
        if ranks == "auto":
            ranks = int(os.environ.get("APM_GPUS", "0")) or _gpu_count()
        self.ranks = int(ranks or 0)
        log_dir = cfg.get("logDir", "/tmp/apm/logs")
        self.argv, self.log_dir, self.state_dir = argv, log_dir, state_dir
        self.procs: List[Proc] = []
        # elastic rank group: the GPUs it may use, the ones retired after repeated failures, the
        # failure times per GPU, and the generation (bumped at every world-size change)
        self.devices: List[int] = [int(d) for d in setting.get("devices", [])] or list(range(self.ranks))
        self.explicit_devices = bool(setting.get("devices"))
        self.bad_devices: set = set()
        self.dev_failures: Dict[int, List[float]] = {}
        self.generation = 0
        if self.ranks:
            self.build_ranks(self.ranks, self.devices[:self.ranks])
        else:
            self.procs.append(Proc(self.name, argv, dict(setting.get("env", {})),
                                   os.path.join(log_dir, f"{self.name}.start.log"),
                                   os.path.join(state_dir, f"{self.name}.pid")))

    def build_ranks(self, world: int, devices: List[int]):
        """(Re)create the rank processes: one per GPU in `devices`, WORLD_SIZE = world."""
        self.ranks = world
        self.active_devices = list(devices)
        port = int(self.s.get("masterPort", 29512)) + self.generation  # fresh rendezvous per generation
        self.procs = []
        for r in range(world):
            env = {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(world),
                   "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "APM_DEVICE": str(devices[r]),
                   "APM_ELASTIC_GENERATION": str(self.generation)}
            if self.explicit_devices or self.generation:
                # LOCAL_RANK r indexes the visible list, so rank r drives physical GPU devices[r]
                env["HIP_VISIBLE_DEVICES"] = ",".join(str(d) for d in devices)
            self.procs.append(Proc(f"{self.name}.rank{r}", self.argv, env,
                                   os.path.join(self.log_dir, f"{self.name}.rank{r}.start.log"),
                                   os.path.join(self.state_dir, f"{self.name}.rank{r}.pid")))

    def device_of(self, p: "Proc") -> Optional[int]:
        v = p.env.get("APM_DEVICE")
        return int(v) if v is not None else None

    def setting(self, key: str, mcfg: Dict[str, Any]):
        """getModuleSetting (:455-464): module value if set (0 counts), else the global one."""
        v = self.s.get(key)
        return v if (v or v == 0) and v is not None else mcfg.get(key)


def _gpu_count() -> int:
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


class Supervisor:
    def __init__(self, cfg: Optional[Dict[str, Any]] = None, config_path: Optional[str] = None,
                 clock: Callable[[], float] = time.time, mailer: Optional[Mailer] = None, annotate=post_annotation):
        self.cfg = cfg if cfg is not None else read_apm_config(config_path, first_run=True)
        self.config_path = config_path or self.cfg.get("apmConfigFilePath")
        self.m = self.cfg["applicationManager"]
        self.clock = clock
        self.mailer = mailer or Mailer(outbox=os.path.join(self.cfg.get("logDir", "/tmp/apm/logs"), "outbox"))
        self.annotate = annotate
        apmlog.set_global_logger(self.cfg.get("logDir"), self.m.get("logFilePrefix", "apm_manager"))
        self.state_dir = self.m.get("stateDir", os.path.join(os.path.dirname(self.cfg.get("logDir", "/tmp/apm/logs")),
                                                             "state"))
        self.modules = [Module(s, self.m, self.cfg, self.state_dir, self.config_path)
                        for s in self.m.get("moduleSettings", []) if as_bool(s.get("enabled", True))]
        self.alert_buffer: List[str] = []
        self.alert_interval = float(self.m.get("alertCollectionIntervalInSeconds", 60))
        self.next_alert = clock() + self.alert_interval
        self.next_inspect = clock()
        self.next_prune = clock()
        self.emails = 0
        self.gc_requests: List[str] = []
        self._hbm_gc_at: Dict[int, float] = {}  # pid -> last HBM-triggered requestGC
        self._stop = False
        self.watcher = (ConfigWatcher(self.cfg, self._reload, ["apmConfigFilePath", "logDir",
                                                               "applicationManager.moduleSettings"])
                        if self.config_path else None)

    # ------------------------------------------------------------------ alerts
    def add_alert(self, text: str):
        self.alert_buffer.append(f"{log_date(self.clock())} ::: {text}")
        log.warning(text)

    def send_alerts(self) -> bool:
        now = self.clock()
        if now < self.next_alert:
            return False
        sent = False
        interval = float(self.m.get("alertCollectionIntervalInSeconds", 60))
        if self.alert_buffer:
            interval = self.alert_interval
            if as_bool(self.m.get("increaseCollectionIntervalAfterAlert", False)) and \
                    interval < float(self.m.get("maxCollectionIntervalInSeconds", 3840)):
                interval *= 2
            body = "".join(f"Alert: {json.dumps(a)}\n" for a in self.alert_buffer)
            body += f"\n\nCooldown until further alerts are sent: {int(interval)} seconds\n"
            if as_bool(self.m.get("emailsEnabled", True)):
                try:
                    self.mailer.send(self.m.get("fromEmail", "apm@localhost"), self.m.get("emailList", ""),
                                     "APM Manager Alerts", f"<pre>{body}</pre>")
                    self.emails += 1
                    sent = True
                except Exception as e:
                    log.error("manager e-mail failed: %s", e)
            self.alert_buffer = []
        self.alert_interval = interval
        self.next_alert = now + interval
        return sent

    # ------------------------------------------------------------------ lifecycle
    def start_all(self):
        self.annotate(self.cfg.get("grafana", {}), "Restarting all modules", ["maintenance"])
        for mod in self.modules:
            for p in mod.procs:
                p.kill_stale()
        now = self.clock()
        for mod in self.modules:
            for p in mod.procs:
                p.start(now)
        log.info("Processes started.")

    def stop_all(self):
        for mod in self.modules:
            for p in mod.procs:
                p.stop()

    def _elastic_degrade(self, mod: Module, p: Proc, code: int, now: float) -> bool:
        """Elastic rank group: a GPU whose rank failed `elasticMaxFailures` times
        within `elasticWindowSeconds` is retired and the group restarts at the largest world size
        the healthy GPUs allow (powers of two by default: 8 -> 4 -> 2 -> 1).  The new ranks shard
        the JVM hosts over the new world; each resumes the tails of the files it now owns from the
        old ranks' offsets (no data gap), and the series that moved rank start a fresh history."""
        flag = mod.setting("elasticDegrade", self.m)
        if not mod.ranks or code in (0, PEER_FAILURE_EXIT) or (flag is not None and not as_bool(flag)):
            return False
        dev = mod.device_of(p)
        if dev is None:
            return False
        window = float(mod.setting("elasticWindowSeconds", self.m) or 900)
        limit = int(mod.setting("elasticMaxFailures", self.m) or 3)
        hist = [t for t in mod.dev_failures.get(dev, []) if now - t <= window] + [now]
        mod.dev_failures[dev] = hist
        if len(hist) < limit:
            return False
        mod.bad_devices.add(dev)
        healthy = [d for d in mod.devices if d not in mod.bad_devices]
        world = len(healthy)
        if str(mod.setting("elasticWorldSizes", self.m) or "pow2") == "pow2" and world:
            world = 1 << (world.bit_length() - 1)
        old_world = mod.ranks
        for q in mod.procs:
            q.stop()
        if world == 0:
            mod.procs = []
            self.add_alert(f"Rank group {mod.name}: every GPU retired (last: {dev}); not restarting")
            return True
        mod.generation += 1
        mod.build_ranks(world, healthy[:world])
        delay = float(self.m.get("restartDelaySeconds", 1))
        for q in mod.procs:
            q.restart_at = now + delay
        text = (f"Rank group {mod.name} degraded from {old_world} to {world} GPUs: GPU {dev} failed "
                f"{len(hist)} times in {int(window)} s (generation {mod.generation}, GPUs {healthy[:world]})")
        self.annotate(self.cfg.get("grafana", {}), text, ["maintenance"])
        self.add_alert(text)
        return True

    def _hung_peer(self, mod: Module, p: Proc) -> Optional[Proc]:
        """A survivor exited PEER_FAILURE_EXIT: some peer stopped answering.  If that peer died,
        it exits with its own code within the grace period and check_children blames it.  If it
        hangs instead (a wedged GPU never lets the process exit), it is the one rank still running
        once every other peer has exited PEER_FAILURE_EXIT: that rank's GPU is the one to blame."""
        grace_end = time.monotonic() + float(self.m.get("groupAbortGraceSeconds", 5))
        peers = [q for q in mod.procs if q is not p and q.restart_at is None]
        while True:
            codes = [(q, q.poll()) for q in peers]
            if any(c not in (None, 0, PEER_FAILURE_EXIT) for _, c in codes):
                return None  # a peer failed on its own: that exit carries the blame
            running = [q for q, c in codes if c is None]
            if not running:
                return None
            if len(running) == 1 and len(peers) > 1 and time.monotonic() >= grace_end:
                return running[0]
            if time.monotonic() >= grace_end:
                return running[0] if len(running) == len(peers) == 1 else None
            time.sleep(0.05)

    def _on_exit(self, mod: Module, p: Proc, code: int, now: float):
        if p not in mod.procs:  # a rank retired by an elastic restart
            return
        log.error("Child exited: code:%s module: %s", code, p.name)
        self.annotate(self.cfg.get("grafana", {}), f"Module exited: {p.name}", ["maintenance"])
        self.add_alert(f"Child module exited: code:{code} module: {p.name}")
        quick = now - p.last_start < float(self.m.get("crashLoopWindowSeconds", 5))
        delay = float(self.m.get("crashLoopDelaySeconds", 60)) if quick else float(self.m.get("restartDelaySeconds", 1))
        if quick:
            log.warning("Time since last restart is under %ss: crash loop suspected, waiting %ss",
                        self.m.get("crashLoopWindowSeconds", 5), delay)
        blame, bcode = p, code
        if mod.ranks and code == PEER_FAILURE_EXIT:
            hung = self._hung_peer(mod, p)
            if hung is not None:
                log.error("Rank %s still running after its peers aborted on it: blamed as hung", hung.name)
                self.add_alert(f"Rank {hung.name} hung (its peers aborted their collectives on it)")
                blame, bcode = hung, HUNG_RANK
        if self._elastic_degrade(mod, blame, bcode, now):
            return
        targets = mod.procs if mod.ranks else [p]
        # A rank group restarts as a whole.  The survivors are expected to notice the dead peer on
        # their own (collective watchdog / peer EOF), abort and exit non-zero: give them
        # `groupAbortGraceSeconds` to do so (their exit codes are reported), then terminate them.
        grace_end = time.monotonic() + float(self.m.get("groupAbortGraceSeconds", 5))
        for q in targets:
            if q is not p and q.restart_at is None:
                qc = q.poll()
                while qc is None and time.monotonic() < grace_end:
                    time.sleep(0.05)
                    qc = q.poll()
                if qc is not None:
                    log.error("Child exited: code:%s module: %s (rank group peer)", qc, q.name)
                    self.add_alert(f"Child module exited: code:{qc} module: {q.name}")
                else:
                    q.stop()
            q.restart_at = now + delay

    def check_children(self):
        now = self.clock()
        for mod in self.modules:
            if mod.ranks:
                # a rank group: when several ranks have exited since the last poll, the one that
                # failed first is the one whose exit is not a survivor's PEER_FAILURE_EXIT (the
                # others aborted their collectives because it died) -- that rank's GPU is blamed
                exited = [(p, p.poll()) for p in mod.procs if p.restart_at is None]
                exited = [(p, c) for p, c in exited if c is not None]
                if exited:
                    first = next(((p, c) for p, c in exited if c not in (0, PEER_FAILURE_EXIT)), exited[0])
                    self._on_exit(mod, first[0], first[1], now)
            for p in mod.procs:
                if p.restart_at is not None:
                    if now >= p.restart_at:
                        p.restarts += 1
                        p.start(now)
                        self.add_alert(f"Process restarted via startProcess: {p.name}")
                    continue
                code = p.poll()
                if code is not None:
                    self._on_exit(mod, p, code, now)

    # ------------------------------------------------------------------ monitoring
    def inspect(self):
        broker_up = self.inspect_broker()
        self.inspect_disk()
        if broker_up:
            self.inspect_queues()
        self.inspect_modules()

    def inspect_disk(self):
        app = self.cfg.get("appDirectory", "/")
        parts = os.path.abspath(app).split(os.sep)
        mount = os.sep + parts[1] if len(parts) > 1 and parts[1] else os.sep
        if not os.path.exists(mount):
            return
        size, used, avail, pct = disk_usage(mount)
        if avail <= float(self.m.get("diskSpaceGBAvailableThreshold", 100)):
            self.add_alert(f"Available disk space is low on mount: {mount} - Size: {size:.0f} GB, Used: {used:.0f} GB,"
                           f" Available: {avail:.0f} GB, PercentUsed: {pct:.0f}%")
        if pct > float(self.m.get("diskSpacePercentageUsedThreshold", 80)):
            self.add_alert(f"Disk space percentage used is high on mount: {mount} - Size: {size:.0f} GB, Used: "
                           f"{used:.0f} GB, Available: {avail:.0f} GB, PercentUsed: {pct:.0f}%")

    # ---- broker supervision (apm_manager.js rabbitMQIsRunning / startRabbitMQ :134-155,
    # inspectQueues :429-453, monitorResourcesRecurs :517-521)
    def _uses_broker(self) -> bool:
        g = self.cfg.get("gpu", {})
        return g.get("outputMode", "inproc") == "amqp" or g.get("inputMode", "logs") == "transactions"

    def _rabbitmqctl(self) -> Optional[str]:
        sbin = self.m.get("rabbitSbinPath")
        p = os.path.join(sbin, "rabbitmqctl") if sbin else None
        return p if p and os.path.exists(p) else None

    def broker_is_running(self) -> bool:
        ctl = self._rabbitmqctl()
        if ctl:
            try:
                return subprocess.run([ctl, "status"], capture_output=True, timeout=30).returncode == 0
            except (OSError, subprocess.TimeoutExpired):
                return False
        try:  # no RabbitMQ tooling (our own broker, or a remote one): an AMQP handshake decides
            from .amqp import Connection
            Connection(self.cfg["amqpConnectionString"], timeout=3).close()
            return True
        except Exception:
            return False

    def start_broker(self):
        log.info("Attempting to start the message broker...")
        sbin = self.m.get("rabbitSbinPath")
        server = os.path.join(sbin, "rabbitmq-server") if sbin else None
        try:
            if server and os.path.exists(server):
                out = subprocess.run([server, "-detached"], capture_output=True, timeout=60)
                log.info("RabbitMQ started! Output: %s", out.stdout.decode(errors="replace").strip())
            elif self.m.get("brokerCommand"):
                # a configured broker command (e.g. python -m apmbackend_amd.runtime.amqp_broker),
                # started detached like rabbitmq-server -detached
                argv = shlex.split(self.m["brokerCommand"])
                with open(os.path.join(self.cfg.get("logDir") or ".", "broker.start.log"), "a") as lf:
                    subprocess.Popen(argv, stdout=lf, stderr=subprocess.STDOUT, start_new_session=True)
            else:
                self.add_alert("Broker is down and neither applicationManager.rabbitSbinPath nor brokerCommand "
                               "is configured to start it")
                return
        except Exception as e:
            log.error("Start of the broker threw an error: %s", e)
            self.add_alert(f"Start of RabbitMQ threw an error: {e}")

    def inspect_broker(self) -> bool:
        """Liveness + auto-start; True when the broker is up."""
        if not self._uses_broker():
            return True
        now = self.clock()
        if self.broker_is_running():
            return True
        if now < getattr(self, "_broker_grace_until", 0.0):
            return False  # a start is in progress (the reference sleeps 30 s here)
        self.add_alert("RabbitMQ is down, attempting to restart it.")
        self.start_broker()
        self._broker_grace_until = now + float(self.m.get("brokerStartGraceSeconds", 30))
        return False

    def _queue_rows(self):
        """(name, messages, memory MB or None) per queue."""
        ctl = self._rabbitmqctl()
        if ctl:
            out = subprocess.run([ctl, "list_queues", "--quiet", "--no-table-headers", "name", "messages_ram",
                                  "message_bytes_ram", "messages_persistent", "message_bytes_persistent", "memory"],
                                 capture_output=True, timeout=60)
            if out.returncode != 0:
                raise RuntimeError(out.stderr.decode(errors="replace").strip())
            rows = []
            for line in out.stdout.decode(errors="replace").splitlines():
                f = line.split()
                if len(f) < 6:
                    continue
                rows.append((f[0], int(f[1]) + int(f[3]), int(f[5]) / 1024.0 / 1024.0))
            return rows
        from .amqp import Connection
        c = Connection(self.cfg["amqpConnectionString"], timeout=3)
        try:
            names = [self.cfg.get("dbInsertQueue", "db_insert"),
                     self.cfg["streamParseTransactions"].get("outQueue", "transactions"),
                     self.cfg["streamCalcStats"].get("outQueue", "stats"),
                     self.cfg["streamCalcZScore"].get("outQueue", "z_score"),
                     self.cfg.get("gpu", {}).get("fleetQueue", "fleet_baseline")]
            rows = []
            for q in dict.fromkeys(names):
                _n, msgs, _c = c.queue_declare(q, durable=True)
                rows.append((q, msgs, None))
            return rows
        finally:
            c.close()

    def inspect_queues(self):
        if not self._uses_broker():
            return
        try:
            rows = self._queue_rows()
        except Exception as e:
            self.add_alert(f"Could not inspect queues via rabbit controller: {e}")
            return
        cnt_thr = float(self.m.get("queueMessageAlertThreshold", 1e6))
        mem_thr = float(self.m.get("queueMemoryAlertThreshold", 1e9))
        for name, msgs, mem_mb in rows:
            log.debug("QUEUE: %s Count: %d MemMb: %s", name, msgs, "-" if mem_mb is None else f"{mem_mb:.1f}")
            if msgs > cnt_thr:
                self.add_alert(f"Queue exceeded the message count threshold - Queue: {name} Threshold: "
                               f"{self.m.get('queueMessageAlertThreshold')} MessageCount: {msgs}")
            if mem_mb is not None and mem_mb > mem_thr:
                self.add_alert(f"Queue exceeded the memory threshold - Queue: {name} Threshold: "
                               f"{self.m.get('queueMemoryAlertThreshold')} MemoryUsed(Mb): {mem_mb:.1f}")

    def inspect_modules(self):
        for mod in self.modules:
            for p in mod.procs:
                if p.restart_at is not None or p.pid is None:
                    continue
                if not pid_exists(p.pid) or p.poll() is not None:
                    continue  # handled by check_children
                mem, swap = pid_mem_swap_mb(p.pid)
                if mem is None:
                    continue
                trigger = False
                mthr = float(mod.setting("moduleMemoryAlertThreshold", self.m) or 1e18)
                if mem > mthr:
                    self.add_alert(f"Child module exceeded the memory threshold - Module: {p.name} Threshold(Mb): "
                                   f"{mthr} MemoryUsed(Mb): {mem:.1f}")
                    trigger = True
                sthr = float(mod.setting("moduleSwapAlertThreshold", self.m) or 1e18)
                if swap > sthr:
                    self.add_alert(f"Child module exceeded the swap threshold - Module: {p.name} Threshold(Mb): "
                                   f"{sthr} SwapUsed(Mb): {swap:.1f}")
                    trigger = True
                gthr = mod.setting("moduleGpuMemoryAlertThreshold", self.m)
                vram = pid_vram_mb(p.pid)
                if gthr and vram > float(gthr):
                    self.add_alert(f"Child module exceeded the GPU memory threshold - Module: {p.name} "
                                   f"Threshold(Mb): {gthr} HBMUsed(Mb): {vram:.1f}")
                    # the child's requestGC trims its grow-only device memory; each trim flushes
                    # the engine and rebuilds the join table, so an HBM-only trigger is sent at most
                    # once per `gpuGcMinIntervalSeconds` (the RSS / swap triggers keep the
                    # reference's every-inspection rule, apm_manager.js:485-508)
                    last = self._hbm_gc_at.get(p.pid)
                    gap = float(mod.setting("gpuGcMinIntervalSeconds", self.m) or 600)
                    if trigger or last is None or self.clock() - last >= gap:
                        trigger = True
                        self._hbm_gc_at[p.pid] = self.clock()
                if trigger:
                    log.info("Sending garbage collection request to module: %s", p.name)
                    self.gc_requests.append(p.name)
                    try:
                        os.kill(p.pid, signal.SIGUSR1)  # requestGC
                    except OSError:
                        pass

    def _reload(self, cfg):
        self.cfg = cfg
        self.m = cfg["applicationManager"]
        apmlog.set_global_logger(cfg.get("logDir"), self.m.get("logFilePrefix", "apm_manager"))

    # ------------------------------------------------------------------ main loop
    def tick(self):
        now = self.clock()
        self.check_children()
        if now >= self.next_inspect:
            self.inspect()
            freq = float(self.m.get("inspectionFrequencySeconds", 60))
            self.next_inspect = now + (freq - (int(now) % 60) % freq if freq < 60 else freq)
        if now >= self.next_prune:
            apmlog.prune_logs(self.cfg.get("logDir", "/tmp/apm/logs"), int(self.m.get("appLogRetentionDays", 7)), now)
            self.next_prune = now + 12 * 3600
        self.send_alerts()
        if self.watcher is not None:
            try:
                self.watcher.check_once()
            except Exception as e:
                log.error("config reload failed: %s", e)

    def run(self, tick_s: float = 0.5, until: Optional[Callable[[], bool]] = None):
        self.start_all()
        try:
            while not self._stop:
                self.tick()
                if until is not None and until():
                    break
                time.sleep(tick_s)
        finally:
            self.stop_all()

    def stop(self, *a):
        self._stop = True


def main(argv=None):  # pragma: no cover - process entry point
    import argparse
    ap = argparse.ArgumentParser(description="apmbackend_amd supervisor (apm_manager equivalent)")
    ap.add_argument("--config", default=None)
    a = ap.parse_args(argv)
    sup = Supervisor(config_path=a.config)
    signal.signal(signal.SIGTERM, sup.stop)
    signal.signal(signal.SIGINT, sup.stop)
    sup.run()


if __name__ == "__main__":  # pragma: no cover
    main()
