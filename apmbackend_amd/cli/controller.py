"""Controller CLI: ``start | stop | restart | status`` of the supervisor (reference
``controller.sh:1-75``).

``start`` launches ``python -m apmbackend_amd.runtime.supervisor`` detached (own session,
output to ``<logDir>/apm_manager.start.log``) unless one is already running; ``stop`` sends
SIGTERM, waits, then SIGKILL, and mails the manager list if the process would not die.  The
running manager is identified by the PID file ``<stateDir>/apm_manager.pid`` *and* its command
line (never by matching process names).

Usage: python -m apmbackend_amd.cli.controller [--config PATH] {start,stop,restart,status} [quiet]
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

from ..runtime.supervisor import pid_exists, proc_cmdline
from ..utils.config import read_apm_config

MARKER = "apmbackend_amd.runtime.supervisor"


def _paths(cfg):
    log_dir = cfg.get("logDir", "/tmp/apm/logs")
    state = cfg["applicationManager"].get("stateDir", os.path.join(os.path.dirname(log_dir), "state"))
    return log_dir, state, os.path.join(state, "apm_manager.pid")


def running_pid(cfg):
    _, _, pidfile = _paths(cfg)
    try:
        pid = int(open(pidfile).read().strip())
    except (OSError, ValueError):
        return None
    return pid if pid_exists(pid) and MARKER in proc_cmdline(pid) else None


def start(cfg, config_path, quiet=False) -> int:
    pid = running_pid(cfg)
    if pid:
        if not quiet:
            print(f"APM manager already running (pid {pid})")
        return 0
    log_dir, state, pidfile = _paths(cfg)
    os.makedirs(log_dir, exist_ok=True)
    os.makedirs(state, exist_ok=True)
    argv = [sys.executable, "-m", MARKER]
    if config_path:
        argv += ["--config", os.path.abspath(config_path)]
    with open(os.path.join(log_dir, "apm_manager.start.log"), "a") as out:
        p = subprocess.Popen(argv, stdin=subprocess.DEVNULL, stdout=out, stderr=subprocess.STDOUT,
                             start_new_session=True)
    with open(pidfile, "w") as f:
        f.write(str(p.pid))
    if not quiet:
        print(f"APM manager started (pid {p.pid})")
    return 0


def stop(cfg, quiet=False, wait_s=30.0) -> int:
    pid = running_pid(cfg)
    if not pid:
        if not quiet:
            print("APM manager is not running")
        return 0
    os.kill(pid, signal.SIGTERM)
    t0 = time.time()
    while time.time() - t0 < wait_s and pid_exists(pid) and MARKER in proc_cmdline(pid):
        time.sleep(0.2)
    if pid_exists(pid) and MARKER in proc_cmdline(pid):
        os.kill(pid, signal.SIGKILL)
        time.sleep(1)
        if pid_exists(pid) and MARKER in proc_cmdline(pid):
            from ..runtime.notifier import Mailer
            m = cfg["applicationManager"]
            Mailer().send(m.get("fromEmail", "apm@localhost"), m.get("emailList", ""), "APM controller",
                          f"<pre>could not stop the APM manager (pid {pid})</pre>")
            print(f"could not stop pid {pid}")
            return 1
    if not quiet:
        print(f"APM manager stopped (pid {pid})")
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="controller")
    ap.add_argument("--config", default=None)
    ap.add_argument("action", choices=["start", "stop", "restart", "status"])
    ap.add_argument("quiet", nargs="?", default=None)
    a = ap.parse_args(argv)
    cfg = read_apm_config(a.config, first_run=True)
    quiet = a.quiet == "quiet"
    if a.action == "start":
        return start(cfg, a.config, quiet)
    if a.action == "stop":
        return stop(cfg, quiet)
    if a.action == "restart":
        rc = stop(cfg, quiet)
        return rc or start(cfg, a.config, quiet)
    pid = running_pid(cfg)
    print(f"running (pid {pid})" if pid else "not running")
    return 0 if pid else 3


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
