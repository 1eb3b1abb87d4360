"""JMX side source: poll WildFly management stats into ``jx`` records (reference
``pull_jvm_stats.js:1-157``, ``entries.js JmxEntry :243-332``).

Every ``pollingIntervalSeconds`` -- aligned to the wall clock, first poll one interval after
start (pullAllJvmStatsRecurs :141-149) -- each host in ``jvmHosts`` is queried with one
``jboss-cli-client.jar --output-json ... commands="<cmd1>,<cmd2>,..."`` call built from
``statCmdMap``.  The concatenated JSON documents are turned into one object keyed by the stat
names (``cli_to_json``, :15-33), converted to a ``jx`` record (host name shortened when
``shortenHostname``) and sent to the ``db_insert`` stream.  A host that fails is skipped for
that round.  The Java client is an external command behind the same contract (its jar is not
part of the reference checkout); ``SyntheticJmx`` produces the same output for tests and
benchmarks.
"""
from __future__ import annotations

import json
import logging
import random
import re
import subprocess
import time
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..utils.records import JmxEntry

log = logging.getLogger("apm.jmx")


def cli_to_json(resources: Sequence[str], output: str) -> Dict[str, Any]:
    """Glue the CLI's back-to-back JSON documents into {resource: document}."""
    res = list(resources)
    f = str(output).replace("\n}\n{", "\n},\n{")
    out = []
    for line in f.split("\n"):
        if re.match(r"^[a-zA-Z]", line):
            out.append("")  # warning line (JS: undefined -> '' in join)
        elif line.startswith("{"):
            out.append(f'"{res.pop(0)}" : {{' if res else '"undefined" : {')
        else:
            out.append(line)
    return json.loads("{" + "\n".join(out) + "}")


def cli_command(host: str, cmds: str, pc: Dict[str, Any]) -> List[str]:
    return ["java", "-jar", pc["clientJarFullPath"], "--output-json", f"--timeout={pc.get('clientTimeoutMs', 2000)}",
            f"--controller={host}:{pc.get('jmxPort', 9990)}", f"--user={pc.get('adminUser', '')}",
            f"--password={pc.get('adminPass', '')}", "--connect", f"commands={cmds}"]


def run_cli(argv: List[str], timeout_s: float) -> str:
    r = subprocess.run(argv, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=timeout_s, check=True)
    return r.stdout.decode("utf-8", "replace")


class JvmStatsPoller:
    def __init__(self, cfg: Dict[str, Any], emit: Callable[[str], None],
                 runner: Callable[[List[str], float], str] = run_cli, clock: Callable[[], float] = time.time):
        self.cfg = cfg
        self.emit = emit
        self.runner = runner
        self.clock = clock
        self.next_due = self._align(clock())
        self.polls = 0

    @property
    def pc(self):
        return self.cfg["pullJvmStats"]

    def _align(self, now: float) -> float:
        iv = int(self.pc.get("pollingIntervalSeconds", 60))
        sec = int(now) % 60
        return now + (iv - (sec % iv))

    def pull(self, host: str) -> Optional[Dict[str, Any]]:
        names = list(self.pc["statCmdMap"].keys())
        cmds = ",".join(self.pc["statCmdMap"].values())
        try:
            out = self.runner(cli_command(host, cmds, self.pc), float(self.pc.get("clientTimeoutMs", 2000)) / 1000 + 30)
            stats = cli_to_json(names, out)
        except Exception as e:
            log.debug("JMX pull failed for %s: %s", host, e)
            return None
        stats["server"] = host
        return stats

    def pull_all(self, ts_ms: int) -> List[str]:
        lines = []
        for host in self.pc.get("jvmHosts", []):
            st = self.pull(host)
            if st is None:
                continue
            server = re.sub(r"\..*", "", st["server"]) if self.pc.get("shortenHostname") else st["server"]
            try:
                line = JmxEntry.from_stats(ts_ms, server, st).to_csv()
            except (KeyError, IndexError, TypeError) as e:
                log.error("unexpected JMX payload from %s: %s", host, e)
                continue
            lines.append(line)
            self.emit(line)
        self.polls += 1
        return lines

    def tick(self) -> List[str]:
        now = self.clock()
        if now < self.next_due:
            return []
        self.next_due = self._align(now)
        return self.pull_all(int(now * 1000))


class SyntheticJmx:
    """Stand-in for the WildFly CLI: deterministic, plausible gauges per host, emitted in the
    CLI's --output-json layout (one JSON document per command, warnings interleaved)."""

    def __init__(self, seed: int = 1):
        self.rng = random.Random(seed)

    def payload(self, host: str) -> Dict[str, Any]:
        r = random.Random(hash((host, self.rng.random())) & 0xFFFFFFFF)
        heap_max = 8 << 30
        return {
            "ds": {"outcome": "success", "result": {"InUseCount": r.randint(0, 40), "ActiveCount": r.randint(10, 60),
                                                    "AvailableCount": r.randint(40, 100)}},
            "heap": {"outcome": "success", "result": {"used": r.randint(1 << 30, heap_max), "committed": heap_max,
                                                      "max": heap_max}},
            "meta": {"outcome": "success", "result": {"used": r.randint(200 << 20, 400 << 20),
                                                      "committed": 512 << 20, "max": -1}},
            "sysload": {"outcome": "success", "result": round(r.uniform(0.1, 12.0), 2)},
            "classcnt": {"outcome": "success", "result": r.randint(20000, 40000)},
            "threading": {"outcome": "success", "result": {"thread-count": r.randint(200, 600),
                                                           "daemon-thread-count": r.randint(100, 300)}},
            "bean": {"outcome": "success", "result": [{"address": [], "outcome": "success", "result": {
                "pool-available-count": r.randint(0, 20), "pool-current-size": r.randint(5, 20),
                "pool-max-size": 20}}]},
        }

    def cli_output(self, names: Sequence[str], host: str) -> str:
        p = self.payload(host)
        docs = ["WARN: picked up JAVA_TOOL_OPTIONS"]
        for n in names:
            docs.append(json.dumps(p[n], indent=4))
        return "\n".join(docs) + "\n"

    def runner(self, argv: List[str], timeout_s: float) -> str:
        host = next(a.split("=", 1)[1].rsplit(":", 1)[0] for a in argv if a.startswith("--controller="))
        cmds = next(a.split("=", 1)[1] for a in argv if a.startswith("commands="))
        n = len(cmds.split(",/"))
        names = ["ds", "heap", "meta", "sysload", "classcnt", "threading", "bean"][:n]
        return self.cli_output(names, host)


def main(argv=None):  # pragma: no cover - process entry point
    import argparse
    from ..utils.config import read_apm_config
    from . import logger as apmlog
    from .queue import QueueManager
    ap = argparse.ArgumentParser(description="JMX poller -> db_insert")
    ap.add_argument("--config", default=None)
    ap.add_argument("--synthetic", action="store_true")
    a = ap.parse_args(argv)
    cfg = read_apm_config(a.config, first_run=True)
    apmlog.set_global_logger(cfg.get("logDir"), cfg["pullJvmStats"].get("logFilePrefix", "pull_jvm_stats"))
    qm = QueueManager(cfg["amqpConnectionString"], cfg.get("statLogIntervalInSeconds", 60))
    q = qm.get_queue(cfg.get("dbInsertQueue", "db_insert"), "p")
    poller = JvmStatsPoller(cfg, q.write_line, runner=SyntheticJmx().runner if a.synthetic else run_cli)
    try:
        while True:
            poller.tick()
            time.sleep(0.5)
    except KeyboardInterrupt:
        qm.shutdown()


if __name__ == "__main__":  # pragma: no cover
    main()
