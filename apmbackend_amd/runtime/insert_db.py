"""Standalone DB insert process (reference ``stream_insert_db.js`` as a process): consume the
``db_insert`` queue and load it with runtime/sinks.DBInserter.  Only needed when the engines run
with ``gpu.outputMode = "amqp"`` (e.g. a DB host separate from the GPU node); in the default
``inproc`` mode each engine process owns its inserter.

Consumption follows the config: ``streamInsertDb.consumeQueue`` toggles start/stop on hot reload
(:100-110), and the queue manager's pause/resume stops and restarts consumption (:118-124).
"""
from __future__ import annotations

import logging
import signal
import threading
import time
from typing import Any, Dict, Optional

from ..utils.config import ConfigWatcher, as_bool, read_apm_config
from . import logger as apmlog
from .queue import QueueManager
from .sinks import DBInserter, Writer

log = logging.getLogger("apm.insert_db")


class InsertDbProcess:
    def __init__(self, cfg: Dict[str, Any], writer: Optional[Writer] = None):
        self.cfg = cfg
        self.lock = threading.Lock()
        self.ins = DBInserter(cfg, writer=writer)
        self.qm = QueueManager(cfg["amqpConnectionString"], cfg.get("statLogIntervalInSeconds", 60))
        self.q = self.qm.get_queue(cfg.get("dbInsertQueue", "db_insert"), "c", self._on_msg)
        self.qm.on("pause", self.q.stop_consume)
        self.qm.on("resume", self.q.start_consume)
        self.watcher = ConfigWatcher(cfg, self.reload) if cfg.get("apmConfigFilePath") else None
        self._stop = False
        if as_bool(cfg["streamInsertDb"].get("consumeQueue", True)):
            self.q.start_consume()

    def _on_msg(self, body: bytes):
        with self.lock:
            self.ins.consume_line(body.decode("utf-8", "replace"))

    def reload(self, cfg):
        self.cfg = cfg
        ic = cfg["streamInsertDb"]
        with self.lock:
            self.ins.limit = int(ic.get("dbInsertBufferLimit", self.ins.limit))
            self.ins.max_wait_s = float(ic.get("dbMaxTimeBetweenInsertsMs", 5000)) / 1000.0
        if not as_bool(ic.get("consumeQueue", True)) and self.q.consuming:
            log.info("Stopping consume from watcher!")
            self.q.stop_consume()
        elif as_bool(ic.get("consumeQueue", True)) and not self.q.consuming:
            log.info("Starting consume from watcher!")
            self.q.start_consume()

    def tick(self):
        with self.lock:
            self.ins.tick()
        if self.watcher:
            self.watcher.check_once()

    def close(self):
        self.q.stop_consume()
        with self.lock:
            self.ins.close()
        self.qm.shutdown()

    def run(self):
        last = time.time()
        while not self._stop:
            self.tick()
            if time.time() - last >= float(self.cfg.get("statLogIntervalInSeconds", 60)):
                self.ins.stats.log_and_reset()
                log.info(self.qm.stats.line())
                last = time.time()
            time.sleep(0.2)
        self.close()


def main(argv=None):  # pragma: no cover
    import argparse
    ap = argparse.ArgumentParser(description="db_insert consumer -> Postgres COPY")
    ap.add_argument("--config", default=None)
    a = ap.parse_args(argv)
    cfg = read_apm_config(a.config, first_run=True)
    apmlog.set_global_logger(cfg.get("logDir"), cfg["streamInsertDb"].get("logFilePrefix", "stream_insert_db"))
    p = InsertDbProcess(cfg)
    signal.signal(signal.SIGTERM, lambda *x: setattr(p, "_stop", True))
    signal.signal(signal.SIGINT, lambda *x: setattr(p, "_stop", True))
    p.run()


if __name__ == "__main__":  # pragma: no cover
    main()
