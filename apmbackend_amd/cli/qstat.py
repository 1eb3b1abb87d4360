"""Queue statistics (reference ``qstat.sh``: ``rabbitmqctl list_queues`` pretty-printed).

Asks the broker for each known queue's depth and consumer count with a passive
``queue.declare`` (works against RabbitMQ and runtime/amqp_broker.py alike).

Usage: python -m apmbackend_amd.cli.qstat [--config PATH] [--url amqp://...] [queue ...]
"""
from __future__ import annotations

import argparse
import sys

from ..runtime.amqp import AMQPError, Connection
from ..utils.config import read_apm_config


def known_queues(cfg):
    names = [cfg["streamParseTransactions"].get("outQueue", "transactions"),
             cfg["streamCalcStats"].get("outQueue", "stats"),
             cfg["streamCalcZScore"].get("outQueue", "z_score"), cfg.get("dbInsertQueue", "db_insert")]
    return list(dict.fromkeys(names))


def queue_table(url: str, names) -> list:
    rows = []
    for n in names:
        c = Connection(url, timeout=5)
        try:
            _q, msgs, cons = c.queue_declare(n, passive=True)
            rows.append((n, msgs, cons))
        except AMQPError:
            rows.append((n, None, None))
        finally:
            c.close()
    return rows


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="qstat")
    ap.add_argument("--config", default=None)
    ap.add_argument("--url", default=None)
    ap.add_argument("queues", nargs="*")
    a = ap.parse_args(argv)
    cfg = read_apm_config(a.config, first_run=True)
    url = a.url or cfg["amqpConnectionString"]
    names = a.queues or known_queues(cfg)
    print("%-20s %12s %10s" % ("name", "messages", "consumers"))
    for n, m, c in queue_table(url, names):
        print("%-20s %12s %10s" % (n, "-" if m is None else m, "-" if c is None else c))
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
