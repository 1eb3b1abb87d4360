"""Queue peek tool (reference ``dequeue.js``): consume a queue without acks and print every
message.  Unlike the reference it does not hard-code the broker URL.

Usage: python -m apmbackend_amd.cli.dequeue [--url amqp://...] [--count N] QUEUE
"""
from __future__ import annotations

import argparse
import sys
import threading
import time

from ..runtime.amqp import Connection
from ..utils.config import read_apm_config


def main(argv=None, out=sys.stdout) -> int:
    ap = argparse.ArgumentParser(prog="dequeue")
    ap.add_argument("--config", default=None)
    ap.add_argument("--url", default=None)
    ap.add_argument("--count", type=int, default=0, help="stop after N messages (0 = run until Ctrl-C)")
    ap.add_argument("--idle-exit", type=float, default=0.0, help="stop after this many idle seconds")
    ap.add_argument("queue")
    a = ap.parse_args(argv)
    url = a.url or read_apm_config(a.config, first_run=True)["amqpConnectionString"]
    c = Connection(url)
    print("AMQP connected.", file=sys.stderr)
    c.queue_declare(a.queue, durable=True)
    print(f" [*] Waiting for messages in {a.queue}. To exit press CTRL+C", file=sys.stderr)
    n = [0]
    last = [time.time()]
    done = threading.Event()

    def cb(m):
        out.write(m.body.decode("utf-8", "replace") + "\n")
        n[0] += 1
        last[0] = time.time()
        if a.count and n[0] >= a.count:
            done.set()

    c.consume(a.queue, cb, no_ack=True)
    try:
        while not done.is_set():
            if a.idle_exit and time.time() - last[0] > a.idle_exit:
                break
            done.wait(0.1)
    except KeyboardInterrupt:
        print("Caught interrupt signal, exiting.", file=sys.stderr)
    c.close()
    return 0


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())
