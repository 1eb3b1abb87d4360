"""A small in-process AMQP 0-9-1 broker (server side of runtime/amqp.py's subset).

RabbitMQ is not installed on this platform; this broker lets the queue bridge, the
``dequeue``/``qstat`` tools and multi-process deployments run (and be tested) without it.
It implements the default exchange only (routing key = queue name, which is all the reference
uses: queue.js:250 ``sendToQueue``), durable-flagged in-memory queues, round-robin delivery with
per-channel prefetch, acks with redelivery of unacked messages when a consumer disconnects,
basic.get, queue.purge, and a memory-alarm style high/low watermark that sends
``connection.blocked`` / ``unblocked`` to publishers (RabbitMQ's flow control, which the
reference's producers turn into pause/resume, queue.js:126-130,230-263).
"""
from __future__ import annotations

import collections
import socket
import socketserver
import struct
import threading
from typing import Deque, Dict, List, Optional, Tuple

from .amqp import (CONFIRM_SELECT, CONFIRM_SELECT_OK, B_ACK, B_CANCEL, B_CANCEL_OK, B_CONSUME, B_CONSUME_OK, B_DELIVER, B_GET, B_GET_EMPTY, B_GET_OK,
                   B_PUBLISH, B_QOS, B_QOS_OK, CH_CLOSE, CH_CLOSE_OK, CH_FLOW_OK, CH_OPEN, CH_OPEN_OK,
                   CONN_BLOCKED, CONN_CLOSE, CONN_CLOSE_OK, CONN_OPEN, CONN_OPEN_OK, CONN_START, CONN_START_OK,
                   CONN_TUNE, CONN_TUNE_OK, CONN_UNBLOCKED, FRAME_BODY, FRAME_HEADER, FRAME_METHOD, PROTOCOL_HEADER,
                   Q_DECLARE, Q_DECLARE_OK, Q_PURGE, Q_PURGE_OK, Reader, Writer, content_frames, method_frame,
                   read_frame)


class _Queue:
    def __init__(self, name: str, durable: bool):
        self.name = name
        self.durable = durable
        self.msgs: Deque[Tuple[bytes, bool]] = collections.deque()  # (body, redelivered)
        self.consumers: List["_Consumer"] = []
        self.rr = 0
        self.published = 0
        self.delivered = 0
        self.bytes = 0  # bodies held (the supervisor's per-queue memory view)


class _Consumer:
    def __init__(self, conn: "_Conn", tag: str, no_ack: bool, queue: _Queue):
        self.conn = conn
        self.tag = tag
        self.no_ack = no_ack
        self.queue = queue


class Broker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, high_water: int = 0, low_water: int = 0,
                 user: str = "guest", password: str = "guest"):
        self.lock = threading.RLock()
        self.queues: Dict[str, _Queue] = {}
        self.conns: List["_Conn"] = []
        self.high_water = high_water
        self.low_water = low_water or high_water // 2
        self.blocked = False
        self.creds = (user, password)
        broker = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                _Conn(broker, self.request).run()

        class Server(socketserver.ThreadingTCPServer):
            allow_reuse_address = True
            daemon_threads = True

        self.server = Server((host, port), Handler)
        self.host, self.port = self.server.server_address[:2]
        self.thread = threading.Thread(target=self.server.serve_forever, name="amqp-broker", daemon=True)

    @property
    def url(self) -> str:
        return f"amqp://{self.creds[0]}:{self.creds[1]}@{self.host}:{self.port}"

    def start(self) -> "Broker":
        self.thread.start()
        return self

    def stop(self):
        self.server.shutdown()
        self.server.server_close()
        with self.lock:
            for c in list(self.conns):
                c.kill()

    def stats(self) -> Dict[str, Dict[str, int]]:
        """rabbitmqctl list_queues equivalent (qstat)."""
        with self.lock:
            return {n: {"messages": len(q.msgs), "message_bytes": sum(len(b) for b, _ in q.msgs),
                        "consumers": len(q.consumers), "published": q.published, "delivered": q.delivered,
                        "durable": q.durable} for n, q in self.queues.items()}

    def total_messages(self) -> int:
        return sum(len(q.msgs) for q in self.queues.values())

    # called with lock held
    def dispatch(self, q: _Queue):
        while q.msgs and q.consumers:
            for _ in range(len(q.consumers)):
                c = q.consumers[q.rr % len(q.consumers)]
                q.rr += 1
                if c.conn.can_take():
                    break
            else:
                return
            body, redelivered = q.msgs.popleft()
            q.delivered += 1
            q.bytes -= len(body)
            c.conn.deliver(c, q, body, redelivered)
        self.check_alarm()

    def check_alarm(self):
        if not self.high_water:
            return
        n = self.total_messages()
        if not self.blocked and n >= self.high_water:
            self.blocked = True
            for c in self.conns:
                c.send_raw(method_frame(0, CONN_BLOCKED, Writer().shortstr("queue high watermark").bytes()))
        elif self.blocked and n <= self.low_water:
            self.blocked = False
            for c in self.conns:
                c.send_raw(method_frame(0, CONN_UNBLOCKED))


class _Conn:
    def __init__(self, broker: Broker, sock: socket.socket):
        self.b = broker
        self.sock = sock
        self.rfile = sock.makefile("rb")
        self.wlock = threading.Lock()
        self.frame_max = 131072
        self.prefetch = 0
        self.unacked: Dict[int, Tuple[_Queue, bytes]] = {}
        self.next_tag = 1
        self.consumers: Dict[str, _Consumer] = {}
        self.pub: Optional[List] = None  # [queue_name, size, body]
        self.alive = True
        self.confirm = False   # confirm.select'ed channel: every publish is acked in order
        self.pub_seq = 0

    def send_raw(self, data: bytes):
        try:
            with self.wlock:
                self.sock.sendall(data)
        except OSError:
            self.alive = False

    def kill(self):
        self.alive = False
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass

    def can_take(self) -> bool:
        return self.alive and (self.prefetch == 0 or len(self.unacked) < self.prefetch)

    def deliver(self, c: _Consumer, q: _Queue, body: bytes, redelivered: bool):
        tag = self.next_tag
        self.next_tag += 1
        if not c.no_ack:
            self.unacked[tag] = (q, body)
        args = Writer().shortstr(c.tag).longlong(tag).bit(redelivered).shortstr("").shortstr(q.name).bytes()
        self.send_raw(method_frame(1, B_DELIVER, args) + content_frames(1, body, self.frame_max))

    def run(self):
        try:
            if self.rfile.read(8) != PROTOCOL_HEADER:
                self.send_raw(PROTOCOL_HEADER)
                return
            self.send_raw(method_frame(0, CONN_START, Writer().octet(0).octet(9).table({"product": "apm-broker"})
                                       .longstr("PLAIN").longstr("en_US").bytes()))
            with self.b.lock:
                self.b.conns.append(self)
            while self.alive:
                ftype, ch, payload = read_frame(self.rfile)
                if ftype == FRAME_METHOD:
                    if not self.on_method(ch, payload):
                        break
                elif ftype == FRAME_HEADER and self.pub is not None:
                    r = Reader(payload)
                    r.short(); r.short()
                    self.pub[1] = r.longlong()
                    if self.pub[1] == 0:
                        self.publish_done()
                elif ftype == FRAME_BODY and self.pub is not None:
                    self.pub[2] += payload
                    if len(self.pub[2]) >= self.pub[1]:
                        self.publish_done()
        except (EOFError, OSError):
            pass
        finally:
            self.cleanup()

    def cleanup(self):
        self.alive = False
        with self.b.lock:
            if self in self.b.conns:
                self.b.conns.remove(self)
            for c in self.consumers.values():
                if c in c.queue.consumers:
                    c.queue.consumers.remove(c)
            # unacked messages go back to the head of their queue, flagged redelivered
            for tag in sorted(self.unacked, reverse=True):
                q, body = self.unacked[tag]
                q.msgs.appendleft((body, True))
                q.bytes += len(body)
            touched = {q for q, _ in self.unacked.values()}
            self.unacked.clear()
            for q in touched:
                self.b.dispatch(q)
        try:
            self.sock.close()
        except OSError:
            pass

    def publish_done(self):
        name, _size, body = self.pub
        self.pub = None
        with self.b.lock:
            q = self.b.queues.get(name)
            if q is not None:  # the default exchange drops unroutable messages (still confirmed)
                q.msgs.append((bytes(body), False))
                q.published += 1
                q.bytes += len(body)
                self.b.dispatch(q)
                self.b.check_alarm()
        if self.confirm:
            self.pub_seq += 1
            self.send_raw(method_frame(1, B_ACK, Writer().longlong(self.pub_seq).bit(False).bytes()))

    def on_method(self, ch: int, payload: bytes) -> bool:
        r = Reader(payload)
        cm = (r.short(), r.short())
        if cm == CONN_START_OK:
            r.table()
            mech = r.shortstr()
            resp = r.longstr()
            parts = resp.split(b"\x00")
            if mech != "PLAIN" or len(parts) != 3 or (parts[1].decode(), parts[2].decode()) != self.b.creds:
                self.send_raw(method_frame(0, CONN_CLOSE, Writer().short(403).shortstr("ACCESS_REFUSED")
                                           .short(10).short(11).bytes()))
                return False
            self.send_raw(method_frame(0, CONN_TUNE, Writer().short(2047).long(self.frame_max).short(0).bytes()))
        elif cm == CONN_TUNE_OK:
            r.short()
            fm = r.long()
            if fm:
                self.frame_max = min(self.frame_max, fm)
        elif cm == CONN_OPEN:
            self.send_raw(method_frame(0, CONN_OPEN_OK, Writer().shortstr("").bytes()))
            if self.b.blocked:
                self.send_raw(method_frame(0, CONN_BLOCKED, Writer().shortstr("queue high watermark").bytes()))
        elif cm == CONN_CLOSE:
            self.send_raw(method_frame(0, CONN_CLOSE_OK))
            return False
        elif cm == CONN_CLOSE_OK:
            return False
        elif cm == CH_OPEN:
            self.send_raw(method_frame(ch, CH_OPEN_OK, Writer().longstr("").bytes()))
        elif cm == CH_CLOSE:
            self.send_raw(method_frame(ch, CH_CLOSE_OK))
        elif cm == CH_FLOW_OK:
            pass
        elif cm == Q_DECLARE:
            r.short()
            name = r.shortstr()
            passive, durable = r.bit(), r.bit()
            with self.b.lock:
                q = self.b.queues.get(name)
                if q is None:
                    if passive:
                        self.send_raw(method_frame(ch, CH_CLOSE, Writer().short(404).shortstr(f"NOT_FOUND - {name}")
                                                   .short(50).short(10).bytes()))
                        return True
                    q = self.b.queues[name] = _Queue(name, durable)
                n_msgs, n_cons = len(q.msgs), len(q.consumers)
            self.send_raw(method_frame(ch, Q_DECLARE_OK, Writer().shortstr(name).long(n_msgs).long(n_cons).bytes()))
        elif cm == Q_PURGE:
            r.short()
            name = r.shortstr()
            with self.b.lock:
                q = self.b.queues.get(name)
                n = len(q.msgs) if q else 0
                if q:
                    q.msgs.clear()
                self.b.check_alarm()
            self.send_raw(method_frame(ch, Q_PURGE_OK, Writer().long(n).bytes()))
        elif cm == B_QOS:
            r.long()
            self.prefetch = r.short()
            self.send_raw(method_frame(ch, B_QOS_OK))
        elif cm == B_CONSUME:
            r.short()
            qname, tag = r.shortstr(), r.shortstr()
            _no_local, no_ack = r.bit(), r.bit()
            with self.b.lock:
                q = self.b.queues.get(qname)
                if q is None:
                    self.send_raw(method_frame(ch, CH_CLOSE, Writer().short(404).shortstr(f"NOT_FOUND - {qname}")
                                               .short(60).short(20).bytes()))
                    return True
                if not tag:
                    tag = f"amq.ctag-{id(self)}-{len(self.consumers)}"
                c = _Consumer(self, tag, no_ack, q)
                self.consumers[tag] = c
                self.send_raw(method_frame(ch, B_CONSUME_OK, Writer().shortstr(tag).bytes()))
                q.consumers.append(c)
                self.b.dispatch(q)
        elif cm == B_CANCEL:
            tag = r.shortstr()
            with self.b.lock:
                c = self.consumers.pop(tag, None)
                if c and c in c.queue.consumers:
                    c.queue.consumers.remove(c)
            self.send_raw(method_frame(ch, B_CANCEL_OK, Writer().shortstr(tag).bytes()))
        elif cm == CONFIRM_SELECT:
            nowait = r.bit()
            self.confirm = True
            if not nowait:
                self.send_raw(method_frame(ch, CONFIRM_SELECT_OK))
        elif cm == B_PUBLISH:
            r.short()
            _exchange, rkey = r.shortstr(), r.shortstr()
            self.pub = [rkey, 0, bytearray()]
        elif cm == B_GET:
            r.short()
            qname = r.shortstr()
            no_ack = r.bit()
            with self.b.lock:
                q = self.b.queues.get(qname)
                if not q or not q.msgs:
                    self.send_raw(method_frame(ch, B_GET_EMPTY, Writer().shortstr("").bytes()))
                    return True
                body, redelivered = q.msgs.popleft()
                q.delivered += 1
                q.bytes -= len(body)
                tag = self.next_tag
                self.next_tag += 1
                if not no_ack:
                    self.unacked[tag] = (q, body)
                left = len(q.msgs)
                self.b.check_alarm()
            args = Writer().longlong(tag).bit(redelivered).shortstr("").shortstr(qname).long(left).bytes()
            self.send_raw(method_frame(ch, B_GET_OK, args) + content_frames(1, body, self.frame_max))
        elif cm == B_ACK:
            tag, multiple = r.longlong(), r.bit()
            with self.b.lock:
                tags = [t for t in self.unacked if t <= tag] if multiple else [tag]
                qs = set()
                for t in tags:
                    e = self.unacked.pop(t, None)
                    if e:
                        qs.add(e[0])
                for q in qs:
                    self.b.dispatch(q)
        return True


def main(argv=None):  # pragma: no cover - CLI
    import argparse
    import time
    ap = argparse.ArgumentParser(description="in-process AMQP 0-9-1 broker (default exchange only)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=5672)
    ap.add_argument("--high-water", type=int, default=1_000_000)
    a = ap.parse_args(argv)
    b = Broker(a.host, a.port, high_water=a.high_water).start()
    print(f"broker listening on {b.url}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        b.stop()


if __name__ == "__main__":  # pragma: no cover
    main()
