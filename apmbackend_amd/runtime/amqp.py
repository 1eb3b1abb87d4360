"""Minimal AMQP 0-9-1 client (the RabbitMQ wire protocol), dependency-free.

The reference moves every record between its five stage processes through RabbitMQ queues with
amqplib (queue.js:1-311).  The fused engine needs no broker, but the queue *contract* stays:
the same queue names and text records can be published to / consumed from a real RabbitMQ
(``amqpConnectionString``) so external consumers, ``dequeue``/``qstat`` style tools and mixed
deployments keep working.  amqplib/pika are not available here, so this module speaks the
protocol directly: connection negotiation (PLAIN auth), one channel per Connection object,
queue.declare, basic.publish, basic.consume / deliver / ack / cancel, basic.qos, and broker flow
control (channel.flow, connection.blocked) surfaced as pause/resume callbacks.

``runtime/amqp_broker.py`` implements the server side of the same subset for tests and for
hosts without RabbitMQ.
"""
from __future__ import annotations

import queue as _queue
import socket
import struct
import threading
import urllib.parse
from typing import Any, Callable, Dict, List, Optional, Tuple

FRAME_METHOD, FRAME_HEADER, FRAME_BODY, FRAME_HEARTBEAT = 1, 2, 3, 8
FRAME_END = 0xCE
PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"

# (class, method) ids
CONN_START, CONN_START_OK, CONN_TUNE, CONN_TUNE_OK = (10, 10), (10, 11), (10, 30), (10, 31)
CONN_OPEN, CONN_OPEN_OK, CONN_CLOSE, CONN_CLOSE_OK = (10, 40), (10, 41), (10, 50), (10, 51)
CONN_BLOCKED, CONN_UNBLOCKED = (10, 60), (10, 61)
CH_OPEN, CH_OPEN_OK, CH_FLOW, CH_FLOW_OK, CH_CLOSE, CH_CLOSE_OK = (20, 10), (20, 11), (20, 20), (20, 21), (20, 40), (20, 41)
Q_DECLARE, Q_DECLARE_OK, Q_PURGE, Q_PURGE_OK = (50, 10), (50, 11), (50, 30), (50, 31)
B_QOS, B_QOS_OK, B_CONSUME, B_CONSUME_OK = (60, 10), (60, 11), (60, 20), (60, 21)
B_CANCEL, B_CANCEL_OK, B_PUBLISH, B_DELIVER = (60, 30), (60, 31), (60, 40), (60, 60)
B_GET, B_GET_OK, B_GET_EMPTY, B_ACK = (60, 70), (60, 71), (60, 72), (60, 80)
B_NACK = (60, 120)
CONFIRM_SELECT, CONFIRM_SELECT_OK = (85, 10), (85, 11)


class AMQPError(RuntimeError):
    pass


# --------------------------------------------------------------------------- codec

class Writer:
    def __init__(self):
        self.b = bytearray()
        self._bits: List[bool] = []

    def _flush_bits(self):
        if self._bits:
            v = 0
            for i, bit in enumerate(self._bits):
                v |= (1 << i) if bit else 0
            self.b += struct.pack("B", v)
            self._bits = []

    def bit(self, v: bool):
        self._bits.append(bool(v))
        if len(self._bits) == 8:
            self._flush_bits()
        return self

    def octet(self, v):
        self._flush_bits(); self.b += struct.pack(">B", v); return self

    def short(self, v):
        self._flush_bits(); self.b += struct.pack(">H", v); return self

    def long(self, v):
        self._flush_bits(); self.b += struct.pack(">I", v); return self

    def longlong(self, v):
        self._flush_bits(); self.b += struct.pack(">Q", v); return self

    def shortstr(self, s):
        self._flush_bits()
        d = s.encode() if isinstance(s, str) else bytes(s)
        if len(d) > 255:
            raise AMQPError("shortstr too long")
        self.b += struct.pack("B", len(d)) + d
        return self

    def longstr(self, s):
        self._flush_bits()
        d = s.encode() if isinstance(s, str) else bytes(s)
        self.b += struct.pack(">I", len(d)) + d
        return self

    def table(self, t: Optional[Dict[str, Any]]):
        self._flush_bits()
        body = Writer()
        for k, v in (t or {}).items():
            body.shortstr(k)
            _write_field(body, v)
        self.b += struct.pack(">I", len(body.b)) + body.b
        return self

    def bytes(self) -> bytes:
        self._flush_bits()
        return bytes(self.b)


def _write_field(w: Writer, v):
    if isinstance(v, bool):
        w.b += b"t" + struct.pack("B", 1 if v else 0)
    elif isinstance(v, int):
        w.b += b"l" + struct.pack(">q", v)
    elif isinstance(v, float):
        w.b += b"d" + struct.pack(">d", v)
    elif isinstance(v, dict):
        w.b += b"F"
        w.table(v)
    elif isinstance(v, (list, tuple)):
        inner = Writer()
        for x in v:
            _write_field(inner, x)
        w.b += b"A" + struct.pack(">I", len(inner.b)) + inner.b
    elif v is None:
        w.b += b"V"
    else:
        w.b += b"S"
        w.longstr(str(v))


class Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.i = 0
        self._bits = 0
        self._nbits = 0

    def _take(self, n):
        if self.i + n > len(self.d):
            raise AMQPError("truncated frame")
        v = self.d[self.i:self.i + n]
        self.i += n
        self._nbits = 0
        return v

    def bit(self) -> bool:
        if self._nbits == 0 or self._nbits == 8:
            self._bits = self.d[self.i]
            self.i += 1
            self._nbits = 0
        v = bool(self._bits & (1 << self._nbits))
        self._nbits += 1
        return v

    def octet(self):
        return struct.unpack(">B", self._take(1))[0]

    def short(self):
        return struct.unpack(">H", self._take(2))[0]

    def long(self):
        return struct.unpack(">I", self._take(4))[0]

    def longlong(self):
        return struct.unpack(">Q", self._take(8))[0]

    def shortstr(self) -> str:
        n = self.octet()
        return self._take(n).decode("utf-8", "replace")

    def longstr(self) -> bytes:
        n = self.long()
        return bytes(self._take(n))

    def table(self) -> Dict[str, Any]:
        n = self.long()
        end = self.i + n
        out = {}
        while self.i < end:
            k = self.shortstr()
            out[k] = self._field()
        return out

    def _field(self):
        t = self._take(1)
        if t == b"t":
            return bool(self.octet())
        if t == b"b":
            return struct.unpack(">b", self._take(1))[0]
        if t == b"B":
            return self.octet()
        if t == b"s":
            return struct.unpack(">h", self._take(2))[0]
        if t == b"u":
            return self.short()
        if t == b"I":
            return struct.unpack(">i", self._take(4))[0]
        if t == b"i":
            return self.long()
        if t in (b"l", b"L"):
            return struct.unpack(">q", self._take(8))[0]
        if t == b"f":
            return struct.unpack(">f", self._take(4))[0]
        if t == b"d":
            return struct.unpack(">d", self._take(8))[0]
        if t == b"D":
            scale = self.octet()
            return struct.unpack(">i", self._take(4))[0] / (10 ** scale)
        if t == b"S":
            return self.longstr().decode("utf-8", "replace")
        if t == b"x":
            return self.longstr()
        if t == b"T":
            return self.longlong()
        if t == b"F":
            return self.table()
        if t == b"A":
            n = self.long()
            end = self.i + n
            arr = []
            while self.i < end:
                arr.append(self._field())
            return arr
        if t == b"V":
            return None
        raise AMQPError(f"unknown field type {t!r}")


def method_frame(channel: int, cm: Tuple[int, int], args: bytes = b"") -> bytes:
    payload = struct.pack(">HH", *cm) + args
    return struct.pack(">BHI", FRAME_METHOD, channel, len(payload)) + payload + bytes([FRAME_END])


def content_frames(channel: int, body: bytes, frame_max: int, class_id: int = 60,
                   delivery_mode: Optional[int] = None) -> bytes:
    flags = 0
    props = b""
    if delivery_mode is not None:  # basic properties: delivery-mode is bit 12
        flags |= 1 << 12
        props += struct.pack("B", delivery_mode)
    hdr = struct.pack(">HHQH", class_id, 0, len(body), flags) + props
    out = struct.pack(">BHI", FRAME_HEADER, channel, len(hdr)) + hdr + bytes([FRAME_END])
    step = max(1, frame_max - 8)
    for i in range(0, len(body), step):
        chunk = body[i:i + step]
        out += struct.pack(">BHI", FRAME_BODY, channel, len(chunk)) + chunk + bytes([FRAME_END])
    return out


def read_frame(sock_file) -> Tuple[int, int, bytes]:
    hdr = sock_file.read(7)
    if len(hdr) < 7:
        raise EOFError("connection closed")
    ftype, ch, size = struct.unpack(">BHI", hdr)
    payload = sock_file.read(size)
    end = sock_file.read(1)
    if len(payload) < size or not end:
        raise EOFError("connection closed")
    if end[0] != FRAME_END:
        raise AMQPError("bad frame end")
    return ftype, ch, payload


def parse_url(url: str) -> Dict[str, Any]:
    u = urllib.parse.urlparse(url or "amqp://localhost:5672")
    vhost = urllib.parse.unquote(u.path[1:]) if u.path and u.path != "/" else "/"
    return {"host": u.hostname or "localhost", "port": u.port or 5672,
            "user": urllib.parse.unquote(u.username or "guest"), "password": urllib.parse.unquote(u.password or "guest"),
            "vhost": vhost}


# --------------------------------------------------------------------------- client

class Message:
    __slots__ = ("body", "delivery_tag", "redelivered", "routing_key", "consumer_tag")

    def __init__(self, body, delivery_tag, redelivered, routing_key, consumer_tag):
        self.body = body
        self.delivery_tag = delivery_tag
        self.redelivered = redelivered
        self.routing_key = routing_key
        self.consumer_tag = consumer_tag


class Connection:
    """One TCP connection with a single channel (1), like each amqplib connection+channel pair
    the reference opens per direction (queue.js:73-79)."""

    def __init__(self, url: str = "amqp://localhost:5672", timeout: float = 10.0,
                 on_pause: Optional[Callable[[], None]] = None, on_resume: Optional[Callable[[], None]] = None):
        p = parse_url(url)
        self.sock = socket.create_connection((p["host"], p["port"]), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.rfile = self.sock.makefile("rb")
        self.timeout = timeout
        self.frame_max = 131072
        self.ch = 1
        self._wlock = threading.Lock()
        self._rpc: "_queue.Queue" = _queue.Queue()
        self._consumers: Dict[str, Callable[[Message], None]] = {}
        self._pending: Optional[list] = None  # deliver/get-ok awaiting header+body
        self.closed = False
        self.blocked = False
        self.flow_active = True
        self.on_pause = on_pause
        self.on_resume = on_resume
        # publisher confirms (confirm.select): broker basic.ack / basic.nack per publish sequence
        self.confirming = False
        self._pub_seq = 0
        self._unconfirmed: set = set()
        self._nacked: list = []
        self._confirm_cv = threading.Condition()
        self._handshake(p)
        self._reader = threading.Thread(target=self._read_loop, name="amqp-reader", daemon=True)
        self._reader.start()
        self._call(CH_OPEN, Writer().shortstr("").bytes(), CH_OPEN_OK)

    # -- plumbing
    def _send(self, data: bytes):
        with self._wlock:
            self.sock.sendall(data)

    def _handshake(self, p):
        self.sock.sendall(PROTOCOL_HEADER)
        ftype, ch, payload = read_frame(self.rfile)
        r = Reader(payload)
        if (r.short(), r.short()) != CONN_START:
            raise AMQPError("expected connection.start")
        r.octet(); r.octet(); r.table()
        mechs = r.longstr().decode().split()
        if "PLAIN" not in mechs:
            raise AMQPError(f"broker offers no PLAIN auth: {mechs}")
        resp = b"\x00" + p["user"].encode() + b"\x00" + p["password"].encode()
        self.sock.sendall(method_frame(0, CONN_START_OK, Writer().table(
            {"product": "apmbackend_amd", "capabilities": {"consumer_cancel_notify": True}})
            .shortstr("PLAIN").longstr(resp).shortstr("en_US").bytes()))
        ftype, ch, payload = read_frame(self.rfile)
        r = Reader(payload)
        if (r.short(), r.short()) != CONN_TUNE:
            raise AMQPError("expected connection.tune")
        ch_max, fmax, _hb = r.short(), r.long(), r.short()
        self.frame_max = min(fmax or 131072, 131072)
        self.sock.sendall(method_frame(0, CONN_TUNE_OK, Writer().short(ch_max or 2047).long(self.frame_max).short(0).bytes()))
        self.sock.sendall(method_frame(0, CONN_OPEN, Writer().shortstr(p["vhost"]).shortstr("").bit(False).bytes()))
        ftype, ch, payload = read_frame(self.rfile)
        r = Reader(payload)
        cm = (r.short(), r.short())
        if cm == CONN_CLOSE:
            code, text = r.short(), r.shortstr()
            raise AMQPError(f"connection refused: {code} {text}")
        if cm != CONN_OPEN_OK:
            raise AMQPError("expected connection.open-ok")
        self.sock.settimeout(None)

    def _call(self, cm, args: bytes, expect, channel=None):
        self._send(method_frame(self.ch if channel is None else channel, cm, args))
        try:
            got, r = self._rpc.get(timeout=self.timeout)
        except _queue.Empty:
            raise AMQPError(f"timeout waiting for {expect}")
        if got == "error":
            raise AMQPError(r)
        if got != expect:
            raise AMQPError(f"expected {expect}, got {got}")
        return r

    def _read_loop(self):
        try:
            while True:
                ftype, ch, payload = read_frame(self.rfile)
                if ftype == FRAME_METHOD:
                    self._on_method(ch, payload)
                elif ftype == FRAME_HEADER and self._pending is not None:
                    r = Reader(payload)
                    r.short(); r.short()
                    self._pending.append(r.longlong())
                    self._pending.append(bytearray())
                    if self._pending[-2] == 0:
                        self._deliver()
                elif ftype == FRAME_BODY and self._pending is not None:
                    self._pending[-1] += payload
                    if len(self._pending[-1]) >= self._pending[-2]:
                        self._deliver()
                elif ftype == FRAME_HEARTBEAT:
                    self._send(struct.pack(">BHI", FRAME_HEARTBEAT, 0, 0) + bytes([FRAME_END]))
        except (EOFError, OSError, AMQPError) as e:
            if not self.closed:
                self._rpc.put(("error", f"connection lost: {e}"))
        finally:
            self.closed = True

    def _deliver(self):
        kind, msg_args, _size, body = self._pending
        self._pending = None
        if kind == "get":
            self._rpc.put((B_GET_OK, (msg_args, bytes(body))))
            return
        tag, dtag, redelivered, _ex, rkey = msg_args
        cb = self._consumers.get(tag)
        if cb is not None:
            cb(Message(bytes(body), dtag, redelivered, rkey, tag))

    def _on_method(self, ch, payload):
        r = Reader(payload)
        cm = (r.short(), r.short())
        if cm == B_DELIVER:
            args = (r.shortstr(), r.longlong(), r.bit(), r.shortstr(), r.shortstr())
            self._pending = ["deliver", args]
        elif cm == B_GET_OK:
            args = (r.longlong(), r.bit(), r.shortstr(), r.shortstr(), r.long())
            self._pending = ["get", args]
        elif cm == CH_FLOW:
            active = r.bit()
            self._send(method_frame(ch, CH_FLOW_OK, Writer().bit(active).bytes()))
            self.flow_active = active
            cb = self.on_resume if active else self.on_pause
            if cb:
                cb()
        elif cm in (CONN_BLOCKED, CONN_UNBLOCKED):
            self.blocked = cm == CONN_BLOCKED
            cb = self.on_pause if self.blocked else self.on_resume
            if cb:
                cb()
        elif cm == CH_CLOSE:
            code, text = r.short(), r.shortstr()
            self._send(method_frame(ch, CH_CLOSE_OK))
            self._rpc.put(("error", f"channel closed by broker: {code} {text}"))
        elif cm == CONN_CLOSE:
            code, text = r.short(), r.shortstr()
            self._send(method_frame(0, CONN_CLOSE_OK))
            self._rpc.put(("error", f"connection closed by broker: {code} {text}"))
        elif cm == B_CANCEL:  # broker-side consumer cancel notification
            self._consumers.pop(r.shortstr(), None)
        elif cm in (B_ACK, B_NACK) and self.confirming:  # publisher confirm
            tag, multiple = r.longlong(), r.bit()
            with self._confirm_cv:
                done = {t for t in self._unconfirmed if t <= tag} if multiple else {tag}
                if cm == B_NACK:
                    self._nacked.extend(sorted(done & self._unconfirmed))
                self._unconfirmed -= done
                self._confirm_cv.notify_all()
        else:
            self._rpc.put((cm, r))

    # -- API
    def queue_declare(self, name: str, durable: bool = True, passive: bool = False) -> Tuple[str, int, int]:
        args = (Writer().short(0).shortstr(name).bit(passive).bit(durable).bit(False).bit(False).bit(False)
                .table({}).bytes())
        r = self._call(Q_DECLARE, args, Q_DECLARE_OK)
        return r.shortstr(), r.long(), r.long()

    def queue_purge(self, name: str) -> int:
        r = self._call(Q_PURGE, Writer().short(0).shortstr(name).bit(False).bytes(), Q_PURGE_OK)
        return r.long()

    def basic_qos(self, prefetch_count: int):
        self._call(B_QOS, Writer().long(0).short(prefetch_count).bit(False).bytes(), B_QOS_OK)

    def publish(self, queue: str, body: bytes, exchange: str = "", persistent: bool = False) -> bool:
        """sendToQueue: default exchange, routing key = queue.  Returns False while the broker
        asked us to stop (flow/blocked), mirroring amqplib's write-buffer-full signal."""
        data = method_frame(self.ch, B_PUBLISH, Writer().short(0).shortstr(exchange).shortstr(queue)
                            .bit(False).bit(False).bytes())
        data += content_frames(self.ch, body, self.frame_max, delivery_mode=2 if persistent else None)
        with self._wlock:  # the confirm sequence number follows the wire order of publishes
            if self.confirming:
                self._pub_seq += 1
                with self._confirm_cv:
                    self._unconfirmed.add(self._pub_seq)
            self.sock.sendall(data)
        return self.flow_active and not self.blocked

    def confirm_select(self):
        """Put the channel in confirm mode (RabbitMQ publisher confirms)."""
        if not self.confirming:
            self._call(CONFIRM_SELECT, Writer().bit(False).bytes(), CONFIRM_SELECT_OK)
            self.confirming = True

    def wait_confirms(self, timeout: float = 30.0) -> bool:
        """Blocks until every publish so far is acked; raises if the broker nacked any or the
        connection died.  Returns False on timeout."""
        import time as _t
        end = _t.monotonic() + timeout
        with self._confirm_cv:
            while self._unconfirmed:
                if self.closed:
                    raise AMQPError("connection lost with unconfirmed publishes")
                left = end - _t.monotonic()
                if left <= 0:
                    return False
                self._confirm_cv.wait(min(left, 0.2))
            if self._nacked:
                n, self._nacked = self._nacked, []
                raise AMQPError(f"broker nacked {len(n)} publishes")
        return True

    def consume(self, queue: str, callback: Callable[[Message], None], consumer_tag: str = "",
                no_ack: bool = False) -> str:
        if not consumer_tag:  # a client-chosen tag: deliveries can race the consume-ok
            import uuid
            consumer_tag = f"apm.ctag-{uuid.uuid4().hex[:12]}"
        self._consumers[consumer_tag] = callback  # registered first: deliveries may race the -ok
        args = (Writer().short(0).shortstr(queue).shortstr(consumer_tag).bit(False).bit(no_ack).bit(False)
                .bit(False).table({}).bytes())
        r = self._call(B_CONSUME, args, B_CONSUME_OK)
        tag = r.shortstr()
        if tag != consumer_tag:
            self._consumers[tag] = self._consumers.pop(consumer_tag)
        return tag

    def cancel(self, consumer_tag: str):
        self._call(B_CANCEL, Writer().shortstr(consumer_tag).bit(False).bytes(), B_CANCEL_OK)
        self._consumers.pop(consumer_tag, None)

    def get(self, queue: str, no_ack: bool = True) -> Optional[bytes]:
        self._send(method_frame(self.ch, B_GET, Writer().short(0).shortstr(queue).bit(no_ack).bytes()))
        got, r = self._rpc.get(timeout=self.timeout)
        if got == B_GET_EMPTY:
            return None
        if got == "error":
            raise AMQPError(r)
        return r[1]

    def ack(self, delivery_tag: int, multiple: bool = False):
        self._send(method_frame(self.ch, B_ACK, Writer().longlong(delivery_tag).bit(multiple).bytes()))

    def close(self):
        if self.closed:
            return
        try:
            self._call(CH_CLOSE, Writer().short(200).shortstr("bye").short(0).short(0).bytes(), CH_CLOSE_OK)
            self._send(method_frame(0, CONN_CLOSE, Writer().short(200).shortstr("bye").short(0).short(0).bytes()))
        except Exception:
            pass
        self.closed = True
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        self.sock.close()
