"""Queue layer with the reference's producer/consumer contract (queue.js:1-311).

* ``QueueStats`` -- per-queue IN/OUT counters logged (and reset) every
  ``statLogIntervalInSeconds``: ``IN<name: n - OUT>name: m`` (queue.js:4-64).
* ``QueueManager`` -- one producer and one consumer connection per process (queue.js:67-189);
  ``pause`` / ``resume`` callbacks fire when a producer hits broker backpressure and when every
  producer buffer drained again.
* ``ProducerQueue`` -- ``write_line``: while paused (or when the broker refuses) lines go to an
  in-memory buffer; ``retry_buffer`` on drain re-sends in order (queue.js:206-264).
* ``ConsumerQueue`` -- ``start_consume`` / ``stop_consume`` with the reference's consumer tag;
  ``ack_before_process=True`` (default) keeps queue.js:277-283 semantics, ``False`` acks after
  the callback returned (at-least-once, the fix suggested in SURVEY §5.2).

Backends: ``amqp://...`` (RabbitMQ or runtime/amqp_broker.py, via runtime/amqp.py) and
``local://`` (in-process queues with a bounded capacity: the same flow-control states without a
broker; used by the single-process pipeline and tests).
"""
from __future__ import annotations

import collections
import logging
import threading
import time
from typing import Callable, Deque, Dict, List, Optional

log = logging.getLogger("apm.queue")

CONSUMER_TAG = "xConsumerTagx"


class QueueStats:
    def __init__(self, interval_s: float = 60.0):
        self.interval = interval_s
        self.counters: Dict[str, List] = {}  # name -> [type, cnt]
        self._lock = threading.Lock()

    def add_counter(self, name: str, qtype: str, init: int = 0):
        with self._lock:
            self.counters[name] = [qtype, init]
        log.info("Init counter: %s Type: %s", name, qtype)

    def incr(self, name: str, n: int = 1):
        with self._lock:
            self.counters[name][1] += n

    def line(self, reset: bool = True) -> str:
        with self._lock:
            parts = []
            for name, c in self.counters.items():
                parts.append(f"{'IN<' if c[0] == 'c' else 'OUT>'}{name}: {c[1]}")
                if reset:
                    c[1] = 0
            return " - ".join(parts)

    def next_delay(self, now: Optional[float] = None) -> float:
        """Seconds to the next log point aligned to the interval (logQueueStatsRecurs :55-63)."""
        now = time.time() if now is None else now
        sec = int(now) % 60
        return self.interval - (sec % self.interval)


# --------------------------------------------------------------------------- local backend

class _LocalHub:
    """Process-wide in-memory broker: bounded deques + condition variables."""

    def __init__(self):
        self.lock = threading.Condition()
        self.queues: Dict[str, Deque[bytes]] = {}
        self.capacity: Dict[str, int] = {}
        self.drain_listeners: List[Callable[[], None]] = []

    def declare(self, name: str, capacity: int = 0):
        with self.lock:
            self.queues.setdefault(name, collections.deque())
            if capacity:
                self.capacity[name] = capacity

    def put(self, name: str, body: bytes) -> bool:
        with self.lock:
            q = self.queues[name]
            q.append(body)
            self.lock.notify_all()
            cap = self.capacity.get(name, 0)
            return not cap or len(q) < cap

    def get(self, name: str, timeout: float) -> Optional[bytes]:
        with self.lock:
            q = self.queues[name]
            if not q:
                self.lock.wait(timeout)
            if not q:
                return None
            body = q.popleft()
            self.lock.notify_all()
            cap = self.capacity.get(name, 0)
            drained = cap and len(q) == cap // 2
        if drained:  # the channel 'drain' event of the producers
            for fn in list(self.drain_listeners):
                fn()
        return body

    def depth(self, name: str) -> int:
        with self.lock:
            return len(self.queues.get(name, ()))

    def below(self, name: str, frac: float = 0.5) -> bool:
        with self.lock:
            cap = self.capacity.get(name, 0)
            return not cap or len(self.queues[name]) <= cap * frac


LOCAL = _LocalHub()


# --------------------------------------------------------------------------- queues

class ProducerQueue:
    type = "p"

    def __init__(self, mgr: "QueueManager", name: str):
        self.mgr = mgr
        self.name = name
        self.buffer: Deque[str] = collections.deque()
        self.paused = False
        mgr.stats.add_counter(name, "p")

    def _send(self, line: str) -> bool:
        return self.mgr._publish(self.name, line.encode("utf-8"))

    def write_line(self, line: str):
        if self.paused:
            self.buffer.append(line)
            return
        if not self._send(line):
            # the message itself was accepted by the transport; it is the *next* ones that wait
            self.mgr.stats.incr(self.name)
            log.info("--- PRODUCER CHANNEL BUFFER FULL (Q=%s) --- Pausing until drain event", self.name)
            self.pause()
        else:
            self.mgr.stats.incr(self.name)

    def write_lines(self, lines):
        for ln in lines:
            self.write_line(ln)

    def pause(self):
        if not self.paused:
            self.paused = True
            self.mgr._on_producer_pause(self)

    def retry_buffer(self):
        self.paused = False
        while self.buffer and not self.paused:
            self.write_line(self.buffer.popleft())
        if self.buffer:
            log.info("Records still remaining in %s buffer, waiting for next drain: %d records", self.name,
                     len(self.buffer))

    def buffer_count(self) -> int:
        return len(self.buffer)


class ConsumerQueue:
    type = "c"

    def __init__(self, mgr: "QueueManager", name: str, callback: Callable[[bytes], None],
                 ack_before_process: bool = True):
        self.mgr = mgr
        self.name = name
        self.cb = callback
        self.ack_before = ack_before_process
        self.consuming = False
        self._thread: Optional[threading.Thread] = None
        self._tag: Optional[str] = None
        mgr.stats.add_counter(name, "c")

    def _handle(self, body: bytes):
        self.mgr.stats.incr(self.name)
        self.cb(body)

    def start_consume(self):
        if self.consuming:
            return
        self.consuming = True
        if self.mgr.backend == "local":
            self._thread = threading.Thread(target=self._local_loop, name=f"consume-{self.name}", daemon=True)
            self._thread.start()
        else:
            conn = self.mgr._consumer_conn()

            def on_msg(m):
                if self.ack_before:
                    conn.ack(m.delivery_tag)
                    self._handle(m.body)
                else:
                    self._handle(m.body)
                    conn.ack(m.delivery_tag)

            self._tag = conn.consume(self.name, on_msg, consumer_tag=CONSUMER_TAG)

    def _local_loop(self):
        while self.consuming:
            body = LOCAL.get(self.name, 0.2)
            if body is not None:
                self._handle(body)

    def stop_consume(self):
        self.consuming = False
        if self._tag is not None:
            try:
                self.mgr._consumer_conn().cancel(self._tag)
            except Exception as e:  # pragma: no cover - broker went away
                log.error("channel.cancel() threw an error: %s", e)
            self._tag = None
        if self._thread is not None:
            self._thread.join(timeout=2)
            self._thread = None


class QueueManager:
    def __init__(self, url: str = "local://", stat_interval_s: float = 60.0, local_capacity: int = 0,
                 confirms: bool = False, persistent: bool = False):
        """``confirms``: publisher confirms on the producer channel (wait_confirms() before the
        caller commits its own progress, e.g. tail offsets -> at-least-once delivery across a
        crash); ``persistent``: delivery_mode 2 (durable queues keep them across a broker restart)."""
        self.url = url
        self.confirms = confirms
        self.persistent = persistent
        self.backend = "local" if url.startswith("local:") else "amqp"
        self.stats = QueueStats(stat_interval_s)
        self.queues: Dict[str, object] = {}
        self.local_capacity = local_capacity
        self._prod = None
        self._cons = None
        self._listeners: Dict[str, List[Callable[[], None]]] = {"pause": [], "resume": []}
        self._paused = False
        self._lock = threading.Lock()

    # events (EventEmitter 'pause' / 'resume')
    def on(self, event: str, fn: Callable[[], None]):
        self._listeners[event].append(fn)

    def _emit(self, event: str):
        for fn in self._listeners[event]:
            fn()

    # connections
    def _producer_conn(self):
        if self._prod is None:
            from .amqp import Connection
            self._prod = Connection(self.url, on_pause=self._broker_pause, on_resume=self._broker_resume)
            if self.confirms:
                self._prod.confirm_select()
        return self._prod

    def _consumer_conn(self):
        if self._cons is None:
            from .amqp import Connection
            self._cons = Connection(self.url)
        return self._cons

    def _broker_pause(self):
        for q in self.queues.values():
            if isinstance(q, ProducerQueue):
                q.pause()

    def _broker_resume(self):  # the drain event
        self.retry_all_buffers()

    def _publish(self, name: str, body: bytes) -> bool:
        if self.backend == "local":
            return LOCAL.put(name, body)
        return self._producer_conn().publish(name, body, persistent=self.persistent)

    def wait_confirms(self, timeout: float = 30.0) -> bool:
        """Every message published so far is safely with the broker (no-op without confirms or
        on the in-process backend)."""
        if self.backend == "local" or not self.confirms or self._prod is None:
            return True
        return self._prod.wait_confirms(timeout)

    def _on_producer_pause(self, q: ProducerQueue):
        with self._lock:
            first = not self._paused
            self._paused = True
        if first:
            log.info("Pausing all queues!")
            self._emit("pause")

    def _maybe_drain(self):
        """Local backend: a consumer made room -> behave like the channel 'drain' event."""
        if self._paused and all(LOCAL.below(n) for n, q in self.queues.items() if isinstance(q, ProducerQueue)):
            self.retry_all_buffers()

    def retry_all_buffers(self):
        for q in list(self.queues.values()):
            if isinstance(q, ProducerQueue):
                q.retry_buffer()
        if sum(q.buffer_count() for q in self.queues.values() if isinstance(q, ProducerQueue)) == 0:
            with self._lock:
                was = self._paused
                self._paused = False
            if was:
                self._emit("resume")

    # queues
    def get_queue(self, name: str, qtype: str, callback: Optional[Callable[[bytes], None]] = None, **kw):
        if name in self.queues:
            return self.queues[name]
        if qtype not in ("p", "c"):
            raise ValueError("queue type must be 'p' or 'c'")
        if qtype == "c" and callback is None:
            raise ValueError("a callback must be provided when consuming a queue")
        if self.backend == "local":
            LOCAL.declare(name, self.local_capacity)
            if qtype == "p" and self._maybe_drain not in LOCAL.drain_listeners:
                LOCAL.drain_listeners.append(self._maybe_drain)
        else:
            conn = self._producer_conn() if qtype == "p" else self._consumer_conn()
            conn.queue_declare(name, durable=True)  # assertQueue(name, {durable: true})
        q = ProducerQueue(self, name) if qtype == "p" else ConsumerQueue(self, name, callback, **kw)
        self.queues[name] = q
        return q

    def depth(self, name: str) -> int:
        if self.backend == "local":
            return LOCAL.depth(name)
        return self._producer_conn().queue_declare(name, durable=True)[1]

    def shutdown(self):
        if self._maybe_drain in LOCAL.drain_listeners:
            LOCAL.drain_listeners.remove(self._maybe_drain)
        for q in self.queues.values():
            if isinstance(q, ConsumerQueue):
                q.stop_consume()
        for c in (self._prod, self._cons):
            if c is not None:
                c.close()
        self._prod = self._cons = None
