"""Queue layer: AMQP 0-9-1 client <-> in-process broker, reference producer/consumer semantics."""
import threading
import time

import pytest

from apmbackend_amd.runtime import amqp
from apmbackend_amd.runtime.amqp_broker import Broker
from apmbackend_amd.runtime.queue import LOCAL, QueueManager, QueueStats


def wait_for(pred, timeout=5.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.01)
    return pred()


@pytest.fixture
def broker():
    b = Broker(port=0).start()
    yield b
    b.stop()


def test_codec_roundtrip():
    w = amqp.Writer().short(7).shortstr("abc").bit(True).bit(False).bit(True).longlong(1 << 40).table(
        {"a": 1, "b": "x", "c": {"d": True}, "e": [1, "y"], "f": 1.5, "g": None})
    r = amqp.Reader(w.bytes())
    assert r.short() == 7 and r.shortstr() == "abc"
    assert (r.bit(), r.bit(), r.bit()) == (True, False, True)
    assert r.longlong() == 1 << 40
    assert r.table() == {"a": 1, "b": "x", "c": {"d": True}, "e": [1, "y"], "f": 1.5, "g": None}
    assert amqp.parse_url("amqp://u:p@h:5772/v")["vhost"] == "v"


def test_publish_consume_ack_and_declare_counts(broker):
    c = amqp.Connection(broker.url)
    assert c.queue_declare("transactions") == ("transactions", 0, 0)
    for i in range(50):
        c.publish("transactions", f"tx|{i}".encode())
    assert c.queue_declare("transactions")[1] == 50
    got = []
    c2 = amqp.Connection(broker.url)
    c2.consume("transactions", lambda m: (got.append(m.body), c2.ack(m.delivery_tag)), consumer_tag="xConsumerTagx")
    assert wait_for(lambda: len(got) == 50)
    assert got == [f"tx|{i}".encode() for i in range(50)]
    big = b"x" * 300000  # spans several body frames
    c.publish("transactions", big)
    assert wait_for(lambda: len(got) == 51) and got[-1] == big
    assert broker.stats()["transactions"]["messages"] == 0
    c.close()
    c2.close()


def test_unacked_messages_are_redelivered(broker):
    c = amqp.Connection(broker.url)
    c.queue_declare("stats")
    for i in range(5):
        c.publish("stats", str(i).encode())
    seen = []
    c2 = amqp.Connection(broker.url)
    c2.basic_qos(2)
    c2.consume("stats", lambda m: seen.append(m.body))  # never acks
    assert wait_for(lambda: len(seen) == 2)
    time.sleep(0.1)
    assert len(seen) == 2  # prefetch window respected
    c2.close()
    assert wait_for(lambda: broker.stats()["stats"]["messages"] == 5)
    assert c.get("stats") == b"0" and c.queue_purge("stats") == 4
    c.close()


def test_bad_credentials_refused(broker):
    with pytest.raises(amqp.AMQPError):
        amqp.Connection(f"amqp://guest:nope@{broker.host}:{broker.port}")


def test_queue_manager_over_amqp_with_flow_control():
    b = Broker(port=0, high_water=20, low_water=5).start()
    try:
        qm = QueueManager(b.url, stat_interval_s=60)
        events = []
        qm.on("pause", lambda: events.append("pause"))
        qm.on("resume", lambda: events.append("resume"))
        p = qm.get_queue("z_score", "p")
        for i in range(60):
            p.write_line(f"fs|{i}")
            time.sleep(0.001)
        assert wait_for(lambda: "pause" in events)
        assert p.buffer_count() > 0
        got = []
        qm2 = QueueManager(b.url)
        c = qm2.get_queue("z_score", "c", lambda body: got.append(body.decode()))
        c.start_consume()
        assert wait_for(lambda: len(got) == 60, timeout=10)
        assert got == [f"fs|{i}" for i in range(60)]  # order kept through pause / buffer / resume
        assert events[-1] == "resume"
        line = qm.stats.line()
        assert line.startswith("OUT>z_score: 60")
        assert qm2.stats.line() == "IN<z_score: 60"
        c.stop_consume()
        qm.shutdown()
        qm2.shutdown()
    finally:
        b.stop()


def test_local_backend_backpressure():
    name = "db_insert_local_test"
    qm = QueueManager("local://", local_capacity=10)
    events = []
    qm.on("pause", lambda: events.append("pause"))
    qm.on("resume", lambda: events.append("resume"))
    p = qm.get_queue(name, "p")
    for i in range(30):
        p.write_line(str(i))
    assert events == ["pause"] and p.buffer_count() == 20
    got = []
    qm2 = QueueManager("local://", local_capacity=10)
    cons = qm2.get_queue(name, "c", lambda b: got.append(int(b)))
    cons.start_consume()
    assert wait_for(lambda: len(got) == 30)
    assert got == list(range(30)) and events[-1] == "resume"
    cons.stop_consume()
    qm.shutdown()
    qm2.shutdown()


def test_queue_stats_alignment():
    s = QueueStats(60)
    assert s.next_delay(now=120.0) == 60
    assert s.next_delay(now=125.0) == 55
    s.add_counter("a", "c")
    s.incr("a", 3)
    assert s.line() == "IN<a: 3" and s.line() == "IN<a: 0"


def test_publisher_confirms_and_persistent_messages(broker):
    """Q15: the bridge publishes persistent messages on a confirm.select'ed channel and can wait
    until the broker acknowledged everything (before committing tail offsets)."""
    qm = QueueManager(broker.url, confirms=True, persistent=True)
    p = qm.get_queue("db_insert", "p")
    for i in range(200):
        p.write_line(f"fs|{i}")
    assert qm.wait_confirms(10.0)
    assert qm._prod._unconfirmed == set() and qm._prod._pub_seq == 200
    assert broker.stats()["db_insert"]["messages"] == 200
    qm.shutdown()
    local = QueueManager("local://", confirms=True)
    assert local.wait_confirms(0.1)  # in-process backend: nothing to wait for
