"""JMX poller (pull_jvm_stats.js) and the standalone db_insert consumer process."""
import time

from apmbackend_amd.runtime import jmx, sinks
from apmbackend_amd.runtime.amqp import Connection
from apmbackend_amd.runtime.amqp_broker import Broker
from apmbackend_amd.runtime.insert_db import InsertDbProcess
from apmbackend_amd.utils.config import default_config
from apmbackend_amd.utils.records import entry_from_csv


def test_cli_to_json_glues_documents_and_drops_warnings():
    out = ('WARN something\n{\n    "outcome" : "success",\n    "result" : {"InUseCount" : 3}\n}\n'
           '{\n    "outcome" : "success",\n    "result" : 1.5\n}\n')
    d = jmx.cli_to_json(["ds", "sysload"], out)
    assert d["ds"]["result"]["InUseCount"] == 3 and d["sysload"]["result"] == 1.5


class Clock:
    t = 1_600_000_010.0

    def __call__(self):
        return self.t


def test_poller_emits_jx_records_aligned_to_interval():
    C = default_config(replay=True)
    C["pullJvmStats"]["jvmHosts"] = ["jvm1.example.com", "jvm2.example.com", "down.example.com"]
    got = []
    syn = jmx.SyntheticJmx(3)

    def runner(argv, t):
        if any("down." in a for a in argv):
            raise RuntimeError("connection refused")
        return syn.runner(argv, t)

    clk = Clock()
    p = jmx.JvmStatsPoller(C, got.append, runner=runner, clock=clk)
    assert p.next_due == 1_600_000_020.0  # 60 s interval aligned to :00 (start at :10 -> +50 s)... 
    assert not p.tick()
    clk.t = p.next_due
    lines = p.tick()
    assert len(lines) == 2 and got == lines
    e = entry_from_csv(lines[0])
    assert e.type == "jx" and e.server == "jvm1" and e.timestamp == int(clk.t * 1000)
    assert len(e.values) == 16 and 0.1 <= e.values[9] <= 12.0
    cmd = jmx.cli_command("h", "a,b", C["pullJvmStats"])
    assert cmd[:3] == ["java", "-jar", C["pullJvmStats"]["clientJarFullPath"]] and cmd[-1] == "commands=a,b"


def test_insert_db_process_consumes_queue():
    b = Broker(port=0).start()
    try:
        C = default_config(replay=True)
        C["amqpConnectionString"] = b.url
        C["apmConfigFilePath"] = None
        C["streamInsertDb"]["bufferResumeFileFullPath"] = None
        C["streamInsertDb"]["dbInsertBufferLimit"] = 2

        class W(sinks.Writer):
            rows = []

            def write(self, table, columns, rows):
                W.rows += [(table, r) for r in rows]

        p = InsertDbProcess(C, writer=W())
        c = Connection(b.url)
        c.queue_declare("db_insert")
        for i in range(5):
            c.publish("db_insert", f"tx|jvm|S:a|[L{i}]|1|1578391200000|1578391200250|250|Y".encode())
        t0 = time.time()
        while len(W.rows) < 4 and time.time() - t0 < 5:
            time.sleep(0.05)
        p.close()
        assert len(W.rows) == 5 and all(t == "tx" for t, _ in W.rows)
        c.close()
    finally:
        b.stop()
