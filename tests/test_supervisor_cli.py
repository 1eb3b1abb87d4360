"""Supervisor tree (apm_manager.js) and the CLI tools, with throw-away child processes."""
import io
import os
import signal
import sys
import time

import pytest

from apmbackend_amd.cli import backup, dequeue, pid_stats, qstat
from apmbackend_amd.runtime import supervisor as sup
from apmbackend_amd.runtime.amqp import Connection
from apmbackend_amd.runtime.amqp_broker import Broker
from apmbackend_amd.runtime.notifier import Mailer
from apmbackend_amd.utils.config import default_config


def wait_for(pred, timeout=10.0):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


def make_cfg(tmp_path, modules, **mgr):
    C = default_config(replay=True)
    C["logDir"] = str(tmp_path / "logs")
    C["appDirectory"] = str(tmp_path)
    C["apmConfigFilePath"] = None
    m = C["applicationManager"]
    m.update({"moduleSettings": modules, "stateDir": str(tmp_path / "state"), "restartDelaySeconds": 0.2,
              "crashLoopWindowSeconds": 1.0, "crashLoopDelaySeconds": 2.0, "inspectionFrequencySeconds": 1,
              "alertCollectionIntervalInSeconds": 1, "diskSpaceGBAvailableThreshold": 0,
              "diskSpacePercentageUsedThreshold": 101})
    m.update(mgr)
    return C


def script(tmp_path, name, body):
    p = tmp_path / name
    p.write_text("import sys, time, signal\n" + body)
    return name


def test_restart_and_crash_loop_damping(tmp_path):
    crash = script(tmp_path, "crash.py", "sys.exit(3)\n")
    sleeper = script(tmp_path, "sleeper.py", "time.sleep(60)\n")
    C = make_cfg(tmp_path, [{"name": "crashy", "relativePath": crash, "passConfig": False},
                            {"name": "steady", "relativePath": sleeper, "passConfig": False}])
    notes = []
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda g, text, tags: notes.append(text))
    s.start_all()
    try:
        crashy = s.modules[0].procs[0]
        assert wait_for(lambda: (s.check_children() or True) and crashy.restart_at is not None)
        # died < crashLoopWindow after start -> long delay
        assert crashy.restart_at - crashy.last_start >= 2.0 - 0.1
        assert "Module exited: crashy" in notes
        assert wait_for(lambda: (s.check_children() or True) and crashy.restarts >= 1, timeout=6)
        steady = s.modules[1].procs[0]
        assert steady.poll() is None and steady.restarts == 0
        assert any("Child module exited" in a for a in s.alert_buffer)
        s.next_alert = 0
        assert s.send_alerts() and s.emails == 1
        assert os.path.exists(tmp_path / "logs" / "crashy.start.log")
        assert open(tmp_path / "state" / "steady.pid").read().strip() == str(steady.pid)
    finally:
        s.stop_all()


def test_rank_group_restarts_together(tmp_path):
    r = script(tmp_path, "rank.py", "import os\nif os.environ['RANK']=='1': time.sleep(0.5); sys.exit(1)\n"
                                    "time.sleep(60)\n")
    C = make_cfg(tmp_path, [{"name": "engine", "relativePath": r, "ranks": 2, "passConfig": False}],
                 crashLoopWindowSeconds=0.1)
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda *a: None)
    s.start_all()
    try:
        p0, p1 = s.modules[0].procs
        assert p0.env["WORLD_SIZE"] == "2" and p1.env["LOCAL_RANK"] == "1"
        assert wait_for(lambda: (s.check_children() or True) and p1.restart_at is not None)
        assert p0.restart_at is not None and p0.poll() is not None  # survivor stopped for the group restart
        assert wait_for(lambda: (s.check_children() or True) and p0.restarts == 1 and p1.restarts == 1)
    finally:
        s.stop_all()


def test_memory_threshold_sends_request_gc(tmp_path):
    body = ("got = []\nsignal.signal(signal.SIGUSR1, lambda *a: open(sys.argv[1], 'w').write('gc'))\n"
            "time.sleep(60)\n")
    g = script(tmp_path, "gc.py", body)
    flag = tmp_path / "gc.flag"
    C = make_cfg(tmp_path, [{"name": "hog", "relativePath": g, "passConfig": False, "args": [str(flag)],
                             "moduleMemoryAlertThreshold": 0.001}])
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda *a: None)
    s.start_all()
    try:
        time.sleep(0.5)
        s.inspect()
        assert s.gc_requests == ["hog"]
        assert any("exceeded the memory threshold" in a for a in s.alert_buffer)
        assert wait_for(lambda: flag.exists())
    finally:
        s.stop_all()


def test_hbm_threshold_request_gc_is_rate_limited(tmp_path, monkeypatch):
    """An HBM-only breach sends requestGC at most once per gpuGcMinIntervalSeconds (each trim
    flushes the engine and rebuilds the join table); RSS / swap keep the every-inspection rule."""
    body = "signal.signal(signal.SIGUSR1, lambda *a: None)\ntime.sleep(60)\n"
    g = script(tmp_path, "gc.py", body)
    C = make_cfg(tmp_path, [{"name": "hbm", "relativePath": g, "passConfig": False,
                             "moduleGpuMemoryAlertThreshold": 1, "gpuGcMinIntervalSeconds": 100}])
    now = [1000.0]
    monkeypatch.setattr(sup, "pid_vram_mb", lambda pid: 5000.0)
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda *a: None, clock=lambda: now[0])
    s.start_all()
    try:
        time.sleep(0.3)
        s.inspect_modules()
        s.inspect_modules()
        assert s.gc_requests == ["hbm"]  # the second breach within the interval: alert only
        assert sum("GPU memory threshold" in a for a in s.alert_buffer) == 2
        now[0] += 101
        s.inspect_modules()
        assert s.gc_requests == ["hbm", "hbm"]
    finally:
        s.stop_all()


def test_stale_pid_only_killed_when_marker_matches(tmp_path):
    import subprocess
    other = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(30)"], start_new_session=True)
    try:
        (tmp_path / "state").mkdir()
        (tmp_path / "state" / "m.pid").write_text(str(other.pid))
        p = sup.Proc("m", [sys.executable, "-c", "pass"], {}, str(tmp_path / "m.log"), str(tmp_path / "state/m.pid"))
        assert p.kill_stale() is None and other.poll() is None  # not ours: untouched
    finally:
        other.kill()
        other.wait()


def test_pid_stats_quiet_format(capsys):
    assert pid_stats.main(["-p", str(os.getpid()), "-S", "-q", "-m"]) == 0
    out = capsys.readouterr().out.split()
    assert out[1] == "MiB" and out[3] == "MiB" and float(out[0]) > 1
    mem, swap = sup.pid_mem_swap_mb(os.getpid())
    assert mem > 1 and swap >= 0


def test_qstat_and_dequeue_against_broker(tmp_path, capsys):
    b = Broker(port=0).start()
    try:
        c = Connection(b.url)
        c.queue_declare("db_insert")
        for i in range(3):
            c.publish("db_insert", f"tx|{i}".encode())
        rows = qstat.queue_table(b.url, ["db_insert", "nope"])
        assert rows == [("db_insert", 3, 0), ("nope", None, None)]
        buf = io.StringIO()
        dequeue.main(["--url", b.url, "--count", "3", "db_insert"], out=buf)
        assert buf.getvalue().splitlines() == ["tx|0", "tx|1", "tx|2"]
        c.close()
    finally:
        b.stop()


def test_backup(tmp_path):
    files = backup.backup(str(tmp_path), stamp="2026101512")
    assert any(f.endswith("apmbackend_amd/runtime/service.py.2026101512") for f in files)
    assert any(f.endswith("config/apm_config.json.2026101512") for f in files)


def test_rank_group_elastic_degrade(tmp_path):
    """A GPU whose rank keeps failing is retired: 4 GPUs -> 3 healthy -> world 2 (powers of two),
    HIP_VISIBLE_DEVICES / WORLD_SIZE / MASTER_PORT of the new generation, alert + annotation."""
    r = script(tmp_path, "rank.py", "import os\n"
                                    "if os.environ['APM_DEVICE']=='1': sys.exit(2)\n"
                                    "time.sleep(60)\n")
    C = make_cfg(tmp_path, [{"name": "engine", "relativePath": r, "ranks": 4, "passConfig": False,
                             "masterPort": 29600}],
                 crashLoopWindowSeconds=0.0, restartDelaySeconds=0.05, elasticMaxFailures=3,
                 elasticWindowSeconds=600)
    notes = []
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda g, text, tags: notes.append(text))
    s.start_all()
    mod = s.modules[0]
    try:
        assert [p.env["APM_DEVICE"] for p in mod.procs] == ["0", "1", "2", "3"]
        assert "HIP_VISIBLE_DEVICES" not in mod.procs[0].env
        assert wait_for(lambda: (s.check_children() or True) and mod.generation == 1, timeout=20)
        assert mod.bad_devices == {1} and mod.ranks == 2
        assert [p.env["WORLD_SIZE"] for p in mod.procs] == ["2", "2"]
        assert all(p.env["HIP_VISIBLE_DEVICES"] == "0,2" for p in mod.procs)
        assert [p.env["APM_DEVICE"] for p in mod.procs] == ["0", "2"]
        assert mod.procs[0].env["MASTER_PORT"] == "29601"
        assert any("degraded from 4 to 2 GPUs" in n for n in notes)
        assert any("degraded from 4 to 2 GPUs" in a for a in s.alert_buffer)
        # the new generation starts and stays up (device 1 is no longer used)
        assert wait_for(lambda: (s.check_children() or True) and all(p.popen is not None for p in mod.procs))
        time.sleep(0.3)
        s.check_children()
        assert all(p.poll() is None for p in mod.procs) and mod.generation == 1
    finally:
        s.stop_all()


def test_hung_rank_is_blamed_when_its_peers_abort(tmp_path):
    """A rank that hangs never exits; its peers' watchdogs abort and exit PEER_FAILURE_EXIT (75).
    The supervisor blames the rank still running after the grace period (its GPU is retired),
    not a survivor, so a wedged GPU cannot restart the group forever."""
    r = script(tmp_path, "rank.py", "import os\n"
                                    "if os.environ['APM_DEVICE']=='2': time.sleep(60)\n"
                                    "time.sleep(0.3); sys.exit(75)\n")
    C = make_cfg(tmp_path, [{"name": "engine", "relativePath": r, "ranks": 4, "passConfig": False,
                             "masterPort": 29640}],
                 crashLoopWindowSeconds=0.0, restartDelaySeconds=0.05, elasticMaxFailures=1,
                 elasticWindowSeconds=600, groupAbortGraceSeconds=1.0)
    notes = []
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda g, text, tags: notes.append(text))
    s.start_all()
    mod = s.modules[0]
    try:
        assert wait_for(lambda: (s.check_children() or True) and mod.generation == 1, timeout=20)
        assert mod.bad_devices == {2} and mod.ranks == 2
        assert any("hung" in a for a in s.alert_buffer)
        assert any("GPU 2 failed" in n for n in notes)
    finally:
        s.stop_all()


def test_elastic_degrade_can_be_disabled(tmp_path):
    r = script(tmp_path, "rank.py", "sys.exit(2)\n")
    C = make_cfg(tmp_path, [{"name": "engine", "relativePath": r, "ranks": 2, "passConfig": False,
                             "elasticDegrade": False}],
                 crashLoopWindowSeconds=0.0, restartDelaySeconds=0.05, elasticMaxFailures=1)
    s = sup.Supervisor(C, mailer=Mailer(sendmail="/nonexistent", outbox=str(tmp_path / "out")),
                       annotate=lambda *a: None)
    s.start_all()
    mod = s.modules[0]
    try:
        assert wait_for(lambda: (s.check_children() or True) and mod.procs[0].restarts >= 1)
        assert mod.generation == 0 and mod.ranks == 2 and not mod.bad_devices
    finally:
        s.stop_all()


def test_broker_liveness_autostart_and_queue_thresholds(tmp_path):
    """monitorResourcesRecurs / rabbitMQIsRunning / startRabbitMQ / inspectQueues
    (apm_manager.js:134-155, 429-453, 517-521) with a stand-in rabbitmqctl + rabbitmq-server."""
    sbin = tmp_path / "sbin"
    sbin.mkdir()
    up = tmp_path / "broker_up"
    (sbin / "rabbitmqctl").write_text(
        "#!/bin/sh\n"
        f"[ -f {up} ] || exit 2\n"
        "if [ \"$1\" = list_queues ]; then\n"
        "  echo 'db_insert 5 100 2000000 900000000 1300000000'\n"
        "  echo 'transactions 3 10 0 0 4096'\n"
        "fi\n")
    (sbin / "rabbitmq-server").write_text(f"#!/bin/sh\ntouch {up}\necho started\n")
    for f in ("rabbitmqctl", "rabbitmq-server"):
        os.chmod(sbin / f, 0o755)
    C = make_cfg(tmp_path, [], rabbitSbinPath=str(sbin), queueMessageAlertThreshold=1000000,
                 queueMemoryAlertThreshold=1000, brokerStartGraceSeconds=0)
    C["gpu"]["outputMode"] = "amqp"
    s = sup.Supervisor(C, mailer=Mailer(outbox=str(tmp_path / "out")))
    assert not s.broker_is_running()
    assert not s.inspect_broker()  # down -> alert + rabbitmq-server -detached
    assert up.exists() and s.broker_is_running()
    s.inspect_queues()
    alerts = "\n".join(s.alert_buffer)
    assert "RabbitMQ is down" in alerts
    assert "message count threshold - Queue: db_insert" in alerts and "MessageCount: 2000005" in alerts
    assert "memory threshold - Queue: db_insert" in alerts and "transactions" not in alerts.split("memory")[-1]
