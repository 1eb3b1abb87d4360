"""Alert e-mail batching (stream_process_alerts.js sendAlertsRecurse) and the rolling logger."""
import datetime as dt
import email
import logging
import os
import time

from apmbackend_amd.runtime import logger as apmlog
from apmbackend_amd.runtime import notifier
from apmbackend_amd.utils.config import default_config
from apmbackend_amd.utils.records import entry_from_csv

FS = ("fs|1578391200000|jvm01|S:getFoo|360|1.20|12000.0:240.1:200.0:280.2:1|13000.0:undefined:undefined:"
      "undefined:0.0|400.0:390.0:380.0:400.0:-1.0")


def al(server="jvm01", service="S:getFoo", ts=1578391200000, lag=360):
    fs = FS.replace("jvm01", server).replace("S:getFoo", service).replace("1578391200000", str(ts)).replace(
        "|360|", f"|{lag}|")
    return f"al|{ts + 1000}|{ts}|{server}|{service}|average exceeded hard ms threshold|" + fs.replace("|", "&")


class Clock:
    t = 1000.0

    def __call__(self):
        return self.t


def test_html_table_matches_reference_layout():
    a = entry_from_csv(al())
    html = notifier.format_alerts_html([a])
    assert html.startswith('<style type="text/css" media="all"> table { border-collapse: collapse; }')
    assert "<td>jvm01</td><td>S:getFoo</td>" in html
    assert '<td class="center">360</td><td>average exceeded hard ms threshold</td>' in html
    # tpm / avg / avgUB / p75 / p75UB with toFixed(1); undefined -> NaN
    assert ('<td class="bbcenter">1.2</td><td class="bbcenter">12000.0</td><td class="bbcenter">280.2</td>'
            '<td class="bbcenter">13000.0</td><td class="bbcenter">NaN</td>') in html
    assert html.endswith("</table>")


def test_grafana_urls():
    g = default_config(replay=True)["grafana"]
    alerts = [entry_from_csv(al()), entry_from_csv(al("jvm02", lag=8640, ts=1578391260000))]
    url, render = notifier.grafana_urls(alerts, now_ms=1578392000000.0, grafana=g)
    assert url.startswith(g["grafanaURL"] + g["alertInspectorRelativeURL"] + "?from=1578390900000&to=1578391560000")
    assert "&var-server=jvm01&var-server=jvm02&var-service=S:getFoo&var-lag=360&var-lag=8640" in url
    assert f"&height={100 + 750 * (2 * 1 * 2 + 1)}" in render and "/render/d/" in render
    # 'to' clamps to now - grafanaNowDelayIntervalMs when the window reaches the present
    url2, _ = notifier.grafana_urls(alerts, now_ms=1578391600000.0, grafana=g)
    assert "&to=1578391510000" in url2


def test_collection_interval_backoff_and_reset(tmp_path):
    C = default_config(replay=True)
    ac = C["streamProcessAlerts"]
    ac.update({"alertCollectionIntervalInSeconds": 60, "maxCollectionIntervalInSeconds": 200,
               "increaseCollectionIntervalAfterAlert": True, "emailsEnabled": "true"})
    clk = Clock()
    mailer = notifier.Mailer(sendmail="/nonexistent/sendmail", outbox=str(tmp_path))
    img = tmp_path / "g.png"
    img.write_bytes(b"\x89PNG\r\n\x1a\nfake")
    n = notifier.AlertNotifier(C, mailer, clock=clk, renderer=lambda url, g: str(img))
    n.add_line(al())
    assert not n.tick()  # not due yet
    clk.t += 60
    assert n.tick() and n.interval == 120
    n.add_line(al())
    clk.t += 120
    assert n.tick() and n.interval == 240  # doubled again (was below max)
    n.add_line(al())
    clk.t += 240
    assert n.tick() and n.interval == 240  # at/above max: no further doubling
    clk.t += 240
    assert not n.tick() and n.interval == 60  # quiet interval resets
    assert n.emails == 3 and len(os.listdir(tmp_path)) == 4  # 3 .eml + the png
    msg = mailer.sent[0]
    assert msg["Subject"] == "APM Alerts Triggered!"
    parts = list(msg.walk())
    assert any(p.get_content_type() == "image/png" for p in parts)
    html = [p for p in parts if p.get_content_type() == "text/html"][0].get_payload(decode=True).decode()
    assert "Cooldown until further alerts are sent out: 2 minutes" in html and 'src="cid:graph_' in html


def test_render_failure_falls_back_to_test_list(tmp_path):
    C = default_config(replay=True)
    clk = Clock()
    mailer = notifier.Mailer(sendmail="/nonexistent/sendmail", outbox=str(tmp_path))

    def boom(url, g):
        raise OSError("grafana down")

    n = notifier.AlertNotifier(C, mailer, clock=clk, renderer=boom)
    n.add_line(al())
    clk.t += 61
    assert n.tick()
    assert mailer.sent[0]["To"] == C["streamProcessAlerts"]["testEmailList"]


def test_emails_disabled_string_false():
    C = default_config(replay=True)
    C["streamProcessAlerts"]["emailsEnabled"] = "false"
    clk = Clock()
    n = notifier.AlertNotifier(C, notifier.Mailer(sendmail="/nonexistent"), clock=clk, renderer=lambda u, g: None)
    n.add_line(al())
    clk.t += 61
    assert not n.tick() and n.buffer  # kept, not mailed


def test_daily_rolling_logger_and_pruning(tmp_path):
    lg = apmlog.set_global_logger(str(tmp_path), "stream_calc_stats", colorize=False)
    lg.getChild("x").info("hello %d", 5)
    lg.getChild("x").warning("careful")
    day = dt.datetime.now().strftime("%Y%m%d")
    path = tmp_path / f"stream_calc_stats.log.{day}"
    lines = path.read_text().splitlines()
    assert lines[0].endswith("INFO hello 5") and lines[1].endswith("WARN careful")
    assert lines[0][:8] == day
    old = tmp_path / "stream_calc_stats.log.20000101"
    old.write_text("x")
    removed = apmlog.prune_logs(str(tmp_path), 7)
    assert removed == [str(old)] and path.exists()
    for h in list(lg.handlers):
        lg.removeHandler(h)
        h.close()


def test_startup_test_email_goes_to_test_list(tmp_path):
    """sendTestEmail at alerts-module start (stream_process_alerts.js:54-56,597)."""
    C = default_config(replay=True)
    mailer = notifier.Mailer(sendmail="/nonexistent/sendmail", outbox=str(tmp_path))
    n = notifier.AlertNotifier(C, mailer, clock=Clock(), renderer=lambda u, g: None)
    out = n.send_test_email()
    assert out and os.path.exists(out)
    msg = mailer.sent[0]
    assert msg["To"] == C["streamProcessAlerts"]["testEmailList"]
    assert msg["Subject"] == "Test APM alert email"
    html = [p for p in msg.walk() if p.get_content_type() == "text/html"][0].get_payload(decode=True).decode()
    assert html == "If you get this email, emails are working!"
    C["streamProcessAlerts"]["sendTestEmailOnStart"] = "false"
    assert n.send_test_email() is None and len(mailer.sent) == 1


def test_shipped_config_uses_the_reference_wall_alert_clock():
    from apmbackend_amd.utils.config import default_config as dc
    assert dc()["gpu"]["alertClock"] == "wall"
    assert dc(replay=True)["gpu"]["alertClock"] == "entry"
