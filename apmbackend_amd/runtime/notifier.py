"""Alert notification: batched HTML e-mails with a Grafana-rendered graph, and Grafana
annotations (reference ``stream_process_alerts.js:50-85,153-333``, ``util_methods.js:359-396``,
``apm_manager.js:224-244``).

``AlertNotifier`` reproduces ``sendAlertsRecurse``: alerts accumulate in a buffer; every
collection interval (``alertCollectionIntervalInSeconds``), if the buffer is non-empty and
e-mails are enabled, one e-mail goes out (HTML table from ``formatAlertsHTML``, Grafana links
from ``generateGrafanaURL``, legend) and -- with ``increaseCollectionIntervalAfterAlert`` --
the next interval doubles up to ``maxCollectionIntervalInSeconds``; an interval without alerts
resets it.  The graph is fetched from Grafana's /render endpoint (bearer token, self-signed
certificates accepted, ``renderTimeout``) and attached inline (cid); if rendering fails the
mail goes to ``testEmailList`` without the image, as the reference does.

Mail is handed to ``/usr/sbin/sendmail -t`` (nodemailer's sendmail transport).  Without a
sendmail binary the message is written to an outbox directory as an .eml file.
"""
from __future__ import annotations

import datetime as _dt
import email.utils
import json
import logging
import os
import shutil
import ssl
import subprocess
import time
import urllib.request
from email.mime.image import MIMEImage
from email.mime.multipart import MIMEMultipart
from email.mime.text import MIMEText
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..utils.config import as_bool
from ..utils.jsfmt import to_fixed
from ..utils.records import AlertEntry, entry_from_csv

log = logging.getLogger("apm.alerts")

DEEP_BLUE, MED_BLUE, LIGHT_BLUE = "#1ab2ff", "#94DBFF", "#e5f8ff"


def log_date(ms: float) -> str:
    """Date.prototype.convertDateToLogDate (util_methods.js:149-176), local time."""
    d = _dt.datetime.fromtimestamp(ms / 1000.0)
    return d.strftime("%Y-%m-%d %H:%M:%S")


def _fx1(x) -> str:
    return to_fixed(x, 1)


def format_alerts_html(alerts: List[AlertEntry]) -> str:
    css = ('<style type="text/css" media="all">'
           ' table { border-collapse: collapse; }'
           ' td { font-family: "Calibri"; font-size: 11pt; white-space: nowrap; }'
           ' td, th { padding: 7px; }'
           ' td.bb, th.bb { border-bottom: 2px solid black }'
           ' td.center { text-align: center; }'
           ' td.right { text-align: right; }'
           ' td.bbcenter { border-bottom: 2px solid black; text-align: center; }  </style>')
    header = (f'<table><tr bgcolor="{DEEP_BLUE}"><th>Server</th><th>Service</th><th>Timestamp</th><th>Lag</th>'
              f'<th>Cause</th></tr><tr bgcolor="{MED_BLUE}"><th class="bb">TPM</th><th class="bb">Avg</th>'
              f'<th class="bb">Avg UB</th><th class="bb">75%</th><th class="bb">75% UB</th></tr>')
    rows = []
    for a in alerts:
        e = a.fs_entry()
        rows.append(f'<tr bgcolor="white"><td>{e.server}</td><td>{e.service}</td><td>{log_date(e.timestamp)}</td>'
                    f'<td class="center">{e.lag}</td><td>{a.cause}</td></tr>'
                    f'<tr bgcolor="{LIGHT_BLUE}"><td class="bbcenter">{_fx1(e.tpm)}</td>'
                    f'<td class="bbcenter">{_fx1(e.average)}</td><td class="bbcenter">{_fx1(e.averageUB)}</td>'
                    f'<td class="bbcenter">{_fx1(e.per75)}</td><td class="bbcenter">{_fx1(e.per75UB)}</td></tr>')
    return css + header + "".join(rows) + "</table>"


def grafana_url_params(alerts: List[AlertEntry], now_ms: float, grafana: Dict[str, Any]) -> Tuple[str, int]:
    """generateGrafanaURLParams (:153-193)."""
    servers, services, lags = [], [], []
    for a in alerts:
        e = a.fs_entry()
        if e.server not in servers:
            servers.append(e.server)
        if e.service not in services:
            services.append(e.service)
        if e.lag not in lags:
            lags.append(e.lag)
    first = alerts[0].fs_entry().timestamp
    last = alerts[-1].fs_entry().timestamp
    frm = first - 300000
    to = last + 300000
    delay = float(grafana.get("grafanaNowDelayIntervalMs", 90000))
    if now_ms - to <= delay:
        to = now_ms - delay
    p = f"from={int(frm)}&to={int(to)}"
    for s in servers:
        p += f"&var-server={s}"
    for s in services:
        p += f"&var-service={s}"
    for l in lags:
        p += f"&var-lag={l}"
    return p, len(servers) * len(services) * len(lags) + len(services)


def grafana_urls(alerts: List[AlertEntry], now_ms: float, grafana: Dict[str, Any]) -> Tuple[str, str]:
    """generateGrafanaURL (:195-206): (dashboard URL, /render URL)."""
    params, hf = grafana_url_params(alerts, now_ms, grafana)
    base, rel = grafana.get("grafanaURL", ""), grafana.get("alertInspectorRelativeURL", "")
    url = f"{base}{rel}?{params}"
    height = 100 + int(grafana.get("renderHeightMultiple", 750)) * hf
    extra = f"&width={grafana.get('renderWidth', 1800)}&height={height}{grafana.get('renderExtraParams', '')}"
    return url, f"{base}/render{rel}?{params}{extra}"


def legend_html(cfg: Dict[str, Any]) -> str:
    sc = cfg["streamCalcStats"]
    win_s = int(sc["intervalLengthInSeconds"]) * int(sc["windowSizeInIntervals"])
    tpm_example = 1 / (win_s // 60) if win_s >= 60 else float("inf")
    tpm_txt = repr(tpm_example) if tpm_example != int(tpm_example) else str(int(tpm_example))
    iv = sc["intervalLengthInSeconds"]
    return (f"<b>Avg</b>: {win_s} second rolling average of elapsed transaction times."
            f"\n<b>Avg UB</b>: Average upper bound. Determined from the Lag value. A Lag of 360 means the upper bound "
            f"is generated from a one hour period of data."
            f"\n\n<b>75%</b>: {win_s} second rolling 75th percentile of elapsed transaction times."
            f"\n<b>75% UB</b>: 75th percentile upper bound. Determined from the Lag value. A Lag of 360 means the upper "
            f"bound is generated from a one hour period of data."
            f"\n\n<b>Lag</b>: Number of intervals (interval = {iv} seconds) over which the z-score algorithm is applied. "
            f"The z-score determines the upper and lower bounds outside of which an alert is triggered."
            f"\n<b>TPM</b>: Transactions per minute. Note this value is calculated over a {win_s} second interval so a "
            f"single transaction in the window will show a value of {tpm_txt} TPM.")


# --------------------------------------------------------------------------- transport

def build_mail(frm: str, to: str, subject: str, html: str, image_path: Optional[str] = None) -> MIMEMultipart:
    msg = MIMEMultipart("related")
    msg["From"] = frm
    msg["To"] = to
    msg["Subject"] = subject
    msg["Date"] = email.utils.formatdate(localtime=True)
    if image_path:
        cid = f"graph_{int(time.time() * 1000)}"
        html += f'<br><br><img src="cid:{cid}"/>'
    msg.attach(MIMEText(html, "html", "utf-8"))
    if image_path:
        with open(image_path, "rb") as f:
            img = MIMEImage(f.read(), name=os.path.basename(image_path))
        img.add_header("Content-ID", f"<{cid}>")
        img.add_header("Content-Disposition", "inline", filename=os.path.basename(image_path))
        msg.attach(img)
    return msg


class Mailer:
    def __init__(self, sendmail: str = "/usr/sbin/sendmail", outbox: str = "/tmp/apm/outbox"):
        self.sendmail = sendmail if (os.path.exists(sendmail) or shutil.which(sendmail)) else None
        self.outbox = outbox
        self.sent: List[MIMEMultipart] = []

    def send(self, frm: str, to: str, subject: str, html: str, image_path: Optional[str] = None):
        msg = build_mail(frm, to, subject, html, image_path)
        log.info("Sending email! to=%s subject=%s", to, subject)
        self.sent.append(msg)
        if self.sendmail:
            r = subprocess.run([self.sendmail, "-t", "-oi"], input=msg.as_bytes(), capture_output=True, timeout=60)
            if r.returncode != 0:
                raise RuntimeError(f"sendmail failed: {r.stderr.decode(errors='replace')}")
            return "sendmail"
        os.makedirs(self.outbox, exist_ok=True)
        path = os.path.join(self.outbox, f"mail_{int(time.time() * 1000)}_{len(self.sent)}.eml")
        with open(path, "wb") as f:
            f.write(msg.as_bytes())
        return path


def _http(url: str, token: Optional[str], timeout_s: float, data: Optional[bytes] = None, method: str = "GET"):
    req = urllib.request.Request(url, data=data, method=method)
    if token:
        req.add_header("Authorization", token)
    if data is not None:
        req.add_header("Content-Type", "application/json")
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE  # rejectUnauthorized: false (self-signed Grafana)
    return urllib.request.urlopen(req, timeout=timeout_s, context=ctx)


def render_graph(render_url: str, grafana: Dict[str, Any], fetch=_http) -> str:
    """renderGraph (:59-85): download the PNG into renderDir; raises on failure."""
    d = grafana.get("renderDir", "/tmp/apm/renders")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"alert_{_dt.datetime.utcnow().isoformat(timespec='milliseconds')}Z.png")
    with fetch(render_url, grafana.get("bearerToken"), float(grafana.get("renderTimeout", 90000)) / 1000.0) as r:
        data = r.read()
    with open(path, "wb") as f:
        f.write(data)
    return path


def post_annotation(grafana: Dict[str, Any], text: str, tags: List[str], now_ms: Optional[float] = None,
                    fetch=_http) -> bool:
    """sendAnnotation (apm_manager.js:224-244): POST /api/annotations."""
    body = {"time": int(now_ms if now_ms is not None else time.time() * 1000), "tags": tags, "text": text}
    try:
        with fetch(f"{grafana.get('grafanaURL', '')}/api/annotations", grafana.get("bearerToken"), 5.0,
                   json.dumps(body).encode(), "POST"):
            return True
    except Exception as e:
        log.error("Grafana annotation failed: %s", e)
        return False


# --------------------------------------------------------------------------- batching

class AlertNotifier:
    def __init__(self, cfg: Dict[str, Any], mailer: Optional[Mailer] = None, clock: Callable[[], float] = time.time,
                 renderer: Callable[[str, Dict[str, Any]], str] = render_graph):
        self.cfg = cfg
        self.mailer = mailer or Mailer()
        self.clock = clock
        self.renderer = renderer
        self.buffer: List[AlertEntry] = []
        self.base = self._ac()["alertCollectionIntervalInSeconds"]
        self.interval = float(self.base)
        self.next_due = clock() + self.interval
        self.emails = 0

    def _ac(self):
        return self.cfg["streamProcessAlerts"]

    def send_test_email(self):
        """sendTestEmail at alerts-module start (stream_process_alerts.js:54-56,597): the
        reference's only "is mail working" probe, sent to ``testEmailList`` on every start
        (``emailsEnabled`` is not consulted there either).  ``sendTestEmailOnStart: false`` in
        the ``streamProcessAlerts`` section turns it off (new key)."""
        ac = self._ac()
        if not as_bool(ac.get("sendTestEmailOnStart", True)):
            return None
        try:
            return self.mailer.send(ac.get("fromEmail", "apm@localhost"),
                                    ac.get("testEmailList", ac.get("emailList", "")),
                                    "Test APM alert email", "If you get this email, emails are working!")
        except Exception as e:  # a broken mailer must not stop the engine
            log.error("test e-mail failed: %s", e)
            return None

    def reload(self, cfg):
        self.cfg = cfg
        self.base = self._ac()["alertCollectionIntervalInSeconds"]

    def add_line(self, line: str):
        e = entry_from_csv(line)
        if isinstance(e, AlertEntry):
            self.buffer.append(e)

    def add_lines(self, lines):
        for ln in lines:
            if ln:
                self.add_line(ln)

    def build_email(self, now_ms: float, interval_s: float) -> Tuple[str, str]:
        grafana = self.cfg.get("grafana", {})
        body = format_alerts_html(self.buffer)
        url, render_url = grafana_urls(self.buffer, now_ms, grafana)
        lh = url.replace(grafana.get("grafanaHostname", "") or "\0", "localhost")
        body += (f'<pre>\n\n<a href="{lh}">(Citi) View Alert Graphs</a> - <i>Requires tunnel</i>\n'
                 f'<a href="{url}">(Acxiom) View Alert Graphs</a>\n\n'
                 f"Cooldown until further alerts are sent out: {to_fixed(interval_s / 60, 0)} minutes\n\n"
                 f"{legend_html(self.cfg)}</pre>")
        return body, render_url

    def tick(self) -> bool:
        """One step of sendAlertsRecurse; returns True when an e-mail went out."""
        now = self.clock()
        if now < self.next_due:
            return False
        ac = self._ac()
        sent = False
        interval = float(self.base)
        if self.buffer and as_bool(ac.get("emailsEnabled", True)):
            interval = self.interval
            if as_bool(ac.get("increaseCollectionIntervalAfterAlert", False)):
                if interval < float(ac.get("maxCollectionIntervalInSeconds", 3840)):
                    interval *= 2
                    log.info("Increasing alert collection interval to %s seconds.", interval)
            body, render_url = self.build_email(now * 1000.0, interval)
            frm = ac.get("fromEmail", "apm@localhost")
            try:
                img = self.renderer(render_url, self.cfg.get("grafana", {}))
                self.mailer.send(frm, ac.get("emailList", ""), "APM Alerts Triggered!", body, img)
            except Exception as e:
                log.error("Error while trying to render graph: %s", e)
                self.mailer.send(frm, ac.get("testEmailList", ac.get("emailList", "")), "APM Alerts Triggered!", body)
            self.buffer = []
            self.emails += 1
            sent = True
        self.interval = interval
        self.next_due = now + interval
        return sent
