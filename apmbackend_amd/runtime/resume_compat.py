"""Importer / exporter for the reference's JSON resume files.

The reference's stateful stages persist themselves as JSON every 60 s and on exit:

* ``stream_calc_stats.js`` (StatParser, :54-87): ``{"servers": {srv: {"services": {svc:
  {"buckets": {label: [elapsed, ...]}}}}}, "latestBucket": "<label>", "minHeap": {"content":
  [TxEntry, ...]}}``;
* ``stream_calc_z_score.js`` (ZScoreParser, :37-64): ``{"servers": {srv: {"services": {svc:
  {"lags": {"<LAG>": {"THRESHOLD", "INFLUENCE", "avgList", "per75List", "per95List"}}}}}}}``
  (NaN serialised as null);
* ``stream_process_alerts.js`` (AlertsManager, :111-142): ``{"alerts": {service: AlertEntry},
  "alertBuffer": [...], "recentAlertCounts": {srv: {svc: {lag: n}}}}``.

``export_reference_resume`` writes the engine's live state in those layouts (a migration path
back, and a human-readable dump); ``import_reference_resume`` seeds a fresh engine from them,
so a running reference deployment can be cut over without losing its 1-day z-score history.
Reference load semantics are kept: THRESHOLD/INFLUENCE come from the current config
(updateAllServiceSettings runs after load), ``recentAlertCounts`` is reset (setProperties :107;
``restore_alert_counts=True`` keeps them instead).  The parser's join caches are not part of
the reference's state (it loses them on restart) and are not touched here.
"""
from __future__ import annotations

import json
import math
import os
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..utils.records import TxEntry, entry_from_csv

STAT_LISTS = ("avgList", "per75List", "per95List")


def _num(v):
    if v is None:
        return None
    if isinstance(v, float):
        if math.isnan(v) or math.isinf(v):
            return None
        if v.is_integer() and abs(v) < 2 ** 53:
            return int(v)
    return v


def _tx_obj(line: str) -> Dict[str, Any]:
    e = entry_from_csv(line)
    return OrderedDict([("server", e.server), ("service", e.service), ("logId", e.logId),
                        ("acctNum", _num(e.acctNum)), ("startTs", _num(e.startTs)), ("endTs", _num(e.endTs)),
                        ("elapsed", _num(e.elapsed)), ("topLevel", e.topLevel), ("type", "tx")])


def export_reference_resume(eng, chunk: int = 4096) -> Tuple[Dict, Dict, Dict]:
    """eng: models.pipeline.APMEngine (or its native Engine).  Returns (stats, zscore, alerts)."""
    nat = getattr(eng, "eng", eng)
    lags = [int(x[0]) if isinstance(x, (list, tuple)) else int(x) for x in eng.ecfg["lags"]] \
        if hasattr(eng, "ecfg") else None
    series = nat.export_series()
    # ---- stats
    latest, s_ids, buckets, counts, values = nat.export_buckets()
    servers: "OrderedDict[str, Any]" = OrderedDict()
    for srv, svc in series:  # creation order == emission order == the reference's key order
        servers.setdefault(srv, {"services": OrderedDict()})["services"].setdefault(svc, {"buckets": OrderedDict()})
    off = 0
    for s, b, c in zip(s_ids, buckets, counts):
        srv, svc = series[s]
        servers[srv]["services"][svc]["buckets"][str(b)] = list(values[off:off + c])
        off += c
    pending = nat.export_pending()
    stats = OrderedDict([("servers", servers), ("latestBucket", str(latest)),
                         ("minHeap", {"content": [_tx_obj(line) for _end, line in pending if line]})])
    # ---- z-score
    zs: "OrderedDict[str, Any]" = OrderedDict()
    n = len(series)
    settings = [np.asarray(nat.export_lag_settings(li)).reshape(-1, 2) if n else None for li in range(len(lags))]
    for li, lag in enumerate(lags):
        for lo in range(0, n, chunk):
            hi = min(n, lo + chunk)
            lens, raw = nat.export_history(li, lo, hi)
            vals = np.frombuffer(raw, dtype=np.float64).reshape(hi - lo, 3, lag)
            for j in range(hi - lo):
                if lens[j] <= 0:
                    continue
                srv, svc = series[lo + j]
                node = zs.setdefault(srv, {"services": OrderedDict()})["services"].setdefault(svc, {"lags": OrderedDict()})
                thr, infl = settings[li][lo + j]
                d = OrderedDict([("THRESHOLD", _num(float(thr))), ("INFLUENCE", _num(float(infl)))])
                for k, name in enumerate(STAT_LISTS):
                    d[name] = [_num(float(v)) for v in vals[j, k, :lens[j]]]
                node["lags"][str(lag)] = d
    zscore = {"servers": zs}
    # ---- alerts
    by_service = nat.cooldown_by_service()
    alerts = OrderedDict()
    for key, ts in sorted(nat.export_cooldowns()):
        if by_service:
            alerts[key] = {"alertTimestamp": _num(ts), "service": key, "type": "al"}
        else:
            srv, svc = key.split("\x01", 1)
            alerts[f"{srv}|{svc}"] = {"alertTimestamp": _num(ts), "server": srv, "service": svc, "type": "al"}
    rac: "OrderedDict[str, Any]" = OrderedDict()
    for li, lag in enumerate(lags):
        for s, c in enumerate(nat.export_alert_counters(li)):
            if c:
                srv, svc = series[s]
                rac.setdefault(srv, OrderedDict()).setdefault(svc, OrderedDict())[str(lag)] = int(c)
    alerts_doc = OrderedDict([("alerts", alerts), ("alertBuffer", []), ("recentAlertCounts", rac)])
    return stats, zscore, alerts_doc


def import_reference_resume(eng, stats: Optional[Dict] = None, zscore: Optional[Dict] = None,
                            alerts: Optional[Dict] = None, restore_alert_counts: bool = False,
                            servers: Optional[set] = None) -> Dict[str, int]:
    """Seed a *fresh* engine (no batches yet) from reference resume documents.  ``servers``
    restricts the import to one rank's JVM hosts (multi-GPU: every rank imports its shard)."""
    keep = (lambda srv: True) if servers is None else (lambda srv: srv in servers)
    nat = getattr(eng, "eng", eng)
    lags = [int(x[0]) if isinstance(x, (list, tuple)) else int(x) for x in eng.ecfg["lags"]]
    ids: Dict[Tuple[str, str], int] = {}

    def sid(srv, svc):
        k = (srv, svc)
        if k not in ids:
            ids[k] = nat.import_series(srv, svc)
        return ids[k]

    out = {"series": 0, "bucket_rows": 0, "pending": 0, "history": 0}
    if stats:
        latest = int(stats.get("latestBucket") or 0)
        s_ids, bks, cnts, vals = [], [], [], []
        for srv, so in stats.get("servers", {}).items():
            if not keep(srv):
                continue
            for svc, sv in so.get("services", {}).items():
                s = sid(srv, svc)
                b = sv.get("buckets", {})
                if not b:  # known series with an empty window still emits st rows
                    s_ids.append(s); bks.append(latest); cnts.append(0)
                for lab, arr in b.items():
                    ints = [int(x) for x in arr if x is not None]
                    s_ids.append(s); bks.append(int(lab)); cnts.append(len(ints)); vals += ints
        nat.import_buckets(latest, s_ids, bks, cnts, vals)
        out["bucket_rows"] = len(s_ids)
        content = (stats.get("minHeap") or {}).get("content", [])
        ends, lines = [], []
        for o in content:
            if not keep(o.get("server")):
                continue
            tx = TxEntry.make(o.get("server"), o.get("service"), o.get("logId"), o.get("acctNum"), o.get("startTs"),
                              o.get("endTs"), o.get("elapsed"), o.get("topLevel"))
            e = tx.endTs
            if e is None or (isinstance(e, float) and math.isnan(e)):
                continue
            ends.append(int(e)); lines.append(tx.to_csv())
        order = sorted(range(len(ends)), key=lambda i: ends[i])
        nat.import_pending([ends[i] for i in order], [lines[i] for i in order])
        out["pending"] = len(ends)
    if zscore:
        per_lag: Dict[int, Tuple[List[int], List[int], List[np.ndarray]]] = {l: ([], [], []) for l in lags}
        for srv, so in zscore.get("servers", {}).items():
            if not keep(srv):
                continue
            for svc, sv in so.get("services", {}).items():
                s = sid(srv, svc)
                for lag_s, lo in sv.get("lags", {}).items():
                    lag = int(float(lag_s))
                    if lag not in per_lag:
                        continue  # removeStaleLagData: LAGs no longer configured are dropped
                    arrs = [[float("nan") if v is None else float(v) for v in lo.get(k) or []][-lag:]
                            for k in STAT_LISTS]
                    m = max(len(a) for a in arrs)
                    block = np.full((3, lag), np.nan)
                    for k, a in enumerate(arrs):
                        block[k, :len(a)] = a
                    per_lag[lag][0].append(s); per_lag[lag][1].append(m); per_lag[lag][2].append(block)
        for li, lag in enumerate(lags):
            s_list, lens, blocks = per_lag[lag]
            if s_list:
                nat.import_history(li, s_list, lens, np.stack(blocks).astype(np.float64).tobytes())
                out["history"] += len(s_list)
    if alerts:
        by_service = nat.cooldown_by_service()
        cds = []
        for key, ae in (alerts.get("alerts") or {}).items():
            ts = (ae or {}).get("alertTimestamp")
            if ts is None:
                continue
            if by_service:
                cds.append((ae.get("service", key), float(ts)))
            elif "server" in ae:
                cds.append((f"{ae['server']}\x01{ae['service']}", float(ts)))
        nat.import_cooldowns(cds)
        if restore_alert_counts:
            for li, lag in enumerate(lags):
                ss, cc = [], []
                for srv, so in (alerts.get("recentAlertCounts") or {}).items():
                    if not keep(srv):
                        continue
                    for svc, lagd in so.items():
                        c = lagd.get(str(lag))
                        if c:
                            ss.append(sid(srv, svc)); cc.append(int(c))
                nat.import_alert_counters(li, ss, cc)
    out["series"] = len(ids)
    return out


def write_docs(directory: str, stats: Dict, zscore: Dict, alerts: Dict, cfg: Optional[Dict] = None) -> List[str]:
    """Write the three documents where the reference's config expects them (or into dir)."""
    names = [("stream_calc_stats.resume", stats), ("stream_calc_z_score.resume", zscore),
             ("stream_process_alerts.resume", alerts)]
    if cfg:
        paths = [cfg["streamCalcStats"].get("resumeFileFullPath"), cfg["streamCalcZScore"].get("resumeFileFullPath"),
                 cfg["streamProcessAlerts"].get("alertsResumeFileFullPath")]
    else:
        paths = [None, None, None]
    out = []
    for (name, doc), p in zip(names, paths):
        p = p or os.path.join(directory, name)
        os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        with open(p + ".tmp", "w") as f:
            json.dump(doc, f)
        os.replace(p + ".tmp", p)
        out.append(p)
    return out


def read_docs(paths: List[str]) -> List[Optional[Dict]]:
    docs = []
    for p in paths:
        if p and os.path.exists(p):
            with open(p) as f:
                docs.append(json.load(f, object_pairs_hook=OrderedDict))
        else:
            docs.append(None)
    return docs
