"""Production-path benchmark (``bench.py --path service``): real log files -> native tailer
(read-ahead into pinned slots) -> engine -> native DB sink (COPY spool) -- the path a deployment
runs, next to the headline which feeds the engine from memory.

The corpus is the headline's (SynthGen, same shard shape); it is appended to real files under
``--service-dir`` (default: a directory next to bench.py, i.e. a disk-backed filesystem, not
tmpfs) before the timed region, so the timed region measures the service catching up on a
backlog: tailer reads, H2D, GPU pipeline, sink encoding and writes, every tail offset committed.
The z-score rings get the same synthetic pre-history as the headline.  As in production: the
incremental checkpoint runs every 60 s of *log* time (the service clock is the engine's log-time
watermark, so the compressed bench takes one every 6 batches; ``--service-ckpt off`` for the A/B),
the fleet exchange + lock-step clocks run as at the headline (``--service-fleet``), and the COPY
spool is on the same disk.  Reported: lines/s through the service, the DB rows/s the sink wrote,
the sink's encode/write share, the checkpoints taken and their ingest stall.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import time
from typing import Any, Dict


def run(args, cfg: Dict[str, Any], N, rank: int = 0) -> Dict[str, Any]:
    from .service import IngestService

    base = args.service_dir or os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), ".service_bench")
    os.makedirs(base, exist_ok=True)
    root = tempfile.mkdtemp(prefix="apm_svc_bench_", dir=base)
    try:
        return _run(args, cfg, N, rank, root, IngestService)
    finally:
        shutil.rmtree(root, ignore_errors=True)


def _run(args, cfg, N, rank, root, IngestService):
    start = 1578391200000
    step_ms = int(args.batch_seconds * 1000)
    # pre-history batches before the synthetic z-score history (as the headline: bench.py
    # --pre-batches): the 31-bucket window is full when the history is drawn
    PRE = max(2, getattr(args, "pre_batches", 33))
    gen = N.SynthGen({"servers": args.servers, "ejb_services": args.ejb, "provider_services": args.providers,
                      "tx_per_sec_per_server": args.tx_rate, "seed": 1 + rank,
                      "server_offset": rank * args.servers,
                      "anomaly_services": args.anomaly_services, "anomaly_factor": args.anomaly_factor,
                      "anomaly_start_ms": start + PRE * step_ms})
    paths = []
    for p, _kind, server in gen.files():
        d = os.path.join(root, "logs", server)
        os.makedirs(d, exist_ok=True)
        fp = os.path.join(d, os.path.basename(p))
        open(fp, "wb").close()
        paths.append(fp)
    fds = [os.open(p, os.O_WRONLY | os.O_APPEND) for p in paths]
    written = [0]

    def append(b0, b1):
        for b in range(b0, b1):
            data, chunks = gen.generate(start + (b + 1) * step_ms, args.gen_threads)
            mv = memoryview(data)
            for fid, lo, hi in chunks:
                os.write(fds[fid], mv[lo:hi])
            written[0] += len(data)

    g = cfg["gpu"]
    ckpt = getattr(args, "service_ckpt", "on") == "on"
    fleet = getattr(args, "service_fleet", "on") == "on"
    g.update({"tailFromStart": True, "tailReadAhead": True, "tailIdleMs": 1.0,
              "tailReadThreads": getattr(args, "tail_read_threads", 8),
              "checkpointDir": os.path.join(root, "ckpt") if ckpt else None, "checkpointEverySeconds": 60,
              "fleetBaseline": fleet, "fleetSingleRank": fleet})
    ic = cfg["streamInsertDb"]
    ic.update({"sink": args.service_sink, "copySinkDir": os.path.join(root, "spool"),
               "encoderThreads": args.encoder_threads, "copySinkRotateBytes": 1 << 62,
               "writerLanes": getattr(args, "writer_lanes", 1)})
    cfg["logDir"] = os.path.join(root, "log")
    cfg["streamParseTransactions"]["tailOffsetFileFullPath"] = os.path.join(root, "state", "tail_offsets.json")
    cfg["streamInsertDb"]["bufferResumeFileFullPath"] = os.path.join(root, "state", "db_resume.json")
    srv_of = lambda p: p.split("/")[-2]  # noqa: E731
    # the service's clock = log time (the engine's watermark): checkpoints / stat lines every 60 s
    # of log time, as a real-time deployment has them, at the bench's compressed pace
    holder = {}

    def log_clock():
        e = holder.get("svc")
        return e.native.watermark() / 1000.0 if e is not None and e.eng is not None else 0.0

    svc = IngestService(cfg, engine="native", files=paths, rank=0, world=1, server_of_path=srv_of, clock=log_clock)
    holder["svc"] = svc

    loop_t = {"step_s": 0.0, "housekeeping_s": 0.0, "idle_s": 0.0, "idles": 0, "cond_s": 0.0}

    def drain():
        # the service loop (IngestService.run): step + housekeeping (checkpoints on the log-time
        # clock, stat lines, sink ticks), idle wait when nothing was read
        while True:
            tz = time.perf_counter()
            more = sum(o[1] for o in svc.tailer.offsets()) < written[0] or svc._held is not None
            ta = time.perf_counter()
            loop_t["cond_s"] += ta - tz
            if not more:
                break
            n = svc.step()
            tb = time.perf_counter()
            svc._housekeeping()
            tc = time.perf_counter()
            loop_t["step_s"] += tb - ta
            loop_t["housekeeping_s"] += tc - tb
            if n == 0:
                svc._idle(0.001)
                loop_t["idle_s"] += time.perf_counter() - tc
                loop_t["idles"] += 1

    append(0, PRE)
    drain()
    svc.eng.eng.flush()
    svc.eng.eng.warm_history(12345 + rank)
    append(PRE, PRE + args.warmup)
    drain()
    svc.eng.eng.flush()
    svc.inserter.flush_all()
    append(PRE + args.warmup, PRE + args.warmup + args.steps)  # the backlog the timed region consumes
    m0 = svc.eng.metrics()
    s0 = svc.inserter.sink_stats()
    ck0 = svc.eng.eng.checkpoint_info() if ckpt else None
    n_ck0 = svc.n_checkpoints if hasattr(svc, "n_checkpoints") else 0
    import torch
    torch.cuda.synchronize()
    if args.trace:
        svc.eng.eng.set_trace(True)
    import gc
    gc.collect()  # (the corpus generation's garbage: not inside the timed region)
    pf0 = dict(svc.perf)
    tl0 = dict(loop_t)
    ts0 = svc.tailer.stats()
    h0 = _host_sample()
    t0 = time.perf_counter()
    drain()
    ta = time.perf_counter()
    svc.eng.eng.flush()
    tb = time.perf_counter()
    svc._drain_outputs()
    t_engine = time.perf_counter() - t0
    tc = time.perf_counter()
    svc.inserter.flush_all()  # every row of the timed batches encoded and written
    dt = time.perf_counter() - t0
    host = _host_delta(h0, _host_sample(), dt)
    tail = {"loop_s": round(ta - t0, 4), "engine_flush_s": round(tb - ta, 4), "drain_outputs_s": round(tc - tb, 4),
            "sink_flush_all_s": round(t0 + dt - tc, 4)}
    m1 = svc.eng.metrics()
    s1 = svc.inserter.sink_stats()
    tstats = svc.tailer.stats()
    ck1 = svc.eng.eng.checkpoint_info() if ckpt else None
    n_ck = (svc.n_checkpoints if hasattr(svc, "n_checkpoints") else 0) - n_ck0
    if args.trace:
        svc.eng.dump_trace(args.trace)
    pf = {k: svc.perf[k] - pf0[k] for k in pf0}
    svc.shutdown()
    for fd in fds:
        os.close(fd)
    lines = m1["lines"] - m0["lines"]
    rows = s1.get("rows", 0) - s0.get("rows", 0)
    return {
        "lines": lines,
        "seconds": dt,
        "lines_per_s": lines / dt,
        "lines_per_s_engine_drained": lines / t_engine,
        "db_rows_per_s": rows / dt,
        "db_rows": rows,
        "db_bytes": s1.get("bytes", 0) - s0.get("bytes", 0),
        "sink": args.service_sink,
        "writer_lanes": s1.get("lanes", 1),
        "sink_write_ms": s1.get("ms", 0.0) - s0.get("ms", 0.0),
        "sink_failures": s1.get("failures", 0),
        "tailer": {**{k: tstats[k] for k in ("batches", "bytes_read", "read_threads")},
                   **{k + "_timed": tstats.get(k, 0) - ts0.get(k, 0) for k in ("batches", "bytes_read", "plan_ms", "read_ms")}},
        "drain_loop": {k: round(loop_t[k] - tl0[k], 4) for k in loop_t},
        "timed_split": tail,  # the drain loop, then the engine's pipeline tail, outputs, the sink's last writes
        "ingest_GB_per_s": (m1["bytes"] - m0["bytes"]) / dt / 1e9,
        "loop": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in pf.items()},
        "mean_batch_MB": round(pf["bytes"] / max(pf["batches"], 1) / 1e6, 3),
        "checkpoints": n_ck,
        "checkpoint_info": {k: ck1[k] for k in ck1} if ck1 else None,
        "fleet": fleet,
        "fs_type": _fs_type(root),
        "host": host,  # what else the host did during the timed region (run-to-run spread attribution)
        "batches": pf["batches"],
        "pre_history_batches": PRE,
    }


def _host_sample() -> Dict[str, Any]:
    """Host-side counters around the timed region: this process's CPU seconds, the page cache's
    dirty / writeback bytes and the kernel's pressure-stall totals (cpu / memory / io, us)."""
    t = os.times()
    out: Dict[str, Any] = {"user_s": t.user, "sys_s": t.system}
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                k, v = line.split(":", 1)
                if k in ("Dirty", "Writeback", "MemFree"):
                    out[k] = int(v.split()[0]) * 1024
    except OSError:
        pass
    for r in ("cpu", "memory", "io"):
        try:
            with open(f"/proc/pressure/{r}") as f:
                for line in f:
                    kind, *fields = line.split()
                    out[f"psi_{r}_{kind}_us"] = int(dict(x.split("=") for x in fields)["total"])
        except (OSError, KeyError, ValueError):
            pass
    try:
        with open("/proc/loadavg") as f:
            out["loadavg1"] = float(f.read().split()[0])
    except OSError:
        pass
    return out


def _host_delta(a: Dict[str, Any], b: Dict[str, Any], dt: float) -> Dict[str, Any]:
    d: Dict[str, Any] = {"cpu_util": round((b["user_s"] + b["sys_s"] - a["user_s"] - a["sys_s"]) / dt, 2),
                         "sys_share": round((b["sys_s"] - a["sys_s"]) / max(b["user_s"] + b["sys_s"] - a["user_s"] - a["sys_s"], 1e-9), 3)}
    for k in ("Dirty", "Writeback", "MemFree"):
        if k in a and k in b:
            d[k + "_MB_before"] = round(a[k] / 1e6, 1)
            d[k + "_MB_after"] = round(b[k] / 1e6, 1)
    for k in a:
        if k.startswith("psi_") and k in b:
            d[k[:-3] + "_pct"] = round(100.0 * (b[k] - a[k]) / 1e6 / dt, 2)  # share of the region stalled
    if "loadavg1" in b:
        d["loadavg1"] = b["loadavg1"]
    return d


def _fs_type(path: str) -> str:
    """Filesystem type of the mount holding `path` (/proc/mounts, longest prefix)."""
    best, typ = "", "?"
    try:
        with open("/proc/mounts") as f:
            for line in f:
                parts = line.split()
                mp, fst = parts[1], parts[2]
                if os.path.abspath(path).startswith(mp) and len(mp) > len(best):
                    best, typ = mp, fst
    except OSError:
        pass
    return typ
