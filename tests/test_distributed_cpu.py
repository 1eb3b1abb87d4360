"""Multi-process data parallelism on CPU (gloo): JVM-host sharding over ranks gives exactly the
single-rank per-series output, and the fleet moment all-reduce equals the global pack."""
import collections
import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from apmbackend_amd.models.oracle import PipelineOracle
from apmbackend_amd.parallel.dist import all_reduce_metrics, rank_of_server, shard_servers
from apmbackend_amd.parallel.fleet import merged_stats, pack_moments_host
from apmbackend_amd.utils.config import default_config
from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks
from apmbackend_amd.utils.timeparse import TzOffset

UTC = TzOffset("UTC")
START = 1578391200000


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def corpus():
    # the same services degrade on JVMs of different shards: the per-service cooldown (default
    # 15 min) must then be decided node-wide, in the single process's emission order
    an = [Anomaly("jvm01", "getSvc0001", START + 100_000, START + 500_000, 30.0),
          Anomaly("jvm02", "getSvc0001", START + 100_000, START + 500_000, 30.0),
          Anomaly("jvm03", "getSvc0002", START + 150_000, START + 500_000, 30.0),
          Anomaly("jvm04", "getSvc0002", START + 200_000, START + 500_000, 30.0)]
    sc = SynthConfig(servers=4, duration_s=600, tx_per_sec_per_server=2, seed=21, ejb_services=3,
                     provider_services=2, anomalies=an)
    return Generator(sc).generate(), sc


def cfg():
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5}]
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 5
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 2
    C["gpu"]["timezone"] = "UTC"
    return C


def run_shard(lines, sc, servers, sync=None, node_exchange=None, server_index=None):
    """One rank's pipeline over its servers.  Batches are cut on the global timeline (all ranks
    ingest the same wall-clock slices) and the watermark clock is the global one, as the
    engine ranks see it through the lock-step exchange."""
    bl = with_watermarks(batches(lines, sc.start_ms, 5.0), UTC)
    mine = [(now, [(fp, ls) for fp, ls in chunks if fp.split("/")[2] in servers]) for now, chunks in bl]
    P = PipelineOracle(copy.deepcopy(cfg()), UTC, node_exchange=node_exchange, server_index=server_index)
    P.run_batches(mine, sync_latest=sync)
    return P


def per_series(stream, key_fields=(2, 3)):
    d = collections.defaultdict(list)
    for l in stream:
        f = l.split("|")
        d[tuple(f[i] for i in key_fields)].append(l)
    return d


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lines, sc = corpus()
        servers = sorted({fp.split("/")[2] for fp in lines})
        mine = shard_servers(servers, world)[rank]
        def sync(latest):  # the engine's per-batch all-reduce(MAX) of the latest bucket
            t = torch.tensor([latest], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return int(t.item())

        def node_exchange(cands):  # the engine's per-batch all-gather of alert candidates
            out = [None] * world
            dist.all_gather_object(out, cands)
            return [c for r in out for c in r]

        P = run_shard(lines, sc, set(mine), sync, node_exchange, {s: i for i, s in enumerate(servers)})
        # fleet moments: per-series baseline means of the last fs rows -> packed per service
        svc_ids = {}
        means, ss = [], []
        for l in P.fs:
            f = l.split("|")
            svc = svc_ids.setdefault(f[3], len(svc_ids))
        all_svcs = sorted({l.split("|")[3] for l in run_shard(lines, sc, set(servers)).fs})
        idx = {s: i for i, s in enumerate(all_svcs)}
        last = {}
        for l in P.fs:
            f = l.split("|")
            last[(f[2], f[3])] = [float(x.split(":")[1]) if x.split(":")[1] != "undefined" else float("nan")
                                  for x in f[6:9]]
        keys = sorted(last)
        series_service = np.array([idx[k[1]] for k in keys], dtype=np.int64)
        m = np.array([[last[k]] for k in keys]).reshape(len(keys), 1, 3) if keys else np.zeros((0, 1, 3))
        mom = torch.from_numpy(pack_moments_host(series_service, m, len(all_svcs)))
        dist.all_reduce(mom, op=dist.ReduceOp.SUM)
        metrics = all_reduce_metrics({"fs": float(len(P.fs)), "al": float(len(P.al))})
        out_q.put((rank, mine, P.stats, P.fs, P.al, mom.numpy(), metrics))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_ranks_reproduce_single_rank_per_series(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    lines, sc = corpus()
    servers = sorted({fp.split("/")[2] for fp in lines})
    full = run_shard(lines, sc, set(servers))
    # disjoint, complete sharding
    owned = sorted(s for r in res for s in r[1])
    assert owned == servers
    for s in servers:
        assert s in res[rank_of_server(s, servers, world)][1]
    # per-series streams identical to the single-rank run
    for idx, name in ((2, "st"), (3, "fs")):
        got = collections.defaultdict(list)
        for r in res:
            for k, v in per_series(r[idx]).items():
                got[k] += v
        assert got == per_series(full.stats if name == "st" else full.fs), name
    # alerts: the node-wide cooldown reproduces the single alerts process (one per service)
    assert sorted(l for r in res for l in r[4]) == sorted(full.al) and len(full.al) >= 2
    alerted = collections.Counter(l.split("|")[4].split(":")[-1] for l in full.al)
    assert set(alerted) == {"getSvc0001", "getSvc0002"}
    # ... and within the cooldown each service alerts from one JVM although two JVMs degrade
    for svc in alerted:
        assert len({l.split("|")[3] for l in full.al if l.split("|")[4].endswith(svc)}) == 1
    # fleet moments: the all-reduced pack equals the pack over every series at once
    all_svcs = sorted({l.split("|")[3] for l in full.fs})
    idx = {s: i for i, s in enumerate(all_svcs)}
    last = {}
    for l in full.fs:
        f = l.split("|")
        last[(f[2], f[3])] = [float(x.split(":")[1]) if x.split(":")[1] != "undefined" else float("nan")
                              for x in f[6:9]]
    keys = sorted(last)
    want = pack_moments_host(np.array([idx[k[1]] for k in keys]), np.array([[last[k]] for k in keys]).reshape(-1, 1, 3),
                             len(all_svcs))
    for r in res:
        np.testing.assert_allclose(r[5], want, rtol=1e-12, atol=0)
        assert r[6] == {"al": float(len(full.al)), "fs": float(len(full.fs))}
    mean, std, n = merged_stats(want)
    assert (n[:, 0, 0] > 0).all()


def _host_coll_worker(rank, world, port, die_rank, out_q):
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    try:
        c = N.HostCollective("127.0.0.1", port, world, rank, 20000.0)
        vals = [float(rank + 1) * 0.1, float(-rank), 2.0 ** -(rank + 3)]
        s = c.all_reduce(vals, False)
        m = c.all_reduce(vals, True)
        g = c.all_gather(bytes([rank]) * 3)
        res = {"sum": s, "max": m, "gather": g}
        if rank == die_rank:
            os._exit(9)  # a crash: no goodbye, the kernel closes the socket
        try:
            c.all_reduce(vals, False)
            res["after"] = "ok"
        except Exception as e:  # the survivors must fail promptly, not hang
            res["after"] = str(e)
        out_q.put((rank, res))
    except Exception as e:  # pragma: no cover - reported to the parent
        out_q.put((rank, {"error": repr(e)}))


@pytest.mark.parametrize("world,die", [(2, -1), (4, -1), (4, 2), (3, 0)])
def test_host_collective_transport_across_processes(world, die):
    """HostCollective (the engine's TCP transport for ranks sharing a GPU): SUM reduced by rank 0
    in rank order (bit-identical on every rank), MAX, all-gather in rank order; a rank process
    that dies makes every survivor's next collective fail at once (peer gone), which is what the
    engine's watchdog turns into abort + non-zero exit."""
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_host_coll_worker, args=(r, world, port, die, q)) for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    alive = world - (1 if die >= 0 else 0)
    res = dict(q.get(timeout=120) for _ in range(alive))
    for p in procs:
        p.join(60)
    assert time.time() - t0 < 60  # no survivor waited for the 20 s collective timeout... twice
    want_sum = [0.0, 0.0, 0.0]
    for r in range(world):
        v = [float(r + 1) * 0.1, float(-r), 2.0 ** -(r + 3)]
        want_sum = [a + b for a, b in zip(want_sum, v)]
    for r, d in res.items():
        assert "error" not in d, d
        assert d["sum"] == want_sum  # same order of additions as rank 0's loop
        assert d["max"] == [world * 0.1, 0.0, 0.125]
        assert d["gather"] == b"".join(bytes([k]) * 3 for k in range(world))
        if die < 0:
            assert d["after"] == "ok"
        else:
            assert "closed its connection" in d["after"] or "connection lost" in d["after"], d["after"]
    if die >= 0:
        assert procs[die].exitcode == 9
