"""Fleet-wide per-service baseline merge over RCCL (xGMI).

Each GPU owns a disjoint set of JVM hosts (``parallel.dist.shard_servers``), so every
(server, service) series -- its exact percentiles and its z-score history -- lives on exactly one
rank and never needs cross-GPU traffic.  What *is* global is the per-service view across all
servers ("is getFoo slow everywhere or on one JVM?"): every interval each rank packs, per service
and per LAG/stat, {#series with a baseline, sum of baseline means, sum of squared means} into a
dense fp64 matrix on the engine's comm stream (``k_service_gram``: per-service Gram matrices on the
MFMA f64 matrix cores, ``k_service_moments`` atomic scatter for the newest series) and one
``all_reduce(SUM)`` merges it.  The collective runs on the engine's second HIP stream, so it
overlaps the next batch's H2D + parse kernels on the main stream; a two-slot buffer ring keeps
the in-flight reduction from being overwritten.

Message size: n_services x n_lags x 3 stats x 3 moments x 8 B = 1.44 MB for 10k services and two
LAGs -- small and latency-bound on xGMI, so one flat all_reduce per interval (no bucketing).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def pack_moments_host(series_service: np.ndarray, means: np.ndarray, n_services: int) -> np.ndarray:
    """CPU twin of k_service_moments: means[s, lag, stat] (NaN = no baseline)."""
    n_lags = means.shape[1]
    out = np.zeros((n_services, n_lags, 3, 3), dtype=np.float64)
    for s, svc in enumerate(series_service):
        for l in range(n_lags):
            for k in range(3):
                m = means[s, l, k]
                if m == m:
                    out[svc, l, k, 0] += 1.0
                    out[svc, l, k, 1] += m
                    out[svc, l, k, 2] += m * m
    return out


def merged_stats(moments: np.ndarray):
    """(fleet mean of baselines, fleet std of baselines, n) per (service, lag, stat)."""
    n = moments[..., 0]
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = moments[..., 1] / n
        var = moments[..., 2] / n - mean * mean
    return mean, np.sqrt(np.maximum(var, 0.0)), n


class FleetBaseline:
    """Native RCCL fleet exchange bound to an engine.

    Rank 0 draws an RCCL unique id, the id travels over the existing torch.distributed group
    (one small object broadcast at start-up), and every rank's engine creates its own RCCL
    communicator.  From then on the engine's ingest thread issues, per batch and in a fixed order,
    the lock-step clock all-reduce, the node-wide registry all-gather (rounds with new services)
    and the fleet-moment all-reduce of the previous batch (packed by the stats thread) -- no
    Python on the hot path (csrc/runtime/engine.cpp, fleet.cpp).
    """

    def __init__(self, engine, world: int, rank: int, max_services: Optional[int] = None, group=None,
                 lockstep: bool = True, local_group=None, servers: Optional[Sequence[str]] = None,
                 backend: Optional[str] = None):
        """``local_group`` (tests): a ``LocalCollGroup`` joining N engines of this process instead
        of RCCL.  ``servers``: the node-wide server list -- each owned server's position in it
        orders the node-wide alert decisions (default: this rank's registration order).
        ``backend``: ``rccl`` (default; ``gpu.collectiveBackend``) or ``host`` -- the TCP host
        transport through rank 0 at MASTER_ADDR : MASTER_PORT + 11 (``APM_HOST_COLL_PORT``
        overrides), for ranks sharing a GPU or nodes without an RCCL path; no torch.distributed
        group is needed for it."""
        self.eng = engine
        self.world = world
        self.n_lags = len(engine.ecfg["lags"])
        self.cap = int(max_services or engine.cfg.get("gpu", {}).get("maxServices", 1 << 16))
        if servers is not None:
            index = {s: i for i, s in enumerate(servers)}
            for s in engine.eng.servers():
                if s in index:
                    engine.eng.set_server_index(s, index[s])
        if local_group is not None:
            engine.eng.fleet_init_local(local_group, rank, self.cap, lockstep)
            return
        backend = backend or str(engine.cfg.get("gpu", {}).get("collectiveBackend", "rccl"))
        if backend == "host":
            import os
            addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
            port = int(os.environ.get("APM_HOST_COLL_PORT") or int(os.environ.get("MASTER_PORT", "29500")) + 11)
            engine.eng.fleet_init_host(addr, port, world, rank, self.cap, lockstep)
            return
        if backend != "rccl":
            raise ValueError(f"unknown collective backend {backend!r} (rccl / host)")
        import torch.distributed as dist
        native = type(engine.eng)
        obj = [(native.fleet_unique_id(), native.fleet_unique_id() if lockstep else b"") if rank == 0 else None]
        if world > 1:  # a single rank needs no rendezvous (bench.py --gpus 1 runs the same per-rank work)
            dist.broadcast_object_list(obj, src=0, group=group)
        uid, clock_uid = obj[0]
        engine.eng.fleet_init(uid, world, rank, self.cap, clock_uid)

    def drain_alerts(self):
        """Collective: decide every queued node-wide alert candidate (end of stream)."""
        self.eng.eng.node_drain()

    @property
    def exchanges(self) -> int:
        return int(self.eng.eng.fleet_rounds())

    def merged(self) -> np.ndarray:
        raw = self.eng.eng.fleet_merged()
        if not raw:
            return np.zeros((self.cap, self.n_lags, 3, 3))
        # (the LAG count is the one of the newest exchanged pack: a reload may have changed it)
        return np.frombuffer(raw, dtype=np.float64).reshape(self.cap, -1, 3, 3).copy()
