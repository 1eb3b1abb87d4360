"""Fleet-wide per-service baseline merge over RCCL (xGMI).

Each GPU owns a disjoint set of JVM hosts (``parallel.dist.shard_servers``), so every
(server, service) series -- its exact percentiles and its z-score history -- lives on exactly one
rank and never needs cross-GPU traffic.  What *is* global is the per-service view across all
servers ("is getFoo slow everywhere or on one JVM?"): every interval each rank packs, per service
and per LAG/stat, {#series with a baseline, sum of baseline means, sum of squared means} into a
dense fp64 matrix on the engine's comm stream (``k_service_moments``) and one
``all_reduce(SUM)`` merges it.  The collective runs on the engine's second HIP stream, so it
overlaps the next batch's H2D + parse kernels on the main stream; a two-slot buffer ring keeps
the in-flight reduction from being overwritten.

Message size: n_services x n_lags x 3 stats x 3 moments x 8 B = 1.44 MB for 10k services and two
LAGs -- small and latency-bound on xGMI, so one flat all_reduce per interval (no bucketing).
"""
from __future__ import annotations

from typing import Optional

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
    def __init__(self, engine, world: int, max_services: Optional[int] = None, group=None):
        import torch
        self.torch = torch
        self.eng = engine
        self.world = world
        self.group = group
        self.n_lags = len(engine.ecfg["lags"])
        self.cap = int(max_services or engine.cfg.get("gpu", {}).get("maxServices", 1 << 16))
        n = self.cap * self.n_lags * 3 * 3
        self.bufs = [torch.zeros(n, dtype=torch.float64, device="cuda") for _ in range(2)]
        self.works = [None, None]
        self.slot = 0
        self.last = None
        self.stream = torch.cuda.ExternalStream(engine.eng.comm_stream_handle())
        self.exchanges = 0

    def exchange(self):
        import torch.distributed as dist
        i = self.slot
        self.slot ^= 1
        buf = self.bufs[i]
        with self.torch.cuda.stream(self.stream):
            if self.works[i] is not None:
                self.works[i].wait()  # comm stream waits for the reduction that last used this slot
            self.eng.eng.pack_service_moments(buf.data_ptr(), self.cap)
            self.works[i] = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.last = i
        self.exchanges += 1

    def merged(self) -> np.ndarray:
        if self.last is None:
            return np.zeros((self.cap, self.n_lags, 3, 3))
        w = self.works[self.last]
        if w is not None:
            w.wait()
        self.stream.synchronize()
        return self.bufs[self.last].view(self.cap, self.n_lags, 3, 3).cpu().numpy()
