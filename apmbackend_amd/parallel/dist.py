"""Multi-GPU data parallelism: one process per GPU, log shards keyed by JVM host.

* ``init_distributed`` -- reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* (torchrun or the
  supervisor's launcher), binds the GPU and creates the process group: backend ``nccl`` (RCCL
  over xGMI) on GPUs, ``gloo`` on CPU-only hosts (tests).
* ``shard_servers`` -- deterministic server -> rank assignment.  A JVM host's soap_io, server and
  app logs, and therefore every (server, service) series, its joins, its exact percentiles and
  its z-score history, stay on one rank: no series is ever split (percentiles cannot be
  all-reduced).  Greedy balancing by expected volume, stable in the host list.
* ``all_reduce_metrics`` -- whole-node counters (lines, tx, alerts) for reporting.
"""
from __future__ import annotations

import hashlib
import os
from typing import Dict, List, Optional, Sequence, Tuple


def dist_env() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0):
    import datetime

    import torch
    import torch.distributed as dist
    rank, world, local = dist_env()
    if world <= 1:
        return None
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {"timeout": datetime.timedelta(seconds=timeout_s)}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    if not dist.is_initialized():
        dist.init_process_group(backend, **kw)
    return dist


def _stable_hash(s: str) -> int:
    return int.from_bytes(hashlib.blake2b(s.encode(), digest_size=8).digest(), "little")


def shard_servers(servers: Sequence[str], world: int, weights: Optional[Dict[str, float]] = None) -> List[List[str]]:
    """Greedy longest-processing-time assignment of JVM hosts to ranks (deterministic)."""
    weights = weights or {}
    order = sorted(servers, key=lambda s: (-weights.get(s, 1.0), _stable_hash(s), s))
    loads = [0.0] * world
    out: List[List[str]] = [[] for _ in range(world)]
    for s in order:
        r = min(range(world), key=lambda i: (loads[i], i))
        out[r].append(s)
        loads[r] += weights.get(s, 1.0)
    for r in range(world):
        out[r].sort()
    return out


def rank_of_server(server: str, servers: Sequence[str], world: int,
                   weights: Optional[Dict[str, float]] = None) -> int:
    for r, lst in enumerate(shard_servers(servers, world, weights)):
        if server in lst:
            return r
    raise KeyError(server)


def all_reduce_metrics(values: Dict[str, float], device=None) -> Dict[str, float]:
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return dict(values)
    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return {k: float(v) for k, v in zip(keys, t.tolist())}
