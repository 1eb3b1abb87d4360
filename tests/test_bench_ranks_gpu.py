"""bench.py's multi-rank launch path, executed (not simulated) on one GPU.

The driver's scaling run launches ``python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N``.  On an 8-GPU node every rank gets its own GPU and the engine exchanges over RCCL; on
the one-GPU box the same launcher puts N ranks on one device, where RCCL refuses duplicate
devices, so bench.py selects the TCP host transport (``--coll auto``).  Everything else -- the
gloo bench group, the server index, the uid/rendezvous, the lock-step clocks, the node-wide
alert decision, the final SUM/MAX reductions and the JSON line -- is the N > 1 code path itself.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_json(stdout: str):
    rows = [l for l in stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(rows) == 1, stdout[-4000:]
    return json.loads(rows[0])


@pytest.mark.parametrize("world", [2, 4])
def test_bench_torchrun_ranks_share_one_gpu(tmp_path, world):
    rep = str(tmp_path / "ranks")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "6", "--warmup", "2", "--rank-report", rep]
    env = dict(os.environ, PYTHONUNBUFFERED="1", OMP_NUM_THREADS="4")
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    out = _bench_json(r.stdout)
    assert out["n_ranks"] == world and out["comm_nranks"] == world
    assert out["collective"] == "host" and out["config"]["parallelism"] == f"dp{world}"
    assert out["n_gpus"] == 1  # honest: the ranks share the box's one GPU
    assert out["steps"] == 6 and out["warmup"] == 2 and out["value"] > 0
    reps = [json.load(open(os.path.join(rep, f"rank{k}.json"))) for k in range(world)]
    assert sorted(x["rank"] for x in reps) == list(range(world))
    for x in reps:
        assert x["comm_ranks"] == world and x["coll"] == "host"
        assert x["node_metrics"] and x["node_metrics"][0] == world  # node-wide counters span every rank
        assert len(x["step_ms"]) == 6
    assert sum(x["lines_timed"] for x in reps) == out["lines_total"]
    # the node-wide line counter (as of the last exchanged interval edge) is a sum over ranks
    assert all(x["node_metrics"][2] == reps[0]["node_metrics"][2] for x in reps)
    assert reps[0]["node_metrics"][2] <= sum(x["lines_total"] for x in reps)
    assert reps[0]["node_metrics"][2] > max(x["lines_total"] for x in reps) * (world - 0.5)
    # fb rows are formatted by every rank (its slice of the node-wide services), off the
    # collective stream: no rank carries the node's fb formatting inside its lock-step exchange
    p50 = [sorted(x["step_ms"])[len(x["step_ms"]) // 2] for x in reps]
    print(f"[{world} ranks] per-rank step p50 {p50}")
    print(f"[{world} ranks] {out['value'] / 1e6:.1f} M lines/s, step p50 {out['step_ms_p50']} ms, "
          f"p99 {out['step_ms_p99']} ms, lockstep {out['t_lockstep_ms']} ms/step ({time.time() - t0:.0f} s)")


_INIT_PROBE = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
import torch
from apmbackend_amd import _native
from apmbackend_amd.models.pipeline import APMEngine
from apmbackend_amd.utils.config import default_config
N = _native.load(build_if_missing=False)
C = default_config(replay=True)
C["gpu"].update({"maxSeries": 4096, "batchBytes": 1 << 20, "maxLinesPerBatch": 1 << 14,
                 "collectiveInitTimeoutSeconds": 6})
eng = APMEngine(C, device=0)
uid = type(eng.eng).fleet_unique_id()
t0 = time.time()
try:
    eng.eng.fleet_init(uid, 2, 0, 1024, uid)  # rank 1 never joins
except RuntimeError as e:
    print("INIT-FAILED after %.1f s: %s" % (time.time() - t0, e), flush=True)
    import os
    os._exit(0)
print("INIT-RETURNED", flush=True)
"""


def test_rccl_init_without_peer_fails_fast(tmp_path):
    """A rank whose peer never joins gets a clear error at the init deadline instead of hanging
    the node (the 8-GPU run must never be the first place a hang is found)."""
    p = tmp_path / "probe.py"
    p.write_text(_INIT_PROBE)
    r = subprocess.run([sys.executable, str(p), ROOT], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, PYTHONUNBUFFERED="1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "INIT-FAILED" in r.stdout and "did not complete within 6 s" in r.stdout, r.stdout
    secs = float(r.stdout.split("INIT-FAILED after ")[1].split(" s")[0])
    assert 5.0 <= secs < 30.0
