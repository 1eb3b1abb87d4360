#!/usr/bin/env python3
"""One rank of a multi-PROCESS native node on a shared GPU (GPU tests, test_node_gpu.py).

Each process owns a shard of the JVM hosts (parallel.dist.shard_servers), runs its own native
engine on GPU 0 and joins the node-wide exchanges (lock-step clocks, node-wide service registry,
fleet moments, node-wide alert cooldown) over the TCP host transport (``gpu.collectiveBackend:
host``) -- the same per-batch collective sequence RCCL carries on a multi-GPU node.

    RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment (supervisor rank group or
    the test's launcher);  node_rank.py OUT_DIR [--ckpt-every K] [--kill RANK:BATCH]
    [--kill-world WORLD:RANK:BATCH] [--first-world N]

Outputs: OUT_DIR/rank<r>.{st,fs,al} (reference wire lines).  Every K batches the rank saves its
engine state to OUT_DIR/ckpt/rank<r>.b<k>.bin with the output file sizes; a restarted rank resumes
from the newest batch index every rank of the group has a checkpoint for, truncates its outputs
to that point, and continues -- so the union of the outputs is exactly-once.  ``--kill R:B``: rank
R dies (os._exit, no cleanup) right after batch B, once (marker file), as a crashed GPU process.
When the corpus is done the rank writes OUT_DIR/done.rank<r> and idles like a tailing service
until it is stopped (a supervisor restarts exited modules).

Elastic degrade: ``--kill-world W:R:B`` makes rank R of a W-rank world die after batch B every time
(a GPU that keeps failing), so the supervisor retires it and restarts the group at a smaller world.
A rank of a world other than ``--first-world`` that finds no checkpoint of its own world merges
the first world's rank checkpoints of the newest batch they all have (merge_checkpoints: the
state of the servers it now owns), truncates the old ranks' outputs it took over to that batch,
and continues into OUT_DIR/w<world>.rank<r>.* -- the union of every file stays exactly-once.  A
rank that stops because a peer died exits PEER_FAILURE_EXIT (75), as the service does.
"""
import argparse
import collections
import copy
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

START = 1578391200000
KINDS = ("st", "fs", "al")


def node_cfg():
    from apmbackend_amd.utils.config import default_config
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                         {"LAG": 30, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 5
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 2
    # perServiceAlertCooldownInMinutes: the default (15)
    C["gpu"].update({"zscoreMeanMode": "exact", "timezone": "UTC", "maxSeries": 4096, "batchBytes": 4 << 20,
                     "maxLinesPerBatch": 1 << 16, "bucketCellCapacity": 8, "bucketOverflowCapacity": 1 << 16,
                     "txTextRingMB": 256, "joinTableSlots": 1 << 16, "collectiveBackend": "host",
                     "collectiveTimeoutSeconds": 60})
    return C


def corpus():
    from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks
    from apmbackend_amd.utils.timeparse import TzOffset
    an = [Anomaly("jvm01", "getSvc0001", START + 100_000, START + 900_000, 30.0),
          Anomaly("jvm02", "getSvc0001", START + 100_000, START + 900_000, 30.0),
          Anomaly("jvm03", "getSvc0002", START + 150_000, START + 900_000, 30.0),
          Anomaly("jvm04", "getSvc0002", START + 200_000, START + 900_000, 30.0),
          Anomaly("jvm02", "getSvc0003", START + 600_000, START + 900_000, 40.0)]
    sc = SynthConfig(servers=4, duration_s=1000, tx_per_sec_per_server=3, seed=21, ejb_services=3,
                     provider_services=2, anomalies=an)
    lines = Generator(sc).generate()
    return lines, with_watermarks(batches(lines, sc.start_ms, 5.0), TzOffset("UTC"))


def server_of(fp):
    return fp.split("/")[2]


def _complete_checkpoint(ck_dir, world, pre=""):
    """Newest batch index every rank saved a checkpoint for (0: none)."""
    per = collections.defaultdict(set)
    for p in glob.glob(os.path.join(ck_dir, f"{pre}rank*.b*.bin")):
        name = os.path.basename(p)[len(pre):]
        r, b = name[4:name.index(".b")], name[name.index(".b") + 2:-4]
        per[int(b)].add(int(r))
    done = [b for b, rs in per.items() if len(rs) == world]
    return max(done, default=0)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--ckpt-every", type=int, default=40)
    ap.add_argument("--kill", default="", help="RANK:BATCH -- that rank dies after that batch, once")
    ap.add_argument("--kill-world", default="", help="WORLD:RANK:BATCH -- that rank of that world dies, every time")
    ap.add_argument("--first-world", type=int, default=0, help="world size of the first generation")
    ap.add_argument("--idle", type=float, default=600.0)
    a, _unknown = ap.parse_known_args(argv)  # the supervisor appends --apm-module=<name>
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    os.environ.pop("HIP_VISIBLE_DEVICES", None)  # (ranks share GPU 0: the supervisor's device list is logical)
    first_world = a.first_world or world
    pre = "" if world == first_world else f"w{world}."
    os.makedirs(a.out, exist_ok=True)
    ck_dir = os.path.join(a.out, "ckpt")
    os.makedirs(ck_dir, exist_ok=True)

    from apmbackend_amd.models.pipeline import APMEngine
    from apmbackend_amd.parallel.dist import shard_servers
    from apmbackend_amd.parallel.fleet import FleetBaseline

    lines, bl = corpus()
    servers = sorted({server_of(fp) for fp in lines})
    mine = set(shard_servers(servers, world)[rank])
    eng = APMEngine(copy.deepcopy(node_cfg()), device=0, keep_text=True)
    start = _complete_checkpoint(ck_dir, world, pre)
    paths = {k: os.path.join(a.out, f"{pre}rank{rank}.{k}") for k in KINDS}
    merged_from = _complete_checkpoint(ck_dir, first_world) if (world != first_world and not start) else 0
    if start:
        extra = json.loads(eng.load_state(os.path.join(ck_dir, f"{pre}rank{rank}.b{start}.bin")).decode())
        assert extra["batch"] == start
        for k in KINDS:  # drop what was emitted after the checkpoint: it is emitted again
            with open(paths[k], "ab") as f:
                f.truncate(extra["sizes"][k])
        print(f"rank {rank}: resumed from the group checkpoint of batch {start}", flush=True)
    elif merged_from:
        # re-shard: the first world's states of this rank's servers, merged at their common batch
        from apmbackend_amd import _native
        N = _native.load(build_if_missing=False)
        olds = [os.path.join(ck_dir, f"rank{j}.b{merged_from}.bin") for j in range(first_world)]
        tmp = os.path.join(ck_dir, f".merge.{pre}rank{rank}.bin")
        info = N.merge_checkpoints(olds, sorted(mine), tmp, b"{}")
        eng.load_state(tmp)
        os.remove(tmp)
        old_shards = shard_servers(servers, first_world)
        for j, ex in enumerate(info["extras"]):
            if old_shards[j] and old_shards[j][0] in mine:  # this rank took over old rank j's outputs
                sizes = json.loads(bytes(ex).decode())["sizes"]
                for k in KINDS:
                    with open(os.path.join(a.out, f"rank{j}.{k}"), "ab") as f:
                        f.truncate(sizes[k])
        for k in KINDS:
            open(paths[k], "wb").close()
        for _now, chunks in bl:
            for fp, _ls in chunks:
                if server_of(fp) in mine and fp not in eng.file_ids:
                    eng.add_file(fp)
        start = merged_from
        print(f"rank {rank}: world {first_world} -> {world}: merged the first world's batch-{start} checkpoints "
              f"({info['series']} series, {info['keys']} join keys, {info['need']} parked, {info['pending']} pending)",
              flush=True)
    else:
        for k in KINDS:
            open(paths[k], "wb").close()
        for _now, chunks in bl:  # this rank's files, in the global layout order
            for fp, _ls in chunks:
                if server_of(fp) in mine and fp not in eng.file_ids:
                    eng.add_file(fp)
    fleet = FleetBaseline(eng, world, rank, max_services=64, servers=servers, backend="host")
    kill_rank, kill_at = (int(x) for x in a.kill.split(":")) if a.kill else (-1, -1)
    kw_world, kw_rank, kw_at = (int(x) for x in a.kill_world.split(":")) if a.kill_world else (-1, -1, -1)
    marker = os.path.join(a.out, "killed")

    def emit():
        for k in KINDS:
            got = eng.take(k)
            if got:
                with open(paths[k], "a") as f:
                    f.write("".join(l + "\n" for l in got))

    for b in range(start, len(bl)):
        now, chunks = bl[b]
        try:
            eng.process_lines([(fp, ls) for fp, ls in chunks if server_of(fp) in mine], now)
        except RuntimeError as e:
            if "peer" in str(e) or "aborted" in str(e):  # a peer died: this rank is healthy
                print(f"rank {rank}: collective peer failure: {e}", flush=True)
                sys.exit(75)
            raise
        emit()
        if rank == kill_rank and b == kill_at and not os.path.exists(marker):
            open(marker, "w").close()
            print(f"rank {rank}: fault injection -- dying after batch {b}", flush=True)
            os._exit(17)
        if world == kw_world and rank == kw_rank and b == kw_at:
            with open(marker, "a") as f:
                f.write(f"{world}:{rank}:{b}\n")
            print(f"rank {rank}: fault injection (world {world}) -- dying after batch {b}", flush=True)
            os._exit(17)
        if a.ckpt_every and (b + 1) % a.ckpt_every == 0 and b + 1 < len(bl):
            sizes = {k: os.path.getsize(paths[k]) for k in KINDS}
            tmp = os.path.join(ck_dir, f".{pre}rank{rank}.b{b + 1}.tmp")
            eng.save_state(tmp, json.dumps({"batch": b + 1, "sizes": sizes}).encode())
            os.replace(tmp, os.path.join(ck_dir, f"{pre}rank{rank}.b{b + 1}.bin"))
    fleet.drain_alerts()
    emit()
    m = eng.metrics()
    with open(os.path.join(a.out, f"done.rank{rank}"), "w") as f:
        json.dump({"alerts": m["alerts"], "alert_candidates": m["alert_candidates"], "start": start,
                   "node_metrics": list(eng.eng.node_metrics())}, f)
    print(f"rank {rank}: done ({len(bl) - start} batches)", flush=True)
    t_end = time.time() + a.idle
    while time.time() < t_end and not os.path.exists(os.path.join(a.out, "stop")):
        time.sleep(0.2)


if __name__ == "__main__":
    main()
