"""State continuity across a world-size change (elastic degrade).

The reference restarts a stage from its resume file with every per-series history intact
(stream_calc_stats.js:54-87, stream_calc_z_score.js:37-64, stream_process_alerts.js:111-142).
Here a 4-rank node (four engines on one GPU joined by an in-process collective group, as in
test_node_gpu.py) runs half the corpus and checkpoints every rank at the same batch; the
checkpoints are merged on the host into the starting state of a 2-rank node (merge.cpp: each new
rank takes the series, join caches and parked records, pending lines, window buckets, z-score
rings and alert counters of the servers it now owns), which runs the rest.  Per series, the st /
fs streams and the alerts equal an uninterrupted 4-rank run of the whole corpus.
"""
import collections
import copy
import os
import sys
import threading

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU containers
    pytest.skip("no GPU", allow_module_level=True)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_node_gpu import corpus, node_cfg, per_series, server_of  # noqa: E402

from apmbackend_amd import _native  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.parallel.dist import shard_servers  # noqa: E402
from apmbackend_amd.parallel.fleet import FleetBaseline  # noqa: E402

KINDS = ("st", "fs", "al", "transactions")


def run_phase(world, bl, servers, load=None, save=None, cfg=None):
    """`world` engines on host threads over an in-process group; `load[r]`: a checkpoint rank r
    starts from; `save[r]`: where rank r checkpoints after the last batch."""
    N = _native.load()
    group = N.LocalCollGroup(world, 120000.0)
    shards = shard_servers(servers, world)
    engs, outs, errs = [], [], []
    for r in range(world):
        eng = APMEngine(copy.deepcopy(cfg or node_cfg()), keep_text=True)
        if load is not None:
            eng.load_state(load[r])
        for _now, chunks in bl:
            for fp, _ls in chunks:
                if server_of(fp) in shards[r]:
                    eng.add_file(fp)
        engs.append(eng)
        outs.append(collections.defaultdict(list))

    def rank_main(r):
        try:
            fb = FleetBaseline(engs[r], world, r, max_services=64, local_group=group, servers=servers)
            for now, chunks in bl:
                engs[r].process_lines([(fp, ls) for fp, ls in chunks if server_of(fp) in shards[r]], now)
                for k in KINDS:
                    outs[r][k] += engs[r].take(k)
            if save is None:
                fb.drain_alerts()
            else:
                engs[r].save_state(save[r], b"{}")
            for k in KINDS:
                outs[r][k] += engs[r].take(k)
        except Exception as e:  # pragma: no cover - reported below
            errs.append((r, repr(e)))

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    assert not errs, errs
    assert all(not t.is_alive() for t in th)
    return engs, outs


def _by_series(outs, kind):
    got = collections.defaultdict(list)
    for o in outs:
        for k, v in per_series(o[kind]).items():
            got[k] += v
    return got


def test_degrade_4_to_2_keeps_every_series_state(tmp_path):
    lines, bl = corpus()
    servers = sorted({server_of(fp) for fp in lines})
    cut = len(bl) // 2
    # uninterrupted reference: the 4-rank node over the whole corpus
    _e, ref = run_phase(4, bl, servers)
    # phase 1: 4 ranks, checkpoint at batch `cut` on every rank
    old = [str(tmp_path / f"old.rank{r}.ckpt") for r in range(4)]
    e1, o1 = run_phase(4, bl[:cut], servers, save=old)
    del e1
    # re-shard: each new rank's state from the old ranks holding its servers
    N = _native.load()
    new = [str(tmp_path / f"new.rank{r}.ckpt") for r in range(2)]
    shards2 = shard_servers(servers, 2)
    infos = []
    for r in range(2):
        info = N.merge_checkpoints(old, shards2[r], new[r], b"{}")
        assert info["servers"] == len(shards2[r]) and info["series"] > 0 and info["keys"] > 0, info
        infos.append(info)
    assert sum(i["series"] for i in infos) > 0
    # phase 2: 2 ranks from the merged states over the rest of the corpus
    e2, o2 = run_phase(2, bl[cut:], servers, load=new)
    # joined transactions: the same multiset (emission order across ranks is free)
    tx_ref = sorted(l for o in ref for l in o["transactions"])
    tx_got = sorted(l for o in o1 + o2 for l in o["transactions"])
    if tx_got != tx_ref:
        import collections as _c
        cg, cr = _c.Counter(tx_got), _c.Counter(tx_ref)
        print("tx only in the re-sharded run:", list((cg - cr).elements())[:5])
        print("tx only in the reference run:", list((cr - cg).elements())[:5])
        for line in list((cg - cr).elements())[:3]:
            lid = line.split("|")[3]
            for name, outs in (("phase 1", o1), ("phase 2", o2), ("reference", ref)):
                print(f"  {lid} {name}:", [l for o in outs for l in o["transactions"] if l.split("|")[3] == lid])
    assert len(tx_got) == len(tx_ref) and tx_got == tx_ref
    for k in ("st", "fs", "al"):
        want = _by_series(ref, k)
        got = _by_series(o1, k)
        for key, v in _by_series(o2, k).items():
            got[key] += v
        assert set(got) == set(want), k
        bad = [key for key in want if got[key] != want[key]]
        for b in bad[:3]:
            g, w = got[b], want[b]
            i = next((j for j in range(min(len(g), len(w))) if g[j] != w[j]), min(len(g), len(w)))
            print(f"{k} {b}: {len(g)} vs {len(w)} lines, first difference at {i} (phase 1 has "
                  f"{len(_by_series(o1, k)[b])}):\n  got  {g[max(0, i - 1):i + 2]}\n  want {w[max(0, i - 1):i + 2]}")
        assert not bad, (k, len(bad), bad[:3])
    assert sum(len(o["al"]) for o in ref) > 0
    # the restored engines hold every series of their servers
    n_series = sum(e.eng.n_series() for e in e2)
    assert n_series == sum(i["series"] for i in infos)
