"""CPU model of the join's in-place key-table rebuild (devjoin.hip k_rebuild_starts /
k_rebuild_inplace), the algorithm alone: per RB_SEG-slot segment the first cluster start is found
before anything moves, then each segment's owner re-inserts the live keys of the clusters that
start in it, in slot order, into the emptied cluster (first free slot at or after the home).
Owners run in a random order here (on the GPU they run concurrently: clusters are disjoint).
Checked: exactly the live keys survive, each reachable from its home by linear probing, and no
key is placed past the slot it was read from (what makes the GPU form safe in place).  The
kernel itself is checked against the reinsert form on the GPU (test_rebuild_gpu.py)."""
import random

import pytest

SEG = 8


def _home(k, mask):
    return (k * 0x9E3779B1) & mask


def _rebuild_model(table, mask, rng):
    cap = mask + 1
    starts = []
    for sg in range(cap // SEG):
        lo, hi = sg * SEG, sg * SEG + SEG
        p = lo
        if table[(lo - 1) & mask] is not None:
            while p < hi and table[p] is not None:
                p += 1
        starts.append(p)
    order = list(range(cap // SEG))
    rng.shuffle(order)
    for sg in order:
        hi, p = sg * SEG + SEG, starts[sg]
        while p < hi:
            if table[p & mask] is None:
                p += 1
                continue
            q = p
            while table[q & mask] is not None and q < p + cap:
                q += 1
            occ = [False] * (q - p)
            for r in range(p, q):
                key, dead = table[r & mask]
                if dead:
                    continue
                i = r - (((r & mask) - _home(key, mask)) & mask) - p
                while i < len(occ) and occ[i]:
                    i += 1
                assert i <= r - p, "a key would land past the slot it was read from"
                occ[i] = True
                table[(p + i) & mask] = (key, False)
            for i, placed in enumerate(occ):
                if not placed:
                    table[(p + i) & mask] = None
            p = q + 1


@pytest.mark.parametrize("cap,load,dead", [(8, 0.75, 0.5), (64, 0.6, 0.3), (4096, 0.5, 0.0), (4096, 0.62, 1.0),
                                           (1 << 15, 0.62, 0.3), (1 << 14, 0.95, 0.2)])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_inplace_rebuild_model(cap, load, dead, seed):
    rng = random.Random(seed * 7919 + cap)
    mask = cap - 1
    table = [None] * cap
    live = set()
    for _ in range(int(load * cap)):
        k = rng.getrandbits(62) | 1
        i = _home(k, mask)
        while table[i] is not None and table[i][0] != k:
            i = (i + 1) & mask
        if table[i] is not None:
            continue
        d = rng.random() < dead
        table[i] = (k, d)
        if not d:
            live.add(k)
    _rebuild_model(table, mask, rng)
    assert {e[0] for e in table if e is not None} == live
    for k in live:
        i = _home(k, mask)
        while table[i][0] != k:
            i = (i + 1) & mask
            assert table[i] is not None, "a live key is no longer reachable from its home"
