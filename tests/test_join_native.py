"""The C++ host join workers (csrc/runtime/join.cpp) against the oracle, on the CPU.

Events are produced by the Python model of the parse kernels (ops/parse_ref.py), i.e. the exact
records the GPU would emit, and fed through ``_apm_native.JoinHarness``."""
import collections

import pytest

from apmbackend_amd import _native
from apmbackend_amd.models.oracle import ParseOracle, file_kind
from apmbackend_amd.ops.parse_ref import parse_batch, tz_table
from apmbackend_amd.utils.synth import Generator, SynthConfig, batches, with_watermarks
from apmbackend_amd.utils.timeparse import TzOffset

UTC = TzOffset("UTC")
KINDS = {"SOAP": 0, "SERVER": 1, "APP": 2}


def run_both(seed, servers=3, duration=300, **kw):
    N = _native.load()
    cfg = SynthConfig(servers=servers, duration_s=duration, tx_per_sec_per_server=3, seed=seed, **kw)
    lines = Generator(cfg).generate()
    bl = with_watermarks(batches(lines, cfg.start_ms, 5.0), UTC)
    want = []
    po = ParseOracle(lambda q, l: want.append((q, l)), tz=UTC)
    for now, chunks in bl:
        po.begin_batch(now)
        for fp, ls in chunks:
            for ln in ls:
                po.read_line(fp, ln)
    h = N.JoinHarness({"tz_table": tz_table(UTC)})
    fid = {fp: h.add_file(fp, KINDS[file_kind(fp)], fp.split("/")[2]) for fp in sorted(lines)}
    got, fo = [], {}
    for now, chunks in bl:
        bch = [(KINDS[file_kind(fp)], ("\n".join(ls) + "\n").encode()) for fp, ls in chunks]
        cf = [fid[fp] for fp, _ in chunks]
        ev, _, _, buf = parse_batch(bch, UTC, fo, cf)
        got += h.process(ev.tobytes(), buf, cf, now)
    return want, got, h.counters(), po.counters


@pytest.mark.parametrize("seed", [1, 5])
def test_native_join_matches_oracle(seed):
    want, got, nc, oc = run_both(seed)
    assert nc["host_fallback"] == 0
    assert nc["need_expired"] == oc["need_expired"] > 0
    assert collections.Counter(want) == collections.Counter(got)
    assert want == got


def test_native_join_heavy_audit_and_late_accounts():
    want, got, nc, oc = run_both(9, servers=2, duration=200, audit_fraction=0.4, soap_late_fraction=0.5,
                                 missing_logid_fraction=0.1, baf_fraction=0.8)
    assert nc["tx_db"] > 0
    assert want == got


def test_js_number_helpers_match_python():
    from apmbackend_amd.utils import jsfmt
    N = _native.load()
    for x in [0.25, 1.45, -0.04, 123.45, 6.2, 1e21, 1.5e-7, 5555000011112222, 0.1 + 0.2, 99.95, 143.6]:
        for f in (0, 1, 2):
            assert N.js_to_fixed(x, f) == jsfmt.to_fixed(x, f), (x, f)
        assert N.js_num_str(x) == jsfmt.js_str(x)
        r = N.js_round_fixed(x, 1)
        assert r == float(jsfmt.to_fixed(x, 1)) or abs(x) >= 1e21
    for s in [" 12ab", "00123", "-7", "abc", "", "5555000011112222", "12345678901234567890", "0x1A"]:
        a, b = N.js_parse_int(s), jsfmt.parse_int(s)
        assert (a != a and b != b) or a == b, s


@pytest.mark.parametrize("key_space", [50, 5000, 1 << 20])
def test_flatmap_and_smallvec_against_std(key_space):
    N = _native.load()
    assert N.flatmap_selftest(200000, 12345 + key_space, key_space)


def test_join_key_hash_python_matches_native():
    """ops.parse_ref.hash_bytes (the model of the kernel's key hash) == the C++ host/device one."""
    import random
    from apmbackend_amd.ops.parse_ref import HASH_SEED, HASH_SEED_EJB, hash_bytes
    N = _native.load()
    rng = random.Random(5)
    for n in list(range(0, 40)) + [63, 64, 65, 200]:
        b = bytes(rng.randrange(256) for _ in range(n))
        for seed in (HASH_SEED, HASH_SEED_EJB):
            assert hash_bytes(b, seed) == N.hash_bytes(b, seed)


def test_native_join_many_services_long_logids():
    """12-20 overlapping provider calls per request, late accounts and 150-byte logIds: the host
    join keeps every open partial and parked record (the reference caches are unbounded Maps,
    stream_parse_transactions.js:215-218,433-437,548-555)."""
    want, got, nc, oc = run_both(11, servers=2, duration=240, sub_calls=(12, 20), overlap_subs=True,
                                 provider_services=30, logid_pad=150, soap_late_fraction=0.6,
                                 audit_fraction=0.1)
    assert max(len(l.split("|")[3]) for _, l in want) > 150
    assert nc["need_expired"] == oc["need_expired"]
    assert want == got
