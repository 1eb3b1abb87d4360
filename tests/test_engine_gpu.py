"""GPU tests: the parse kernels and the full engine against the CPU models.

* K1/K2 device events == ops.parse_ref (the Python transliteration of the kernels);
* full pipeline (parse -> join -> stats -> z-score -> alerts) == PipelineOracle, record for
  record in the reference wire formats (tx / st / fs / al), exact-mean mode;
* rolling-mean mode agrees with exact mode on signals/alerts and to 1 dp on the printed means.
"""
import collections
import os
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU containers
    pytest.skip("no GPU", allow_module_level=True)

from apmbackend_amd import _native  # noqa: E402
from apmbackend_amd.models.oracle import PipelineOracle, file_kind  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.ops.parse_ref import EVENT_DTYPE, parse_batch  # noqa: E402
from apmbackend_amd.utils.config import default_config  # noqa: E402
from apmbackend_amd.utils.synth import Anomaly, Generator, SynthConfig, batches, with_watermarks  # noqa: E402
from apmbackend_amd.utils.timeparse import TzOffset  # noqa: E402

UTC = TzOffset("UTC")
KINDS = {"SOAP": 0, "SERVER": 1, "APP": 2}
START = 1578391200000


def small_cfg(mode="exact"):
    C = default_config(replay=True)
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                         {"LAG": 30, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    C["streamCalcZScore"]["overrides"]["services"]["S:getSvc0002"] = {"6": {"THRESHOLD": 4.0, "INFLUENCE": 0.25}}
    C["streamProcessAlerts"]["rollingAlertWindowSizeInIntervals"] = 10
    C["streamProcessAlerts"]["requiredNumberBadIntervalsInAlertWindowToTrigger"] = 3
    C["streamProcessAlerts"]["perServiceAlertCooldownInMinutes"] = 2
    C["gpu"].update({"emulateOverrideAliasing": True, "zscoreMeanMode": mode, "timezone": "UTC",
                     "maxSeries": 4096, "batchBytes": 4 << 20, "maxLinesPerBatch": 1 << 16,
                     "bucketCellCapacity": 8, "bucketOverflowCapacity": 1 << 16})
    return C


def synth_batches(seed=1, duration=1200, servers=2):
    an = [Anomaly("jvm00", "getSvc0001", START + 400_000, START + 1100_000, 30.0)]
    cfg = SynthConfig(servers=servers, duration_s=duration, tx_per_sec_per_server=3, seed=seed,
                      ejb_services=4, provider_services=3, anomalies=an)
    lines = Generator(cfg).generate()
    return lines, with_watermarks(batches(lines, cfg.start_ms, 5.0), UTC)


@pytest.mark.parametrize("mode", ["tile", "line"])
def test_parse_kernel_matches_model(mode, monkeypatch):
    monkeypatch.setenv("APM_PARSE", mode)
    lines, bl = synth_batches(3, duration=120)
    C = small_cfg()
    eng = APMEngine(C, keep_text=False)
    fo = {}
    for now, chunks in bl[:12]:
        eng.process_lines(chunks, now)
        got = np.frombuffer(eng.eng.last_events(), dtype=EVENT_DTYPE)
        bch = [(KINDS[file_kind(fp)], ("\n".join(ls) + "\n").encode()) for fp, ls in chunks]
        cf = [eng.file_ids[fp] for fp, _ in chunks]
        want, _, _, _ = parse_batch(bch, UTC, fo, cf)
        assert len(got) == len(want)
        for name in EVENT_DTYPE.names:
            a, b = got[name], want[name]
            if a.dtype.kind == "f":
                assert np.array_equal(a, b, equal_nan=True), name
            else:
                assert np.array_equal(a, b), name


def _run_engine(C, bl):
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
            out[k] += eng.take(k)
    return eng, out


def _run_engine_ptr(C, bl, stage):
    """The bench's feeding: every batch in one pinned block, the next batch passed for the parse
    prefetch, and (stage) the batch after that's input copied ahead with stage_batch_ptr."""
    from apmbackend_amd import _native
    N = _native.load(build_if_missing=False)
    eng = APMEngine(C, keep_text=True)
    blobs = []
    for now, chunks in bl:
        parts, table, off = [], [], 0
        for fp, ls in chunks:
            if not ls:
                continue
            data = ("\n".join(ls) + "\n").encode()
            table.append((eng.add_file(fp), off, off + len(data)))
            parts.append(data)
            off += len(data)
        blobs.append((now, b"".join(parts), table))
    total = sum(len(b) + 64 for _, b, _ in blobs)
    base = N.alloc_pinned(total)
    ptrs, off = [], 0
    for now, b, table in blobs:
        N.memcpy_to(base, b, off)
        ptrs.append((base + off, len(b), table, now))
        off += len(b) + 64
    out = collections.defaultdict(list)
    try:
        for i, (ptr, n, table, now) in enumerate(ptrs):
            if i + 1 < len(ptrs):
                nptr, nn, nt, _ = ptrs[i + 1]
                eng.eng.process_batch_ptr(ptr, n, table, now, nptr, nn, nt)
            else:
                eng.eng.process_batch_ptr(ptr, n, table, now)
            if stage and i + 2 < len(ptrs):
                eng.eng.stage_batch_ptr(ptrs[i + 2][0], ptrs[i + 2][1])
            for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
                out[k] += eng.take(k)
        eng.eng.flush()
        for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
            out[k] += eng.take(k)
        staged = int(eng.eng.metrics().get("staged_batches", 0))
    finally:
        del eng
        N.free_pinned(base)
    return out, staged


def test_two_ahead_input_staging_matches_the_plain_feed():
    """Engine::stage_batch: the H2D of the batch after next on its own stream into a third device
    buffer that the later parse launch takes over.  Outputs equal the unstaged prefetch feed and the
    plain per-batch feed; every batch but the first two is parsed from a staged copy."""
    lines, bl = synth_batches(5, duration=600)
    C = small_cfg("exact")
    _, plain = _run_engine(C, bl)
    unstaged, n0 = _run_engine_ptr(C, bl, stage=False)
    staged, n1 = _run_engine_ptr(C, bl, stage=True)
    assert n0 == 0 and 0 < n1 <= len(bl) - 2, (n0, n1, len(bl))
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert staged[k] == unstaged[k] == plain[k], k
    assert sorted(staged["db"]) == sorted(unstaged["db"]) == sorted(plain["db"])


def test_pipeline_matches_oracle_exact():
    lines, bl = synth_batches(1)
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng, out = _run_engine(C, bl)
    assert out["transactions"] == P.tx_out
    assert out["audit_db"] == P.audit_db
    assert out["st"] == P.stats
    assert out["fs"] == P.fs
    assert out["al"] == P.al and len(P.al) > 0
    # released tx: same records, endTs-ordered (ties may differ from the JS heap order)
    assert collections.Counter(out["db"]) == collections.Counter(P.tx_db[:len(out["db"])]) or \
        sorted(out["db"]) == sorted(P.tx_db)
    ends = [int(l.split("|")[6]) for l in out["db"]]  # tx|server|service|logId|acct|start|END|...
    assert ends == sorted(ends)
    m = eng.metrics()
    assert m["rollovers"] > 50 and m["join"]["host_fallback"] == 0


def _al_decisions(al):
    # al|alertTs|entryTs|server|service|causes|<embedded fs>: the embedded fs carries printed
    # means, which may differ by one ulp-tie between mean modes
    return [l.split("|")[:6] for l in al]


def _fs_means(fs):
    out = []
    for l in fs:
        f = l.split("|")
        out.append([float(v) if v not in ("undefined", "NaN") else float("nan")
                    for part in f[6:9] for v in part.split(":")[1:4]])
    return np.array(out)


def _fs_signals(fs):
    return np.array([[float(part.split(":")[4]) for part in l.split("|")[6:9]] for l in fs])


@pytest.mark.parametrize("resync", [360, 4])
def test_rolling_mode_matches_exact_decisions(resync):
    lines, bl = synth_batches(2)
    _, ex = _run_engine(small_cfg("exact"), bl)
    C = small_cfg("rolling")
    C["gpu"]["exactRecomputeEveryIntervals"] = resync
    _, ro = _run_engine(C, bl)
    assert _al_decisions(ex["al"]) == _al_decisions(ro["al"])
    assert len(ex["fs"]) == len(ro["fs"])
    # The rolling sum differs from the JS left-to-right sum by a few ulps, so a mean that is an
    # exact decimal tie (common: LAG-6 means of 1-dp values are k/60) may print the other way;
    # signals can only flip when |x - mean| == T*sigma to the ulp.
    sig_a, sig_b = _fs_signals(ex["fs"]), _fs_signals(ro["fs"])
    assert (sig_a != sig_b).sum() <= max(2, sig_a.size // 2000)
    a, b = _fs_means(ex["fs"]), _fs_means(ro["fs"])
    np.testing.assert_allclose(a, b, rtol=0, atol=0.1001, equal_nan=True)  # tie printed either way


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_reduced_ring_dtype_runs_and_tracks(dtype):
    lines, bl = synth_batches(5)
    _, ex = _run_engine(small_cfg("exact"), bl)
    C = small_cfg("rolling")
    C["gpu"]["ringDtype"] = dtype
    C["gpu"]["exactRecomputeEveryIntervals"] = 8
    _, ro = _run_engine(C, bl)
    assert len(ex["fs"]) == len(ro["fs"]) and len(ex["st"]) == len(ro["st"])
    assert ex["st"] == ro["st"]  # window stats do not depend on the ring dtype
    a, b = _fs_means(ex["fs"]), _fs_means(ro["fs"])
    ok = ~np.isnan(a)
    assert np.array_equal(ok, ~np.isnan(b))
    # printed at 1 dp: a decimal tie can flip by 0.1 on top of the storage rounding
    tol = 0.1001 + (1e-5 if dtype == "float32" else 1e-2) * np.abs(a[ok])
    assert np.all(np.abs(a[ok] - b[ok]) <= tol)


def test_native_fleet_exchange_single_rank():
    """RCCL communicator owned by the engine (nranks=1): the all-reduced moments of the newest
    batch equal a direct pack of the same state."""
    lines, bl = synth_batches(4, duration=300)
    C = small_cfg("rolling")
    eng = APMEngine(C, keep_text=False)
    cap = 64
    eng.eng.fleet_init(type(eng.eng).fleet_unique_id(), 1, 0, cap)
    for now, chunks in bl:
        eng.process_lines(chunks, now)
    got = np.frombuffer(eng.eng.fleet_merged(), dtype=np.float64)
    assert eng.eng.fleet_rounds() == len(bl)
    buf = torch.zeros(got.size, dtype=torch.float64, device="cuda")
    eng.eng.pack_service_moments(buf.data_ptr(), cap)  # one rank, no lock-step: rows = dictionary ids
    torch.cuda.synchronize()  # device-wide: covers the engine's comm stream
    want = buf.cpu().numpy()
    assert got.sum() > 0
    np.testing.assert_allclose(got, want, rtol=0, atol=0)


def test_fleet_moments_mfma_gram_matches_atomic_scatter():
    """The MFMA per-service Gram pack (v_mfma_f64_16x16x4f64, one wave per service) yields the
    same {n, sum, sum^2} per (service, LAG, stat) as the per-series fp64 atomic scatter, and is
    bitwise reproducible across calls -- including series created after the CSR snapshot, which
    go through the per-batch tail CSR (a 9th JVM that starts logging late)."""
    lines, bl = synth_batches(5, duration=300, servers=9)
    bl = list(bl)
    C = small_cfg("rolling")
    eng = APMEngine(C, keep_text=False)
    cap = 64
    n = cap * 2 * 3 * 3
    cut = (len(bl) * 3) // 5
    late = "jvm08"
    for now, chunks in bl[:cut]:
        eng.process_lines([(fp, ls) for fp, ls in chunks if late not in fp], now)
    # snapshot the per-service CSR: jvm08's series arrive afterwards (1/9 of the table)
    early = torch.zeros((n,), dtype=torch.float64, device="cuda")
    eng.eng.pack_service_moments(early.data_ptr(), cap)
    for now, chunks in bl[cut:]:
        eng.process_lines(chunks, now)
    bufs = [torch.full((n,), -1.0, dtype=torch.float64, device="cuda") for _ in range(3)]
    eng.eng.pack_service_moments(bufs[0].data_ptr(), cap, atomic_path=True)
    eng.eng.pack_service_moments(bufs[1].data_ptr(), cap)
    assert eng.eng.gram_tail_series() > 0  # the tail CSR path really ran
    eng.eng.pack_service_moments(bufs[2].data_ptr(), cap)
    torch.cuda.synchronize()
    ref, got, again = (b.cpu().numpy().reshape(cap, 2, 3, 3) for b in bufs)
    assert ref[..., 0].sum() > 10  # series with baselines on both LAGs
    np.testing.assert_array_equal(got[..., 0], ref[..., 0])            # counts: exact
    np.testing.assert_allclose(got[..., 1:], ref[..., 1:], rtol=1e-12, atol=1e-9)
    np.testing.assert_array_equal(got, again)                          # deterministic


def test_gpu_to_fixed_matches_host():
    """K12 number printer (device) == js::to_fixed (host, verified against node) incl. ties."""
    N = _native.load()
    rng = np.random.default_rng(7)
    xs = list(rng.uniform(-1e6, 1e6, 4000)) + list(rng.uniform(0, 10, 2000))
    xs += [k / 20.0 for k in range(-400, 400)] + [k / 200.0 for k in range(-400, 400)]  # x.x5 / x.xx5 ties
    xs += [k / 60.0 for k in range(0, 3000)] + [0.0, -0.0, 1e-9, -1e-9, 0.05, 0.15, 1.005, 2.675, 1e12 + 0.05]
    xs += [float("nan")]
    for f in (1, 2):
        got = N.gpu_to_fixed(xs, f)
        want = ["undefined" if x != x else N.js_to_fixed(x, f) for x in xs]
        bad = [(x, g, w) for x, g, w in zip(xs, got, want) if g != w]
        assert not bad, bad[:5]


@pytest.mark.parametrize("mode", ["exact", "rolling"])
def test_checkpoint_resume_is_seamless(tmp_path, mode):
    """save_state mid-stream -> fresh engine -> load_state -> continue == uninterrupted run."""
    lines, bl = synth_batches(6, duration=900)
    C = small_cfg(mode)
    _, full = _run_engine(C, bl)
    cut = len(bl) // 2
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    for now, chunks in bl[:cut]:
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)  # "db" left pending on purpose: it must survive the checkpoint
    ck = str(tmp_path / "engine.ckpt")
    assert eng.save_state(ck) > 0
    del eng
    eng2 = APMEngine(C, keep_text=True)
    eng2.load_state(ck)
    for now, chunks in bl[cut:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
            out[k] += eng2.take(k)
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert out[k] == full[k], k
    assert collections.Counter(out["db"]) == collections.Counter(full["db"])


def test_lockstep_clock_communicator_single_rank_is_transparent():
    """fleet_init with lock-step clocks (nranks=1): every batch runs the {watermark, newest
    bucket} all-reduce and the moments all-reduce of the previous batch, all on the ingest
    thread's communicator; with one rank the output must be unchanged."""
    lines, bl = synth_batches(9, duration=400)
    C = small_cfg("exact")
    _, plain = _run_engine(C, bl)
    eng = APMEngine(C, keep_text=True)
    E = type(eng.eng)
    eng.eng.fleet_init(E.fleet_unique_id(), 1, 0, 64, E.fleet_unique_id())
    out = collections.defaultdict(list)
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        for k in ("transactions", "st", "fs", "al"):
            out[k] += eng.take(k)
    m = eng.metrics()
    # device join: a batch's fleet exchange is enqueued during the next batch's join kernels, so
    # the last two batches' rounds are still open here (node_drain / fleet_merged close them)
    assert m["lockstep_rollovers"] == 0 and eng.eng.fleet_rounds() == len(bl) - 2
    # node-wide cooldown: the last batches' alert candidates are decided by the drain
    eng.eng.node_drain()
    out["al"] += eng.take("al")
    for k in ("transactions", "st", "fs", "al"):
        assert out[k] == plain[k], k
    assert len(eng.eng.fleet_merged()) > 0 and eng.eng.fleet_rounds() >= len(bl)


@pytest.mark.parametrize("servers", [2, 70])
def test_server_rollup_fuses_window_stats_with_jmx_gauges(servers):
    """K14: per-JVM rollup (sx) == aggregate of that interval's st rows, joined with the JVM's
    JMX gauges.  70 JVMs exceed the block-local (LDS) accumulators: global-atomic path."""
    from apmbackend_amd.runtime.jmx import SyntheticJmx
    from apmbackend_amd.utils.records import JmxEntry
    lines, bl = synth_batches(10, duration=500 if servers <= 2 else 200, servers=servers)
    C = small_cfg("exact")
    # 70 JVMs' hot series overflow small_cfg's 64k-entry spill area: the lists grow (no sample is
    # lost), and st is checked against the CPU oracle so the rollup sees exact window statistics
    eng = APMEngine(C, keep_text=True)
    syn = SyntheticJmx(5)
    jx = JmxEntry.from_stats(START, "jvm00", syn.payload("jvm00")).to_csv()
    sx, st = [], []
    for i, (now, chunks) in enumerate(bl):
        eng.process_lines(chunks, now)
        if i == 3:
            assert eng.set_server_context(jx, vm_load=1.5)
            assert not eng.eng.set_server_context("nope", 0.0, [0.0] * 16, 0.0)
        sx += eng.take("sx")
        st += eng.take("st")
    assert sx
    assert eng.metrics()["spill_dropped"] == 0
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    assert st == P.stats
    by_ts = collections.defaultdict(list)
    for l in st:
        f = l.split("|")
        by_ts[(f[1], f[2])].append(f)
    e = entry_from = None
    from apmbackend_amd.utils.records import entry_from_csv
    g = entry_from_csv(jx)
    heap = g.values[3] / g.values[5]
    checked = 0
    for l in sx:
        f = l.split("|")
        ts, srv = f[1], f[2]
        rows = by_ts[(ts, srv)]
        assert int(f[3]) == len(rows)
        tpm = sum(float(r[4]) for r in rows)
        assert abs(float(f[4]) - tpm) <= 0.01 * len(rows) + 1e-9
        ns = [float(r[4]) * 5 for r in rows]  # tpm = n / 5 for the 30 x 10 s window
        avgs = [float(r[5]) if r[5] != "undefined" else 0.0 for r in rows]
        if sum(ns) > 0:
            want = sum(a * n for a, n in zip(avgs, ns)) / sum(ns)
            # sx prints the exact window mean with toFixed(1); the st rows it is checked against
            # print their means with toFixed(1) too: each side is off by <= 0.05
            assert abs(float(f[5]) - want) <= 0.1 + 1e-9
        if srv == "jvm00" and f[9] != "undefined":
            assert abs(float(f[9]) - heap) < 1e-3 and float(f[16]) == 1.5
            checked += 1
        if srv != "jvm00":
            assert f[9] == "undefined"
    assert checked > 0


def _regroup(bl, sizes):
    """Concatenate consecutive batches (per file, in order) into groups of the given sizes."""
    out, i, k = [], 0, 0
    while i < len(bl):
        n = sizes[k % len(sizes)]
        k += 1
        grp = bl[i:i + n]
        i += n
        per_file = collections.OrderedDict()
        for _, chunks in grp:
            for fp, ls in chunks:
                per_file.setdefault(fp, []).extend(ls)
        out.append((grp[-1][0], [(fp, ls) for fp, ls in per_file.items() if ls]))
    return out


@pytest.mark.parametrize("shape", ["uniform", "growing"])
def test_parse_prefetch_pipelining_is_transparent(shape):
    """process_batch(i, next=i+1) launches batch i+1's parse before batch i's join: outputs
    must be identical to the plain sequence.  "growing" alternates small and very large batches
    so the speculative event D2H behind a prefetched parse (last count + 25 % + 1024) falls
    short and finish_parse has to copy the remainder."""
    lines, bl = synth_batches(11, duration=400)
    if shape == "growing":
        bl = _regroup(bl, [1, 1, 24, 1, 30])
    C = small_cfg("exact")
    _, plain = _run_engine(C, bl)
    eng = APMEngine(C, keep_text=True)
    N = eng.N
    bufs = []
    for now, chunks in bl:
        parts, table, off = [], [], 0
        for fp, ls in chunks:
            data = ("\n".join(ls) + "\n").encode()
            fid = eng.add_file(fp)
            parts.append(data)
            table.append((fid, off, off + len(data)))
            off += len(data)
        blob = b"".join(parts)
        p = N.alloc_pinned(len(blob) + 64)
        N.memcpy_to(p, blob, 0)
        bufs.append((p, len(blob), table, now))
    out = collections.defaultdict(list)
    for i, (p, n, table, now) in enumerate(bufs):
        if i + 1 < len(bufs):
            q, m, t2, _ = bufs[i + 1]
            eng.eng.process_batch_ptr(p, n, table, now, q, m, t2)
        else:
            eng.eng.process_batch_ptr(p, n, table, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert out[k] == plain[k], k
    for p, *_ in bufs:
        N.free_pinned(p)


@pytest.mark.parametrize("dtype", ["float64", "bfloat16"])
def test_deterministic_replay(dtype):
    """Same input, two engines: every output stream is bitwise identical (device atomics in
    K7 / K14 and the K9 sort must not leak scheduling order into the results)."""
    lines, bl = synth_batches(21, duration=500, servers=3)
    C = small_cfg("rolling")
    C["gpu"]["ringDtype"] = dtype
    _, a = _run_engine(C, bl)
    _, b = _run_engine(copy.deepcopy(C), bl)
    for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
        assert a[k] == b[k], k
    assert len(a["fs"]) > 100


def test_sink_fds_match_in_memory_streams(tmp_path):
    """The output lane (released tx, st, fs) and the stats thread (tx, audit, al) write their
    streams straight to sink fds: the files equal the in-memory streams of a second engine."""
    lines, bl = synth_batches(5, duration=600)
    C = small_cfg("exact")
    _, want = _run_engine(C, bl)
    eng = APMEngine(copy.deepcopy(C), keep_text=True)
    kinds = ("transactions", "audit_db", "db", "st", "fs", "al")
    files = {k: open(tmp_path / f"{k}.out", "wb") for k in kinds}
    for k in kinds:
        eng.eng.set_sink_fd(k, files[k].fileno())
    for now, chunks in bl:
        eng.process_lines(chunks, now)
    eng.eng.flush()
    for k in kinds:
        files[k].close()
        got = (tmp_path / f"{k}.out").read_text().splitlines()
        assert got == want[k], k
        assert eng.eng.sink_bytes(k) == (tmp_path / f"{k}.out").stat().st_size


def test_interleaved_server_chunks_match_oracle():
    """Chunks of different JVMs interleaved inside a batch: the engine lays the batch out in its
    canonical order (grouped by JVM, caller's order otherwise), i.e. the oracle run on that
    order."""
    lines, bl = synth_batches(8, duration=600, servers=3)
    inter = []
    for now, chunks in bl:
        by_base = sorted(chunks, key=lambda c: (c[0].rsplit("/", 1)[-1], c[0]))
        inter.append((now, by_base))
    assert any(len({fp.split("/")[2] for fp, _ in ch[:3]}) > 1 for _, ch in inter)
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches([(now, sorted(ch, key=lambda c: c[0].split("/")[2])) for now, ch in inter])
    eng, out = _run_engine(C, inter)
    assert out["transactions"] == P.tx_out
    assert out["audit_db"] == P.audit_db
    assert out["st"] == P.stats
    assert out["fs"] == P.fs


_HOT = {}


def _hot_corpus():
    """One JVM, one EJB service at 200 tx/s (+2 provider sub-services hit 1-3x per tx): the
    service's 31-bucket window holds ~62k samples -- far past K8's LDS tile (16k), so the
    multi-pass radix select runs -- and its buckets overflow small cells into the spill list."""
    if "bl" not in _HOT:
        sc = SynthConfig(servers=1, duration_s=390, tx_per_sec_per_server=200, ejb_services=1, provider_services=2,
                         seed=5, noise_lines_per_tx=0, audit_fraction=0.0)
        lines = Generator(sc).generate()
        _HOT["bl"] = with_watermarks(batches(lines, sc.start_ms, 5.0), UTC)
        C = small_cfg("exact")
        C["gpu"]["emulateOverrideAliasing"] = False
        C["streamCalcZScore"]["overrides"]["services"] = {}
        P = PipelineOracle(copy.deepcopy(C), UTC)
        P.run_batches(_HOT["bl"])
        _HOT["P"] = P
    return _HOT["bl"], _HOT["P"]


@pytest.mark.parametrize("cells", [8, 64])
def test_hot_series_and_spill_match_oracle(cells):
    bl, P = _hot_corpus()
    C = small_cfg("exact")
    C["gpu"]["emulateOverrideAliasing"] = False
    C["streamCalcZScore"]["overrides"]["services"] = {}
    C["gpu"].update({"bucketCellCapacity": cells, "bucketOverflowCapacity": 1 << 21, "batchBytes": 16 << 20,
                     "maxLinesPerBatch": 1 << 18})
    eng, out = _run_engine(C, bl)
    # the hot series really is hot: ~60k samples in its last window
    last = [l for l in P.stats if "getSvc0000" in l][-1].split("|")
    assert float(last[4]) * 5 > 55000  # tpm x 5 min
    assert out["st"] == P.stats
    assert out["fs"] == P.fs
    m = eng.metrics()
    assert m["spill_dropped"] == 0 and m["series_overflow_tx"] == 0


def _nan_corpus(rate=0.03, seed=1):
    """synth corpus with some CommonTiming::Stop lines carrying a non-numeric elapsed: the tx is
    still emitted, its elapsed parses to NaN (stream_calc_stats.js:131)."""
    import random
    rng = random.Random(seed)
    lines, _ = synth_batches(seed)
    out = {}
    for fp, rows in lines.items():
        out[fp] = [(a, b, ln.replace(" - total time ", " - total time x", 1)
                    if "CommonTiming::Stop:" in ln and rng.random() < rate else ln) for a, b, ln in rows]
    return with_watermarks(batches(out, START, 5.0), UTC)


def test_nan_elapsed_matches_oracle():
    """NaN elapsed samples: counted in tpm, average undefined, and the p75/p95 of every window
    holding one read the JS binaryInsert order (device: ordered K7 append while a NaN is live,
    K8 JS-insertion replay)."""
    bl = _nan_corpus()
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    nan_st = [l for l in P.stats if l.split("|")[5] == "undefined" and l.split("|")[4] != "0.00"]
    assert len(nan_st) > 20
    eng, out = _run_engine(C, bl)
    assert out["transactions"] == P.tx_out
    assert out["st"] == P.stats
    assert out["fs"] == P.fs
    assert out["al"] == P.al
    m = eng.metrics()
    assert m["nan_windows_clipped"] == 0


@pytest.mark.parametrize("mode", ["exact", "rolling"])
def test_incremental_checkpoint_chain_resume(tmp_path, mode):
    """checkpoint_async: a base, then increments holding only the ring rows written since the
    previous checkpoint (one per rollover per LAG); a fresh engine restored from the chain
    manifest (base + increments) continues exactly like the uninterrupted run."""
    lines, bl = synth_batches(6, duration=900)
    C = small_cfg(mode)
    _, full = _run_engine(C, bl)
    cut = [len(bl) // 4, len(bl) // 2, (2 * len(bl)) // 3]
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    prefix = str(tmp_path / "engine.rank0")
    infos = []
    for i, (now, chunks) in enumerate(bl[:cut[-1]]):
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
        if i + 1 in cut:
            assert eng.checkpoint_async(prefix, b'{"tail": {"x": [%d, 0]}}' % i) > 0
            eng.checkpoint_wait()
            infos.append(eng.checkpoint_info())
    assert infos[0]["last_base"] and not infos[1]["last_base"] and not infos[2]["last_base"]
    assert infos[2]["chain_len"] == 3
    # the base carries every ring row (LAG 6 + 30); increments only the rows of their rollovers
    assert infos[0]["last_ring_rows"] == 36
    assert 0 < infos[1]["last_ring_rows"] < 36 and 0 < infos[2]["last_ring_rows"] < 36
    manifest = open(prefix + ".ckpt", "rb").read()
    assert manifest.startswith(b"APMCHAIN") and manifest.count(b".ckpt") == 3
    del eng
    eng2 = APMEngine(C, keep_text=True)
    extra = eng2.load_state(prefix + ".ckpt")
    assert extra == b'{"tail": {"x": [%d, 0]}}' % (cut[-1] - 1)
    for now, chunks in bl[cut[-1]:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "db", "st", "fs", "al"):
            out[k] += eng2.take(k)
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert out[k] == full[k], k


def test_base_checkpoint_keeps_the_previous_chain(tmp_path):
    """a new base keeps the chain it replaces as <prefix>.prev.ckpt (a lock-step peer
    that died while the node wrote an aligned base still shares a batch with the survivors); the
    chain before that one is deleted.  Restoring from the previous chain continues exactly like
    the uninterrupted run."""
    lines, bl = synth_batches(7, duration=900)
    C = small_cfg("exact")
    _, full = _run_engine(C, bl)
    n = len(bl)
    cuts = {n // 5: False, (2 * n) // 5: False, (3 * n) // 5: True, (4 * n) // 5: True}  # batch -> force base
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    upto = collections.defaultdict(list)  # outputs through the third checkpoint (base B)
    prefix = str(tmp_path / "engine.rank0")
    chains = []
    for i, (now, chunks) in enumerate(bl[:max(cuts)]):
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
        if i + 1 in cuts:
            assert eng.checkpoint_async(prefix, b"%d" % i, cuts[i + 1]) > 0
            eng.checkpoint_wait()
            chains.append(open(prefix + ".ckpt").read().split()[2:])
            if i + 1 == (3 * n) // 5:
                upto = {k: list(v) for k, v in out.items()}
    a_files, b_files, c_files = chains[1], chains[2], chains[3]
    assert len(a_files) == 2 and len(b_files) == 1 and len(c_files) == 1
    assert open(prefix + ".prev.ckpt").read().split()[2:] == b_files
    for f in a_files:  # the chain before the previous one is gone
        assert not os.path.exists(os.path.join(str(tmp_path), f))
    for f in b_files + c_files:
        assert os.path.exists(os.path.join(str(tmp_path), f))
    del eng
    eng2 = APMEngine(C, keep_text=True)
    assert eng2.load_state(prefix + ".prev.ckpt") == b"%d" % ((3 * n) // 5 - 1)
    for now, chunks in bl[(3 * n) // 5:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            upto[k] += eng2.take(k)
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert upto[k] == full[k], k


@pytest.mark.parametrize("row_delay_us,cap_kb", [(0, 10), (20000, 1)])
def test_streamed_base_checkpoint_under_a_staging_cap(tmp_path, monkeypatch, row_delay_us, cap_kb):
    """Verdict r5 #4: rings sized toward HBM do not fit a snapshot's staging.  With
    gpu.checkpointStageMB far below the rings' size the base streams: the rows the next rollovers
    overwrite first are staged, the writer reads the rest from the live ring, and (with a slow
    writer: 20 ms per row, a 1 KB cap that stages at most one row, while a rollover comes every
    ~12 batches) rollovers that reach a row not yet written copy it aside first or wait.
    The engine keeps running during the write; a fresh engine restored from the file continues
    exactly like the uninterrupted run."""
    monkeypatch.setenv("APM_CK_ROW_DELAY_US", str(row_delay_us))
    lines, bl = synth_batches(8, duration=900)
    C = small_cfg("exact")
    C["streamCalcZScore"]["defaults"] = [{"LAG": 6, "THRESHOLD": 3.0, "INFLUENCE": 0.5},
                                         {"LAG": 120, "THRESHOLD": 2.0, "INFLUENCE": 0.0}]
    # ring rows: (6 + 120) positions x 3 stats x n series x 8 B (tens of KB); staging capped below
    C["gpu"]["checkpointStageMB"] = cap_kb / 1024
    _, full = _run_engine(C, bl)
    cut = len(bl) // 2
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    prefix = str(tmp_path / "engine.rank0")
    for i, (now, chunks) in enumerate(bl):
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
        if i + 1 == cut:
            at_cut = {k: len(v) for k, v in out.items()}
            assert eng.checkpoint_async(prefix, b"%d" % i, True) > 0
    eng.checkpoint_wait()
    info = eng.checkpoint_info()
    assert info["streamed"] == 1 and info["streamed_live_rows"] > 0, info
    assert info["stage_bytes"] <= cap_kb * 1024, info
    if row_delay_us:
        assert info["side_rows"] + info["guard_stalls"] > 0, info  # rollovers overtook the writer
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert out[k] == full[k], k
    eng2 = APMEngine(C, keep_text=True)
    assert eng2.load_state(prefix + ".ckpt") == b"%d" % (cut - 1)
    rest = collections.defaultdict(list)
    for now, chunks in bl[cut:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            rest[k] += eng2.take(k)
    for k in ("transactions", "audit_db", "st", "fs", "al"):
        assert out[k][:at_cut[k]] + rest[k] == full[k], k


def test_host_join_tx_staging_grows_instead_of_failing():
    """Host-join mode with a tiny per-batch tx staging: the engine doubles it mid-batch (was: a
    'too many tx in one batch' exception) and the output is unchanged."""
    lines, bl = synth_batches(1, duration=600)
    C = small_cfg("exact")
    C["gpu"]["joinOnDevice"] = False
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    C["gpu"]["maxTxPerBatch"] = 16
    eng, out = _run_engine(C, bl)
    assert out["transactions"] == P.tx_out
    assert out["st"] == P.stats and out["fs"] == P.fs
    assert eng.metrics()["tx_capacity_grows"] > 0


def test_fs_copy_rows_on_gpu_match_host_encoder():
    """K12 in COPY mode (the DB sink's row encoding fused into the GPU formatter): every fs row
    equals what the host COPY encoder (copyenc.cpp / sinks.copy_encode_lines) makes of the wire
    line -- numbers re-printed JS-style, NaN -> null, names COPY-escaped."""
    from apmbackend_amd.runtime import sinks
    lines, bl = synth_batches(3, duration=700)
    C = small_cfg("exact")
    _, wire = _run_engine(C, bl)
    eng = APMEngine(C, keep_text=True)
    eng.eng.set_fs_copy(True)
    got = []
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        got += eng.take("fs")
    want = [r.rstrip("\n") for r in sinks.copy_encode_lines(wire["fs"])["fs"]]
    assert len(want) > 100 and got == want
    assert any("null" in r for r in got)  # undefined window stats


def test_resync_on_matrix_cores_matches_valu_resync():
    """Rolling mode's staggered exact re-sum as MFMA tile reductions (v_mfma_f64_16x16x4f64
    over [16 series x 2 window rows] with a ones/squares B operand) vs the VALU Neumaier walk:
    same signals and alerts; printed means agree (fp64 sums, different order)."""
    lines, bl = synth_batches(8, duration=900)
    res = {}
    for mfma in (True, False):
        C = small_cfg("rolling")
        C["gpu"]["exactRecomputeEveryIntervals"] = 3
        C["gpu"]["resyncOnMatrixCores"] = mfma
        _, out = _run_engine(C, bl)
        res[mfma] = out
    assert _al_decisions(res[True]["al"]) == _al_decisions(res[False]["al"])
    a, b = res[True]["fs"], res[False]["fs"]
    assert len(a) == len(b) > 100
    diff = sum(x != y for x, y in zip(a, b))
    assert diff <= len(a) // 200, diff


def test_spill_lists_grow_and_match_oracle():
    """48 JVMs with a 64k-entry spill area (1638 per bucket slot): hot series' window samples
    overflow it.  The reference window is unbounded (stream_calc_stats.js:127-131): the engine
    grows the spill lists between appends from the device's fill levels (was: samples dropped and
    counted in spill_dropped), and the sorted-by-series lists give K8 each series' run by binary
    search.  st / fs equal the CPU oracle."""
    lines, bl = synth_batches(10, duration=120, servers=48)
    C = small_cfg("exact")
    assert C["gpu"]["bucketOverflowCapacity"] == 1 << 16
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng, out = _run_engine(C, bl)
    m = eng.metrics()
    assert m["spill_grows"] > 0 and m["spill_dropped"] == 0, m
    assert m["spill_capacity"] > (1 << 16) // 40
    assert out["st"] == P.stats
    assert out["fs"] == P.fs


def _capacity_corpus(seed=12, servers=2, duration=300):
    """Requests touching 12-20 provider services that all open before any closes (up to 20 open
    partials per logId), late SOAP accounts (up to 20 parked records per logId) and 130-byte
    logIds: past every inline capacity of the device join (5 partials, 7 parked records, 80
    logId bytes), which the reference does not have (unbounded Maps,
    stream_parse_transactions.js:215-218,433-437,548-555)."""
    cfg = SynthConfig(servers=servers, duration_s=duration, tx_per_sec_per_server=3, seed=seed,
                      ejb_services=4, provider_services=30, sub_calls=(12, 20), overlap_subs=True,
                      logid_pad=120, soap_late_fraction=0.6, audit_fraction=0.1, no_acct_fraction=0.05)
    lines = Generator(cfg).generate()
    return with_watermarks(batches(lines, cfg.start_ms, 5.0), UTC)


def _assert_streams(out, P):
    assert out["transactions"] == P.tx_out
    assert out["audit_db"] == P.audit_db
    assert out["st"] == P.stats
    assert out["fs"] == P.fs
    assert out["al"] == P.al


def test_join_overflow_chains_match_oracle():
    bl = _capacity_corpus()
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    assert max(len(l.split("|")[3]) for l in P.tx_out) > 120
    eng, out = _run_engine(C, bl)
    _assert_streams(out, P)
    j = eng.metrics()["join"]
    assert j["partial_overflow"] == 0 and j["need_overflow"] == 0 and j["table_full"] == 0
    assert j["pool_exhausted"] == 0
    # the chains were really used: > 5 open partials, > 7 parked records, logIds > 80 bytes
    assert j["chain_partial_blocks"] > 0 and j["chain_need_blocks"] > 0 and j["chain_logid_blocks"] > 0


def test_hot_logid_groups_match_oracle():
    """Keys with thousands of ops in one batch.  The join groups a batch's ops by key with slot
    lists (devjoin.hip k_claim / k_group_walk): a key with more than 16 ops is walked by
    k_group_walk_big, which sorts its members in LDS up to 4096 and in global memory above --
    these logIds carry 40 to 4850 provider lines in one batch."""
    cfg = SynthConfig(servers=1, duration_s=40, tx_per_sec_per_server=0.5, seed=5, sub_calls=(20, 2500),
                      ejb_services=2, provider_services=8, audit_fraction=0.0, soap_late_fraction=0.3)
    lines = Generator(cfg).generate()
    bl = with_watermarks(batches(lines, cfg.start_ms, 5.0), UTC)
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng, out = _run_engine(C, bl)
    _assert_streams(out, P)
    j = eng.metrics()["join"]
    assert j["partial_overflow"] == 0 and j["table_full"] == 0 and j["pool_exhausted"] == 0


@pytest.mark.parametrize("restore", [True, False], ids=["ckpt", "same"])
def test_join_tables_grow_instead_of_failing(tmp_path, restore):
    """Key table, need arena and chain pool all start at 1024 entries: each batch's worst case
    exceeds them, so the join grows them between batches (was: a throw once live keys passed half
    of gpu.joinTableSlots, and silently dropped parked records past the arena).  A checkpoint
    taken mid-run with the grown tables and live chains restores into an engine of default size
    and continues identically."""
    bl = _capacity_corpus(seed=13)
    C = small_cfg("exact")
    C["gpu"].update({"joinTableSlots": 1024, "needArenaEntries": 1024, "joinChainBlocks": 1024})
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    cut = len(bl) // 2
    prefix = str(tmp_path / "engine.rank0")
    marks = []  # tx lines out after each batch
    for i, (now, chunks) in enumerate(bl[:cut]):
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
        marks.append(len(out["transactions"]))
    j = eng.metrics()["join"]
    assert j["table_grows"] > 0 and j["arena_grows"] > 0 and j["pool_grows"] > 0, j
    assert j["table_slots"] > 1024 and j["need_arena_entries"] > 1024 and j["chain_pool_blocks"] > 1024
    if restore:
        eng.save_state(prefix + ".bin")
        del eng
        C2 = small_cfg("exact")
        eng2 = APMEngine(C2, keep_text=True)
        eng2.load_state(prefix + ".bin")
    else:
        eng2 = eng
    for now, chunks in bl[cut:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng2.take(k)
        marks.append(len(out["transactions"]))
    got, want = out["transactions"], P.tx_out
    d = next((i for i, (a, b) in enumerate(zip(got, want)) if a != b), min(len(got), len(want)))
    if d < max(len(got), len(want)):
        at = next((b for b, m in enumerate(marks) if m > d), len(marks))
        bad = sum(1 for a, b in zip(got, want) if a != b)
        pytest.fail(f"tx stream differs first at line {d} (batch {at}, cut {cut}; {bad} lines differ, "
                    f"{len(got)} vs {len(want)}): {got[d][:160] if d < len(got) else None!r} != "
                    f"{want[d][:160] if d < len(want) else None!r}")
    _assert_streams(out, P)
    j2 = eng2.metrics()["join"]
    assert j2["partial_overflow"] == 0 and j2["need_overflow"] == 0 and j2["table_full"] == 0
    assert j2["pool_exhausted"] == 0


def _burst_then_trickle(seed=21):
    """jvm00: a burst of 40 tx/s (2-5 provider calls each) in the first 30 s, then silence;
    jvm01: 1 tx/s from 200 s on.  The burst grows the join tables; once the trickle has moved the
    watermark past the 120 s TTLs, the burst's keys are dead."""
    a = Generator(SynthConfig(servers=2, duration_s=420, tx_per_sec_per_server=40, seed=seed, ejb_services=6,
                              provider_services=8, sub_calls=(2, 5))).generate()
    b = Generator(SynthConfig(servers=2, duration_s=420, tx_per_sec_per_server=1, seed=seed + 1,
                              ejb_services=6, provider_services=8)).generate()
    lines = {}
    for f, v in a.items():
        if "/jvm00/" in f:
            lines[f] = [x for x in v if x[0] < START + 30_000]
    for f, v in b.items():
        if "/jvm01/" in f:
            lines[f] = [x for x in v if x[0] >= START + 200_000]
    return with_watermarks(batches(lines, START, 5.0), UTC)


def test_bursty_all_new_key_batches_never_fill_the_table():
    """a burst of all-new logIds, a quiet stretch (its keys expire), new keys again, on
    a 1024-slot key table.  The stream-ordered rebuild is only taken when the worst case -- every
    key claimed since the last live count still live, plus the batch -- fits 5/8 of the table;
    otherwise the join waits for the count and grows.  No op may be dropped (table_full == 0) and
    the streams equal the oracle."""
    bl = _burst_then_trickle()
    C = small_cfg("exact")
    C["gpu"].update({"joinTableSlots": 1024, "needArenaEntries": 1024, "joinChainBlocks": 1024})
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng, out = _run_engine(C, bl)
    _assert_streams(out, P)
    j = eng.metrics()["join"]
    assert j["table_full"] == 0 and j["partial_overflow"] == 0 and j["need_overflow"] == 0, j
    assert j["table_rebuilds"] > 2 and j["table_grows"] > 0, j


def test_request_gc_trims_device_memory():
    """requestGC for HBM (util_methods.js:398-417 runGC, apm_manager.js:475-512): a burst grows
    the join's key table; once its keys expired, trim_device_memory at a batch boundary shrinks
    the table back to its live entries (never below the configured size) and frees the
    checkpoint scratch, and the pipeline continues with outputs equal to the oracle."""
    bl = _burst_then_trickle(seed=31)
    C = small_cfg("exact")
    C["gpu"].update({"joinTableSlots": 1024, "needArenaEntries": 1024, "joinChainBlocks": 1024})
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    cut = next(i for i, (now, _c) in enumerate(bl) if now > START + 360_000)
    for now, chunks in bl[:cut]:
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
    j0 = eng.metrics()["join"]
    assert j0["table_slots"] > 1024, j0
    before, after = eng.eng.trim_device_memory()
    j1 = eng.metrics()["join"]
    assert after < before and eng.eng.device_bytes() == after, (before, after)
    assert j1["trims"] == 1 and j1["table_slots"] < j0["table_slots"], (j0["table_slots"], j1["table_slots"])
    assert j1["table_slots"] >= 1024 and j1["need_arena_entries"] >= 1024
    assert j1["table_grows"] == j0["table_grows"]  # (a shrink is not counted as growth)
    for now, chunks in bl[cut:]:
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
    _assert_streams(out, P)
    j2 = eng.metrics()["join"]
    assert j2["table_full"] == 0 and j2["partial_overflow"] == 0 and j2["need_overflow"] == 0


def test_fatal_error_leaves_a_state_dump(tmp_path):
    """A fatal engine error (here: a batch larger than gpu.batchBytes -- the same path as a HIP
    error or a capacity throw) leaves a host-side state dump next to the checkpoints before the
    non-zero exit: the reference's heapdump / node-oom-heapdump (apm_manager.js:12-18)."""
    from apmbackend_amd.runtime.service import read_state_dump, write_fatal_dump
    lines, bl = synth_batches(1, duration=200)
    C = small_cfg("exact")
    eng = APMEngine(C, keep_text=True)
    for now, chunks in bl[:10]:
        eng.process_lines(chunks, now)
    fp = bl[3][1][0][0]
    with pytest.raises(RuntimeError) as ei:
        eng.process_lines([(fp, ["x" * 4096] * 4096)], bl[10][0])  # 16 MB > batchBytes (4 MB)
    path = write_fatal_dump(eng.eng, str(tmp_path), 0, ei.value)
    d = read_state_dump(path)
    assert "larger than" in d["reason"]
    m = eng.metrics()
    assert d["batches"] == m["batches"] and d["lines"] == m["lines"] and d["n_series"] == eng.eng.n_series()
    assert d["rollovers"] == m["rollovers"] > 0 and d["join_table_slots"] >= 1024
    assert len(d["slot_bucket"]) == 40 and d["tx_ring_head"] > 0
    # per-series device state (SEC_DUMP_SERIES): read back and checked against the engine
    sd = d["series"]
    assert sd["device_readable"] and sd["n"] == eng.eng.n_series() and sd["lags"] == [6, 30]
    assert list(zip(sd["server"], sd["service"])) == [tuple(x) for x in eng.eng.export_series()]
    assert (sd["window"][:, 5] == 1).sum() > 0 and sd["window"].shape == (sd["n"], 6)
    for li, lag in enumerate(sd["lags"]):
        pl = sd["per_lag"][lag]
        assert 0 < pl["len"].max() <= min(lag, m["rollovers"]) and list(pl["counter"]) == list(eng.eng.export_alert_counters(li))


def _edge_corpus(seed, n=4000):
    """Realistic lines with tokenizer edge cases mixed in: leading / trailing whitespace (space,
    tab, VT, FF), CR and CR CR before LF, whitespace-only and empty lines, non-ASCII bytes,
    repeated INFO, '<' tags at the line end, 20+ tokens, and 1-6 KB lines (they cross the
    parse kernel's per-block stage boundaries)."""
    import random
    rng = random.Random(seed)
    ts = "2020-01-07 10:00:{:02d},{:03d}"
    server, app, soap = [], [], []
    for i in range(n):
        lid = f"id{rng.randint(0, 50):04d}"
        t = ts.format(rng.randint(0, 59), rng.randint(0, 999))
        pre = "[baf][x:y:1234] " if rng.random() < 0.3 else ""
        svc = f"Provider[p{rng.randint(0, 3)}]"
        r = rng.random()
        if r < 0.2:
            line, dst = f"[{lid}] {t} INFO  [CommonTiming] The EJB call started for bean Delegation method: ejb{i % 5}", server
        elif r < 0.35:
            line, dst = f"[{lid}] {t} INFO  [CommonTiming] Total time taken for: ejb{i % 5} - {rng.randint(1, 900)} ms", server
        elif r < 0.5:
            line, dst = f"[{lid}] {t} {pre}INFO  CommonTiming::Start: {svc} begin", app
        elif r < 0.65:
            line, dst = f"[{lid}] {t} {pre}INFO  CommonTiming::Stop: {svc} - total time {rng.randint(0, 500)} ms", app
        elif r < 0.7:
            line, dst = f"[{lid}] {t} [baf][x:1] INFO  auditTrailId=A{i:07d}", app
        elif r < 0.73:
            line, dst = rng.choice(["Audit Trail id : A1", "Audit Trail id   :A2", "]", "<stopWatchList>",
                                    "</stopWatchList>", f"  <name>{svc}</name>",
                                    "  <startTime>2020-01-07T10:00:00.000Z</startTime>",
                                    "  <stopTime>2020-01-07T10:00:00.010Z</stopTime>",
                                    f"[{lid}] {t} INFO  com.acme.Audit: RequestTrace [stopWatchList="]), app
        elif r < 0.8:
            line, dst = rng.choice([f"=== jbossId={lid} IO=I", f"=== jbossId={lid} IO=O",
                                    "      <key>AccountNumber</key>", "      <value>123</value>",
                                    "      <ACCOUNTNUMBER>99</ACCOUNTNUMBER>", "<acc", "x <key"]), soap
        else:
            line = f"[{lid}] {t} DEBUG noise " + " ".join(f"w{k}" for k in range(rng.randint(0, 24)))
            dst = rng.choice([server, app, soap])
        m = rng.random()
        if m < 0.08:
            line = rng.choice([" ", "\t", "  ", "\x0b", "\x0c "]) + line
        elif m < 0.16:
            line = line + rng.choice([" ", "\t", "\r", "  \r", "\r\r", " x", "\x0c"])
        elif m < 0.2:
            line = line.replace(" ", rng.choice(["\t", "  ", " \t "]), rng.randint(1, 4))
        elif m < 0.23:
            line = rng.choice(["", " ", "\t\t", "\r", "   \r"])
        elif m < 0.26:
            line = line[: len(line) // 2] + "é€" + line[len(line) // 2:]
        elif m < 0.29:
            line = line + " INFO again INFO" + rng.choice(["", " <", " <na", " <name>", " <sto"])
        elif m < 0.31:
            line = line + " pad" * rng.randint(250, 1500)
        elif m < 0.32:
            line = "x" * rng.randint(1000, 6000) + " " + line
        dst.append(line)
    return {"/logs/jvm00/server.log": server, "/logs/jvm00/app.log": app, "/logs/jvm00/soap_io.log": soap}


@pytest.mark.parametrize("mode", ["line"])
@pytest.mark.parametrize("seed", [3, 4])
def test_parse_kernel_edge_lines_match_model(seed, mode, monkeypatch):
    """K1/K2 on lines built to hit the tokenizer's and the pattern scan's corner cases (see
    _edge_corpus) == the Python model, field for field; the default K2 kernel (one lane per
    line).  The experimental cooperative-tile kernel (APM_PARSE=tile) is not run here: on seed 3
    it emits 23 events the model does not (tools/diag/parse_edge_diff.py)."""
    monkeypatch.setenv("APM_PARSE", mode)
    files = _edge_corpus(seed)
    C = small_cfg()
    eng = APMEngine(C, keep_text=False)
    raw = [(fp, ("\n".join(ls) + "\n").encode("utf-8")) for fp, ls in files.items()]
    eng.process(raw, START + 60_000)
    got = np.frombuffer(eng.eng.last_events(), dtype=EVENT_DTYPE)
    bch = [(KINDS[file_kind(fp)], b) for fp, b in raw]
    cf = [eng.file_ids[fp] for fp, _ in raw]
    want, _, _, _ = parse_batch(bch, UTC, {}, cf)
    assert len(got) == len(want)
    for name in EVENT_DTYPE.names:
        a, b = got[name], want[name]
        if a.dtype.kind == "f":
            assert np.array_equal(a, b, equal_nan=True), name
        else:
            bad = np.flatnonzero(a != b)
            assert bad.size == 0, (name, bad[:5], a[bad[:5]], b[bad[:5]])


def _audit_corpus(seed, n_req=600, per_batch=37):
    """App-log audit trails (parseAppLine, stream_parse_transactions.js:578-731) with the state
    machine's corner cases: map lines long before their block, blocks interleaved with other
    lines and split across batches at arbitrary lines, duplicate services in one block, a
    startTime / stopTime for a service with no queued entry, headers with no (or an already
    consumed) map entry, unterminated blocks, re-used auditTrailIds, empty / 'Z' / offset-less /
    garbage timestamps, non-ASCII names and elapsed values (those lines take the host's HOP_AUD
    path), BAF accounts that are not digits, and map lines with no account at all."""
    import random
    rng = random.Random(seed)
    app = "/logs/jvm00/app.log"
    base = 1578391200000
    lines = []
    pending = []  # (autr, logId, services) whose block is still to come

    def ts(ms):
        s, m = divmod(ms, 1000)
        import datetime
        d = datetime.datetime.utcfromtimestamp(s)
        return d.strftime("%Y-%m-%d %H:%M:%S") + f",{m:03d}"

    def iso(ms, form):
        import datetime
        d = datetime.datetime.utcfromtimestamp(ms // 1000)
        core = d.strftime("%Y-%m-%dT%H:%M:%S") + f".{ms % 1000:03d}"
        return {0: core + "Z", 1: core + "-06:00", 2: core, 3: "", 4: "2020-13-01T00:00:00Z", 5: "not a date"}[form]

    t = base
    for r in range(n_req):
        t += rng.randint(1, 400)
        lid = f"L{seed}{r:05d}" + ("é" if rng.random() < 0.03 else "")
        autr = f"A{r % 450:04d}"  # ids come back (a later map line replaces an unconsumed entry)
        acct = rng.choice(["12345", "999", "x1", "", "007"])
        pre = f"[baf][x:{acct}] " if acct or rng.random() < 0.5 else ""
        if rng.random() < 0.93:
            lines.append(f"[{lid}] {ts(t)} {pre}INFO  auditTrailId={autr}")
        svcs = [rng.choice(["Provider[cb-a]", "Provider[cb-b]", "RulesEngine", "Lookup", "Provider[cb-é]"])
                for _ in range(rng.randint(1, 6))]
        pending.append((autr, lid, svcs, t))
        lines.append(f"[{lid}] {ts(t)} INFO  [CommonTiming] noise line {r}")
        while pending and (rng.random() < 0.45 or len(pending) > 8):
            a, l, sv, t0 = pending.pop(rng.randrange(len(pending)))
            if rng.random() < 0.04:
                a = "A9999"  # header without a map entry
            lines.append(f"Audit Trail id : {a}")
            lines.append(f"[{l}] {ts(t)} INFO  com.acme.Audit: RequestTrace [stopWatchList=")
            for s in sv:
                el = rng.choice([str(rng.randint(0, 900)), str(rng.randint(0, 900)), "", "12é", "[7]"])
                lines.append(f"  {s}:[{el} millis] ok")
            if rng.random() < 0.05:
                lines.append(f"[{l}] {ts(t)} INFO  unrelated line inside the section")
            lines.append("]")
            lines.append("<stopWatchList>")
            order = sv[:] + ([rng.choice(["Ghost", "Lookup"])] if rng.random() < 0.1 else [])
            rng.shuffle(order)
            for s in order:
                lines.append(f"  <name>{s}</name>")
                if rng.random() < 0.9:
                    lines.append(f"  <startTime>{iso(t0 + 1, rng.choice([0, 1, 1, 1, 2, 3, 4, 5]))}</startTime>")
                lines.append(f"  <stopTime>{iso(t0 + rng.randint(2, 300), rng.choice([0, 1, 1, 1, 1, 2, 3, 5]))}</stopTime>")
            if rng.random() < 0.95:
                lines.append("</stopWatchList>")
    out, i, now = [], 0, base + 60_000
    while i < len(lines):
        k = rng.randint(1, 2 * per_batch)
        out.append((now, [(app, lines[i:i + k])]))
        i += k
        now += 1000
    return out


@pytest.mark.parametrize("seed", [21, 22])
def test_audit_trail_state_machine_on_device_matches_oracle(tmp_path, seed):
    """K5 on the GPU (map/header matching by key, one lane per audit block, carried blocks and
    map entries across batches, host-derived fields for the lines it cannot read) == the
    reference state machine, tx for tx; a checkpoint taken mid-run (open blocks and live map
    entries carried in it) restores into a fresh engine and continues identically."""
    bl = _audit_corpus(seed)
    C = small_cfg("exact")
    P = PipelineOracle(copy.deepcopy(C), UTC)
    P.run_batches(bl)
    assert len(P.audit_db) > 100 and len(P.tx_out) > 100
    eng = APMEngine(C, keep_text=True)
    out = collections.defaultdict(list)
    cut = len(bl) // 2
    for now, chunks in bl[:cut]:
        eng.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng.take(k)
    path = str(tmp_path / "aud.bin")
    eng.save_state(path)
    j1 = eng.metrics()["join"]
    del eng
    eng2 = APMEngine(small_cfg("exact"), keep_text=True)
    eng2.load_state(path)
    for now, chunks in bl[cut:]:
        eng2.process_lines(chunks, now)
        for k in ("transactions", "audit_db", "st", "fs", "al"):
            out[k] += eng2.take(k)
    _assert_streams(out, P)
    j = eng2.metrics()["join"]
    assert j["host_fallback"] > 0 or j["host_events"] > 0  # the HOP_AUD path ran
    assert j1["audit_errors"] > 0 and j["audit_errors"] >= j1["audit_errors"]
