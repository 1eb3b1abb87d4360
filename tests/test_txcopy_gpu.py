"""GPU tests: the released `db` rows encoded as COPY rows of the transactions table on the GPU
(txcopy.hip) against the host encoder (copyenc.cpp, itself pinned to runtime/sinks.py
copy_encode_lines and the reference's TransactionEntry.toPostgresObject).

* edge cases of the wire text: '|' inside a name, COPY escapes, NaN / Infinity / exponent-form
  and negative numbers, -0, leading zeros, missing and extra fields, pre-1970 and far-future
  timestamps -- byte for byte;
* lines outside the GPU encoder's domain are counted (the engine then encodes the release on
  the host);
* the engine's db stream in COPY mode == the host encoding of its wire db stream, on the GPU
  path and on the forced host-fallback path.
"""
import collections
import random

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU containers
    pytest.skip("no GPU", allow_module_level=True)

from apmbackend_amd import _native  # noqa: E402
from apmbackend_amd.models.pipeline import APMEngine  # noqa: E402
from apmbackend_amd.runtime import sinks  # noqa: E402

from test_engine_gpu import _run_engine, small_cfg, synth_batches  # noqa: E402

N = _native.load(build_if_missing=False)

EDGE = [
    "tx|srv1|svcA|lid-1|12345|1700000000000|1700000000123|123|Y",
    "tx|srv\\x|svc\tB|lid\\2|NaN|1700000000000|1700000000456|-5|N",
    "tx|s|n|l|1.2345e+21|0|-1|0|Y",
    "tx|s|n|l|-0|86399999|1|007|Y",
    "tx|s|n|l|999999999999999|999999999999999|-999999999999999|1|Y",
    "tx|s|n|l|1321867455355857|8640000000000000|8640000000000001|9007199254740993|Y",
    "tx|s|n|l|9999999999999999999|-8640000000000000|99999999999999999|-12345678901234567|Y",
    "tx|s|n|l|-62135596800000|-62135596800001|-62198755200000|000000000000000000001|Y",
    "tx|s|n|l",
    "tx|s",
    "tx",
    "tx|a|b|c|d|e|f|g|h|i|j",
    "tx|a||c|+5|+1700000000000|Infinity|-Infinity|",
    "tx|a|b|c|12abc|1700000000000x|1|2|Y",
    "tx|a|b|c|-|+|--5|+-5|Y",
    "tx|a|b|c|5|1700000000000|1700000000000|5|\\\\\\t",
    "tx|" + "x" * 300 + "|n|" + "L" * 700 + "|1|2|3|4|Y",
]

OUTSIDE = [
    "tx|a|b|c| 5|1|1|1|Y",
    "tx|a|b|c|12345678901234567890|1|1|1|Y",
    "tq|a|b|c|1|1|1|1|Y",
    "tx|a|b|c|0x10|1|1|1|Y",
    "tx|a|b|c|1|\t1|1|1|Y",
]


def _host(lines):
    return N.copy_encode("".join(l + "\n" for l in lines).encode())["tx"][0]


def _gpu(lines):
    rows, fb = N.txcopy_lines("".join(l + "\n" for l in lines).encode())
    return rows, fb


def test_txcopy_edge_cases_equal_host_encoder():
    rows, fb = _gpu(EDGE)
    assert fb == 0
    want = _host(EDGE)
    assert rows.count(b"\n") == len(EDGE)
    for g, w in zip(rows.split(b"\n"), want.split(b"\n")):
        assert g == w, (g, w)
    assert rows == want


@pytest.mark.parametrize("line", OUTSIDE)
def test_txcopy_flags_lines_outside_its_domain(line):
    _, fb = _gpu(EDGE[:3] + [line] + EDGE[3:5])
    assert fb == 1


def test_txcopy_random_lines_equal_host_encoder():
    rng = random.Random(7)
    alphabet = "abcXYZ019\\\t-._:"

    def piece():
        s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 20)))
        return rng.choice("abcXYZ._:\\") + s

    def name():
        # (a '|' inside a name shifts the fields, so a piece of a name may land in a numeric
        # field: no piece starts the way a field outside the GPU domain does -- tab, long digits)
        return "|".join(piece() for _ in range(rng.choice([1, 1, 1, 2])))

    def num():
        r = rng.random()
        if r < 0.5:  # up to 19 digits: above 2^53 the parsed Number is rounded, then printed
            return str(rng.randint(-10 ** rng.randint(1, 19) + 1, 10 ** rng.randint(1, 19) - 1))
        if r < 0.6:
            return "NaN"
        if r < 0.7:
            return "%d.%de+%d" % (rng.randint(1, 9), rng.randint(0, 999), rng.randint(21, 30))
        if r < 0.8:
            return "0" * rng.randint(1, 4) + str(rng.randint(0, 99999))
        return rng.choice(["", "-", "+7", "-0", "Infinity", "12x", "x12"])

    lines = []
    for _ in range(5000):
        f = ["tx", name(), name(), name(), num(), num(), num(), num(), rng.choice("YN")]
        lines.append("|".join(f[:rng.choice([9, 9, 9, 9, 5, 3])]))
    rows, fb = _gpu(lines)
    assert fb == 0
    assert rows == _host(lines)


@pytest.mark.parametrize("force_fallback", [False, True])
def test_engine_db_copy_rows_equal_host_encoding(monkeypatch, force_fallback):
    """The engine's released db rows in COPY mode (GPU encoder, or the host path a release takes
    when one of its lines is outside the GPU domain -- forced here) == the host encoding of the
    wire db stream of an identical engine."""
    lines, bl = synth_batches(2, duration=900)
    C = small_cfg("exact")
    _, wire = _run_engine(C, bl)
    assert len(wire["db"]) > 100
    if force_fallback:
        monkeypatch.setenv("APM_TXCOPY_FORCE_FALLBACK", "1")
    eng = APMEngine(C, keep_text=True)
    assert eng.eng.set_db_copy(True)
    got = []
    for now, chunks in bl:
        eng.process_lines(chunks, now)
        got += eng.take("db")
    want = [r.rstrip("\n") for r in sinks.copy_encode_lines(wire["db"])["tx"]]
    assert got == want
    m = eng.metrics()
    if force_fallback:
        assert m["db_copy_fallbacks"] > 0 and m["db_copy_rows"] == 0
    else:
        assert m["db_copy_rows"] == len(want) and m["db_copy_fallbacks"] == 0
