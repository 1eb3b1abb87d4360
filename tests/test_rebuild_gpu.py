"""Key-table rebuild in place (devjoin.hip k_rebuild_starts / k_rebuild_inplace) against the
reinsert-into-a-zeroed-copy form (k_rebuild): the same survivors, each reachable from its home
by linear probing with the payload it had, no dead key left, the device's live count exact --
across loads, dead fractions and a table small enough that clusters wrap past its end."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from apmbackend_amd import _native  # noqa: E402


@pytest.mark.parametrize("cap,load,dead,seed", [
    (8, 0.75, 0.5, 1),          # one segment: every cluster wraps
    (64, 0.6, 0.3, 2),
    (1 << 12, 0.5, 0.0, 3),     # nothing dead: nothing may move
    (1 << 12, 0.62, 1.0, 4),    # everything dead: an empty table
    (1 << 16, 0.62, 0.3, 5),
    (1 << 20, 0.55, 0.4, 6),
])
@pytest.mark.parametrize("copy", [False, True], ids=["inplace", "copy"])
def test_rebuild_keeps_live_keys_reachable(cap, load, dead, seed, copy):
    r = _native.load(build_if_missing=False).dj_rebuild_selftest(cap, load, dead, seed, copy)
    assert r["live"] == r["want_live"], r
    assert r["found"] == r["want_live"], r
    assert r["dead_left"] == 0, r
    assert r["occupied"] == r["want_live"], r
    if dead == 0.0:
        assert r["probes_after"] == r["probes_before"], r


def test_rebuild_inplace_is_faster_at_headline_size():
    """2M slots at the headline's steady-state load: the in-place compaction against the reinsert
    (which the async rebuild ran every ~32 batches, the periodic p99 step)."""
    lib = _native.load(build_if_missing=False)
    cap = 1 << 21
    lib.dj_rebuild_selftest(cap, 0.55, 0.2, 7, False)  # (first launch: code object load)
    lib.dj_rebuild_selftest(cap, 0.55, 0.2, 7, True)
    a = min(lib.dj_rebuild_selftest(cap, 0.55, 0.2, 8 + i, False)["us"] for i in range(3))
    b = min(lib.dj_rebuild_selftest(cap, 0.55, 0.2, 8 + i, True)["us"] for i in range(3))
    print(f"rebuild 2M slots: in place {a:.0f} us, reinsert {b:.0f} us (+ a 256 MB memset)")
    assert a < b, (a, b)
