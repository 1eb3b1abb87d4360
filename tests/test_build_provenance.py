"""The native extension is tied to the sources it was built from (csrc hash embedded at link)."""
import types

import pytest

from apmbackend_amd import _native
from apmbackend_amd.build_native import csrc_hash


def test_in_tree_extension_matches_sources():
    N = _native.load(build_if_missing=False)
    assert N.csrc_hash() == csrc_hash()


def test_stale_extension_is_refused_when_strict():
    fake = types.SimpleNamespace(csrc_hash=lambda: "0" * 32, __file__="_apm_native.fake.so")
    with pytest.raises(RuntimeError, match="stale native extension"):
        _native.check_provenance(fake, strict=True)
    with pytest.warns(UserWarning, match="stale native extension"):
        _native.check_provenance(fake, strict=False)


def test_hash_changes_with_any_source(tmp_path, monkeypatch):
    import apmbackend_amd.build_native as bn
    (tmp_path / "kernels").mkdir()
    (tmp_path / "kernels" / "a.hip").write_text("x")
    monkeypatch.setattr(bn, "CSRC", str(tmp_path))
    h0 = bn.csrc_hash()
    (tmp_path / "kernels" / "a.hip").write_text("y")
    assert bn.csrc_hash() != h0
