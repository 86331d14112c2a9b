"""The C-ABI library loads, exports every symbol include/pdp_hip.h declares,
and its host-side calibration matches the reference known answers (no GPU
compute here)."""
import math
import os
import re

import numpy as np
import pytest

import pdp_oracle as o
from golden_util import known_answers
from pipelinedp_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "pdp_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pdp_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = native.lib()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    bound = {name for name, _, _ in native.SIGNATURES}
    assert set(syms) == bound, set(syms) ^ bound
    assert lib.pdp_abi_version() == native.ABI_VERSION


def test_gaussian_sigma_known_answers():
    for c in known_answers()["gaussian_sigma"]:
        l2 = c["l2"] if "l2" in c else math.sqrt(c["l0"]) * c["linf"]
        assert native.gaussian_sigma(c["eps"], c["delta"], l2) == pytest.approx(c["sigma"], abs=1e-12)


@pytest.mark.parametrize("eps,delta,k", [(1.0, 1e-5, 1), (0.5, 1e-6, 4), (2.0, 1e-8, 32), (0.05, 1e-3, 2)])
def test_truncated_geometric_table_matches_oracle(eps, delta, k):
    t = np.array(native.truncated_geometric_table(eps, delta, k))
    r = o.truncated_geometric_table(eps, delta, k)
    assert len(t) == len(r)
    np.testing.assert_array_equal(t, r)


@pytest.mark.parametrize("sel,eps,delta,k", [(2, 1.0, 1e-5, 1), (2, 0.3, 1e-6, 5), (3, 1.0, 1e-5, 3),
                                             (3, 2.0, 1e-8, 10)])
def test_selection_thresholds_match_oracle(sel, eps, delta, k):
    thr, scale = native.selection_threshold(sel, eps, delta, k)
    if sel == 2:
        rt, rs = o.laplace_threshold(eps, delta, k)
    else:
        rt, rs = o.gaussian_threshold(eps, delta, k)
    assert thr == pytest.approx(rt, rel=1e-9)
    assert scale == pytest.approx(rs, rel=1e-12)


def test_metric_fields_match_metrics_tuple_order():
    names = {"count": 1, "sum": 2, "mean": 4, "variance": 8, "privacy_id_count": 16}
    import itertools
    for r in range(1, 6):
        for combo in itertools.combinations(names, r):
            mask = sum(names[c] for c in combo)
            assert native.metric_fields(mask) == o.metric_field_order(combo), combo


def test_library_fails_loudly_when_missing(monkeypatch, tmp_path):
    monkeypatch.setattr(native, "_lib", None)
    monkeypatch.setattr(native, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(native.NativeError):
        native.lib()


@pytest.mark.parametrize("k", [1, 2, 4, 32])
def test_one_delta_adjustment_for_all_selection_strategies(k):
    # truncated geometric p(1) = adjusted delta (from p(0) = 0), and the
    # Laplace threshold inverts the same adjusted delta: one per-partition
    # (eps / k, 1 - (1 - delta)^(1/k)) rule for the three strategies.
    eps, delta = 1.0, 1e-5
    adj = o.adjusted_delta(delta, k)
    assert adj == (delta if k == 1 else pytest.approx(1 - (1 - delta)**(1 / k), rel=1e-9))
    assert abs(adj - delta / k) <= delta**2
    t = native.truncated_geometric_table(eps, delta, k)
    assert t[1] == pytest.approx(adj, rel=1e-12)
    thr, b = native.selection_threshold(2, eps, delta, k)
    assert b == k / eps
    # P(1 + Lap(b) > thr) == adjusted delta (Laplace tail)
    assert 0.5 * math.exp(-(thr - 1) / b) == pytest.approx(adj, rel=1e-9)


def test_shard_symbols_reject_bad_args():
    import ctypes
    n = ctypes.c_size_t(0)
    assert native.lib().pdp_shard_workspace_size(1000, 0, ctypes.byref(n)) != 0
    assert native.lib().pdp_shard_workspace_size(1000, 65, ctypes.byref(n)) != 0
    assert native.lib().pdp_shard_workspace_size(1000, 8, ctypes.byref(n)) == 0 and n.value > 0
