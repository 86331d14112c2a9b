"""GPU parity of the bounding sweep (pdp_bound_accumulate_sweep): one sort by
privacy id, then bounding + accumulation per configuration -- the batched
form of the utility-analysis runs over many AggregateParams
(analysis/utility_analysis_engine.py:88-173, BASELINE.json config c5).

Each configuration's accumulators must equal a single pdp_bound_accumulate
with the same parameters and seed (counts bit-exact, fp64 sums to 1e-9
relative: same kept rows, atomics order differs) and the CPU oracle
(oracle/pdp_oracle.py:bound_and_accumulate).  A forced generic-path
configuration in the middle checks that the sorted rows survive it.
"""
import numpy as np
import pytest

import pdp_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ex():
    from pipelinedp_amd.executor import HipExecutor
    return HipExecutor(0)


def _cfgs(mask):
    from pipelinedp_amd.executor import BoundConfig
    out = []
    for i, (l0, linf) in enumerate([(1, 1), (2, 1), (4, 2), (8, 3), (32, 1), (3, 8), (70, 2), (4, 2)]):
        out.append(BoundConfig(mask, l0, linf, 0.0 if i % 2 else -1.0, 10.0 - i, sampling_seed=100 + i,
                               debug_force_fallback=(i == 3)))
    return out


@pytest.mark.parametrize("shape", [(60000, 800, 3000, 1.1), (30000, 3, 40, 0.0), (40000, 20000, 500, 0.0)])
def test_sweep_matches_single_runs_and_oracle(ex, shape):
    import torch
    n, U, P, z = shape
    mask = 1 | 2 | 4 | 8 | 16
    pid, pk, val = o.synth_rows(n, U, P, seed=77, zipf_s=z)
    val = val * 1.3 - 1.0  # some values outside the bounds (clipping)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    tp, tk, tv = d(pid), d(pk), d(val)
    cfgs = _cfgs(mask)
    accs = ex.accumulate_sweep(tp, tk, tv, U, P, cfgs)
    torch.cuda.synchronize()
    assert len(accs) == len(cfgs)
    for c, a in zip(cfgs, accs):
        single = ex.accumulate(tp, tk, tv, U, P, c)
        torch.cuda.synchronize()
        assert torch.equal(a.row_count, single.row_count)
        assert torch.equal(a.count, single.count)
        for f in ("x", "y"):
            g, s = getattr(a, f), getattr(single, f)
            assert bool(((g - s).abs() <= 1e-9 * (s.abs() + a.count.to(torch.float64) * 100 + 1)).all())
        ref = o.bound_and_accumulate(pid, pk, val, P,
                                     o.BoundParams(c.max_partitions_contributed, c.max_contributions_per_partition,
                                                   c.min_value, c.max_value), "hash", seed=c.sampling_seed)
        np.testing.assert_array_equal(a.row_count.cpu().numpy(), ref.row_count)
        np.testing.assert_array_equal(a.count.cpu().numpy(), ref.count)
        tol = 1e-9 * ((ref.count + 1) * 200.0) + 1e-9
        assert np.all(np.abs(a.x.cpu().numpy() - ref.nsum) <= tol)
        assert np.all(np.abs(a.y.cpu().numpy() - ref.nsumsq) <= tol * 100)


def test_sweep_rejects_enforced_bounds(ex):
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig
    pid = torch.zeros(4, dtype=torch.int64, device="cuda")
    val = torch.zeros(4, dtype=torch.float64, device="cuda")
    cfg = BoundConfig(1, 1, 1, bounds_already_enforced=True, sampling_seed=1)
    with pytest.raises(native.NativeError):
        ex.accumulate_sweep(pid, pid.clone(), val, 1, 1, [cfg])
