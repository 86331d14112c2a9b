"""Bounding sweep host layer (pipelinedp_amd/analysis.py).

CPU: MultiParameterConfiguration validation and parameter substitution, as
the reference's analysis/tests/data_structures_test.py checks them.
GPU: bounded_accumulators_sweep on Python rows equals, per configuration, the
CPU oracle (oracle/pdp_oracle.py:bound_and_accumulate) with the same seed.
"""
import numpy as np
import pytest

import pdp_oracle as o
from pipelinedp_amd import AggregateParams, DataExtractors, Metrics
from pipelinedp_amd.analysis import MultiParameterConfiguration, bounded_accumulators_sweep


def _params():
    return AggregateParams(metrics=[Metrics.COUNT, Metrics.SUM], max_partitions_contributed=1,
                           max_contributions_per_partition=1, min_value=0.0, max_value=5.0)


def test_multi_config_validation():
    with pytest.raises(ValueError, match="at least 1"):
        MultiParameterConfiguration()
    with pytest.raises(ValueError, match="same length"):
        MultiParameterConfiguration(max_partitions_contributed=[1, 2], max_contributions_per_partition=[1])
    with pytest.raises(ValueError, match="both set"):
        MultiParameterConfiguration(min_sum_per_partition=[0.0])


def test_get_aggregate_params_substitutes_bounds():
    m = MultiParameterConfiguration(max_partitions_contributed=[1, 2], max_contributions_per_partition=[10, 11])
    assert m.size == 2
    p = m.get_aggregate_params(_params(), 1)
    assert (p.max_partitions_contributed, p.max_contributions_per_partition) == (2, 11)
    assert p.min_value == 0.0 and p.metrics == [Metrics.COUNT, Metrics.SUM]
    base = _params()
    m.get_aggregate_params(base, 0)
    assert base.max_partitions_contributed == 1  # the input is not modified


@pytest.mark.gpu
def test_sweep_on_rows_matches_oracle():
    n, U, P = 20000, 400, 300
    pid, pk, val = o.synth_rows(n, U, P, seed=31, zipf_s=1.1)
    rows = list(zip(pid.tolist(), pk.tolist(), (val * 0.7).tolist()))
    ext = DataExtractors(privacy_id_extractor=lambda r: r[0], partition_extractor=lambda r: r[1],
                         value_extractor=lambda r: r[2])
    multi = MultiParameterConfiguration(max_partitions_contributed=[1, 3, 8],
                                        max_contributions_per_partition=[1, 2, 5])
    res = bounded_accumulators_sweep(rows, _params(), ext, multi, sampling_seed=50)
    assert len(res) == 3
    # encode_rows numbers pids and partitions in first-appearance order
    pid_order = {p: i for i, p in enumerate(dict.fromkeys(pid.tolist()))}
    pk_order = {k: i for i, k in enumerate(dict.fromkeys(pk.tolist()))}
    pid_dense = np.array([pid_order[p] for p in pid.tolist()])
    pk_dense = np.array([pk_order[k] for k in pk.tolist()])
    keys = list(pk_order)
    for i, got in enumerate(res):
        bp = o.BoundParams(multi.max_partitions_contributed[i], multi.max_contributions_per_partition[i], 0.0, 5.0)
        ref = o.bound_and_accumulate(pid_dense, pk_dense, val * 0.7, len(keys), bp, "hash", seed=50 + i)
        for j, key in enumerate(keys):
            if ref.row_count[j] == 0:
                assert key not in got
                continue
            a = got[key]
            assert (a.privacy_id_count, a.count) == (int(ref.row_count[j]), int(ref.count[j]))
            assert abs(a.sum - ref.sum[j]) <= 1e-9 * (abs(ref.sum[j]) + 1)
