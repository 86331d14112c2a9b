"""Host-side checks of bench.py (no GPU): the workload presets carry the
BASELINE.json / SURVEY.md 8(d) shapes, explicit flags override them, and the
CPU-baseline leg runs on a tiny sample for every workload."""
import sys

import pytest

import bench


def _parse(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_default_is_headline_c3():
    a = _parse()
    assert a.workload == "c3"
    assert (a.rows, a.partitions, a.pids, a.zipf, a.l0, a.linf) == (1e9, 1e6, 1e7, 1.1, 4, 2)


def test_flags_override_presets():
    a = _parse("--workload", "c2", "--rows", "1e6", "--l0", "3")
    assert (a.rows, a.partitions, a.l0, a.linf) == (1e6, 1e5, 3, 4)
    assert bench.WORKLOADS["c2"]["public"]


def test_sweep_grid_is_64_configs():
    assert len(bench.SWEEP) == 64
    assert {l0 for l0, _ in bench.SWEEP} == {1, 2, 4, 8, 16, 32, 64, 128}
    assert {linf for _, linf in bench.SWEEP} == set(range(1, 9))


@pytest.mark.parametrize("w", ["c2", "c3", "c5"])
def test_cpu_baseline_leg_runs(w):
    a = _parse("--workload", w, "--cpu-sample", "3000", "--partitions", "500")
    res = bench.cpu_baseline(a, int(a.partitions))
    assert res["value"] > 0 and res["kind"] == "port" and res["plan_item"] == 3
    # every host core (up to the GPU box's 16-core share), reported with the CPU model
    assert 1 <= res["cores"] <= 16 and res["host_cpus_visible"] >= res["cores"]
    assert res["sample"].startswith(w)
