"""pdp_bound_accumulate is stream-ordered ("no host sync inside
except optional debug").

* Every count the kernels need (the L0 pre-filter's survivors, K2's slots,
  K4's pairs and chunk) lives in device memory, so a call waits for its stream
  once, to copy the status back (pdp_stats.host_waits == 1), and never with
  PDP_BOUND_ASYNC (host_waits == 0; pdp_get_status reports afterwards).
* An asynchronous accumulate + release is captured in a hipGraph (torch's
  CUDAGraph on ROCm) and replayed: bit for bit the eager results, also after
  the input columns are overwritten in place between replays.
* Tied truncated priorities go to k_segments_big inside the launch sequence,
  not to the host-driven generic path; an input that does need the generic
  path (a privacy id with more rows than the wave kernels hold) is finished
  by a redone, "careful" call in sync mode and reported as ERR_NEEDS_SYNC in
  async mode.
Reference: the lazy, stream-ordered DPEngine.aggregate contract
(pipeline_dp/dp_engine.py:66-109); results as tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

import pdp_oracle as o

pytestmark = pytest.mark.gpu

MASK = 1 | 2 | 4 | 16  # COUNT, SUM, MEAN, PRIVACY_ID_COUNT


@pytest.fixture(scope="module")
def ex():
    from pipelinedp_amd.executor import HipExecutor
    return HipExecutor(0)


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _c3_like(seed=5):
    # the headline's shape at 2^22 rows: ~100 rows per privacy id, L0 = 4 -> the L0 pre-filter runs
    n, P = 1 << 22, 50_000
    U = n // 100
    pid, pk, val = o.synth_rows(n, U, P, seed=seed, zipf_s=1.1, value_lo=-2, value_hi=12)
    return pid, pk, val, U, P


def test_one_host_wait_per_call_and_none_async(ex):
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig
    pid, pk, val, U, P = _c3_like()
    cfg = BoundConfig(MASK, 4, 2, 0.0, 10.0, sampling_seed=7)
    d = [_dev(a) for a in (pid, pk, val)]
    a1 = ex.accumulate(*d, U, P, cfg)
    st = ex.stats()
    assert st.filter_rows > 0 and st.fallback_rows == 0
    assert st.host_waits == 1
    a2 = ex.accumulate(*d, U, P, cfg, sync=False)
    torch.cuda.synchronize()
    assert ex.status() == 0
    st2 = ex.stats()
    assert st2.host_waits == 0
    # (k4_pairs, the records that reach K4's pair passes, depends on which partitions claimed K2's
    # hot-partition slots first; the accumulators do not)
    assert st2.filter_rows == st.filter_rows
    for name in ("row_count", "count", "x"):
        assert torch.equal(getattr(a1, name), getattr(a2, name)), name
    ref = o.bound_and_accumulate(pid, pk, val, P, o.BoundParams(4, 2, 0.0, 10.0), "hash", seed=7)
    np.testing.assert_array_equal(a2.row_count.cpu().numpy(), ref.row_count)
    # the c4-like path (L0 = 32: full pid sort, k_lean sorted) is stream-ordered too
    cfg32 = BoundConfig(MASK, 32, 4, 0.0, 10.0, sampling_seed=8)
    ex.accumulate(*d, U, P, cfg32)
    assert ex.stats().host_waits == 1 and ex.stats().fallback_rows == 0
    assert native.ERR_NEEDS_SYNC == -6


def test_hip_graph_capture_and_replay(ex):
    """accumulate(sync=False) + release captured once, replayed: the eager
    results bit for bit; new data written into the captured input buffers is
    picked up by the next replay."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, ReleaseConfig
    pid, pk, val, U, P = _c3_like(seed=11)
    pid2, pk2, val2, _, _ = _c3_like(seed=12)
    cfg = BoundConfig(MASK, 4, 2, 0.0, 10.0, sampling_seed=3)
    eps = [0.0, 0.0, 0.4, 0.0, 0.3, 0.3]
    delta = [0.0] * 5 + [1e-5]
    rel = ReleaseConfig(MASK, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, 1,
                        add_noise=True, noise_seed=9)
    d_pid, d_pk, d_val = _dev(pid), _dev(pk), _dev(val)

    def step():
        acc = ex.accumulate(d_pid, d_pk, d_val, U, P, cfg, sync=False)
        return ex.release(acc, rel, cfg)

    want_keep, want_out, _ = step()  # eager (also caches the workspace and the selection table)
    torch.cuda.synchronize()
    assert ex.status() == 0
    want_keep, want_out = want_keep.clone(), want_out.clone()
    # eager results of the second input, for the replay after the in-place overwrite
    e_pid, e_pk, e_val = _dev(pid2), _dev(pk2), _dev(val2)
    acc2 = ex.accumulate(e_pid, e_pk, e_val, U, P, cfg)
    k2, o2, _ = ex.release(acc2, rel, cfg)
    torch.cuda.synchronize()
    want2 = (k2.clone(), o2.clone())

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        keep, out, _ = step()
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        assert ex.status() == 0
        assert torch.equal(keep, want_keep)
        same = (out == want_out) | (torch.isnan(out) & torch.isnan(want_out))
        assert bool(same.all())
    d_pid.copy_(e_pid)
    d_pk.copy_(e_pk)
    d_val.copy_(e_val)
    g.replay()
    torch.cuda.synchronize()
    assert ex.status() == 0
    assert torch.equal(keep, want2[0])
    same = (out == want2[1]) | (torch.isnan(out) & torch.isnan(want2[1]))
    assert bool(same.all())


def test_captured_release_survives_later_releases_with_larger_tables():
    """A captured pdp_release points at the context's truncated-geometric
    table.  Round 5 rewrote that table in place for another (eps, delta, L0),
    or freed it for a larger one, so a graph captured earlier replayed the
    wrong keep probabilities or a dangling pointer.  Tables are now immutable
    per (eps, delta, L0) until the context is destroyed, and prepare_release
    builds one outside the capture.  Capture accumulate + release; run eager
    releases that need LARGER tables on the same executor; replay: bit for bit
    the result of a fresh eager run.  An unprepared table under capture is
    ERR_NEEDS_SYNC, not a host synchronisation inside the capture."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig
    ex3 = HipExecutor(0)
    pid, pk, val, U, P = _c3_like(seed=21)
    cfg = BoundConfig(MASK, 4, 2, 0.0, 10.0, sampling_seed=5)
    eps = [0.0, 0.0, 0.4, 0.0, 0.3, 0.3]
    delta = [0.0] * 5 + [1e-5]
    rel = ReleaseConfig(MASK, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, 1,
                        add_noise=True, noise_seed=13)
    # the later, eager releases: smaller selection eps / delta and larger L0 -> longer keep tables
    others = [(0.05, 1e-8, 8), (0.02, 1e-9, 16)]
    n0 = len(native.truncated_geometric_table(0.3, 1e-5, 4))
    assert all(len(native.truncated_geometric_table(e, d, k)) > n0 for e, d, k in others)
    d_pid, d_pk, d_val = _dev(pid), _dev(pk), _dev(val)

    ex3.prepare_release(rel, cfg)  # the table, built outside the capture
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ex3.accumulate(d_pid, d_pk, d_val, U, P, cfg, sync=False)  # warm-up: sizes the workspace
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    rel_new = ReleaseConfig(MASK, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps,
                            [0.0] * 5 + [3e-6], 1, add_noise=True, noise_seed=13)
    with torch.cuda.graph(g):
        acc = ex3.accumulate(d_pid, d_pk, d_val, U, P, cfg, sync=False)
        keep, out, _ = ex3.release(acc, rel, cfg)
        # an unprepared table inside the capture: refused, nothing enqueued, the capture stays valid
        with pytest.raises(native.NativeError, match=r"\(-6\)"):
            ex3.release(acc, rel_new, cfg)
    for e, d, k in others:  # eager releases that need larger tables, on the same context
        cfg_k = BoundConfig(MASK, k, 2, 0.0, 10.0, sampling_seed=5)
        acc_k = ex3.accumulate(d_pid, d_pk, d_val, U, P, cfg_k)
        ex3.release(acc_k, ReleaseConfig(MASK, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC,
                                         [0.0, 0.0, 0.4, 0.0, 0.3, e], [0.0] * 5 + [d], 1, add_noise=True,
                                         noise_seed=13), cfg_k)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    assert ex3.status() == 0
    # a fresh executor, eager
    ex4 = HipExecutor(0)
    acc4 = ex4.accumulate(d_pid, d_pk, d_val, U, P, cfg)
    k4, o4, _ = ex4.release(acc4, rel, cfg)
    torch.cuda.synchronize()
    assert int(k4.sum()) > 0 and int(k4.sum()) < P
    assert torch.equal(keep, k4)
    assert bool(((out == o4) | (torch.isnan(out) & torch.isnan(o4))).all())


def test_generic_path_input_redone_in_sync_mode_and_flagged_async(ex):
    """Privacy ids with > 2048 rows in a wave kernel need the host-driven
    generic path: a sync call redoes itself careful (more than one host wait,
    oracle-exact result; the next call starts careful), an async call leaves
    ERR_NEEDS_SYNC in pdp_get_status."""
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor
    ex2 = HipExecutor(0)  # a fresh context: not yet careful
    n, U, P = 25000, 3, 7
    pid, pk, val = o.synth_rows(n, U, P, seed=105, zipf_s=0.0, value_lo=-5, value_hi=15)
    cfg = BoundConfig(1 | 2 | 4 | 16, 2, 5, 1.0, 5.0, sampling_seed=9)
    d = [_dev(a) for a in (pid, pk, val)]
    ex2.accumulate(*d, U, P, cfg, sync=False)
    torch.cuda.synchronize()
    assert ex2.status() == native.ERR_NEEDS_SYNC
    acc = ex2.accumulate(*d, U, P, cfg)
    st = ex2.stats()
    assert st.fallback_rows > 0 and st.host_waits > 1
    ref = o.bound_and_accumulate(pid, pk, val, P, o.BoundParams(2, 5, 1.0, 5.0), "hash", seed=9)
    np.testing.assert_array_equal(acc.row_count.cpu().numpy(), ref.row_count)
    np.testing.assert_array_equal(acc.count.cpu().numpy(), ref.count)
    kx, _ = o.k4_finalize(o.k4_partials(ref, P, o.BoundParams(2, 5, 1.0, 5.0), 1 | 2 | 4 | 16),
                          o.BoundParams(2, 5, 1.0, 5.0), 1 | 2 | 4 | 16)
    np.testing.assert_array_equal(acc.x.cpu().numpy(), kx)
