"""The multi-GPU path (World.aggregate: rank-local bound+accumulate, RCCL
reduce-scatter of the [P] accumulators, owner-side release) on the nccl
(= RCCL) backend with real device tensors.  One GPU box => world size 1, so
this checks the collective calls (dtypes, shapes, layouts) on RCCL; the
world-size-2 data flow is covered by the gloo tests (tests/test_distributed.py).
Must equal the single-process path bit-exactly: the reduce-scatter of one rank
is the identity and Philox noise is keyed by the global partition id."""
import socket

import numpy as np
import pytest

import pdp_oracle as o

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world_aggregate_on_rccl_matches_single_process():
    import torch
    import torch.distributed as dist
    from pipelinedp_amd import native
    from pipelinedp_amd.distributed import World
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        ex = HipExecutor(0)
        n, U, P = 50000, 900, 777
        pid, pk, val = o.synth_rows(n, U, P, seed=21, zipf_s=1.1)
        d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
        mask = native.METRIC_COUNT | native.METRIC_SUM | native.METRIC_MEAN | native.METRIC_PRIVACY_ID_COUNT
        bounds = BoundConfig(mask, 3, 2, 0.0, 10.0, sampling_seed=5)
        eps = [0.0] * native.NUM_MECH
        delta = [0.0] * native.NUM_MECH
        eps[native.MECH_MEAN], eps[native.MECH_PRIVACY_ID_COUNT] = 0.4, 0.3
        eps[native.MECH_SELECTION], delta[native.MECH_SELECTION] = 0.3, 1e-5
        rel = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta,
                            noise_seed=9)
        world = World(0, 1)
        k1, m1, f1 = world.aggregate(ex, d(pid), d(pk), d(val), U, P, bounds, rel, gather=True)
        acc = ex.accumulate(d(pid), d(pk), d(val), U, P, bounds)
        k2, m2, f2 = ex.release(acc, rel, bounds)
        torch.cuda.synchronize()
        assert f1 == f2
        np.testing.assert_array_equal(k1.cpu().numpy(), k2[:P].cpu().numpy())
        kept = k2[:P].bool().cpu().numpy()
        a, b = m1.cpu().numpy()[:, kept], m2[:, :P].cpu().numpy()[:, kept]
        np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-9)
    finally:
        dist.destroy_process_group()
