"""Staged hipGraph capture/replay check of the aggregate path (GPU box), one
stage per process so a failing stage names itself:
    python tools/graph_stages.py release|enforced|nofilter|filter
Each stage: eager run (reference), capture in a torch CUDAGraph (after a
side-stream warm-up), replay twice, compare bit for bit, print OK."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pdp_oracle as o  # noqa: E402  (input generator only)
from pipelinedp_amd import native  # noqa: E402
from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig  # noqa: E402

stage = sys.argv[1]
ex = HipExecutor(0)
MASK = 1 | 2 | 4 | 16
if stage == "filter":
    n, P = 1 << 22, 50_000
    U = n // 100
    L0, Linf = 4, 2
else:
    n, U, P = 50_000, 2_000, 700
    L0, Linf = 3, 2
pid, pk, val = o.synth_rows(n, U, P, seed=11, zipf_s=1.1, value_lo=-2, value_hi=12)
d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (pid, pk, val)]
cfg = BoundConfig(MASK, L0, Linf, 0.0, 10.0, bounds_already_enforced=stage == "enforced", sampling_seed=3)
rel = ReleaseConfig(MASK if stage != "enforced" else 1 | 2 | 4, native.NOISE_LAPLACE,
                    native.SELECTION_TRUNCATED_GEOMETRIC, [0.3, 0.3, 0.4, 0.0, 0.3, 0.3], [0.0] * 5 + [1e-5],
                    Linf if stage == "enforced" else 1, add_noise=True, noise_seed=9)
if stage == "enforced":
    cfg.metrics_mask = 1 | 2 | 4
pre = ex.accumulate(*d, U, P, cfg)  # synchronous: also the reference accumulators


def step():
    acc = pre if stage == "release" else ex.accumulate(*d, U, P, cfg, sync=False)
    return ex.release(acc, rel, cfg)


k0, m0, _ = step()
torch.cuda.synchronize()
assert ex.status() == 0
k0, m0 = k0.clone(), m0.clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print(stage, "captured ...", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    keep, out, _ = step()
for i in range(2):
    g.replay()
    torch.cuda.synchronize()
    assert ex.status() == 0
    assert torch.equal(keep, k0), stage
    assert bool(((out == m0) | (torch.isnan(out) & torch.isnan(m0))).all()), stage
    print(stage, "replay", i, "ok", flush=True)
print(stage, "OK", flush=True)
