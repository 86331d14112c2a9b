"""Captures one asynchronous accumulate + release (the c3 shape at 2^22 rows)
in a torch CUDAGraph and writes its DOT dump WITHOUT replaying it: inspects
which nodes (kernels, memsets, copies) a captured call holds.  GPU box:
    python tools/graph_dump.py gpurun_out/<dir>/graph.dot"""
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

out_path = sys.argv[1]
ex = HipExecutor(0)
n, P = 1 << 22, 50_000
U = n // 100
pid, pk, val = o.synth_rows(n, U, P, seed=11, zipf_s=1.1, value_lo=-2, value_hi=12)
d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (pid, pk, val)]
cfg = BoundConfig(1 | 2 | 4 | 16, 4, 2, 0.0, 10.0, sampling_seed=3)
rel = ReleaseConfig(1 | 2 | 4 | 16, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC,
                    [0.0, 0.0, 0.4, 0.0, 0.3, 0.3], [0.0] * 5 + [1e-5], 1, add_noise=True, noise_seed=9)


def step():
    acc = ex.accumulate(*d, U, P, cfg, sync=False)
    return ex.release(acc, rel, cfg)


step()
torch.cuda.synchronize()
print("eager status", ex.status(), flush=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
print("side-stream status", ex.status(), flush=True)
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g):
    keep, out, _ = step()
g.debug_dump(out_path)
print("dumped", out_path, os.path.getsize(out_path), flush=True)
