import sys, time, json
sys.path.insert(0, "/root/repo")
import torch
from pipelinedp_amd import native
from pipelinedp_amd.executor import BoundConfig, HipExecutor
ex = HipExecutor(0)
n, U, P = 100_000_000, 1_000_000, 100_000
pid, pk, val = ex.generate(n, U, P, seed=1, zipf_s=1.1)
ex.profile(True)
out = {}
for l0 in (1, 4, 16, 32, 64, 65, 128):
    for linf in (1, 8):
        cfg = BoundConfig(native.METRIC_COUNT, l0, linf, sampling_seed=3)
        ex.accumulate(pid, pk, val, U, P, cfg)
        torch.cuda.synchronize()
        ex.profile_read(reset=True)
        for _ in range(3):
            ex.accumulate(pid, pk, val, U, P, cfg)
        torch.cuda.synchronize()
        prof = ex.profile_read(reset=True)
        out[f"L0={l0},Linf={linf}"] = round(prof["buckets"][0] / max(prof["buckets"][1], 1), 3)
print(json.dumps(out))
