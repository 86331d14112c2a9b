"""Diagnostic (GPU box, debug library): ONE look-back radix pass over a large
input.  pid = i mod 256 (U = 256: one 8-bit pass), pk = i // 256 (P = 2^25).
SORT_ONLY call; recs_a = the pass output: row j must be
pid = j // (n / 256), pk = (j mod (n / 256)) mod P.  Args: n:debug_flags ..."""
import sys

import torch

sys.path.insert(0, ".")
from pipelinedp_amd.executor import BoundConfig, HipExecutor  # noqa: E402

ex = HipExecutor(0)
P = 1 << 25  # > n / 256: pk = i // 256 exactly
for spec in sys.argv[1:]:
    a, b = spec.split(":")
    n, dbg = int(float(a)), int(b)
    assert n % 256 == 0
    m = n // 256
    # this torch build's elementwise kernels fill only numel mod 2^32 elements of a > 2^32-element
    # tensor (what this script first found): the columns are built in slices, and checked
    probe = torch.arange(n, dtype=torch.int64, device="cuda")
    print("torch.arange(n)[-1] =", int(probe[-1]), "want", n - 1, flush=True)
    del probe
    pid = torch.empty(n, dtype=torch.int64, device="cuda")
    pk = torch.empty(n, dtype=torch.int64, device="cuda")
    for c0 in range(0, n, 1 << 30):
        r = torch.arange(c0, min(n, c0 + (1 << 30)), dtype=torch.int64, device="cuda")
        pid[c0:c0 + r.numel()] = r.remainder(256)
        pk[c0:c0 + r.numel()] = r.div_(256, rounding_mode="floor")
        del r
    cfg = BoundConfig(1 | 16, 4, 1, sampling_seed=5)
    ex.set_debug(16384 | dbg)
    ex._ws = None
    torch.cuda.empty_cache()
    ex.accumulate(pid, pk, None, 256, P, cfg)
    torch.cuda.synchronize()
    print(n, dbg, "passes", ex.stats().sort_passes, flush=True)
    rb = (n * 16 + 255) // 256 * 256
    hist = ex._ws[2 * rb:2 * rb + 12 * 257 * 8].view(torch.int64).view(12, 257)
    off = ex._ws[2 * rb + 24832:2 * rb + 24832 + 12 * 257 * 8].view(torch.int64).view(12, 257)
    ctr = ex._ws[2 * rb + 2 * 24832:2 * rb + 2 * 24832 + 8 * 24].view(torch.int64)
    print("  hist", hist[0, :3].tolist(), hist[0, 254:].tolist(), "off", off[0, :3].tolist(), off[0, 254:].tolist(),
          "ctr", ctr.tolist(), flush=True)
    del hist, off, ctr
    del pid, pk
    recs = ex._ws[0:n * 16].view(torch.int32).view(n, 4)
    for j in (0, 1, 16, m - 1, m, 1 << 31, (1 << 32) - 1, 1 << 32, n - 1):
        if j < n:
            print("  row", j, "got", recs[j, :2].tolist(), "want", [j // m, (j % m) % P], flush=True)
    bad, first = 0, None
    C = 1 << 28
    for c0 in range(0, n, C):
        c1 = min(n, c0 + C)
        j = torch.arange(c0, c1, dtype=torch.int64, device="cuda")
        got_pid = recs[c0:c1, 0].to(torch.int64) & 0xFFFFFFFF
        got_pk = recs[c0:c1, 1].to(torch.int64) & 0xFFFFFFFF
        mm = (got_pid != j // m) | (got_pk != (j % m) % P)
        k = int(mm.sum())
        if k and first is None:
            i = int(torch.nonzero(mm)[0])
            first = c0 + i
        bad += k
        del j, got_pid, got_pk, mm
    print("  mismatches", bad, "first", first, flush=True)
    del recs
ex.set_debug(0)
