"""PCIe-inclusive rate of the path when the caller hands over HOST columns
(Measurement): times host->device copies of int64 pid, int64 pk
and f64 value from pinned memory, then the same rows through
pdp_bound_accumulate + pdp_release on device, and reports both rates and the
end-to-end rate with the copy included (not overlapped).

  python tools/pcie_rate.py [rows]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor, ReleaseConfig

    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 200_000_000
    U, P = max(1, n // 100), 1_000_000
    ex = HipExecutor(0)
    pid, pk, val = ex.generate(n, U, P, seed=20250204, zipf_s=1.1, lo=0.0, hi=10.0)
    host = [t.cpu().pin_memory() for t in (pid, pk, val)]
    dev = [torch.empty_like(t) for t in (pid, pk, val)]
    mask = native.METRIC_COUNT | native.METRIC_SUM | native.METRIC_MEAN
    bounds = BoundConfig(mask, 4, 2, 0.0, 10.0, sampling_seed=1)
    eps, delta = [0.0] * native.NUM_MECH, [0.0] * native.NUM_MECH
    eps[native.MECH_MEAN] = 0.5
    eps[native.MECH_SELECTION], delta[native.MECH_SELECTION] = 0.5, 1e-6
    rel = ReleaseConfig(mask, native.NOISE_LAPLACE, native.SELECTION_TRUNCATED_GEOMETRIC, eps, delta, noise_seed=2)

    def h2d():
        for d, h in zip(dev, host):
            d.copy_(h, non_blocking=True)

    def kernels():
        acc = ex.accumulate(dev[0], dev[1], dev[2], U, P, bounds)
        ex.release(acc, rel, bounds)

    res = {}
    for name, fn in (("h2d", h2d), ("kernels", kernels)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / 3
    line = {"rows": n, "h2d_s": res["h2d"], "h2d_GBs": 24 * n / res["h2d"] / 1e9,
            "kernel_rows_per_s": n / res["kernels"], "pcie_inclusive_rows_per_s": n / (res["h2d"] + res["kernels"])}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
