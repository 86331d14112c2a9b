"""K4 vs the fp64-atomic accumulation (PDP_K4=0) on the same device inputs:
counts / privacy-id counts bit-exact, sums to 1e-9 relative.  Diagnostic for
the GPU box; prints one line per shape as it goes.

  python tools/k4_check.py "rows,pids,parts,zipf,l0,linf,public[,metrics]" ...
metrics: mean (COUNT+SUM+MEAN, default), count_sum, variance."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor
    ex = HipExecutor(0)
    bad = 0
    for spec in sys.argv[1:]:
        f = spec.split(",")
        n, U, P = int(float(f[0])), int(float(f[1])), int(float(f[2]))
        zipf, l0, linf, public = float(f[3]), int(f[4]), int(f[5]), int(f[6])
        metrics = f[7] if len(f) > 7 else "mean"
        pid, pk, val = ex.generate(n, U, P, seed=7, zipf_s=zipf, lo=0.0, hi=10.0)
        if public:  # every other partition public: the other rows drop
            pk = torch.where(pk % 2 == 0, pk // 2, torch.full_like(pk, -1))
            P = (P + 1) // 2
        mask = native.METRIC_COUNT | native.METRIC_SUM
        if metrics == "mean":
            mask |= native.METRIC_MEAN
        elif metrics == "variance":
            mask |= native.METRIC_VARIANCE | native.METRIC_MEAN
        cfg = BoundConfig(mask, l0, linf, 0.0, 10.0, sampling_seed=3)
        res = {}
        for k4 in ("1", "0"):
            os.environ["PDP_K4"] = k4
            t0 = time.perf_counter()
            try:
                acc = ex.accumulate(pid, pk, val, U, P, cfg)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                print(f"{spec} K4={k4}: ERROR {e}", flush=True)
                res[k4] = None
                continue
            st = ex.stats()
            res[k4] = [None if t is None else t.cpu().numpy() for t in (acc.row_count, acc.count, acc.x, acc.y)]
            print(f"{spec} K4={k4}: {time.perf_counter() - t0:.2f}s filter_rows={st.filter_rows} "
                  f"k4_slots={st.k4_slots} k4_pairs={st.k4_pairs} fallback_rows={st.fallback_rows}", flush=True)
        os.environ.pop("PDP_K4", None)
        if res.get("1") is None or res.get("0") is None:
            bad += 1
            continue
        a, b = res["1"], res["0"]
        ok = np.array_equal(a[0], b[0]) and (a[1] is None or np.array_equal(a[1], b[1]))
        msg = []
        if not ok:
            d = np.flatnonzero(a[0] != b[0])
            msg.append(f"row_count differs at {len(d)} partitions, e.g. {d[:5].tolist()} "
                       f"{a[0][d[:5]].tolist()} vs {b[0][d[:5]].tolist()}")
        for i, nm in ((2, "x"), (3, "y")):
            if a[i] is not None:
                err = np.abs(a[i] - b[i])
                tol = 1e-9 * (np.abs(b[i]) + 1.0)
                if not np.all(err <= tol):
                    ok = False
                    msg.append(f"{nm} max err {err.max():.3e}")
        bad += not ok
        print(f"{spec}: {'OK' if ok else 'MISMATCH ' + '; '.join(msg)} (pairs {int(a[0].sum())})", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
