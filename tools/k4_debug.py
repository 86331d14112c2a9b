"""Which K2 / K4 combination disagrees with the oracle?  Small forced-filter
inputs (oracle-sized), each kernel mode against oracle/pdp_oracle.py:
  thin+K4, lean+K4 (kDebugNoThin), thin (PDP_K4=0), nofilter+K4.
Prints per mode: row_count / count mismatches and max |x| error.  GPU-box
diagnostic (test infrastructure: imports the oracle as the checker)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

FORCE_FILTER, NO_THIN, NO_FILTER = 268435456, 536870912, 134217728


def main():
    import numpy as np
    import torch

    import pdp_oracle as o
    from pipelinedp_amd import native
    from pipelinedp_amd.executor import BoundConfig, HipExecutor
    ex = HipExecutor(0)
    bad = 0
    shapes = [(200000, 3000, 500, 0.0, 8, 4), (200000, 3000, 500, 1.1, 4, 2), (300000, 2000, 20000, 1.1, 8, 3),
              (1 << 20, 20000, 5000, 0.0, 8, 4)]
    for n, U, P, z, l0, linf in shapes:
        pid, pk, val = o.synth_rows(n, U, P, seed=11, zipf_s=z)
        mask = native.METRIC_COUNT | native.METRIC_SUM | native.METRIC_PRIVACY_ID_COUNT
        ref = o.bound_and_accumulate(pid, pk, val, P, o.BoundParams(l0, linf, 0.0, 10.0), "hash", seed=5)
        d = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
        for name, flags, k4 in (("thin+K4", FORCE_FILTER, "1"), ("lean+K4", FORCE_FILTER | NO_THIN, "1"),
                                ("thin-K4", FORCE_FILTER, "0"), ("nofilter+K4", NO_FILTER, "1"),
                                ("nofilter-K4", NO_FILTER, "0")):
            os.environ["PDP_K4"] = k4
            cfg = BoundConfig(mask, l0, linf, 0.0, 10.0, sampling_seed=5, debug_flags=flags)
            try:
                acc = ex.accumulate(d(pid), d(pk), d(val), U, P, cfg)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001
                print(f"{(n, U, P, z, l0, linf)} {name}: ERROR {e}", flush=True)
                bad += 1
                if "illegal" in str(e):
                    sys.exit(3)
                continue
            st = ex.stats()
            rc, cnt, x = acc.row_count.cpu().numpy(), acc.count.cpu().numpy(), acc.x.cpu().numpy()
            drc = np.flatnonzero(rc != ref.row_count)
            dc = np.flatnonzero(cnt != ref.count)
            ex_ = np.abs(x - ref.sum).max()
            ok = len(drc) == 0 and len(dc) == 0 and ex_ <= 1e-6
            bad += not ok
            print(f"{(n, U, P, z, l0, linf)} {name}: {'OK' if ok else 'BAD'} filter_rows={st.filter_rows} "
                  f"k4_pairs={st.k4_pairs} rc_diff={len(drc)} {drc[:6].tolist()} "
                  f"{rc[drc[:6]].tolist()} vs {ref.row_count[drc[:6]].tolist()} cnt_diff={len(dc)} "
                  f"x_err={ex_:.3e} pairs={int(rc.sum())} vs {int(ref.row_count.sum())}", flush=True)
        os.environ.pop("PDP_K4", None)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
