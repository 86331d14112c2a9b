"""Prints the last pipeline step of a rocprofv3 kernel trace: every dispatch
with its duration and the idle gap before it (GPU time not in kernels).

  python tools/timeline.py gpurun_out/<dir>   (searches *kernel_trace.csv)
"""
import csv
import glob
import sys


def main(d):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    rows = []
    for p in paths:
        rows += list(csv.DictReader(open(p)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].split("<")[0].replace("(anonymous namespace)::", "")  # noqa: E731
    starts = [i for i, r in enumerate(rows) if name(r).startswith("k_histogram")]
    step = rows[starts[-2]:starts[-1]] if len(starts) > 1 else rows[starts[-1]:]
    t0 = int(step[0]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        print(f"{(s - t0) / 1e6:9.3f} ms  gap {(s - prev_end) / 1e3:8.1f} us  dur {(e - s) / 1e3:9.1f} us  {name(r)}")
        prev_end = e
    span = prev_end - t0
    print(f"step span {span / 1e6:.3f} ms, kernels {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
