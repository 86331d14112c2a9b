"""Per-kernel summary of a rocprofv3 --pmc counter_collection.csv (SQ counters
per wave).   python tools/pmc_summary.py gpurun_out/<dir>"""
import collections
import csv
import glob
import sys


def kname(s):
    s = s.replace("void ", "").replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("<")[0]


agg = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        agg[kname(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
for n, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    w = c.get("SQ_WAVES", 0) or 1
    print(f"{n[:24]:24s} waves {c.get('SQ_WAVES', 0):9.0f} " +
          " ".join(f"{k.replace('SQ_INSTS_', '').replace('SQ_', '')}/w {v / w:8.0f}" for k, v in sorted(c.items())
                   if k != "SQ_WAVES"))
