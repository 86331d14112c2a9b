"""Helpers to load the committed golden fixtures (tests/golden/*.npz)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def aggregate_cases():
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))
    return [n for n in names if not n.startswith(("binding_", "select_partitions_", "analysis_", "aggregate_"))]


def known_answers():
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        return json.load(f)


def encode_case(d):
    """Dense-encode a golden case the same way the host layer does:
    public partitions first (in given order), then observed keys."""
    pk_raw = d["pk"]
    if bool(d["has_public"]):
        keys = d["public"]
        lut = {int(k): i for i, k in enumerate(keys)}
        pk = np.array([lut.get(int(k), -1) for k in pk_raw], dtype=np.int64)
    else:
        keys, pk = np.unique(pk_raw, return_inverse=True)
    pid = d["pid"]
    if len(pid):
        _, pid = np.unique(pid, return_inverse=True)
    return pid.astype(np.int64), pk.astype(np.int64), np.asarray(keys, dtype=np.int64)


def sum_tolerance(expected, scale):
    """Float sums may differ only by summation order: |a-b| <= 1e-9 *
    (sum of |terms|) + 1e-9.  ``scale`` is an upper bound of sum |terms|."""
    return 1e-9 * np.abs(scale) + 1e-9
