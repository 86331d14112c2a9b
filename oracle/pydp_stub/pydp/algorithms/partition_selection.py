"""Test-only stub of pydp.algorithms.partition_selection.

should_keep(n): keep-all by default, so the reference LocalBackend output is
deterministic; with PDP_STUB_SELECT_THRESHOLD=T in the environment it keeps
exactly the partitions with n >= T (golden vectors of select_partitions that
pin the privacy-id counting).

probability_of_keep(n) (used by the reference's utility analysis,
analysis/combiners.py:124-141) is the oracle's restatement of PyDP's
strategies: the truncated-geometric keep table, and P(n + noise > threshold)
for Laplace / Gaussian thresholding (pdp_oracle.py; parity unpinned for
k > 1 and for the thresholding strategies).
"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", ".."))
import pdp_oracle as _o  # noqa: E402


class PartitionSelectionStrategy:

    def __init__(self, prob_fn=None):
        self._prob_fn = prob_fn

    def should_keep(self, n):
        t = os.environ.get("PDP_STUB_SELECT_THRESHOLD")
        return True if t is None else n >= int(t)

    def probability_of_keep(self, n):
        return 1.0 if self._prob_fn is None else self._prob_fn(n)


def create_truncated_geometric_partition_strategy(eps, delta, k):
    table = _o.truncated_geometric_table(eps, delta, k)
    return PartitionSelectionStrategy(lambda n: float(table[n]) if 0 <= n < len(table) else (1.0 if n > 0 else 0.0))


def create_laplace_partition_strategy(eps, delta, k):
    thr, b = _o.laplace_threshold(eps, delta, k)

    def prob(n):  # P(n + Laplace(b) > thr)
        if n <= 0:
            return 0.0
        x = thr - n
        return 0.5 * math.exp(-x / b) if x >= 0 else 1.0 - 0.5 * math.exp(x / b)

    return PartitionSelectionStrategy(prob)


def create_gaussian_partition_strategy(eps, delta, k):
    thr, sigma = _o.gaussian_threshold(eps, delta, k)

    def prob(n):  # P(n + N(0, sigma^2) > thr)
        if n <= 0:
            return 0.0
        return 0.5 * math.erfc((thr - n) / (sigma * math.sqrt(2.0)))

    return PartitionSelectionStrategy(prob)
