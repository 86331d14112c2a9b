"""Test-only stub of pydp.algorithms.partition_selection: keep-all."""


class PartitionSelectionStrategy:

    def should_keep(self, n):
        return True

    def probability_of_keep(self, n):
        return 1.0


def create_truncated_geometric_partition_strategy(eps, delta, k):
    return PartitionSelectionStrategy()


def create_laplace_partition_strategy(eps, delta, k):
    return PartitionSelectionStrategy()


def create_gaussian_partition_strategy(eps, delta, k):
    return PartitionSelectionStrategy()
