from . import numerical_mechanisms, partition_selection, quantile_tree  # noqa
