"""Backend plugin boundary.

``PipelineBackend`` keeps the reference's collection-op interface
(pipeline_dp/pipeline_backend.py:38-191) so the engine and callers see the
same seam.  ``HipBackend`` is the new MI355X plugin: it advertises the fused
columnar aggregate capability that ``DPEngine.aggregate`` dispatches to.  Its
per-element collection ops are host plumbing for post-processing results
(e.g. ``make_private(...).mean`` extracting ``.mean``) and the complete
element-wise op set of the reference ABC on the host; the hot path itself
(bounding + combining + selection + noise) runs fused on the GPU.
"""
import abc
import collections
import functools
import itertools
from typing import Callable, Iterable

_annotators = []


class Annotator(abc.ABC):
    """Pipeline annotation hook (reference :791-814)."""

    @abc.abstractmethod
    def annotate(self, col, stage_name: str, **kwargs):
        pass


def register_annotator(annotator: Annotator):
    _annotators.append(annotator)


class PipelineBackend(abc.ABC):
    """Collection operations a DP pipeline is built from."""

    #: set by backends that implement ``aggregate_columnar``
    supports_columnar_aggregate = False

    def to_collection(self, collection_or_iterable, col, stage_name: str):
        return collection_or_iterable

    def to_multi_transformable_collection(self, col):
        return col

    @abc.abstractmethod
    def map(self, col, fn, stage_name: str = None):
        pass

    @abc.abstractmethod
    def flat_map(self, col, fn, stage_name: str = None):
        pass

    @abc.abstractmethod
    def map_tuple(self, col, fn, stage_name: str = None):
        pass

    @abc.abstractmethod
    def map_values(self, col, fn, stage_name: str = None):
        pass

    @abc.abstractmethod
    def group_by_key(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def filter(self, col, fn, stage_name: str = None):
        pass

    @abc.abstractmethod
    def filter_by_key(self, col, keys_to_keep, stage_name: str = None):
        pass

    @abc.abstractmethod
    def keys(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def values(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def sample_fixed_per_key(self, col, n: int, stage_name: str = None):
        pass

    @abc.abstractmethod
    def count_per_element(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def sum_per_key(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def combine_accumulators_per_key(self, col, combiner, stage_name: str = None):
        pass

    @abc.abstractmethod
    def reduce_per_key(self, col, fn: Callable, stage_name: str = None):
        pass

    @abc.abstractmethod
    def flatten(self, cols: Iterable, stage_name: str = None):
        pass

    @abc.abstractmethod
    def distinct(self, col, stage_name: str = None):
        pass

    @abc.abstractmethod
    def to_list(self, col, stage_name: str = None):
        pass

    def annotate(self, col, stage_name: str, **kwargs):
        for a in _annotators:
            col = a.annotate(col, stage_name, **kwargs)
        return col


class HipBackend(PipelineBackend):
    """MI355X backend: DPEngine.aggregate / select_partitions run as the fused
    HIP pipeline of libpdp_hip.so on ``device`` (default: torch's current
    device).  ``world`` (optional) is a ``pipelinedp_amd.distributed.World``
    for multi-GPU execution over RCCL.

    ``sampling_seed`` / ``noise_seed`` fix the Philox / Feistel keys for
    reproducible runs (default: fresh 64-bit secrets per aggregation).
    ``_unsafe_disable_noise_for_testing`` releases exact values and must only
    be used by parity tests."""

    supports_columnar_aggregate = True

    def __init__(self, device=None, world=None, sampling_seed=None, noise_seed=None,
                 _unsafe_disable_noise_for_testing=False, _debug_force_fallback=False):
        self._device = device
        self._executor = None
        self.world = world
        self.sampling_seed = sampling_seed
        self.noise_seed = noise_seed
        self._disable_noise = bool(_unsafe_disable_noise_for_testing)
        self._debug_force_fallback = bool(_debug_force_fallback)

    @property
    def executor(self):
        if self._executor is None:
            from .executor import HipExecutor
            self._executor = HipExecutor(self._device)
        return self._executor

    # -- host collection plumbing (lazy generators) --------------------------
    def map(self, col, fn, stage_name=None):
        return map(fn, col)

    def flat_map(self, col, fn, stage_name=None):
        return (y for x in col for y in fn(x))

    def map_tuple(self, col, fn, stage_name=None):
        return (fn(*x) for x in col)

    def map_values(self, col, fn, stage_name=None):
        return ((k, fn(v)) for k, v in col)

    def group_by_key(self, col, stage_name=None):

        def gen():
            groups = collections.defaultdict(list)
            for k, v in col:
                groups[k].append(v)
            yield from groups.items()

        return gen()

    def filter(self, col, fn, stage_name=None):
        return filter(fn, col)

    def filter_by_key(self, col, keys_to_keep, stage_name=None):
        keep = keys_to_keep if isinstance(keys_to_keep, (set, frozenset, dict)) else set(keys_to_keep)
        return (kv for kv in col if kv[0] in keep)

    def keys(self, col, stage_name=None):
        return (k for k, _ in col)

    def values(self, col, stage_name=None):
        return (v for _, v in col)

    def count_per_element(self, col, stage_name=None):
        return iter(collections.Counter(col).items())

    def sum_per_key(self, col, stage_name=None):
        return self.map_values(self.group_by_key(col), sum)

    def reduce_per_key(self, col, fn, stage_name=None):
        return self.map_values(self.group_by_key(col), lambda vs: functools.reduce(fn, vs))

    def flatten(self, cols, stage_name=None):
        return itertools.chain(*cols)

    def distinct(self, col, stage_name=None):
        return iter(set(col))

    def to_list(self, col, stage_name=None):
        return iter([list(col)])

    # -- per-key sampling / combining, element-wise on the host ---------------
    # DPEngine.aggregate / select_partitions never call these: bounding and
    # combining run fused on the GPU.  They complete the PipelineBackend seam
    # (the reference's 17 abstract ops) for callers that build their own
    # element-wise graphs, with LocalBackend's semantics.
    def sample_fixed_per_key(self, col, n, stage_name=None):
        """Per key, a uniform sample of <= n values without replacement
        (LocalBackend.sample_fixed_per_key, pipeline_backend.py:504-520)."""
        import numpy as np

        def gen():
            rng = np.random.default_rng(self.sampling_seed)
            for key, values in self.group_by_key(col):
                if len(values) > n:
                    idx = rng.choice(len(values), n, replace=False)
                    values = [values[i] for i in idx]
                yield key, values

        return gen()

    def combine_accumulators_per_key(self, col, combiner, stage_name=None):
        """Per key, the accumulators merged with combiner.merge_accumulators
        (LocalBackend.combine_accumulators_per_key, pipeline_backend.py:528-538)."""
        return self.map_values(self.group_by_key(col),
                               lambda accs: functools.reduce(combiner.merge_accumulators, accs))
