"""ctypes binding of libpdp_hip.so (C ABI: include/pdp_hip.h).

The library is built in-tree by ``pipelinedp_amd/build.py`` (hipcc,
--offload-arch=gfx950).  There is no CPU fallback: if the library is missing
every call raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PDP_HIP_LIB") or os.path.join(_HERE, "libpdp_hip.so")  # env: experiment builds

PDP_OK = 0
ERR_OUT_OF_RANGE, ERR_INTERNAL, ERR_NEEDS_SYNC = -4, -5, -6
BOUND_ASYNC = 1  # pdp_bound_params.flags: no host synchronisation (pdp_get_status afterwards)
ABI_VERSION = 4
METRIC_COUNT, METRIC_SUM, METRIC_MEAN, METRIC_VARIANCE, METRIC_PRIVACY_ID_COUNT = 1, 2, 4, 8, 16
FIELD_NAMES = {0: "variance", 1: "mean", 2: "count", 3: "sum", 4: "privacy_id_count"}
NOISE_LAPLACE, NOISE_GAUSSIAN = 0, 1
SELECTION_NONE, SELECTION_TRUNCATED_GEOMETRIC, SELECTION_LAPLACE, SELECTION_GAUSSIAN = 0, 1, 2, 3
MECH_COUNT, MECH_SUM, MECH_MEAN, MECH_VARIANCE, MECH_PRIVACY_ID_COUNT, MECH_SELECTION = range(6)
NUM_MECH = 6

# Debug flags (pdp_bound_params.reserved / pdp_ctx_set_debug; testing only): alternative forms of a
# stage with identical results, and the forced-path switches of the parity suite.
DEBUG_NO_K4 = 1  # round-2 fp64-atomic accumulation instead of K4 (last bits of sums differ)
DEBUG_K4_P16 = 2
DEBUG_K4_SOA = 4
DEBUG_ODD_GRID = 8
DEBUG_SORT_TILESCAN = 16
DEBUG_ANA_NPART_ATOMICS = 32
DEBUG_ANA_PACK = 64
DEBUG_ANA_FLAGS = 128
DEBUG_ANA_SEL_LDS = 256
DEBUG_DEV_OCC2 = 512  # device-sized look-back passes at 2 blocks per CU
DEBUG_K4_COMPACT = 1024  # K2 claims compacted K4 pair slots (one atomic counter; measured slower)
DEBUG_THIN2 = 67108864  # K4 on: the LDS-staged k_thin2 instead of k_thin (measured slower)
# second flag word (pdp_bound_params.reserved2)
DEBUG2_OVERFLOW_FULL1 = 1  # a second overflow range already sets the "redo everything on the generic path" flag
DEBUG2_FILTER_REC8 = 2  # L0 pre-filter bucket pass with 8-byte {pk, row index} records (measured slower, r06c)
DEBUG2_NO_GROUP = 4  # survivor grouping by a second look-back pass instead of the LDS grouping (k_group)
DEBUG2_GROUP_FALLBACK = 8  # the LDS grouping hands every sub-run to that look-back pass (device-side fallback)
DEBUG2_NO_CLASS_SPLIT = 16  # bucket pass without the low-level-first order inside a tile's bucket run
DEBUG2_THIN_CHUNK_2048 = 32  # K2 k_thin with 2048-row wave chunks whatever the expected survivor count
DEBUG_NO_HOT_CACHE = 524288  # K2 without its hot-partition table (K4 off: LDS atomics cache; K4 on: K4Hot)

c_i32, c_i64, c_u64, c_f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
c_vp = ctypes.c_void_p


class Columns(ctypes.Structure):
    _fields_ = [("pid", c_vp), ("pk", c_vp), ("value", c_vp), ("num_rows", c_i64),
                ("num_privacy_ids", c_i64), ("num_partitions", c_i64)]


class BoundParams(ctypes.Structure):
    _fields_ = [("metrics", c_i32), ("bounds_already_enforced", c_i32),
                ("max_partitions_contributed", c_i64), ("max_contributions_per_partition", c_i64),
                ("has_value_bounds", c_i32), ("has_partition_bounds", c_i32),
                ("min_value", c_f64), ("max_value", c_f64),
                ("min_sum_per_partition", c_f64), ("max_sum_per_partition", c_f64),
                ("sampling_seed", c_u64), ("debug_force_fallback", c_i32), ("reserved", c_i32),
                ("flags", c_i32), ("reserved2", c_i32), ("pid_base", c_i64)]


class Accumulators(ctypes.Structure):
    _fields_ = [("row_count", c_vp), ("count", c_vp), ("x", c_vp), ("y", c_vp)]


class Partials(ctypes.Structure):
    _fields_ = [("row_count", c_vp), ("count", c_vp), ("x_hi", c_vp), ("x_lo", c_vp), ("y_hi", c_vp),
                ("y_lo", c_vp), ("nan", c_vp)]


class ReleaseParams(ctypes.Structure):
    _fields_ = [("metrics", c_i32), ("noise_kind", c_i32), ("selection", c_i32), ("add_noise", c_i32),
                ("max_partitions_contributed", c_i64), ("max_contributions_per_partition", c_i64),
                ("has_value_bounds", c_i32), ("has_partition_bounds", c_i32),
                ("min_value", c_f64), ("max_value", c_f64),
                ("min_sum_per_partition", c_f64), ("max_sum_per_partition", c_f64),
                ("eps", c_f64 * NUM_MECH), ("delta", c_f64 * NUM_MECH),
                ("max_rows_per_privacy_id", c_i64), ("noise_seed", c_u64)]


class Outputs(ctypes.Structure):
    _fields_ = [("keep", c_vp), ("metrics", c_vp)]


class AnalysisConfig(ctypes.Structure):
    _fields_ = [("max_partitions_contributed", c_i64), ("max_contributions_per_partition", c_i64),
                ("min_sum_per_partition", c_f64), ("max_sum_per_partition", c_f64),
                ("selection", c_i32), ("reserved", c_i32), ("selection_eps", c_f64), ("selection_delta", c_f64)]


class AnalysisOutputs(ctypes.Structure):
    _fields_ = [("metrics", c_vp), ("prob_keep", c_vp), ("privacy_ids", c_vp)]


class AggregateParams(ctypes.Structure):
    _fields_ = [("num_configs", c_i32), ("metrics", c_i32), ("num_quantiles", c_i32), ("reserved", c_i32),
                ("quantiles", c_vp), ("std_noise", c_vp), ("noise_kind", c_vp)]


AGG_NUM_FIELDS = 20  # PDP_AGG_NUM_FIELDS; field order = pdp_hip.h PDP_AGG_* enum
AGG_FIELDS = ("num_partitions", "kept_partitions_expected", "total_aggregate", "data_dropped_l0",
              "data_dropped_linf", "data_dropped_partition_selection", "error_l0_expected", "error_linf_expected",
              "error_linf_min_expected", "error_linf_max_expected", "error_l0_variance", "error_variance",
              "rel_error_l0_expected", "rel_error_linf_expected", "rel_error_linf_min_expected",
              "rel_error_linf_max_expected", "rel_error_l0_variance", "rel_error_variance",
              "error_expected_w_dropped_partitions", "rel_error_expected_w_dropped_partitions")


class Stats(ctypes.Structure):
    _fields_ = [("kept_rows_in", c_i64), ("fallback_rows", c_i64), ("fallback_ranges", c_i64),
                ("sort_passes", c_i32), ("bucket_low_bits", c_i32), ("sweep_cycles", c_i64 * 4),
                ("sweep_tiles", c_i64), ("filter_rows", c_i64), ("k4_slots", c_i64), ("k4_pairs", c_i64),
                ("k4_passes", c_i32), ("host_waits", c_i32)]


# Every symbol declared in include/pdp_hip.h: (name, restype, argtypes).
SIGNATURES = [
    ("pdp_abi_version", c_i32, []),
    ("pdp_last_error", ctypes.c_char_p, []),
    ("pdp_ctx_create", c_vp, [c_i32]),
    ("pdp_ctx_destroy", None, [c_vp]),
    ("pdp_ctx_set_debug", c_i32, [c_vp, c_i32]),
    ("pdp_workspace_size", c_i32, [ctypes.POINTER(Columns), ctypes.POINTER(BoundParams),
                                   ctypes.POINTER(ctypes.c_size_t)]),
    ("pdp_bound_accumulate", c_i32, [c_vp, ctypes.POINTER(Columns), ctypes.POINTER(BoundParams),
                                     ctypes.POINTER(Accumulators), c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_bound_accumulate_partials", c_i32, [c_vp, ctypes.POINTER(Columns), ctypes.POINTER(BoundParams),
                                              ctypes.POINTER(Partials), c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_finalize_partials", c_i32, [c_vp, ctypes.POINTER(Partials), c_i64, ctypes.POINTER(BoundParams),
                                      ctypes.POINTER(Accumulators), c_vp]),
    ("pdp_sweep_workspace_size", c_i32, [ctypes.POINTER(Columns), ctypes.POINTER(ctypes.c_size_t)]),
    ("pdp_bound_accumulate_sweep", c_i32, [c_vp, ctypes.POINTER(Columns), ctypes.POINTER(BoundParams), c_i32,
                                           ctypes.POINTER(Accumulators), c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_release", c_i32, [c_vp, ctypes.POINTER(Accumulators), c_i64, c_i64, ctypes.POINTER(ReleaseParams),
                            ctypes.POINTER(Outputs), c_vp]),
    ("pdp_prepare_release", c_i32, [c_vp, ctypes.POINTER(ReleaseParams)]),
    ("pdp_metric_fields", c_i32, [c_i32, ctypes.POINTER(c_i32)]),
    ("pdp_gaussian_sigma", c_f64, [c_f64, c_f64, c_f64]),
    ("pdp_truncated_geometric_table", c_i32, [c_f64, c_f64, c_i64, ctypes.POINTER(c_f64), c_i64,
                                              ctypes.POINTER(c_i64)]),
    ("pdp_selection_threshold", c_i32, [c_i32, c_f64, c_f64, c_i64, ctypes.POINTER(c_f64),
                                        ctypes.POINTER(c_f64)]),
    ("pdp_analysis_workspace_size", c_i32, [c_i64, c_i64, c_i64, ctypes.POINTER(AnalysisConfig), c_i32,
                                            ctypes.POINTER(ctypes.c_size_t)]),
    ("pdp_utility_analysis", c_i32, [c_vp, ctypes.POINTER(Columns), c_i64, c_i32, ctypes.POINTER(AnalysisConfig),
                                     c_i32, ctypes.POINTER(AnalysisOutputs), c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_utility_aggregate", c_i32, [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(AggregateParams), c_vp, c_vp,
                                      c_vp]),
    ("pdp_utility_analysis_preaggregated", c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i32,
                                                   ctypes.POINTER(AnalysisConfig), c_i32,
                                                   ctypes.POINTER(AnalysisOutputs), c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_preaggregate", c_i32, [c_vp, ctypes.POINTER(Columns), c_i64, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64),
                                 c_vp, ctypes.c_size_t, c_vp]),
    ("pdp_shard_workspace_size", c_i32, [c_i64, c_i32, ctypes.POINTER(ctypes.c_size_t)]),
    ("pdp_shard_rows", c_i32, [c_vp, ctypes.POINTER(Columns), c_i32, c_vp, c_vp, c_vp, ctypes.POINTER(c_i64), c_vp,
                               ctypes.c_size_t, c_vp]),
    ("pdp_generate_synthetic", c_i32, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_f64, c_i32, c_f64,
                                       c_f64, c_u64, c_vp]),
    ("pdp_stream_copy", c_i32, [c_vp, c_vp, c_i64, c_vp]),
    ("pdp_fp64_probe", c_i32, [ctypes.POINTER(c_f64), c_vp]),
    ("pdp_get_stats", c_i32, [c_vp, ctypes.POINTER(Stats)]),
    ("pdp_get_status", c_i32, [c_vp, ctypes.POINTER(c_i32)]),
    ("pdp_profile_enable", c_i32, [c_vp, c_i32]),
    ("pdp_profile_read", c_i32, [c_vp, ctypes.POINTER(c_f64), ctypes.POINTER(c_i64), c_i32]),
]

STAGES = ["histogram", "onesweep_first", "onesweep_rest", "buckets", "generic", "release", "enforced",
          "tile_counts", "analysis_pairs", "analysis_metrics", "filter", "survivor_sort", "pair_pass", "reduce",
          "analysis_sort", "analysis_aggregate", "analysis_select", "survivor_group"]

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpdp_hip.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"{LIB_PATH} is missing: build it with `python -m pipelinedp_amd.build` "
                              "(hipcc --offload-arch=gfx950); there is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(handle, name, None)
            if fn is None and os.environ.get("PDP_HIP_LIB"):
                continue  # an experiment build of an older ABI
            if fn is None:
                raise NativeError(f"{LIB_PATH} does not export {name}: rebuild it")
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != PDP_OK:
        msg = lib().pdp_last_error()
        raise NativeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def metric_fields(mask: int):
    buf = (c_i32 * 5)()
    n = lib().pdp_metric_fields(mask, buf)
    return [FIELD_NAMES[buf[i]] for i in range(n)]


def gaussian_sigma(eps: float, delta: float, l2: float) -> float:
    return lib().pdp_gaussian_sigma(eps, delta, l2)


def truncated_geometric_table(eps: float, delta: float, k: int):
    n = c_i64(0)
    check(lib().pdp_truncated_geometric_table(eps, delta, k, None, 0, ctypes.byref(n)), "table size")
    buf = (c_f64 * n.value)()
    n2 = c_i64(0)
    check(lib().pdp_truncated_geometric_table(eps, delta, k, buf, n.value, ctypes.byref(n2)), "table")
    return list(buf)


def selection_threshold(selection: int, eps: float, delta: float, k: int):
    thr, scale = c_f64(0), c_f64(0)
    check(lib().pdp_selection_threshold(selection, eps, delta, k, ctypes.byref(thr), ctypes.byref(scale)),
          "selection threshold")
    return thr.value, scale.value
