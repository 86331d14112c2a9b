/*
 * pdp_hip.h — C ABI of libpdp_hip.so, the MI355X (gfx950) implementation of
 * PipelineDP's DPEngine.aggregate hot path.
 *
 * Reference interfaces replaced (paths under /root/reference):
 *   pdp_bound_accumulate   <- SamplingCrossAndPerPartitionContributionBounder
 *                             .bound_contributions (pipeline_dp/contribution_bounders.py:66-105)
 *                             + CompoundCombiner.create_accumulator/merge_accumulators
 *                             (pipeline_dp/combiners.py:558-573)
 *                             + LocalBackend.combine_accumulators_per_key
 *                             (pipeline_dp/pipeline_backend.py:528-538)
 *                             + the contribution_bounds_already_enforced branch
 *                             (pipeline_dp/dp_engine.py:139-150)
 *                             + _drop_not_public_partitions / _add_empty_public_partitions
 *                             (pipeline_dp/dp_engine.py:283-310): pk < 0 rows are dropped,
 *                             every partition in [0, num_partitions) gets an accumulator.
 *   pdp_release            <- DPEngine._select_private_partitions_internal
 *                             (pipeline_dp/dp_engine.py:312-362) + partition_selection.py:19-33
 *                             + CompoundCombiner.compute_metrics (combiners.py:575-597)
 *                             -> dp_computations.compute_dp_count/sum/mean/var
 *                             (pipeline_dp/dp_computations.py:255-459)
 *   pdp_gaussian_sigma     <- dp_computations.compute_sigma (dp_computations.py:98-108; PyDP)
 *   pdp_truncated_geometric_table / pdp_selection_threshold
 *                          <- PyDP partition-selection strategies (partition_selection.py:24-33)
 *   pdp_metric_fields      <- MetricsTuple field order (combiners.py:575-597, 652-720)
 *
 * Conventions: every pointer in the column/accumulator/output structs is a
 * DEVICE pointer owned by the caller; `stream` is a hipStream_t (NULL = null
 * stream).  The library allocates nothing on the hot path except a rarely
 * used fallback (overflowing privacy-id buckets).  Functions return 0 on
 * success and a negative PDP_ERR_* code on failure; pdp_last_error() gives a
 * thread-local message.  No exceptions cross the ABI.
 */
#ifndef PDP_HIP_H_
#define PDP_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDP_ABI_VERSION 4

enum {
  PDP_OK = 0,
  PDP_ERR_INVALID_ARG = -1,
  PDP_ERR_HIP = -2,
  PDP_ERR_WORKSPACE = -3,
  PDP_ERR_OUT_OF_RANGE = -4,
  PDP_ERR_INTERNAL = -5,
  PDP_ERR_NEEDS_SYNC = -6, /* pdp_get_status: an asynchronous call needed the generic path; redo it without
                              PDP_BOUND_ASYNC */
};

/* pdp_bound_params.flags */
enum {
  /* No host synchronisation at all: the call only enqueues work on `stream` (it can be captured in a
   * hipGraph).  Errors and statistics are read with pdp_get_status after the stream has drained.  An
   * input that needs the generic path (privacy ids with more rows than the wave kernels hold) is not
   * completed: pdp_get_status returns PDP_ERR_NEEDS_SYNC. */
  PDP_BOUND_ASYNC = 1,
};

/* Metric bitmask (aggregate_params.py:54-65). */
enum {
  PDP_METRIC_COUNT = 1,
  PDP_METRIC_SUM = 2,
  PDP_METRIC_MEAN = 4,
  PDP_METRIC_VARIANCE = 8,
  PDP_METRIC_PRIVACY_ID_COUNT = 16,
};

/* Output field ids, in MetricsTuple naming. */
enum {
  PDP_FIELD_VARIANCE = 0,
  PDP_FIELD_MEAN = 1,
  PDP_FIELD_COUNT = 2,
  PDP_FIELD_SUM = 3,
  PDP_FIELD_PRIVACY_ID_COUNT = 4,
};

enum { PDP_NOISE_LAPLACE = 0, PDP_NOISE_GAUSSIAN = 1 }; /* aggregate_params.py:68-76 */

enum { /* aggregate_params.py:92-95; NONE = public partitions */
  PDP_SELECTION_NONE = 0,
  PDP_SELECTION_TRUNCATED_GEOMETRIC = 1,
  PDP_SELECTION_LAPLACE_THRESHOLDING = 2,
  PDP_SELECTION_GAUSSIAN_THRESHOLDING = 3,
};

/* Budget slots (one MechanismSpec each, combiners.py:652-720, dp_engine.py:328). */
enum {
  PDP_MECH_COUNT = 0,
  PDP_MECH_SUM = 1,
  PDP_MECH_MEAN = 2,
  PDP_MECH_VARIANCE = 3,
  PDP_MECH_PRIVACY_ID_COUNT = 4,
  PDP_MECH_SELECTION = 5,
  PDP_NUM_MECH = 6,
};

/* Dictionary-encoded input columns (device).  pid in [0, num_privacy_ids),
 * pk in [0, num_partitions); pk < 0 marks a row of a non-public partition
 * (dropped).  value may be NULL for COUNT / PRIVACY_ID_COUNT only; pid may be
 * NULL when bounds_already_enforced. */
typedef struct pdp_columns {
  const int64_t* pid;
  const int64_t* pk;
  const double* value;
  int64_t num_rows;
  int64_t num_privacy_ids;
  int64_t num_partitions;
} pdp_columns;

/* AggregateParams subset that drives bounding (aggregate_params.py:98-296). */
typedef struct pdp_bound_params {
  int32_t metrics;                          /* PDP_METRIC_* mask */
  int32_t bounds_already_enforced;          /* contribution_bounds_already_enforced */
  int64_t max_partitions_contributed;       /* L0 */
  int64_t max_contributions_per_partition;  /* L_inf */
  int32_t has_value_bounds;                 /* min_value/max_value set */
  int32_t has_partition_bounds;             /* min/max_sum_per_partition set */
  double min_value, max_value;
  double min_sum_per_partition, max_sum_per_partition;
  uint64_t sampling_seed;                   /* keys the uniform sampling permutations */
  int32_t debug_force_fallback;             /* testing: route every bucket through the
                                               generic sorted-stream path */
  int32_t reserved;                         /* testing: debug flags (pdp_ctx_set_debug); 0 */
  int32_t flags;                            /* PDP_BOUND_* */
  int32_t reserved2;                        /* testing: second debug-flag word; 0 */
  /* ABI 3: the columns' privacy ids are (id - pid_base): the sampling hashes pid_base + pid (DESIGN.md
   * 4), so a rank can pass its contiguous range of global ids rebased to [0, num_privacy_ids) -- which
   * sizes the L0 pre-filter by its own ids -- and get the result of the global ids bit for bit.  0
   * otherwise. */
  int64_t pid_base;
} pdp_bound_params;

/* Dense per-partition accumulators [num_partitions] (device).  row_count is the
 * CompoundCombiner row count (= privacy-id count; rows when bounds already
 * enforced).  x = nsum (MEAN/VARIANCE: sum of clip(v)-middle) or sum (SUM only:
 * sum of clip(v), or of per-(pid,pk) clipped sums); y = nsumsq (VARIANCE). */
typedef struct pdp_accumulators {
  int64_t* row_count;
  int64_t* count;
  double* x;
  double* y;
} pdp_accumulators;

typedef struct pdp_release_params {
  int32_t metrics;
  int32_t noise_kind;
  int32_t selection;
  int32_t add_noise;                 /* 0 = noise-free (explain / testing) */
  int64_t max_partitions_contributed;
  int64_t max_contributions_per_partition;
  int32_t has_value_bounds;
  int32_t has_partition_bounds;
  double min_value, max_value;
  double min_sum_per_partition, max_sum_per_partition;
  double eps[PDP_NUM_MECH];
  double delta[PDP_NUM_MECH];
  int64_t max_rows_per_privacy_id;   /* dp_engine.py:163-169 */
  uint64_t noise_seed;
} pdp_release_params;

typedef struct pdp_outputs {
  uint8_t* keep;    /* [num_partitions] 1 = partition released */
  double* metrics;  /* [num_fields][num_partitions], order from pdp_metric_fields */
} pdp_outputs;

typedef struct pdp_ctx pdp_ctx;

int pdp_abi_version(void);
const char* pdp_last_error(void);

pdp_ctx* pdp_ctx_create(int device);
void pdp_ctx_destroy(pdp_ctx* ctx);

/* Testing only: flags that select an alternative form of a stage with
 * identical results (the parity tests A/B them), OR-ed into every later call
 * on ctx; the same bits as pdp_bound_params.reserved.  0 (the default) is the
 * shipped path.  Timing-ablation flags (results invalid) are refused unless
 * the library was built with -DPDP_DEBUG_BUILD. */
int pdp_ctx_set_debug(pdp_ctx* ctx, int32_t flags);

/* Bytes of device workspace pdp_bound_accumulate needs for these columns. */
int pdp_workspace_size(const pdp_columns* cols, const pdp_bound_params* bp, size_t* bytes);

/* Rows -> dense per-partition accumulators (zeroed first).  For L0 <= 8 with
 * enough rows per privacy id the library first drops, after one bucket
 * radix pass, the rows of partitions their privacy id cannot keep (the L0
 * pre-filter); the result is identical either way, and
 * pdp_get_stats reports the surviving rows in filter_rows.
 * Stream-ordered: the kernels read every intermediate count from device
 * memory, so the call waits for the stream once, at the end, to return the
 * status (none with PDP_BOUND_ASYNC).  An input that needs the generic path
 * takes one more wait after the bounding kernels (the context then starts
 * that way until an input no longer needs it). */
int pdp_bound_accumulate(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bp,
                         const pdp_accumulators* acc, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Multi-GPU form of pdp_bound_accumulate: the per-partition sums are exported
 * in K4's 64-bit fixed point instead of as doubles, so that the partials of
 * several ranks add up exactly (an int64 SUM reduce-scatter) before ONE
 * conversion on the owning rank -- the combine_accumulators_per_key merge
 * (pipeline_dp/pipeline_backend.py:528-538) across GPUs, with a result that
 * equals one GPU's bit for bit.  Per partition p:
 *   x = (x_hi[p] + (x_lo[p] >> 32)) * 2^(32-F) + (x_lo[p] mod 2^32) * 2^-F
 * (F from the contribution bounds, pdp_finalize_partials applies it); x_lo is
 * in [0, 2^32) per rank.  nan[p] counts NaN terms: + 1 per x NaN, + 2^32 per
 * y NaN.  Arrays are [num_partitions] int64; row_count / count / x_* / y_* /
 * nan as the metrics need them (x: SUM / MEAN / VARIANCE, y: VARIANCE, nan:
 * with x).  Any row count (with >= 2^32 rows: L_inf < 131072). */
typedef struct pdp_partials {
  int64_t* row_count;
  int64_t* count;
  int64_t* x_hi;
  int64_t* x_lo;
  int64_t* y_hi;
  int64_t* y_lo;
  int64_t* nan;
} pdp_partials;

int pdp_bound_accumulate_partials(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bp,
                                  const pdp_partials* parts, void* workspace, size_t workspace_bytes,
                                  void* stream);

/* Summed partials of num_partitions partitions -> accumulators for
 * pdp_release (bp: the bounds pdp_bound_accumulate_partials ran with).
 * acc->row_count / count may alias parts->row_count / count (then no copy). */
int pdp_finalize_partials(pdp_ctx* ctx, const pdp_partials* parts, int64_t num_partitions,
                          const pdp_bound_params* bp, const pdp_accumulators* acc, void* stream);

/* Bounding sweep (utility analysis over many bounding configurations, the
 * per-configuration DPEngine runs of analysis/utility_analysis_engine.py:
 * 88-173 with MultiParameterConfiguration, analysis/data_structures.py):
 * rows are sorted by privacy id ONCE, then bounded and accumulated per
 * configuration into accs[c].  bps[c] may differ in L0, L_inf, value / sum
 * bounds, metrics and sampling seed; accs[c] follows pdp_bound_accumulate.
 * Result c equals pdp_bound_accumulate(cols, &bps[c], &accs[c]).
 * contribution_bounds_already_enforced is rejected.  Workspace:
 * pdp_sweep_workspace_size (one more record buffer than a single run). */
int pdp_sweep_workspace_size(const pdp_columns* cols, size_t* bytes);
int pdp_bound_accumulate_sweep(pdp_ctx* ctx, const pdp_columns* cols, const pdp_bound_params* bps,
                               int32_t num_configs, const pdp_accumulators* accs, void* workspace,
                               size_t workspace_bytes, void* stream);

/* Accumulators of partitions [pk_offset, pk_offset + num_partitions) ->
 * selection + noisy metrics.  Philox counters use the global partition id
 * (pk_offset + i), so the result does not depend on how partitions are
 * distributed over ranks. */
int pdp_release(pdp_ctx* ctx, const pdp_accumulators* acc, int64_t num_partitions, int64_t pk_offset,
                const pdp_release_params* rp, const pdp_outputs* out, void* stream);

/* Builds (synchronously) the device-side data pdp_release needs for rp -- the truncated-geometric keep
 * table of (eps, delta, max_partitions_contributed) -- in the context's cache, so that a later
 * pdp_release on a capturing stream (hipGraph) enqueues kernels only.  Cached tables are immutable and
 * live until pdp_ctx_destroy: a captured pdp_release stays valid whatever later calls release.
 * pdp_release under capture without a prepared table returns PDP_ERR_NEEDS_SYNC (ABI 4). */
int pdp_prepare_release(pdp_ctx* ctx, const pdp_release_params* rp);

/* Field order of MetricsTuple for a metric mask; returns the count. */
int pdp_metric_fields(int32_t metrics, int32_t* fields_out /* >= 5 */);

/* Host-side calibration (no GPU needed). */
double pdp_gaussian_sigma(double eps, double delta, double l2_sensitivity);
int pdp_truncated_geometric_table(double eps, double delta, int64_t max_partitions, double* out,
                                  int64_t capacity, int64_t* length);
int pdp_selection_threshold(int32_t selection, double eps, double delta, int64_t max_partitions,
                            double* threshold, double* scale);

/* Utility analysis (BASELINE.json configs[4]): the per-partition metrics of
 * the reference's UtilityAnalysisEngine.analyze
 * (analysis/utility_analysis_engine.py:53-173) for many bounding
 * configurations in one launch sequence:
 *   rows -> per (privacy id, partition) (count, sum, n_partitions)
 *     (SamplingL0LinfContributionBounder, analysis/contribution_bounders.py:38-75;
 *      analysis/pre_aggregation.py:preaggregate)
 *   -> per configuration c and partition p, for each of SUM, COUNT,
 *      PRIVACY_ID_COUNT in mask order SUM, COUNT, PRIVACY_ID_COUNT:
 *      (sum, per_partition_error_min, per_partition_error_max,
 *       expected_cross_partition_error, var_cross_partition_error)
 *      (SumCombiner / CountCombiner / PrivacyIdCountCombiner,
 *       analysis/combiners.py:228-310; std = sqrt(var))
 *   -> with private selection: the keep probability
 *      (PartitionSelectionCombiner + Poisson binomial, analysis/combiners.py:
 *       99-225, analysis/poisson_binomial.py:39-83).
 * metrics[C][nb][5][P] and prob_keep[C][P] are device arrays; nb = number of
 * metrics in the mask.  Every configuration uses private selection
 * (selection != NONE: partitions present in the data) or none does (public
 * partitions: pk in [0, P) are the public partitions; rows with pk < 0 are
 * dropped, every partition gets the empty accumulator's pseudo-contribution
 * (0, 0, 0) as in analysis/combiners.py:337-342).  Partition sampling:
 * partitions [num_sampled_partitions, P) count toward n_partitions but are
 * not analysed (ValueSampler, pipeline_dp/sampling_utils.py:38-51, decided on
 * the host).  std_noise is host arithmetic (dp_computations.py:462-481). */
typedef struct pdp_analysis_config {
  int64_t max_partitions_contributed;       /* L0: keep probability q = min(1, L0 / n_partitions) */
  int64_t max_contributions_per_partition;  /* COUNT clip [0, L_inf] */
  double min_sum_per_partition, max_sum_per_partition;  /* SUM clip */
  int32_t selection;                        /* PDP_SELECTION_*; NONE = public partitions */
  int32_t reserved;
  double selection_eps, selection_delta;    /* the GENERIC mechanism's budget */
} pdp_analysis_config;

typedef struct pdp_analysis_outputs {
  double* metrics;         /* [num_configs][nb][5][num_partitions] */
  double* prob_keep;       /* [num_configs][num_partitions]; private selection only */
  int64_t* privacy_ids;    /* [num_partitions] privacy ids with data in the partition (optional) */
} pdp_analysis_outputs;

int pdp_analysis_workspace_size(int64_t num_rows, int64_t num_privacy_ids, int64_t num_partitions,
                                const pdp_analysis_config* cfgs, int32_t num_configs, size_t* bytes);
int pdp_utility_analysis(pdp_ctx* ctx, const pdp_columns* cols, int64_t num_sampled_partitions, int32_t metrics,
                         const pdp_analysis_config* cfgs, int32_t num_configs, const pdp_analysis_outputs* out,
                         void* workspace, size_t workspace_bytes, void* stream);
/* Pre-aggregated input (options.pre_aggregated_data, NoOpContributionBounder,
 * analysis/contribution_bounders.py:78-88): one row per (privacy id,
 * partition) with (count, sum, n_partitions).  Workspace:
 * pdp_analysis_workspace_size(num_pairs, num_pairs, ...). */
int pdp_utility_analysis_preaggregated(pdp_ctx* ctx, const int64_t* pk, const int64_t* count, const double* sum,
                                       const int64_t* n_partitions, int64_t num_pairs, int64_t num_partitions,
                                       int32_t metrics, const pdp_analysis_config* cfgs, int32_t num_configs,
                                       const pdp_analysis_outputs* out, void* workspace, size_t workspace_bytes,
                                       void* stream);

/* Cross-partition aggregation of the utility analysis: the device side of
 * analysis.perform_utility_analysis (analysis/utility_analysis.py:27-161),
 * i.e. AggregateErrorMetricsCompoundCombiner over every partition of the
 * per-partition result (analysis/combiners.py:385-723).  Inputs are the
 * outputs of pdp_utility_analysis (device pointers): metrics
 * [C][nb][5][P], prob_keep [C][P] (NULL: public partitions, p = 1) and
 * privacy_ids [P] (NULL: every partition is in the result; else only those
 * with privacy ids -- private selection).  Outputs (device):
 *   out_errors [C][nb][PDP_AGG_NUM_FIELDS + 2 Q]: per (configuration,
 *     metric) the sums over partitions of the AggregateErrorMetricsAccumulator
 *     fields (:385-416), then error_quantiles[Q], rel_error_quantiles[Q];
 *     the caller divides as compute_metrics does (:590-640);
 *   out_selection [C][3] (private only): partitions, sum p, sum p (1 - p)
 *     (PrivatePartitionSelectionAggregateErrorMetricsCombiner, :677-715).
 * As in the reference (create_accumulator, :470-480) the metric rows of
 * every configuration weight partitions by configuration 0's keep
 * probability.  Laplace error quantiles are the exact quantiles of
 * Laplace(std_noise / sqrt 2) + N(0, std_cross^2), where the reference draws
 * 10^3 Monte-Carlo samples (analysis/probability_computations.py:20-36).
 * Sums are reduced in a fixed order (run-to-run identical).  Synchronises
 * the stream before returning. */
enum {
  PDP_AGG_NUM_PARTITIONS = 0,
  PDP_AGG_KEPT_PARTITIONS_EXPECTED = 1,
  PDP_AGG_TOTAL_AGGREGATE = 2,
  PDP_AGG_DATA_DROPPED_L0 = 3,
  PDP_AGG_DATA_DROPPED_LINF = 4,
  PDP_AGG_DATA_DROPPED_PARTITION_SELECTION = 5,
  PDP_AGG_ERROR_L0_EXPECTED = 6,
  PDP_AGG_ERROR_LINF_EXPECTED = 7,
  PDP_AGG_ERROR_LINF_MIN_EXPECTED = 8,
  PDP_AGG_ERROR_LINF_MAX_EXPECTED = 9,
  PDP_AGG_ERROR_L0_VARIANCE = 10,
  PDP_AGG_ERROR_VARIANCE = 11,
  PDP_AGG_REL_ERROR_L0_EXPECTED = 12,
  PDP_AGG_REL_ERROR_LINF_EXPECTED = 13,
  PDP_AGG_REL_ERROR_LINF_MIN_EXPECTED = 14,
  PDP_AGG_REL_ERROR_LINF_MAX_EXPECTED = 15,
  PDP_AGG_REL_ERROR_L0_VARIANCE = 16,
  PDP_AGG_REL_ERROR_VARIANCE = 17,
  PDP_AGG_ERROR_EXPECTED_W_DROPPED = 18,
  PDP_AGG_REL_ERROR_EXPECTED_W_DROPPED = 19,
  PDP_AGG_NUM_FIELDS = 20,
  PDP_AGG_MAX_QUANTILES = 8,
};
typedef struct pdp_aggregate_params {
  int32_t num_configs;        /* C */
  int32_t metrics;            /* the analysis' PDP_METRIC_* mask: blocks SUM, COUNT, PRIVACY_ID_COUNT (those set) */
  int32_t num_quantiles;      /* Q <= PDP_AGG_MAX_QUANTILES */
  int32_t reserved;
  const double* quantiles;    /* [Q] host: error quantiles as perform_utility_analysis takes them (0.1, 0.5, ...) */
  const double* std_noise;    /* [C][nb] host: SumMetrics.std_noise of each (configuration, metric) */
  const int32_t* noise_kind;  /* [C] host: PDP_NOISE_* */
} pdp_aggregate_params;
int pdp_utility_aggregate(pdp_ctx* ctx, const double* metrics, const double* prob_keep, const int64_t* privacy_ids,
                          int64_t num_partitions, const pdp_aggregate_params* params, double* out_errors,
                          double* out_selection, void* stream);

/* analysis/pre_aggregation.py:preaggregate: one (pk, count, sum, n_partitions)
 * per (privacy id, partition) of a sampled partition (pk < num_sampled), in
 * (pk, privacy id) order; out_* hold num_rows entries, *num_pairs (host) is
 * set.  Workspace: pdp_analysis_workspace_size with one configuration of
 * selection NONE. */
int pdp_preaggregate(pdp_ctx* ctx, const pdp_columns* cols, int64_t num_sampled_partitions, int64_t* out_pk,
                     int64_t* out_count, double* out_sum, int64_t* out_n_partitions, int64_t* num_pairs,
                     void* workspace, size_t workspace_bytes, void* stream);

/* Multi-GPU ingestion of rows that are not sharded by privacy id: the device
 * side of the reference's group-by-pid shuffles (BeamBackend / SparkRDDBackend
 * / LocalBackend.group_by_key, pipeline_dp/pipeline_backend.py:261, 401,
 * 476-485).  Stable counting sort of the rows by destination rank
 * shard_of(pid) = splitmix64(pid ^ 0x9E3779B97F4A7C15) % world_size into
 * out_pid / out_pk / out_value (device, num_rows each; rank 0's rows first,
 * input order kept within a rank); rows_per_rank[world_size] is HOST memory.
 * The caller then moves the runs with an RCCL all-to-all.  value / out_value
 * may both be NULL.  world_size <= 64. */
int pdp_shard_workspace_size(int64_t num_rows, int32_t world_size, size_t* bytes);
int pdp_shard_rows(pdp_ctx* ctx, const pdp_columns* cols, int32_t world_size, int64_t* out_pid, int64_t* out_pk,
                   double* out_value, int64_t* rows_per_rank, void* workspace, size_t workspace_bytes,
                   void* stream);

/* Synthetic workload (bench / tests): rows [row_offset, row_offset+n) of the
 * generator specified in oracle/pdp_oracle.py:synth_rows. */
int pdp_generate_synthetic(int64_t* pid, int64_t* pk, double* value, int64_t n, int64_t row_offset,
                           int64_t num_privacy_ids, int64_t num_partitions, double zipf_s,
                           int32_t value_kind, double value_lo, double value_hi, uint64_t seed,
                           void* stream);

/* Device-to-device copy of `bytes` (a multiple of 16) with a 16-B-per-lane
 * streaming kernel: bench.py's achievable-HBM ceiling (no reference
 * counterpart; measurement only). */
int pdp_stream_copy(const void* src, void* dst, int64_t bytes, void* stream);

/* fp64 FMA-chain probe: the device's achievable fp64 vector rate in TFLOP/s
 * (2 FLOP per FMA), timed with hipEvents on `stream` (synchronises).
 * Measurement only: the denominator of the utility analysis' roofline. */
int pdp_fp64_probe(double* tflops, void* stream);

/* Statistics of the last pdp_bound_accumulate on this ctx (host values). */
typedef struct pdp_stats {
  int64_t kept_rows_in;        /* rows after dropping non-public partitions */
  int64_t fallback_rows;       /* rows routed through the generic path */
  int64_t fallback_ranges;
  int32_t sort_passes;
  int32_t bucket_low_bits;
  int64_t sweep_cycles[4];     /* radix passes, debug stamps only: load, rank, look-back/bases, scatter */
  int64_t sweep_tiles;
  int64_t filter_rows;         /* rows that survived the L0 pre-filter (0: the filter did not run) */
  int64_t k4_slots;            /* K4: pair slots written by K2 (+ generic-path groups); 0: K4 off */
  int64_t k4_pairs;            /* K4: (pid, pk) pair records reduced */
  int32_t k4_passes;           /* K4: radix passes on the partition block */
  int32_t host_waits;          /* times the call waited for its stream (1: the final status copy;
                                  0 with PDP_BOUND_ASYNC; more when the generic path ran) */
} pdp_stats;
int pdp_get_stats(pdp_ctx* ctx, pdp_stats* out);

/* Status of the last pdp_bound_accumulate(_partials) on ctx, for PDP_BOUND_ASYNC calls: call after the
 * stream they were enqueued on has drained (reads the context's device status block).  *call_status = 0,
 * or the PDP_ERR_* code the call would have returned synchronously, or PDP_ERR_NEEDS_SYNC. */
int pdp_get_status(pdp_ctx* ctx, int32_t* call_status);

/* Per-stage device timing with hipEvents recorded on the launch stream (for
 * bench.py's roofline).  Stages: */
enum {
  PDP_STAGE_HISTOGRAM = 0,       /* K0 */
  PDP_STAGE_ONESWEEP_FIRST = 1,  /* K1 pass 0 (reads the int64/int64/f64 columns) */
  PDP_STAGE_ONESWEEP_REST = 2,   /* K1 passes >= 1 */
  PDP_STAGE_BUCKETS = 3,         /* K2 */
  PDP_STAGE_GENERIC = 4,         /* KF (fallback) */
  PDP_STAGE_RELEASE = 5,         /* K5/K6 */
  PDP_STAGE_ENFORCED = 6,        /* bounds already enforced accumulate */
  PDP_STAGE_TILE_COUNTS = 7,     /* K1u per-tile digit counts (passes >= 1) + tile-offset scans */
  PDP_STAGE_ANALYSIS_PAIRS = 8,  /* utility analysis: (pk, pid) sort + per-pair pre-aggregation */
  PDP_STAGE_ANALYSIS_METRICS = 9, /* utility analysis: per-configuration partition metrics + selection */
  PDP_STAGE_FILTER = 10,        /* K1f L0 pre-filter (one workgroup per privacy-id bucket) */
  PDP_STAGE_SURVIVOR_SORT = 11, /* radix sort of the pre-filter's survivors */
  PDP_STAGE_PAIR_PASS = 12,     /* K4 pair-record radix passes by partition block */
  PDP_STAGE_REDUCE = 13,        /* K4 per-partition fixed-point reduction (+ shared-block zero / finalize) */
  PDP_STAGE_ANALYSIS_SORT = 14, /* utility analysis: the (pk, pid) radix sort inside ANALYSIS_PAIRS */
  PDP_STAGE_ANALYSIS_AGGREGATE = 15, /* utility analysis: cross-partition aggregate error metrics */
  PDP_STAGE_ANALYSIS_SELECT = 16, /* utility analysis: Poisson-binomial keep probability (inside ANALYSIS_METRICS) */
  PDP_STAGE_SURVIVOR_GROUP = 17, /* ABI 4: the survivors' last grouping step in LDS (k_group) */
  PDP_NUM_STAGES = 18,
};
int pdp_profile_enable(pdp_ctx* ctx, int enable);
/* Waits for recorded events; adds into ms_out/launches_out[PDP_NUM_STAGES]
 * the totals since the last reset. */
int pdp_profile_read(pdp_ctx* ctx, double* ms_out, int64_t* launches_out, int reset);

#ifdef __cplusplus
}
#endif
#endif /* PDP_HIP_H_ */
