/*
 * pmx.h — C ABI of the MI355X-native ICP inner loop (the drop-in boundary).
 *
 * One pmx_ctx per ICP object (and per GPU rank).  It owns a HIP stream, the
 * device-resident reference / reading clouds, the k x N match and weight
 * arrays, and (optionally) an RCCL communicator.  Not thread-safe — exactly
 * like the reference's ICP object (pointmatcher/PointMatcher.h:652-764 keeps
 * mutable per-object state).  Plain pointers and sizes only: no torch/HIP
 * types cross this boundary.
 *
 * Each entry point replaces one reference interface (paths relative to the
 * libpointmatcher repository root):
 *
 *   pmx_set_reference   Matcher::init(filteredReference)
 *                         pointmatcher/PointMatcher.h:481, MatchersImpl.cpp:77-83
 *                         (+ the centred reference of ICP.cpp:291-302)
 *   pmx_set_reading     the once-per-compute reading copy + transformations.apply
 *                         (ICP.cpp:337-347)
 *   pmx_match           transformations.apply(stepReading, T_iter) fused with
 *                         Matcher::findClosests (ICP.cpp:381-387,
 *                         PointMatcher.h:484, MatchersImpl.cpp:85-101)
 *   pmx_outlier_*       OutlierFilter::compute and the chain product
 *                         (PointMatcher.h:504-512, OutlierFilter.cpp:63-103,
 *                          OutlierFiltersImpl.cpp:51-223)
 *   pmx_p2plane_system  ErrorElements + PointToPlane normal equations
 *                         (ErrorMinimizer.cpp:58-193, PointToPlane.cpp:171-243)
 *   pmx_p2point_system  ErrorElements + PointToPoint weighted moments
 *                         (PointToPoint.cpp:61-81)
 *   pmx_get_matches /   lazy host mirrors of Matches / OutlierWeights for
 *   pmx_get_weights       CPU modules and inspectors (PointMatcher.h:371-391)
 *
 * The 6x6 / 3x3 solves, the transform update and the convergence checks stay
 * on the host (PointToPlane.cpp:108-161, ICP.cpp:411-427).
 *
 * Errors: every call returns 0 or a negative PMX_E_* code; pmx_last_error()
 * gives the message.  The host shim maps codes to the reference exception
 * types (PointMatcher.h:83-100):
 *   PMX_E_NO_POINTS       -> ConvergenceError("ErrorMnimizer: no point to minimize")
 *   PMX_E_EMPTY_QUANTILE  -> ConvergenceError("no outlier to filter")
 *   PMX_E_BAD_PARAM       -> InvalidParameter
 *   PMX_E_TRANSFORMATION  -> TransformationError (device loop)
 *   PMX_E_CONVERGENCE     -> ConvergenceError (device loop checkers)
 *   PMX_E_HIP / PMX_E_RCCL / PMX_E_STATE -> std::runtime_error
 */
#ifndef PMX_H
#define PMX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pmx_ctx pmx_ctx;

enum { PMX_F32 = 0, PMX_F64 = 1 };

enum {
    PMX_OK = 0,
    PMX_E_NO_POINTS = -1,
    PMX_E_EMPTY_QUANTILE = -2,
    PMX_E_BAD_PARAM = -3,
    PMX_E_TRANSFORMATION = -4, /* device loop: T_iter not rigid */
    PMX_E_CONVERGENCE = -5,    /* device loop: a checker raised ConvergenceError */
    PMX_E_HIP = -10,
    PMX_E_RCCL = -11,
    PMX_E_STATE = -12,
    PMX_E_NO_DEVICE = -13
};

/* per-iteration statistics (ErrorElements, ErrorMinimizer.cpp:133-192;
 * ICP.cpp:432-436).  Counts are global over all ranks. */
typedef struct pmx_stats {
    int64_t kept;               /* ErrorElements columns P: dist != inf && w != 0 */
    int64_t nonzero_weights;    /* (w != 0).count()                 ErrorMinimizer.cpp:75 */
    int64_t rejected_matches;   /* nbRejectedMatches                ErrorMinimizer.cpp:191 */
    int64_t rejected_points;    /* nbRejectedPoints                 ErrorMinimizer.cpp:192 */
    double sum_w;               /* sum of kept weights (weightedPointUsedRatio * k * N) */
    double limit;               /* last quantile threshold (diagnostic, T value) */
    int64_t n_total;            /* k * N over all ranks */
    int64_t visited;            /* pair evaluations of the iteration's match (PointCountTouched) */
    int64_t fallback_queries;   /* grid tile search: queries re-run by the per-lane shell search
                                   (diagnostic; local to this rank) */
} pmx_stats;

/* ------------------------------------------------------------ context --- */
/* device: HIP device ordinal; dtype: PMX_F32 | PMX_F64. */
int pmx_ctx_create(int device, int dtype, pmx_ctx** out);
int pmx_ctx_destroy(pmx_ctx* ctx);
/* One developer option of the context (README "Options": switches between
 * measured alternatives and test hooks; the defaults are the tuned path).
 * Also read at pmx_ctx_create from PMX_OPTS="name=value,...".  No reference
 * counterpart: the reference's tuning is its YAML parameters, which the host
 * chain (include/pmx_icp.h) maps as they are.  PMX_E_BAD_PARAM for an
 * unknown name or a malformed value. */
int pmx_ctx_set_option(pmx_ctx* ctx, const char* name, const char* value);
const char* pmx_last_error(const pmx_ctx* ctx);
/* number of visible HIP devices (0 when no GPU / driver) */
int pmx_device_count(void);
/* library build string, e.g. "pmx 0.1 gfx950" */
const char* pmx_version(void);

/* ---------------------------------------------------------- multi-GPU --- */
/* RCCL unique id (128 bytes) generated on rank 0 and broadcast by the
 * launcher; every rank then calls pmx_comm_init.  With a communicator set,
 * pmx_set_reading takes the rank's shard of the reading cloud and every
 * exchange step (quantile histograms or window segments, VarTrimmed's
 * distances, the normal equations) is a collective on the context stream
 * over RCCL/xGMI — issued whenever a communicator exists, also at nranks 1.
 * (The reference is single-process: these have no reference counterpart;
 * the sharded results equal the single-process ones) */
int pmx_comm_unique_id(void* out128);
int pmx_comm_init(pmx_ctx* ctx, const void* uid128, int nranks, int rank);
/* Host-staged collectives: the caller's transport (MPI, gloo, a test
 * harness) instead of RCCL.  The library copies the device buffer to pinned
 * host memory, synchronises its stream, calls the callback and copies the
 * result back.  allreduce: in place over `count` elements of `type`
 * (PMX_COLL_*) with `op`; allgather: `bytes` from every rank into recv, in
 * rank order.  A callback returns 0 on success.  Exclusive with
 * pmx_comm_init; call before pmx_set_reading. */
enum { PMX_COLL_F64 = 0, PMX_COLL_U32 = 1, PMX_COLL_U64 = 2 };
enum { PMX_COLL_SUM = 0, PMX_COLL_MAX = 1 };
typedef int (*pmx_allreduce_fn)(void* user, void* buf, int64_t count, int type, int op);
typedef int (*pmx_allgather_fn)(void* user, const void* send, void* recv, int64_t bytes);
int pmx_comm_init_host(pmx_ctx* ctx, int nranks, int rank, pmx_allreduce_fn allreduce, pmx_allgather_fn allgather,
                       void* user);
/* kind: 0 none, 1 RCCL, 2 host callbacks */
int pmx_comm_size(const pmx_ctx* ctx, int* nranks, int* rank, int* kind);
/* Collectives this context has issued since creation (all-reduces,
 * all-gathers; 0 without a communicator).  A sharded iteration whose
 * quantile was resolved inside the exchanged key window issues two: the
 * window segments' all-gather and the normal equations' all-reduce. */
int pmx_comm_stats(const pmx_ctx* ctx, uint64_t* allreduces, uint64_t* allgathers);
/* How a sharded device loop synchronised (no reference counterpart: the
 * reference has one process, ICP.cpp:371-430).  verdict_syncs: iterations
 * whose window verdict the host read back (one stream synchronisation each;
 * only while the window is settling: after a miss, until two hits in a row);
 * async_iterations: iterations enqueued without reading it (zero host
 * synchronisations: a miss stalls the device loop); stalls: those misses,
 * each replayed at the next batch check (its radix passes and histogram
 * all-reduces, then the rest of the iteration). */
int pmx_comm_loop_stats(const pmx_ctx* ctx, uint64_t* verdict_syncs, uint64_t* async_iterations, uint64_t* stalls);

/* ------------------------------------------------------------ clouds --- */
/* feat: rows x M column-major (point-major) T array, rows = D + 1 with the
 * homogeneous row last (D = 2 or 3).  The caller passes the CENTRED
 * reference (ICP.cpp:299).  normals: D x M (point-major) or NULL.  Copied
 * to HBM once and kept resident across iterations and ICP calls. */
int pmx_set_reference(pmx_ctx* ctx, const void* feat, int rows, int64_t M, const void* normals);
/* The same with the centring done on the device: offset = the D reference
 * means (T values, ICP.cpp:291-292), subtracted from every point in T as
 * ICP.cpp:299 does (features.topRows(dim - 1) -= mean).  The caller then
 * needs no centred host copy of the reference. */
int pmx_set_reference_centred(pmx_ctx* ctx, const void* feat, int rows, int64_t M, const void* normals,
                              const void* offset);
/* pmx_set_reference_centred by the cloud's own mean: the mean in T, each
 * coordinate summed sequentially in point order and divided by M
 * (ICP.cpp:291-292), is computed on a host thread while the cloud and its
 * normals upload, written to mean_out (rows - 1 T values) and subtracted on
 * the device.  Replaces ICP::compute's host mean + centring (ICP.cpp:291-299)
 * followed by Matcher::init (:302). */
int pmx_set_reference_mean_centred(pmx_ctx* ctx, const void* feat, int rows, int64_t M, const void* normals,
                                   void* mean_out);
/* reading shard: rows x N.  T0 (rows x rows, row-major T) is applied once on
 * the device (T_refMean_dataIn, ICP.cpp:345-347). */
int pmx_set_reading(pmx_ctx* ctx, const void* feat, int rows, int64_t N, const void* T0);
/* KDTreeVarDistMatcher (MatchersImpl.cpp:106-150): a maximum search radius
 * per reading point (its maxDistField descriptor, N T values in the order of
 * pmx_set_reading's points; NULL clears).  While set, pmx_match uses these
 * radii (squared in T, as libnabo does) instead of its maxDist.  Cleared by
 * the next pmx_set_reading. */
int pmx_set_reading_radii(pmx_ctx* ctx, const void* radii);

/* ------------------------------------------------------------- match --- */
/* search structure, mirroring KDTreeMatcher's searchType
 * (MatchersImpl.h:85; libnabo: 0 brute force, 1/2 kd-tree): 0 = brute force
 * over all N*M pairs (LDS-tiled), 1 or 2 = uniform grid with exact shell
 * search (default).  Both return identical results (same arithmetic, same
 * lowest-index tie rule).  Takes effect at the next pmx_match. */
int pmx_set_search(pmx_ctx* ctx, int search_type);

/* T_iter: rows x rows row-major T.  knn >= 1 (KDTreeMatcher's bound,
 * MatchersImpl.h:83; k > 16 on the wave-per-query search, lists past 1024
 * entries in chunks of 1024; N * knn entries must fit in device memory),
 * maxDist: radius (inclusive, squared in T; +inf = none), epsilon: the
 * search is exact, so any epsilon >= 0 is satisfied.  visited (may be NULL)
 * receives the pair evaluations of this call when they are known at launch
 * (brute force: N*M; grid: 0 — the exact count is returned in
 * pmx_stats.visited by the next system call).  Results stay on the device. */
int pmx_match(pmx_ctx* ctx, const void* T_iter, int knn, double maxDist, double epsilon,
              uint64_t* visited);

/* ----------------------------------------------------- outlier filters --- */
/* chain_pos 0 writes the weights, chain_pos > 0 multiplies into them
 * (OutlierFilter.cpp:90-99).  pmx_outlier_default = empty chain
 * (w = dist != inf, OutlierFilter.cpp:70-85). */
int pmx_outlier_default(pmx_ctx* ctx);
int pmx_outlier_null(pmx_ctx* ctx, int chain_pos);
int pmx_outlier_maxdist(pmx_ctx* ctx, int chain_pos, double maxDist);
int pmx_outlier_mindist(pmx_ctx* ctx, int chain_pos, double minDist);
int pmx_outlier_mediandist(pmx_ctx* ctx, int chain_pos, double factor);
int pmx_outlier_trimmed(pmx_ctx* ctx, int chain_pos, double ratio);
int pmx_outlier_vartrimmed(pmx_ctx* ctx, int chain_pos, double minRatio, double maxRatio,
                           double lambda);
/* RobustOutlierFilter::robustFiltering (OutlierFiltersImpl.cpp:494-598):
 * real-valued weights w = robust(e^2), e^2 = dist / scale^2; at most one per
 * chain.  robust_fct: PMX_RF_*; tuning: k (after the berg substitution,
 * :419-433); approximation: the unsquared threshold (+inf = none); the
 * scale of this call (the filter's iteration state stays with the caller,
 * :500-531): PMX_RS_NONE (1), _MAD sqrt(median |d - median d|), _STD
 * sqrt(std), _BERG_FIRST 1.9 sqrt(quantile(0.5)), _BERG_NEXT 0.85 (s -
 * berg_target) + berg_target, _KEEP the previous call's scale at this chain
 * position; point2plane: distanceType point2plane (needs reference normals).
 * The scale stays on the device; pmx_robust_scale reads it back. */
enum { PMX_RF_CAUCHY = 0, PMX_RF_WELSCH = 1, PMX_RF_SC = 2, PMX_RF_GM = 3, PMX_RF_TUKEY = 4, PMX_RF_HUBER = 5,
       PMX_RF_L1 = 6, PMX_RF_STUDENT = 7 };
enum { PMX_RS_NONE = 0, PMX_RS_MAD = 1, PMX_RS_STD = 2, PMX_RS_BERG_FIRST = 3, PMX_RS_BERG_NEXT = 4,
       PMX_RS_KEEP = 5 };
int pmx_outlier_robust(pmx_ctx* ctx, int chain_pos, int robust_fct, double tuning, double approximation,
                       int scale_mode, double berg_target, int point2plane);
int pmx_robust_scale(pmx_ctx* ctx, int chain_pos, double* scale);

/* ---------------------------------------------------------- minimizers --- */
/* Point-to-plane normal equations for the step transform of the last
 * pmx_match: A (n x n row-major, n = 6 in 3D / 3 in 2D, full matrix, not
 * symmetrised: A = sum w F F^T) and b = -sum w F (d . n), accumulated in
 * double from T-precision products.  Synchronises the stream.  Returns
 * PMX_E_EMPTY_QUANTILE if a quantile filter of this iteration had no finite
 * distance, PMX_E_NO_POINTS if no weight is non-zero. */
int pmx_p2plane_system(pmx_ctx* ctx, double* A, double* b, pmx_stats* st);
/* Point-to-point: mean_p, mean_q (D each, T values), m = sum (qc w) pc^T
 * (D x D row-major, double sums of T products). */
int pmx_p2point_system(pmx_ctx* ctx, double* mean_p, double* mean_q, double* m, pmx_stats* st);

/* ---------------------------------------------------------- host mirrors --- */
/* dists: k x N T (point-major), ids: k x N int32 (this rank's shard) */
int pmx_get_matches(pmx_ctx* ctx, void* dists, int32_t* ids);
int pmx_get_weights(pmx_ctx* ctx, void* w);
/* The last VarTrimmedDist filter's partial sums (OutlierFiltersImpl.cpp:
 * 196-198: std::partial_sum in T over the sorted finite positive distances):
 * *count of them, copied into out when out != NULL and capacity suffices.
 * Diagnostic (the sequential rounding the device reproduces in parallel). */
int pmx_vartrim_partial_sums(pmx_ctx* ctx, void* out, int64_t capacity, int64_t* count);
/* shape of the current match arrays */
int pmx_get_shape(const pmx_ctx* ctx, int64_t* n_local, int* knn);
/* Grid level `level` of the reference (the spatial index Matcher::init
 * builds, MatchersImpl.cpp:77-83), once its build on any stream is complete
 * (built on demand if it was not): *count records; ids (count int32) the
 * original reference index of each record, points (count x 4 T) and normals
 * (count x 4 T, only with normals on the reference) the records the matcher
 * and the point-to-plane reduction read.  Any of the three may be NULL.
 * Diagnostic (tests check the records against the input clouds). */
int pmx_grid_level_records(pmx_ctx* ctx, int level, int64_t* count, int32_t* ids, void* points, void* normals);

/* ------------------------------------------------------------- timing --- */
/* HIP-event timing of the dominant kernel (the match kernel) on the context
 * stream: enable, then read the accumulated device time and launch count. */
int pmx_timing_enable(pmx_ctx* ctx, int on);
int pmx_timing_read(pmx_ctx* ctx, double* match_ms, int64_t* match_launches, double* other_ms);
int pmx_sync(pmx_ctx* ctx);

/* ------------------------------------------------- device-resident loop --- */
/* The ICP loop body (ICP.cpp:371-430) with the step solve, the T_iter update
 * (ICP.cpp:419) and the transformation checkers (TransformationChecker.cpp,
 * TransformationCheckersImpl.cpp:45-225) on the device: iterations are
 * enqueued back to back and the host synchronises once per pmx_loop_run.
 * Requirements: a grid matcher (pmx_set_search 1/2, per-lane kernel), filters
 * among default / Null / MaxDist / MinDist / MedianDist / TrimmedDist /
 * VarTrimmedDist / Robust (at most one; with PointToPoint only its
 * point2point distance), PointToPlane (no force2D / force4DOF) or
 * PointToPoint, checkers among Counter / Differential (smoothLength < 64) /
 * Bound.  Otherwise pmx_loop_begin returns PMX_E_BAD_PARAM and the caller
 * keeps the per-module calls. */
enum { PMX_CHECK_COUNTER = 0, PMX_CHECK_DIFFERENTIAL = 1, PMX_CHECK_BOUND = 2 };
enum { PMX_FILTER_DEFAULT = 0, PMX_FILTER_NULL = 1, PMX_FILTER_MAXDIST = 2, PMX_FILTER_MINDIST = 3,
       PMX_FILTER_MEDIANDIST = 4, PMX_FILTER_TRIMMED = 5, PMX_FILTER_VARTRIMMED = 6, PMX_FILTER_ROBUST = 7 };
/* RobustOutlierFilter's scale estimator in a loop configuration */
enum { PMX_RSE_NONE = 0, PMX_RSE_MAD = 1, PMX_RSE_STD = 2, PMX_RSE_BERG = 3 };
typedef struct pmx_loop_cfg {
    int knn;
    double max_dist;
    int n_filters;              /* 0: the empty chain's default (dist != inf) */
    int filter_kind[8];         /* PMX_FILTER_* */
    double filter_p[8][3];      /* maxDist / minDist / factor / ratio / (minRatio, maxRatio, lambda) */
    int minimizer;              /* 0 PointToPlane, 1 PointToPoint */
    int n_checkers;
    int checker_kind[8];        /* PMX_CHECK_* */
    double checker_p[8][3];     /* Counter: max; Differential: rot, trans, smoothLength; Bound: rot, trans */
    int keep_trace;             /* record T_iter of every iteration (pmx_loop_trace) */
    /* PMX_FILTER_ROBUST (OutlierFiltersImpl.cpp:380-598): the filter's
     * parameters and its call counter at the loop's start.  The scale of
     * iteration i is recomputed while robust_first_call + i <=
     * robust_nb_iter_for_scale (or always when that is 0), berg's first
     * computation at call 1 — robustFiltering's schedule (:500-531). */
    int robust_fct;             /* PMX_RF_* */
    int robust_estimator;       /* PMX_RSE_* */
    int robust_p2pl;            /* distanceType point2plane */
    int robust_nb_iter_for_scale;
    int robust_first_call;      /* the filter's iteration counter before the loop (1: never called) */
    double robust_tuning;       /* after berg's tuning substitution (:419-433) */
    double robust_approx;       /* approximation (inf: none) */
    double robust_berg_target;  /* berg: the target scale */
} pmx_loop_cfg;
typedef struct pmx_loop_status {
    int iterations;             /* iterations completed (IterationsCount) */
    int done;                   /* the loop has stopped */
    int reason;                 /* 1 Counter (MaxNumIterationsReached), 2 Differential, 3 error */
    int error;                  /* 0 or a PMX_E_* code; pmx_last_error has the reference's message */
    int64_t point_count_touched;/* sum of the iterations' pair evaluations */
    pmx_stats last;             /* statistics of the last iteration that reached the minimiser */
    double T_iter[16];          /* rows x rows */
    double cond[8][2];          /* checkers' condition variables */
} pmx_loop_status;
/* reset the loop: configuration, initial T_iter (rows x rows, T values;
 * normally the identity) — the checkers' init (ICP.cpp:368-369) */
int pmx_loop_begin(pmx_ctx* ctx, const pmx_loop_cfg* cfg, const void* T_iter0);
/* run up to n more iterations (fewer if a checker stops the loop or an error
 * is raised) and fill *st.  Iterations are enqueued in small batches with one
 * batch in flight ahead of the host's check of the stop flag.  Returns 0, or
 * the error the ICP raised (st->error, message in pmx_last_error), or a
 * HIP / RCCL / state error. */
int pmx_loop_run(pmx_ctx* ctx, int n, pmx_loop_status* st);
/* T_iter after each completed iteration (keep_trace): count x rows x rows T */
int pmx_loop_trace(pmx_ctx* ctx, int first, int count, void* out);
/* Quantile window statistics of the device loop (no reference counterpart;
 * diagnostics): iterations whose TrimmedDist / MedianDist quantile (chain
 * position 0) was resolved inside the match's key window, and iterations
 * that ran the radix passes instead.  Both results are exact; counts
 * accumulate over the loops of this context since the last pmx_loop_begin. */
int pmx_loop_select_stats(pmx_ctx* ctx, uint64_t* window_hits, uint64_t* window_misses);
/* Per-iteration diagnostics of the device loop (no reference counterpart):
 * for iterations [first, first + count) of the current loop (at most the
 * last 1024), 4 int64 each: the grid level the match ran on, the quantile
 * window verdict (1 resolved in the window, 0 radix passes, -1 no window),
 * the pairs the match evaluated (MatchersImpl.cpp:98's visit count) and the
 * queries that needed a full search (the rest were certified by temporal
 * reuse).  Synchronises the context stream. */
int pmx_loop_diag(pmx_ctx* ctx, int first, int count, int64_t* out);

/* ------------------------------------------------------ data filters --- */
/* SurfaceNormalDataPointsFilter::inPlaceFilter
 * (DataPointsFilters/SurfaceNormal.cpp:80-290) on the GPU: the self k-NN of
 * the cloud on the exact grid matcher (the filter's KDTreeMatcher with
 * ALLOW_SELF_MATCH, :158-162), then one kernel for the per-point statistics.
 * Standalone (a temporary context on `device`); pmx_last_error(NULL) has the
 * message of a failed call.
 *   feat: rows x n point-major T (dtype PMX_F32 / PMX_F64), rows = D + 1
 *   knn >= 1 (SurfaceNormal.h:68), maxDist: neighbour radius (+inf = none)
 *   outputs (point-major T, each may be NULL): normals D x n, densities n,
 *   eig_values D x n (ascending), eig_vectors D*D x n (serializeEigVec,
 *   row-major; column j = eigenvector of eig_values[j], largest component
 *   positive), matched_ids knn x n (reference indices as T, -1 = none),
 *   mean_dists n; degenerate (may be NULL): points whose C failed the rank test.
 *   flags: PMX_SN_SMOOTH = smoothNormals (sequential in point order, as the
 *   reference; needs normals). */
enum { PMX_SN_SMOOTH = 1 };
int pmx_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, int knn, double maxDist,
                        unsigned flags, void* normals, void* densities, void* eig_values, void* eig_vectors,
                        void* matched_ids, void* mean_dists, int64_t* degenerate);

/* SamplingSurfaceNormalDataPointsFilter::inPlaceFilter
 * (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342) on the GPU: the
 * recursive median split (buildNew) level by level over all boxes, the leaf
 * statistics (fuseRange) one thread per leaf; the sampling (samplingMethod 0:
 * rand() < ratio per point of every fitted leaf, the process's rand() state;
 * 1: the leaf's mean) and the output assembly on the host.  Standalone (a
 * temporary context on `device`); pmx_last_error(NULL) on failure.
 * Deterministic where the reference is implementation-defined: ties of the
 * median split broken by point index, a leaf's points in index order.
 *   feat: rows x n point-major T; desc: desc_dim x n point-major T (may be
 *   NULL when desc_dim = 0) — averaged per leaf with PMX_SSN_AVERAGE and
 *   samplingMethod 1, else the kept point's own
 *   outputs (point-major, sized for n points, each may be NULL): feat_out
 *   rows x n_out, desc_out desc_dim x n_out, normals D x n_out, densities
 *   n_out, eig_values D x n_out (ascending), eig_vectors D*D x n_out
 *   (serializeEigVec, row-major); unfit: points of dropped leaves. */
enum { PMX_SSN_NORMALS = 1, PMX_SSN_DENSITIES = 2, PMX_SSN_EIGVALUES = 4, PMX_SSN_EIGVECTORS = 8,
       PMX_SSN_AVERAGE = 16 };
int pmx_sampling_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc,
                                 int desc_dim, int knn, int sampling_method, double ratio, double max_box_dim,
                                 unsigned flags, void* feat_out, void* desc_out, void* normals, void* densities,
                                 void* eig_values, void* eig_vectors, int64_t* n_out, int64_t* unfit);

/* VoxelGridDataPointsFilter (DataPointsFilters/VoxelGrid.cpp:60-343): one
 * point per occupied voxel (vsize: vSizeX, vSizeY, vSizeZ), the voxel's
 * first point, with useCentroid its features replaced by the voxel mean, else
 * feature rows 1..3 set to the voxel centre as the reference does; descriptors
 * (desc_dim x n, may be NULL) averaged when average_desc.  Kept points in
 * index order; feat_out / desc_out hold n points.  Bit-identical to the
 * reference (sequential T sums in point order). */
int pmx_voxel_grid(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc, int desc_dim,
                   const double* vsize, int use_centroid, int average_desc, void* feat_out, void* desc_out,
                   int64_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* PMX_H */
