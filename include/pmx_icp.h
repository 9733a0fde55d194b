/*
 * pmx_icp.h — C ABI of the host ICP chain (libpmx_icp.so).
 *
 * A flat front-end over the C++ restatement of PointMatcher<T>::ICP
 * (libpointmatcher_amd/csrc/host/pm_icp.h) for non-C++ callers (the Python
 * tests and bench, a ctypes / cgo / JNI binding).  The chain is configured
 * exactly like the reference: ICPChainBase::setDefault (ICP.cpp:99-113) or a
 * libpointmatcher YAML chain (ICPChainBase::loadFromYaml, ICP.cpp:116-167).
 *
 * Clouds: rows x n point-major T arrays (rows = D + 1, homogeneous row last);
 * reference normals D x M point-major or NULL.  Transforms: rows x rows
 * row-major T.
 *
 * Errors: 0 on success, otherwise the negative code of the exception the
 * reference would throw; pmx_icp_last_error() holds its message.
 */
#ifndef PMX_ICP_H
#define PMX_ICP_H

#include <stdint.h>

#include "pmx.h" /* pmx_allreduce_fn / pmx_allgather_fn */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pmx_icp pmx_icp;

enum {
    PMX_ICP_OK = 0,
    PMX_ICP_CONVERGENCE_ERROR = -1,   /* PointMatcher<T>::ConvergenceError */
    PMX_ICP_INVALID_PARAMETER = -3,   /* Parametrizable::InvalidParameter */
    PMX_ICP_TRANSFORMATION_ERROR = -4,/* TransformationError */
    PMX_ICP_INVALID_ELEMENT = -5,     /* InvalidElement (unknown module name) */
    PMX_ICP_INVALID_MODULE_TYPE = -6, /* ICPChainBase::InvalidModuleType */
    PMX_ICP_CONFIGURATION_ERROR = -7, /* ConfigurationError / YAML syntax */
    PMX_ICP_RUNTIME_ERROR = -10       /* std::runtime_error (incl. HIP/RCCL failures) */
};

typedef struct pmx_icp_stats {
    int64_t iterations;            /* IterationsCount */
    int64_t point_count_touched;   /* PointCountTouched (pair evaluations) */
    double overlap_ratio;          /* OverlapRatio = weightedPointUsedRatio */
    double point_used_ratio;
    int64_t kept;                  /* ErrorElements columns of the last iteration */
    int64_t rejected_matches, rejected_points;
    double convergence_duration;   /* s, wall clock of the loop */
    double reference_preprocessing_duration;
    double reading_preprocessing_duration;
    int max_iterations_reached;
} pmx_icp_stats;

/* dtype: 0 = float, 1 = double; device: HIP ordinal */
int pmx_icp_create(int dtype, int device, pmx_icp** out);
void pmx_icp_destroy(pmx_icp* icp);
const char* pmx_icp_last_error(const pmx_icp* icp);

int pmx_icp_set_default(pmx_icp* icp);
int pmx_icp_load_yaml(pmx_icp* icp, const char* yaml_text);
/* multi-GPU: call before the first compute; uid from pmx_comm_unique_id */
int pmx_icp_comm_init(pmx_icp* icp, const void* uid128, int nranks, int rank);
/* multi-rank over the caller's host collectives (pmx_comm_init_host in pmx.h):
 * every rank passes its shard of the reading to compute/prepare */
int pmx_icp_comm_init_host(pmx_icp* icp, int nranks, int rank, pmx_allreduce_fn allreduce, pmx_allgather_fn allgather,
                           void* user);
int pmx_icp_keep_trace(pmx_icp* icp, int on);

/* ICP::compute (ICP.cpp:265-449): T_out = transform of reading into reference */
int pmx_icp_compute(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* reference, int64_t M,
                    const void* ref_normals, const void* T_init, void* T_out);

/* DataPoints descriptors (PointMatcher.h:207-358) for the next compute /
 * prepare: cloud 0 = reading, 1 = reference; span rows x n points,
 * point-major, dtype of the ICP (e.g. the reading's "maxSearchDist" for
 * KDTreeVarDistMatcher).  Consumed by that call. */
int pmx_icp_add_descriptor(pmx_icp* icp, int cloud, const char* name, int span, const void* values, int64_t n);

/* DataPoints::load (IO.cpp:374-389; loadCSV :535-800, loadVTK :948-1252):
 * a .csv or .vtk cloud with the reference's label mapping; features
 * (rows x n, homogeneous row last) and descriptors (desc_dim x n), both
 * point-major.  Errors: PMX_ICP_RUNTIME_ERROR, message in
 * pmx_cloud_last_error(). */
typedef struct pmx_cloud pmx_cloud;
int pmx_cloud_load(const char* path, int dtype, pmx_cloud** out);
void pmx_cloud_destroy(pmx_cloud* cloud);
const char* pmx_cloud_last_error(void);
int pmx_cloud_info(const pmx_cloud* cloud, int64_t* n, int* rows, int* desc_dim, int* n_feature_labels,
                   int* n_descriptor_labels);
/* which: 0 feature labels, 1 descriptor labels */
int pmx_cloud_label(const pmx_cloud* cloud, int which, int i, char* name, int cap, int* span);
int pmx_cloud_data(const pmx_cloud* cloud, void* features, void* descriptors);

/* the same loop in phases (bench: time the iterations alone) */
int pmx_icp_prepare(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* reference, int64_t M,
                    const void* ref_normals, const void* T_init);
/* run up to n iterations; *done = 1 once a checker stopped the loop */
int pmx_icp_iterate(pmx_icp* icp, int n, int* done);
int pmx_icp_finish(pmx_icp* icp, void* T_out);

int pmx_icp_stats_get(const pmx_icp* icp, pmx_icp_stats* out);
/* T_iter after each iteration (rows x rows each), returns count written */
int pmx_icp_trace_get(const pmx_icp* icp, void* out, int max_iters);
/* HIP-event device time of the match kernel over the last iterations */
int pmx_icp_timing(pmx_icp* icp, int on);
int pmx_icp_timing_read(pmx_icp* icp, double* match_ms, int64_t* match_launches);
/* quantile window statistics of the device loop (pmx_loop_select_stats):
 * iterations since the last prepare whose TrimmedDist / MedianDist quantile
 * was resolved inside the match's key window, and iterations that ran the
 * radix passes.  Diagnostics only (no reference counterpart). */
int pmx_icp_select_stats(pmx_icp* icp, uint64_t* window_hits, uint64_t* window_misses);
/* per-iteration diagnostics of the device loop since the last prepare
 * (pmx_loop_diag): 4 int64 per iteration for iterations [first, first +
 * count).  Diagnostics only (no reference counterpart). */
int pmx_icp_loop_diag(pmx_icp* icp, int first, int count, int64_t* out);
/* multi-rank: the context's collectives and loop synchronisations since
 * creation (pmx_comm_stats, pmx_comm_loop_stats).  Diagnostics only. */
int pmx_icp_comm_stats(pmx_icp* icp, uint64_t* allreduces, uint64_t* allgathers, uint64_t* verdict_syncs,
                       uint64_t* async_iterations, uint64_t* stalls);

/* ICPSequence (PointMatcher.h:730-764, ICP.cpp:455-609).  set_map replaces
 * ICPSequence::setMap: the map is centred on its mean, filtered by the
 * referenceDataPointsFilters and indexed once; it stays resident on the
 * device.  accepted = 0 for an empty map (ignored, as the reference).
 * Descriptors staged with pmx_icp_add_descriptor(cloud = 1) go to the map.
 * sequence_compute replaces ICPSequence::compute(cloudIn, T_refIn_dataIn)
 * (T_init may be NULL: identity): the reading against the resident map; with
 * no map T_out is the identity.  sequence_prepare is its first phase
 * (prepared = 0 without a map), followed by pmx_icp_iterate / pmx_icp_finish.
 * get_map: the prefiltered map in global coordinates (ICP.cpp:543-554),
 * rows x n features, point-major, into `features` of `capacity` values;
 * features NULL returns n and rows only, a capacity below n * rows is
 * PMX_ICP_INVALID_PARAMETER (nothing written).  A load_yaml / set_default
 * re-indexes a held map (ICP.cpp:520-539). */
int pmx_icp_set_map(pmx_icp* icp, const void* map, int rows, int64_t M, const void* normals, int* accepted);
int pmx_icp_clear_map(pmx_icp* icp);
int pmx_icp_has_map(const pmx_icp* icp, int* has);
int pmx_icp_get_map(pmx_icp* icp, void* features, int64_t capacity, int64_t* n, int* rows);
int pmx_icp_sequence_prepare(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* T_init,
                             int* prepared);
int pmx_icp_sequence_compute(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* T_init,
                             void* T_out);

#ifdef __cplusplus
}
#endif
#endif
