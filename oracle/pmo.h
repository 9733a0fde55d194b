/*
 * pmo — CPU ORACLE for the libpointmatcher ICP inner loop.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * CPU path (libpointmatcher v1.3.1 + the documented semantics of libnabo and
 * Eigen, which are not vendored in /root/reference).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the CPU baseline.  The product (libpointmatcher_amd)
 * never links or calls it.
 *
 * Parity pinning: the reference's C++ cannot be compiled here (Eigen3, Boost
 * and libnabo are absent), so this restatement is pinned by the reference's
 * own known-answer tests and fixtures (utest/utest.cpp validT2d/validT3d,
 * icpSingular, icpIdentity, utest/ui/Outliers.cpp VarTrimmed KAT, the
 * examples/data/icp_data *.ref_trans regression fixtures) and cross-checked
 * against numpy/scipy (cKDTree) golden vectors — see tests/.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference repository root).
 */
#ifndef PMO_H
#define PMO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes (mirrors the exception types of the reference). */
enum {
    PMO_OK = 0,
    PMO_E_NO_POINTS = -1,       /* ConvergenceError("ErrorMnimizer: no point to minimize") ErrorMinimizer.cpp:75-77 */
    PMO_E_EMPTY_QUANTILE = -2,  /* ConvergenceError("no outlier to filter") Matches.cpp:76-77 */
    PMO_E_BAD_PARAM = -3,       /* InvalidParameter / ConvergenceError("quantile must be between 0 and 1") */
    PMO_E_TRANSFORMATION = -4,  /* TransformationError TransformationsImpl.cpp:62-63 */
    PMO_E_NAN = -5,             /* ConvergenceError("abs rotation norm not a number") TransformationCheckersImpl.cpp:154-157 */
};

/* Outlier filter types (OutlierFiltersImpl.h). */
enum {
    PMO_OF_NULL = 0,        /* NullOutlierFilter            OutlierFiltersImpl.cpp:51-58 */
    PMO_OF_MAXDIST = 1,     /* MaxDistOutlierFilter(maxDist)  :66-84 */
    PMO_OF_MINDIST = 2,     /* MinDistOutlierFilter(minDist)  :87-103 */
    PMO_OF_MEDIANDIST = 3,  /* MedianDistOutlierFilter(factor) :108-128 */
    PMO_OF_TRIMMED = 4,     /* TrimmedDistOutlierFilter(ratio) :132-150 */
    PMO_OF_VARTRIMMED = 5,  /* VarTrimmedDistOutlierFilter(minRatio,maxRatio,lambda) :153-223 */
    PMO_OF_ROBUST = 6,      /* RobustOutlierFilter (pmo_cfg.robust) :394-598 */
};

/* RobustOutlierFilter (OutlierFiltersImpl.cpp:394-598).  The parameters as
 * the YAML gives them; the filter's state (iteration, scale, the berg
 * substitution of the tuning, :419-433) lives in the struct: zero it before
 * the first call, as a freshly constructed filter. */
enum { PMO_RF_CAUCHY = 0, PMO_RF_WELSCH, PMO_RF_SC, PMO_RF_GM, PMO_RF_TUKEY, PMO_RF_HUBER, PMO_RF_L1, PMO_RF_STUDENT };
enum { PMO_RS_NONE = 0, PMO_RS_MAD = 1, PMO_RS_STD = 2, PMO_RS_BERG = 3 };
typedef struct pmo_robust {
    int fct;             /* PMO_RF_* (robustFct) */
    int scale_est;       /* PMO_RS_* (scaleEstimator) */
    int nb_iter;         /* nbIterationForScale */
    int point2plane;     /* distanceType */
    double tuning;
    double approximation;  /* +inf = none */
    /* state */
    int iteration;       /* 0 = not constructed yet */
    double k, target, scale;  /* T values */
} pmo_robust;

enum { PMO_MIN_P2PLANE = 0, PMO_MIN_P2POINT = 1 };
enum { PMO_KNN_BRUTE = 0, PMO_KNN_KDTREE = 1 };
#define PMO_KNN_MAX (1 << 20)  /* largest k of pmo_knn / the ICP's matcher (k-lists past 256 on the heap) */
/* accumulation mode of the minimizer sums:
 *   0 = T-precision products accumulated in double (the build's semantics)
 *   1 = T-precision products accumulated sequentially in T (reference-like,
 *       used only to quantify the float-accumulation gap). */
enum { PMO_ACC_F64 = 0, PMO_ACC_T = 1 };

#define PMO_MAX_FILTERS 8

typedef struct pmo_cfg {
    /* matcher: KDTreeMatcher params (MatchersImpl.h:80-88) */
    int knn;
    double maxDist;          /* radius (not squared); +inf = none */
    int knn_method;          /* PMO_KNN_BRUTE | PMO_KNN_KDTREE */
    int knn_threads;         /* >1 = parallel over queries (CPU baseline only) */
    /* outlier chain (OutlierFilter.cpp:63-103) */
    int n_filters;
    int filter_type[PMO_MAX_FILTERS];
    double filter_p[PMO_MAX_FILTERS][3];
    /* error minimizer */
    int minimizer;           /* PMO_MIN_* */
    int acc_mode;            /* PMO_ACC_* */
    /* transformation checkers (TransformationCheckersImpl.cpp:45-158) */
    int counter_max;         /* <0 = no Counter checker */
    int diff_enabled;
    double diff_rot, diff_trans;
    int diff_smooth;
    pmo_robust robust;       /* the chain's PMO_OF_ROBUST filter (at most one) */
} pmo_cfg;

typedef struct pmo_stats {
    int64_t iterations;          /* IterationsCount  ICP.cpp:432 */
    int64_t kept;                /* P of the last iteration (ErrorElements columns) */
    int64_t nonzero_weights;     /* (w != 0).count()  ErrorMinimizer.cpp:75 */
    int64_t rejected_matches;    /* nbRejectedMatches ErrorMinimizer.cpp:191 */
    int64_t rejected_points;     /* nbRejectedPoints  ErrorMinimizer.cpp:192 */
    int64_t touched;             /* PointCountTouched ICP.cpp:433 */
    double sum_w;                /* sum of kept weights */
    double point_used_ratio;     /* ErrorMinimizer.cpp:139 */
    double weighted_point_used_ratio; /* OverlapRatio ErrorMinimizer.cpp:140 */
    int max_iter_reached;        /* ICP.cpp:426 */
    int error;                   /* PMO_E_* */
    double last_limit;           /* last quantile threshold (diagnostic) */
    double loop_seconds;         /* wall time of the iteration loop (CPU baseline) */
} pmo_stats;

/* ---------- float (T = float) ---------- */
/* rows = D+1 (homogeneous row included); points are stored point-major,
 * i.e. the memory layout of the reference's column-major (D+1) x N
 * features matrix.  normals are D values per point. */
int64_t pmo_knn_f32(const float* ref, int rows, int64_t M, const float* query, int64_t N,
                    int k, float maxDist, int method, int threads, float* dists, int32_t* ids);
int pmo_quantile_f32(const float* dists, int64_t n, float q, float* out);
int pmo_outlier_f32(int type, const double* p, const float* dists, int k, int64_t N, float* w);
int pmo_outlier_chain_f32(int n, const int* types, const double* params, const float* dists,
                          int k, int64_t N, float* w);
/* RobustOutlierFilter::compute: w (k x N) of one call, state updated.
 * step: the transformed reading (point-major, rows); ref / normals (D per
 * point) only for point2plane */
int pmo_robust_weights_f32(pmo_robust* r, const float* dists, const int32_t* ids, int k, int64_t N, const float* step,
                           int rows, const float* ref, const float* normals, float* w);
int pmo_vartrimmed_ratio_f32(const float* dists, int64_t n, float minRatio, float maxRatio,
                             float lambda, float* ratio_out);
void pmo_transform_f32(const float* T, int rows, const float* pts, int64_t N, float* out);
int pmo_p2plane_system_f32(int rows, const float* reading_t, const float* ref, const float* normals,
                           const float* dists, const int32_t* ids, const float* w, int k, int64_t N,
                           int acc_mode, double* A, double* b, pmo_stats* st);
int pmo_p2plane_solve_f32(int rows, const double* A, const double* b, float* dT);
int pmo_p2point_f32(int rows, const float* reading_t, const float* ref, const float* dists,
                    const int32_t* ids, const float* w, int k, int64_t N, int acc_mode,
                    float* dT, pmo_stats* st);
int pmo_icp_f32(const pmo_cfg* cfg, const float* reading, int rows, int64_t N,
                const float* ref, int64_t M, const float* ref_normals,
                const float* T_init, float* T_out, pmo_stats* st, float* trace);
/* the same, cfg->robust being a RobustOutlierFilter object kept across
 * calls (its iteration count and scale updated, OutlierFiltersImpl.cpp:500-540) */
int pmo_icp_keep_f32(pmo_cfg* cfg, const float* reading, int rows, int64_t N,
                     const float* ref, int64_t M, const float* ref_normals,
                     const float* T_init, float* T_out, pmo_stats* st, float* trace);
/* SurfaceNormalDataPointsFilter (DataPointsFilters/SurfaceNormal.cpp:80-290):
 * outputs point-major, any may be NULL (see pmo_impl.inc for the eigen
 * convention); smooth = smoothNormals */
/* SamplingSurfaceNormalDataPointsFilter (pmo_impl.inc): flags */
enum { PMO_SSN_NORMALS = 1, PMO_SSN_DENSITIES = 2, PMO_SSN_EIGVALUES = 4, PMO_SSN_EIGVECTORS = 8, PMO_SSN_AVERAGE = 16 };
int pmo_sampling_surface_normals_f32(const float* pts, int rows, int64_t n, const float* desc, int desc_dim, int knn,
                                     int sampling_method, float ratio, float max_box_dim, unsigned flags,
                                     float* feat_out, float* desc_out, float* normals, float* dens, float* evals,
                                     float* evecs, int64_t* n_out, int64_t* unfit);
int pmo_sampling_surface_normals_f64(const double* pts, int rows, int64_t n, const double* desc, int desc_dim,
                                     int knn, int sampling_method, double ratio, double max_box_dim, unsigned flags,
                                     double* feat_out, double* desc_out, double* normals, double* dens,
                                     double* evals, double* evecs, int64_t* n_out, int64_t* unfit);
/* VoxelGridDataPointsFilter (DataPointsFilters/VoxelGrid.cpp:60-343), the
 * reference's walk restated: outputs capacity n, returns 0 or PMO_E_BAD_PARAM */
int pmo_voxel_grid_f32(const float* pts, int rows, int64_t n, const float* desc, int desc_dim, const double* vsize,
                       int use_centroid, int average_desc, float* feat_out, float* desc_out, int64_t* n_out);
int pmo_voxel_grid_f64(const double* pts, int rows, int64_t n, const double* desc, int desc_dim, const double* vsize,
                       int use_centroid, int average_desc, double* feat_out, double* desc_out, int64_t* n_out);
int pmo_surface_normals_f32(const float* pts, int rows, int64_t n, int k, float maxDist, int threads, int smooth,
                            float* normals, float* dens, float* evals, float* evecs, float* ids, float* mdist,
                            int64_t* degenerate);

/* ---------- double (T = double) ---------- */
int64_t pmo_knn_f64(const double* ref, int rows, int64_t M, const double* query, int64_t N,
                    int k, double maxDist, int method, int threads, double* dists, int32_t* ids);
int pmo_quantile_f64(const double* dists, int64_t n, double q, double* out);
int pmo_outlier_f64(int type, const double* p, const double* dists, int k, int64_t N, double* w);
int pmo_outlier_chain_f64(int n, const int* types, const double* params, const double* dists,
                          int k, int64_t N, double* w);
int pmo_robust_weights_f64(pmo_robust* r, const double* dists, const int32_t* ids, int k, int64_t N,
                           const double* step, int rows, const double* ref, const double* normals, double* w);
int pmo_vartrimmed_ratio_f64(const double* dists, int64_t n, double minRatio, double maxRatio,
                             double lambda, double* ratio_out);
void pmo_transform_f64(const double* T, int rows, const double* pts, int64_t N, double* out);
int pmo_p2plane_system_f64(int rows, const double* reading_t, const double* ref, const double* normals,
                           const double* dists, const int32_t* ids, const double* w, int k, int64_t N,
                           int acc_mode, double* A, double* b, pmo_stats* st);
int pmo_p2plane_solve_f64(int rows, const double* A, const double* b, double* dT);
int pmo_p2point_f64(int rows, const double* reading_t, const double* ref, const double* dists,
                    const int32_t* ids, const double* w, int k, int64_t N, int acc_mode,
                    double* dT, pmo_stats* st);
int pmo_icp_f64(const pmo_cfg* cfg, const double* reading, int rows, int64_t N,
                const double* ref, int64_t M, const double* ref_normals,
                const double* T_init, double* T_out, pmo_stats* st, double* trace);
/* the same, cfg->robust being a RobustOutlierFilter object kept across
 * calls (its iteration count and scale updated, OutlierFiltersImpl.cpp:500-540) */
int pmo_icp_keep_f64(pmo_cfg* cfg, const double* reading, int rows, int64_t N,
                     const double* ref, int64_t M, const double* ref_normals,
                     const double* T_init, double* T_out, pmo_stats* st, double* trace);
int pmo_surface_normals_f64(const double* pts, int rows, int64_t n, int k, double maxDist, int threads, int smooth,
                            double* normals, double* dens, double* evals, double* evecs, double* ids, double* mdist,
                            int64_t* degenerate);

#ifdef __cplusplus
}
#endif
#endif
