// pmx_internal.h — shared device types and launcher declarations for libpmx.
//
// HBM layout:
//   reference  P4<T>[M_pad]  (x, y, z, h) — AoS, 16 B (f32) / 32 B (f64) per
//              point, padded with +inf points to a multiple of kTile so every
//              LDS tile load is full and branch-free;
//   normals    P4<T>[M]      (nx, ny, nz, 0);
//   grid       the reference (and its normals) sorted by cell, + cell starts;
//   reading    P4<T>[N]      already transformed by T_refMean_dataIn, in SLOT
//              order (Morton order of the initial cell; slot -> query index
//              kept on the host for the mirrors);
//   dists / weights T[N * k], ids int32[N * k], slot-major (the memory order
//              of the reference's column-major k x N Eigen matrices, up to the
//              slot permutation).  ids are reference indices after a brute-
//              force match and grid positions after a grid match.
// 2-D clouds (rows = 3) are embedded as (x, y, 0, h) with the 3x3 transform
// embedded in a 4x4; adding the +0 z-term is exact, so distances equal the
// 2-D sums bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

namespace pmx {

template <typename T>
struct alignas(4 * sizeof(T)) P4 {
    T x, y, z, w;
};

// Loads through explicitly global pointers.  Pointers read from device
// tables (the grid-level table of the device loop) are generic, and generic
// loads compile to flat_load (which also waits on lgkmcnt, serialising with
// LDS / scalar traffic); these helpers make every gather a global_load.
template <typename T>
struct Vec4Of;
template <>
struct Vec4Of<float> {
    typedef float V __attribute__((ext_vector_type(4)));
};
template <>
struct Vec4Of<double> {
    typedef double V __attribute__((ext_vector_type(4)));
};
// Workgroup index remapped so that consecutive indices share an XCD: blocks
// are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, "Workgroup
// dispatch, XCD placement"), so without it the neighbouring tiles of the slot
// order, which gather the same reference lines, sit in eight different L2s.
// A bijection on [0, gridDim.x) for any grid size; performance only.
__device__ __forceinline__ uint32_t xcd_block() {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u, i = b >> 3;
    return x < r ? x * (q + 1u) + i : r * (q + 1u) + (x - r) * q + i;
}

template <typename T>
__device__ __forceinline__ P4<T> gld(const P4<T>* p, int64_t i) {
    typedef typename Vec4Of<T>::V V;
    const V v = ((const __attribute__((address_space(1))) V*)p)[i];
    return P4<T>{v.x, v.y, v.z, v.w};
}
// 32-bit element index: the byte offset stays 32-bit, so the load is
// `global_load v, v_off, s[base]` (no 64-bit address arithmetic per lane).
// Callers guarantee count * sizeof(element) < 4 GiB (pmx_set_reference
// checks the reference; the grid arrays are sized from it).
template <typename T>
__device__ __forceinline__ P4<T> gld32(const P4<T>* p, uint32_t i) {
    typedef typename Vec4Of<T>::V V;
    const uint32_t off = i * (uint32_t)sizeof(P4<T>);
    const V v = *(const __attribute__((address_space(1))) V*)((const __attribute__((address_space(1))) char*)p + off);
    return P4<T>{v.x, v.y, v.z, v.w};
}
template <typename E>
__device__ __forceinline__ E gld32(const E* p, uint32_t i) {
    const uint32_t off = i * (uint32_t)sizeof(E);
    return *(const __attribute__((address_space(1))) E*)((const __attribute__((address_space(1))) char*)p + off);
}
__device__ __forceinline__ uint32_t gld(const uint32_t* p, int64_t i) {
    return ((const __attribute__((address_space(1))) uint32_t*)p)[i];
}
__device__ __forceinline__ int32_t gld(const int32_t* p, int64_t i) {
    return ((const __attribute__((address_space(1))) int32_t*)p)[i];
}

// Stores of per-query outputs the NEXT kernel reads (match distances, ids,
// safe radii): plain stores (write-through agent-scope stores measured the
// same)
template <typename V>
__device__ __forceinline__ void st_out(V* p, V v) {
    *p = v;
}

template <typename T>
struct Mat4 {
    T m[16];  // row-major
};

constexpr int kBlock = 256;   // threads per block (4 waves of 64)
constexpr int kTile = 1024;   // reference points per LDS tile
constexpr int kSub = 32;      // sub-block of the min-then-rescan k=1 scheme

// device-side select state for quantile filters (one per context)
struct SelectState {
    unsigned long long prefix;   // key bits resolved so far
    unsigned long long rank;     // rank still to find inside the current prefix
    unsigned long long count;    // number of finite keys (global)
    double limit;                // resolved threshold (T value)
    double ratio;                // quantile ratio (T value)
    int err;                     // PMX_E_EMPTY_QUANTILE etc.
    int pad;
};

// ---- match (pmx_match.hip) ----
template <typename T>
void launch_match(const P4<T>* ref, int64_t M_pad, const P4<T>* rd, int64_t N, const Mat4<T>& Tm,
                  int knn, T maxR2, T* dists, int32_t* ids, T* part_d, int32_t* part_i,
                  int64_t part_cap, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, int cu_count);
template <typename T>
int64_t match_part_elems(int64_t N, int64_t M_pad, int knn, int cu_count);
// KDTreeVarDistMatcher after the brute-force match: entries beyond their
// query's radius become (inf, -1) (the k nearest within a radius are the
// prefix of the k nearest)
template <typename T>
void launch_apply_radii(T* dists, int32_t* ids, const T* radii, int64_t N, int k, hipStream_t s);
// dst[s] = src[order[s]] (order == null: a copy)
template <typename T>
void launch_gather_scalar(const T* src, const int32_t* order, int64_t n, T* dst, hipStream_t s);

template <typename T>
void launch_transform(const P4<T>* in, P4<T>* out, int64_t N, const Mat4<T>& Tm, hipStream_t s);

// quantile window fused into the grid match (pmx_spec.h); null = off
struct SpecSel;

// ---- grid levels and the device-resident loop ----
struct GridGeom {
    double lo[3];
    double h, inv_h;
    int g[3];
};
// one grid level as the kernels see it (device table, indexed by LoopCtl::level)
template <typename T>
struct GridDesc {
    const P4<T>* gpts;
    const P4<T>* gpn;  // point, normal interleaved (2 P4 per position; null without normals)
    const int32_t* gidx;
    const uint32_t* start;
    GridGeom G;
};
// Per-context control word of the device-resident ICP loop (pmx_loop.hip):
// every kernel of an enqueued iteration reads it first.  done != 0 makes the
// kernels of the iterations enqueued past convergence return at once; T is
// the step transform (embedded 4x4, T values) and level the grid level of
// this iteration's match, both written by the previous iteration's step.
// A sharded loop that enqueues iterations without reading the window verdict
// back (pmx_loop_capi.hip) marks a window miss done = kCtlStalled: the rest of
// the enqueued iterations return at once (every kernel tests done != 0), and
// the host replays the stalled iteration's radix passes at its batch check.
constexpr int kCtlStalled = 2;
struct LoopCtl {
    int done;
    int level;
    int prev_level;  // level of the match the output buffers hold (-1: none; temporal reuse, pmx_grid.hip)
    int use_tile;    // the next match runs the tile kernel's warm form (tile dispatch, pmx_step.h)
    double T[16];
    double Tprev[16];  // the step transform of that previous match
};
// temporal reuse of the grid match (pmx_grid.hip): mode 0 off, 1 store the
// safe radii, 2 store and certify from the previous match made at Tprev
template <typename T>
struct GridReuse {
    int mode = 0;
    T* safe = nullptr;
    Mat4<T> Tprev{};
    // a block whose misses are at most this many searches each with a whole
    // wave (pmx_grid.hip coop_search); more take the per-lane search
    int coop_max = 0;
    // k = 1: each query's neighbour record (the grid point, its position in
    // w), written by every search that leaves a safe radius, so that the
    // certificate reads it with the query instead of gathering it by id
    // (null: off).  With the level's interleaved point / normal records
    // (gpn) the normals follow at nbr + N, for the point-to-plane reduction.
    P4<T>* nbr = nullptr;
    const P4<T>* gpn = nullptr;
};
template <typename T>
__device__ __forceinline__ void ctl_transform(const LoopCtl* ctl, Mat4<T>& Tm) {
#pragma unroll
    for (int i = 0; i < 16; ++i) Tm.m[i] = (T)ctl->T[i];
}

// k-NN for k > kLaneMaxK (pmx_knn_wide.hip): one wave per query, the k-list
// spread over the wave.  start == null: brute force over pts[0, M) (ids are
// indices); otherwise a grid level (ids are positions), G its geometry.
constexpr int kLaneMaxK = 16;   // the per-lane searches' largest k-list (wider: the wave-per-query search)
template <typename T>
void launch_knn_wide(const P4<T>* pts, const int32_t* gidx, const uint32_t* start, const GridGeom* G, int64_t M,
                     const P4<T>* rd, int64_t N, const Mat4<T>& Tm, int k, T maxR2, const T* radii, T* out_d,
                     int32_t* out_i, unsigned long long* visited, const LoopCtl* ctl, const GridDesc<T>* gd,
                     SpecSel* spec, hipStream_t s);


// ---- grid match (pmx_grid.hip) ----
// mode 0 = wave-cooperative LDS tiles, 1 = per-lane shell search (default).
// ids written are positions in gpts;
// launch_pos_to_index maps them back.  ctl / gd (device loop, modes 1-2):
// transform and level are read on the device.  cold: a new reading's first
// match (no previous match to certify from) on the tile kernel's cold form.
// vout null: no counter-sum launch after the match (its counter phase is
// merged into the select launch that follows, launch_select_all).
void set_tile_prof(unsigned long long* buf);
template <typename T>
void launch_grid_match(int mode, const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const double* lo,
                       double h, const int* g, const P4<T>* rd, int64_t N, const uint32_t* waves, int64_t n_waves,
                       const Mat4<T>& Tm, int knn, T maxR2, uint32_t max_pts, T* dists, int32_t* ids,
                       unsigned long long* vpart, unsigned long long* vout, int* iter_err, const GridReuse<T>& ru,
                       const LoopCtl* ctl, const GridDesc<T>* gd, SpecSel* spec, SelectState* spec_st,
                       unsigned long long* xseg, const T* radii, bool cold, bool tile_disp, hipEvent_t ev_start,
                       hipEvent_t ev_end, hipStream_t s);
// several ranks: the quantile window's pick over the all-gathered segments
// (pmx_spec.h); xseg above is this rank's segment, packed by the counter sum.
// stall: a miss sets ctl->done = kCtlStalled (the host did not read the
// verdict; it replays the iteration).  force_miss: treat the window as
// missed (test hook, option force_miss).
template <typename T>
void launch_spec_pick(const unsigned long long* segs, int nseg, SpecSel* spec, SelectState* st, LoopCtl* ctl,
                      int stall, int force_miss, hipStream_t s);
// ---- once-per-compute setup on the device (pmx_setup.hip) ----
// a uniform grid shape as the host sizes it (cells = g0 * g1 * g2)
struct SetupShape {
    double lo[3];
    double h;
    int g[3];
    int64_t cells;
};
// scratch of the setup sorts (keys32 / keys32_out alias keys64 / keys64_out)
struct SetupScratch {
    unsigned long long* keys64 = nullptr;
    unsigned long long* keys64_out = nullptr;
    uint32_t* keys32 = nullptr;
    uint32_t* keys32_out = nullptr;
    int32_t* idx = nullptr;
    int32_t* idx_out = nullptr;
    uint32_t* counts = nullptr;  // cells + 1
    void* temp = nullptr;        // hipcub temporary storage
    size_t temp_bytes = 0;
};
template <typename T>
struct Off3 {
    T v[3];
    int on;
};
// offset (may be null): rows - 1 values subtracted per axis in T (centring)
template <typename T>
void launch_pack_p4(const T* raw, int rows, int64_t n, int64_t n_pad, P4<T>* out, hipStream_t s,
                    const T* offset = nullptr);
template <typename T>
void launch_pack_nrm(const T* raw, int D, int64_t n, P4<T>* out, hipStream_t s);
template <typename T>
void launch_bbox(const P4<T>* p, int64_t n, double* scratch, double* out, hipStream_t s);
size_t bbox_scratch_bytes();
template <typename T>
void launch_occupancy(const P4<T>* p, int64_t n, const SetupShape& s, void* scratch, hipStream_t st);
size_t occupancy_bytes(int64_t cells);  // the scratch of launch_occupancy (count first)
// the largest trial grid launch_occupancy takes: build_grid's trial sizes are
// maxe/64 and maxe/128, i.e. at most 129 cells per axis
constexpr int64_t kOccMaxCells = (int64_t)129 * 129 * 129;
template <typename T>
int build_level_device(const P4<T>* pts, int64_t M, const P4<T>* nrm, const SetupShape& s, int64_t valid,
                       const SetupScratch& sc, P4<T>* gp, P4<T>* gpn, int32_t* gi, uint32_t* gstart, hipStream_t st);
template <typename T>
int reading_order_device(const P4<T>* raw, int64_t n, const Mat4<T>& M0, const SetupShape& s, bool morton,
                         const SetupScratch& sc, P4<T>* sorted, hipStream_t st);
size_t setup_temp_bytes(int64_t n, int64_t max_cells);
void launch_unpermute(const void* src, const int32_t* order, int64_t n, int span, size_t esz, void* dst,
                      hipStream_t s);
// SamplingSurfaceNormalDataPointsFilter's recursive median split and
// per-leaf statistics (pmx_ssn.hip).  Returns the point order (leaves
// contiguous, index order inside), the leaves (first, count), their fit flag
// and records (mean D, normal D, density, eigen values D, eigen vectors D*D);
// 0 or a PMX_E_* code with err set.
template <typename T>
int ssn_run(const P4<T>* d_pts, int D, int64_t n, int knn, T max_box, bool want_eig, hipStream_t st,
            std::vector<int32_t>& perm, std::vector<int32_t>& leaf_first, std::vector<int32_t>& leaf_cnt,
            std::vector<int32_t>& fit, std::vector<T>& rec, std::string& err);
// VoxelGridDataPointsFilter (pmx_voxel.hip): device in / out, capacity n
template <typename T>
int voxel_run(const T* d_f, int rows, int64_t n, const T* d_desc, int desc_dim, const double vsize[3], bool centroid,
              bool avg, T* d_of, T* d_od, int64_t* n_out, hipStream_t st, std::string& err);
// code-object preloads (one per translation unit, called by pmx_ctx_create)
void preload_setup();
void preload_ssn();
void preload_match();
void preload_grid();
void preload_select();
void preload_reduce();
void preload_loop();
void preload_normals();
// SurfaceNormalDataPointsFilter statistics over a self-match (pmx_normals.hip)
template <typename T>
void launch_surface_normals(const P4<T>* pts, const P4<T>* gpts, const int32_t* ids, const T* dists, int64_t N,
                            int k, int D, T* o_nrm, T* o_dens, T* o_eval, T* o_evec, T* o_mdist,
                            unsigned long long* degenerate, hipStream_t s);
// spread pair / fallback counters of the grid kernels (bytes; zero-initialised once)
size_t grid_counter_bytes();
void launch_pos_to_index(const int32_t* pos, const int32_t* gidx, int32_t* out, int64_t n, hipStream_t s);

// ---- outlier weights as a predicate chain ----
// Every supported OutlierFilter produces 0/1 weights and a chain multiplies
// them (OutlierFilter.cpp:63-103), so the chain is a conjunction of
// predicates on the distance.  It is evaluated inline by the reductions (no
// weight array is written or read on the hot path) and materialised only for
// the host mirror (pmx_get_weights).
// The RobustOutlierFilter (OutlierFiltersImpl.cpp:394-598) is the one
// filter with real-valued weights: w = robust(e^2), e^2 = dist / scale^2,
// multiplied with the predicates' 0/1 (kWPRobust, at most one per chain; the
// reductions take the weighted path only then).
enum WPred { kWPDefault = 0, kWPNull = 1, kWPLe = 2, kWPGe = 3, kWPState = 4, kWPRobust = 5 };
enum RobustFct { kRFCauchy = 0, kRFWelsch = 1, kRFSC = 2, kRFGM = 3, kRFTukey = 4, kRFHuber = 5, kRFL1 = 6,
                 kRFStudent = 7 };
constexpr int kMaxChain = 8;
template <typename T>
struct WChain {
    int n = 0;
    int type[kMaxChain] = {};
    T thr[kMaxChain] = {};                        // kWPLe / kWPGe: threshold; kWPState: scale
    const SelectState* st[kMaxChain] = {};        // kWPState: resolved quantile (limit)
    // kWPRobust (robust != 0): function, tuning k, squared approximation,
    // the scale (device, T value), point-to-plane distance
    int robust = 0;
    int rb_fct = 0;
    T rb_k = 1;
    T rb_sqa = 0;
    const double* rb_scale = nullptr;
    int rb_p2pl = 0;
    const T* w_arr = nullptr;  // materialised weights (a robust point-to-plane distance, point-to-point minimiser)
};
// robustFiltering's weight of one scaled squared error (OutlierFiltersImpl.cpp:541-596)
template <typename T>
__device__ __forceinline__ T robust_weight(int fct, T k, T sqa, T e2) {
    const T k2 = k * k;
    T w;
    switch (fct) {
    case kRFCauchy: w = (T)1 / ((T)1 + e2 / k2); break;
    case kRFWelsch: w = exp(-e2 / k2); break;
    case kRFSC: {
        const T s = k + e2;
        w = e2 >= k ? (T)(4.0 * (double)k2) * ((T)1 / (s * s)) : (T)1;
        break;
    }
    case kRFGM: {
        const T s = k + e2;
        w = k2 * ((T)1 / (s * s));
        break;
    }
    case kRFTukey: {
        const T a = (T)1 - e2 / k2;
        w = e2 >= k2 ? (T)0 : a * a;
        break;
    }
    case kRFHuber: w = e2 >= k2 ? k * ((T)1 / sqrt(e2)) : (T)1; break;
    case kRFL1: w = (T)1 / sqrt(e2); break;
    default: {  // Student, d = 3
        const T d = 3;
        const T p = pow((T)1 + e2 / k, -(k + d) / (T)2);
        w = p * (k + d) * ((T)1 / (k + e2));
        break;
    }
    }
    // ARBITRARY_SMALL_VALUE (1e-50 as T: 0 in float), then the approximation
    const T tiny = (T)1e-50;
    w = w <= tiny ? tiny : w;
    if (sqa != (T)__builtin_huge_val() && e2 >= sqa) w = 0;
    return w;
}
// per-thread resolved thresholds (kWPState: scale * limit in T, as the
// reference's `factor * quantile`, OutlierFiltersImpl.cpp:121-122)
// A conjunction of `d <= t` / `d >= t` / `d != inf` predicates is one
// interval test: keep = (d != inf if required) && lo <= d && d <= hi with
// hi = min of the upper thresholds, lo = max of the lower ones.  A NaN
// threshold (failed quantile) rejects everything, as `d <= NaN` does; the
// min/max below propagate it.
template <typename T>
struct WRange {
    T lo, hi;
    bool finite;
};
template <typename T>
__device__ __forceinline__ WRange<T> chain_resolve(const WChain<T>& c) {
    WRange<T> r{-(T)__builtin_huge_val(), (T)__builtin_huge_val(), false};
    for (int i = 0; i < c.n; ++i) {  // uniform, once per thread
        const int t = c.type[i];
        if (t == kWPDefault) {
            r.finite = true;
        } else if (t == kWPGe) {
            const T v = c.thr[i];
            r.lo = (v != v || r.lo != r.lo) ? v + r.lo : (v > r.lo ? v : r.lo);
        } else if (t == kWPLe || t == kWPState) {
            const T v = t == kWPState ? c.thr[i] * (T)c.st[i]->limit : c.thr[i];
            r.hi = (v != v || r.hi != r.hi) ? v + r.hi : (v < r.hi ? v : r.hi);
        }
    }
    return r;
}
template <typename T>
__device__ __forceinline__ bool chain_keep(const WRange<T>& r, T d) {
    return (!r.finite || d != (T)__builtin_huge_val()) && d >= r.lo && d <= r.hi;
}

// ---- robust scale estimators (pmx_robust.hip) ----
// the exact median index count / 2 (Matches::getMedianAbsDeviation's
// nth_element, Matches.cpp:110-120) instead of the quantile rule
// (size_t)((T)count * ratio): passed as the select's ratio
constexpr double kRatioMedianIndex = 2.0;
enum RobustScaleMode { kRSNone = 0, kRSMad = 1, kRSStd = 2, kRSBergFirst = 3, kRSBergNext = 4, kRSKeep = 5 };
// dev[i] = |d[i] - median| for finite d (median: st->limit), +inf otherwise
template <typename T>
void launch_abs_dev(const T* d, int64_t n, const SelectState* st, T* dev, const LoopCtl* ctl, hipStream_t s);
// sum of d (pass 0) / of (d - mean)^2 with mean = (T)(sum / n) (pass 1) into
// partials (kRedBlocks x 1), summed by launch_finalize
template <typename T>
void launch_moment(const T* d, int64_t n, int pass, const double* sum, double* partials, int64_t n_total,
                   const LoopCtl* ctl, hipStream_t s);
// the scale (a T value stored as double) of the iteration, from the mode
template <typename T>
void launch_robust_scale(int mode, const SelectState* st, const double* sums, int64_t n, double target,
                         double* scale, const LoopCtl* ctl, hipStream_t s);

// ---- quantile / weights (pmx_select.hip) ----
// one radix-select pass: histogram of digit `pass` among keys matching the
// resolved prefix.  hist must be zero on entry (select zeroes it on exit).
template <typename T>
void launch_select_hist(const T* d, int64_t n, uint32_t* hist, const SelectState* st, int pass,
                        const LoopCtl* ctl, const SpecSel* spec, hipStream_t s);
// resolve the digit of `pass`; pass 0 also computes count and the target
// rank from ratio (host value, or *ratio_dev when non-null).
// spec (may be null): skipped when the window resolved the quantile; the
// last pass re-centres the window
template <typename T>
void launch_select_pick(uint32_t* hist, SelectState* st, int pass, double ratio,
                        const double* ratio_dev, int* iter_err, const LoopCtl* ctl, SpecSel* spec, hipStream_t s);
template <typename T>
int select_passes();
// every pass in one launch (single rank; pmx_select.hip select_all_kernel):
// selx = selx_bytes() of zeroed device memory per context, re-zeroed whenever
// the launch's block count changes (select_all_blocks)
size_t selx_bytes();
int64_t select_all_blocks(int64_t n);
constexpr int kSelTimeout = -30;  // iteration error: a select_all wait timed out
// vpart / vout (may be null): the match's counter phase merged into this
// launch (pmx_selectall.h counter_merged); the spread counters are then
// zeroed by the next point-to-plane launch (launch_p2plane_partial's vzero)
template <typename T>
void launch_select_all(const T* d, int64_t n, void* selx, SelectState* st, double ratio, const double* ratio_dev,
                       int* iter_err, const LoopCtl* ctl, SpecSel* spec, const unsigned long long* vpart,
                       unsigned long long* vout, hipStream_t s);
int select_bins(int pass, int key_bits);

// VarTrimmed pieces
// development trace of the VarTrimmed walk (PMX_VT_TRACE=1): printed by
// pmx_vartrim_partial_sums
extern int g_vt_trace;
template <typename T>
size_t vartrim_trace_offset(int64_t n);
int vartrim_trace_max();
template <typename T>
void launch_vartrim(const T* d, int64_t n, int points_nbr, T minRatio, T maxRatio, const T* deno,
                    void* scratch, size_t scratch_bytes, double* ratio_dev, int* err_dev, SelectState* st,
                    const LoopCtl* ctl, hipStream_t s);
template <typename T>
size_t vartrim_scratch_bytes(int64_t n);
size_t vartrim_scratch_head();  // leading bytes of that scratch that must be zero at allocation
int vartrim_hdr_copy();     // int offset of the last call's counters in that scratch (pmx_vartrim_partial_sums)

// ---- reductions (pmx_reduce.hip) ----
constexpr int kRedBlocks = 512;  // fixed reduction grid (deterministic sums; 256 / 1024 measured slower)
constexpr int kNVMax = 48;
// point-to-plane result layout: upper triangle of A (NS), b (NF), then kept,
// nonzero weights, rejected matches, rejected points, sum of the weights
constexpr int p2plane_nv(int dim) { return dim == 3 ? 21 + 6 + 5 : 6 + 3 + 5; }
// the weighted (robust) variant: full A (NF x NF) instead of the upper triangle
constexpr int p2plane_nv_full(int dim) { return dim == 3 ? 36 + 6 + 5 : 9 + 3 + 5; }
// ctl / gd (device loop, may be null): early exit, step transform and the
// grid level whose positions the ids are (ref / nrm then come from gd)
// rs: index stride of ref / nrm (1: separate arrays; 2: a grid level's
// interleaved point / normal records, ref = gpn, nrm = gpn + 1)
// vzero (may be null): the match's spread counters, zeroed by block 0 (a
// counter phase merged into the select launch read them)
template <typename T>
void launch_p2plane_partial(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const P4<T>* nrm, int rs,
                            const T* d, const int32_t* ids, const WChain<T>& chain, int k, int64_t N, int dim,
                            double* partials, const LoopCtl* ctl, const GridDesc<T>* gd, unsigned long long* vzero,
                            hipStream_t s, const P4<T>* nbr = nullptr);
void launch_finalize(const double* partials, int nblocks, int nv, double* out, const LoopCtl* ctl, hipStream_t s);
template <typename T>
void launch_p2point_pass1(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d,
                          const int32_t* ids, const WChain<T>& chain, int k, int64_t N, double* partials,
                          const LoopCtl* ctl, const GridDesc<T>* gd, hipStream_t s);
template <typename T>
void launch_p2point_means(const double* sums, T* means_dev, int dim, const LoopCtl* ctl, hipStream_t s);
// both passes' sums in one (device loop; the step centres the moments,
// pmx_step.h): 20 values, layout in pmx_reduce.hip
template <typename T>
void launch_p2point_moments(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d, const int32_t* ids,
                            const WChain<T>& chain, int k, int64_t N, double* partials, const LoopCtl* ctl,
                            const GridDesc<T>* gd, hipStream_t s);
template <typename T>
void launch_p2point_pass2(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d,
                          const int32_t* ids, const WChain<T>& chain, int k, int64_t N, const T* means_dev,
                          double* partials, const LoopCtl* ctl, const GridDesc<T>* gd, hipStream_t s);
template <typename T>
void launch_weights_chain(const T* d, T* w, int64_t n, const WChain<T>& chain, const P4<T>* rd, const Mat4<T>& Tm,
                          const P4<T>* ref, const P4<T>* nrm, int rs, const int32_t* ids, int k, hipStream_t s);

}  // namespace pmx
