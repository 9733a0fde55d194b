// pmx_capi.hip — the C ABI declared in include/pmx.h.
//
// Owns the per-ICP-object device state (stream, resident clouds, match /
// weight arrays, select state, reduction buffers, RCCL communicator) and
// sequences the kernels of pmx_match.hip / pmx_select.hip / pmx_reduce.hip on
// one HIP stream.  Host synchronisation happens once per ICP iteration, in
// pmx_p2plane_system / pmx_p2point_system, when the ~400-byte system is
// copied back for the host solve (PointToPlane.cpp:108-161).
#include "pmx_internal.h"
#include "pmx_spec.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pmx.h"
#include "pmx_loop.h"

using namespace pmx;

// iteration block layout (see pmx_ctx_create)
constexpr size_t kBlkSel = 1024;
constexpr size_t kBlkIterErr = kBlkSel + sizeof(SelectState);
constexpr size_t kBlkRatio = 1152;
constexpr size_t kBlkVisited = 1216;
constexpr size_t kBlkMeans = 1280;
constexpr size_t kBlkCopy = 1344;
constexpr size_t kBlkBytes = 2048;
static_assert(kBlkIterErr + sizeof(int) <= kBlkRatio, "iteration block layout");
// The status block: the iteration block, then the loop's control word and
// state, in one allocation, so one copy returns everything the host reads
// after a batch of device-loop iterations.
constexpr size_t kStatCtl = kBlkBytes;
constexpr size_t kStatLoop = kStatCtl + 512;
constexpr size_t kStatBytes = (kStatLoop + sizeof(LoopState<double>) + 255) & ~(size_t)255;
static_assert(sizeof(LoopCtl) <= 512, "status block layout");

// one resolution of the uniform grid over the reference (pmx_grid.hip)
struct GridLevel {
    void* gpts = nullptr;        // P4<T>[valid] sorted by cell (x fastest)
    void* gpn = nullptr;         // point / normal records in the same order (point-to-plane gathers)
    int32_t* gidx = nullptr;     // original reference index of each position
    uint32_t* gstart = nullptr;  // first position of each cell, + end
    double lo[3] = {0, 0, 0};
    double h = 1.0;
    int dim[3] = {1, 1, 1};
    double ppc = 0.0;
    void release() {
        for (void* b : {gpts, gpn, (void*)gidx, (void*)gstart})
            if (b) (void)hipFree(b);
        gpts = gpn = nullptr;
        gidx = nullptr;
        gstart = nullptr;
    }
};

struct pmx_ctx {
    int device = 0;
    int dtype = PMX_F32;
    int cu_count = 256;
    hipStream_t stream = nullptr;
    std::string err;

    // reference (Matcher::init)
    int rows = 0, dim = 0;
    int64_t M = 0, M_pad = 0;
    void* d_ref = nullptr;
    void* d_nrm = nullptr;
    bool has_normals = false;

    // uniform grid over the reference (exact shell search, pmx_grid.hip)
    int search_type = 1;
    int grid_mode = 1;            // 1 = per-lane shell search (default), 0 = LDS tiles (PMX_GRID_MODE=tile)
    uint32_t tile_max = 4096;     // largest per-wave box scanned from LDS (PMX_GRID_TILE_MAX)
    // Grid levels of increasing cell size (points per occupied cell:
    // level_ppc, PMX_GRID_LEVELS).  Every level answers exactly; the level of
    // the next match is chosen from the last match's pair count (adaptive:
    // converged iterations want small cells, misaligned ones or large k want
    // large cells, see choose_level).
    std::vector<GridLevel> levels;
    std::vector<double> level_ppc{2.0, 4.0, 8.0, 16.0, 32.0, 64.0};
    int level = 0;      // level of the next grid match
    double first_ppc = 8.0;   // level of a new reading's first (cold) match (PMX_GRID_FIRST_PPC)
    int ids_level = 0;  // level whose positions the current match ids are
    std::vector<double> level_cells;   // last cells-per-query seen at each level
    std::vector<int64_t> level_seen;   // match count when it was seen (0: never)
    int64_t match_count = 0;
    bool adaptive = true;
    bool reuse_on = true;         // temporal reuse of the grid match (pmx_grid.hip; PMX_GRID_REUSE=0: off)
    bool safe_valid = false;      // d_safe holds the safe radii of the match in d_dists / d_ids
    void* d_safe = nullptr;       // T[N]: safe radius per query
    int64_t safe_cap = 0;
    bool grid_ready = false;
    const GridLevel& lv(int i) const { return levels[(size_t)i]; }
    std::vector<int32_t> slot_query;  // host copy of d_order (host mirrors only; filled on demand)
    int32_t* d_order = nullptr;       // slot -> reading index (has_order; else identity)
    size_t order_bytes = 0;
    bool has_order = false;
    // once-per-compute setup on the device (pmx_setup.hip)
    SetupScratch setup;
    int64_t setup_n = 0, setup_cells = 0;
    void* d_raw = nullptr;            // upload staging of a caller's cloud
    size_t raw_bytes = 0;
    void* d_bbox = nullptr;
    size_t bbox_bytes = 0;
    void* d_occ = nullptr;            // occupancy bitmap + counter
    size_t occ_bytes = 0;
    uint32_t* d_waves = nullptr;      // tile-kernel wave table: first slot of each wave (+ N)
    int64_t n_waves = 0;
    bool ids_grid = false;            // last match wrote grid positions
    unsigned long long* d_visited = nullptr;  // [pairs, fallbacks] in the iteration block
    unsigned long long* d_vpart = nullptr;    // spread per-wave counters (pmx_grid.hip)
    uint64_t visited_host = 0;   // brute force: known at launch

    // reading shard
    int64_t N = 0, N_total = 0, N_max = 0;
    void* d_rd = nullptr;
    // KDTreeVarDistMatcher: per-point search radii in slot order (pmx_set_reading_radii)
    void* d_radii = nullptr;
    size_t radii_bytes = 0;
    bool has_radii = false;

    // matches / weights
    int knn = 0;
    int64_t match_cap = 0;  // elements
    void* d_dists = nullptr;
    int32_t* d_ids = nullptr;
    void* d_w = nullptr;
    int64_t part_cap = 0;
    void* d_part_d = nullptr;
    int32_t* d_part_i = nullptr;
    double Tstep[16] = {0};  // step transform (embedded 4x4, T values)
    double Tprev[16] = {0};  // the previous match's (the grid match's warm start)
    bool have_match = false;

    // outlier weight chain (WChain): predicates recorded by the filter calls
    int chain_n = 0;
    int chain_type[kMaxChain] = {};
    double chain_thr[kMaxChain] = {};
    bool w_valid = false;  // d_w holds the chain's weights (mirror only)
    // RobustOutlierFilter (at most one per chain): its parameters, and the
    // device block of its scale state: SelectState (the MAD's second
    // select), then the scale of each chain position, then the moment sums
    int rb_pos = -1, rb_fct = 0, rb_p2pl = 0;
    double rb_k = 1.0, rb_sqa = INFINITY;
    void* d_rob = nullptr;
    void* d_rdev = nullptr;  // |d - median| (T[n])
    size_t rdev_bytes = 0;
    double* rob_scale(int pos) const { return (double*)((char*)d_rob + 256) + pos; }
    double* rob_sums() const { return (double*)((char*)d_rob + 256) + kMaxChain; }
    SelectState* rob_sel() const { return (SelectState*)d_rob; }

    // quantile select: SelectState followed by the per-iteration error word;
    // chain positions >= 1 use their own states (d_sel_more)
    SelectState* d_sel_more = nullptr;
    SelectState* sel_slot(int pos) const { return pos == 0 ? d_sel : d_sel_more + (pos - 1); }
    SelectState* d_sel = nullptr;
    int* d_iter_err = nullptr;
    uint32_t* d_hist = nullptr;
    void* d_selx = nullptr;            // select_all_kernel's arrivals / publications / per-pass bins
    int64_t selx_grid = 0;             // its block count of the last launch (0: zeroed)
    double* d_ratio = nullptr;

    // VarTrimmed scratch + cached pow table
    void* d_vt = nullptr;
    size_t vt_bytes = 0;
    void* d_deno = nullptr;
    size_t deno_bytes = 0;
    int deno_pts = -1, deno_min = -1, deno_max = -1;
    double deno_lambda = NAN;
    void* d_gather = nullptr;  // multi-rank all-gathered distances
    size_t gather_bytes = 0;

    // reductions
    double* d_partials = nullptr;
    double* d_result = nullptr;  // [0..63] system, [64..127] second pass
    void* d_means = nullptr;
    double* h_result = nullptr;  // pinned

    // multi-GPU: the collectives of a sharded ICP (coll_*).  RCCL over
    // xGMI (pmx_comm_init), or caller-provided host collectives
    // (pmx_comm_init_host: device buffers staged through pinned memory).
    // Once either is set up every exchange step is issued, whatever nranks.
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    pmx_allreduce_fn host_ar = nullptr;
    pmx_allgather_fn host_ag = nullptr;
    void* host_user = nullptr;
    void* h_stage = nullptr;      // pinned staging of the host collectives
    int* h_flags = nullptr;       // pinned: the window verdict a sharded select reads back
    bool spec_exchanged = false;  // this match all-gathered the window segments and picked
    bool shard_done_seen = false; // a sharded loop read back its stop flag: no more iterations to enqueue
    uint64_t n_allreduce = 0, n_allgather = 0;  // collectives issued (pmx_comm_stats)
    size_t h_stage_cap = 0;
    unsigned long long* d_specx = nullptr;  // quantile window exchange: own segment, then nranks gathered

    // device-resident loop (pmx_loop.hip)
    LoopCtl* d_ctl = nullptr;     // control word read by every kernel in loop mode
    void* d_gdesc = nullptr;      // GridDesc<T>[levels]
    void* d_loop = nullptr;       // LoopState<T>
    void* d_loop_T0 = nullptr;    // initial T_iter (upload)
    void* d_trace = nullptr;      // T_iter per iteration (keep_trace)
    int64_t trace_cap = 0;        // iterations
    bool loop_on = false;         // enqueueing loop iterations
    // quantile window fused into the grid match (pmx_spec.h): device loop,
    // single rank, quantile filter at chain position 0 (PMX_SPEC_SELECT=0: off)
    SpecSel* d_spec = nullptr;
    void* d_spec_keys = nullptr;
    bool spec_allowed = true;
    bool spec_on = false;
    SpecSel spec_init{};  // (host staging of the reset)
    SpecSel* spec_now() const { return spec_on && loop_on ? d_spec : nullptr; }
    bool loop_begun = false;
    pmx_loop_cfg loop_cfg{};
    LoopCfg loop_dev{};
    void* h_loop = nullptr;       // pinned: two copies of the status block (the batches in flight)
    hipEvent_t loop_ev[2] = {nullptr, nullptr};  // end of the batches in flight
    int64_t loop_issued = 0;      // iterations enqueued since pmx_loop_begin
    int loop_iters = 0;           // iterations completed (last status)
    bool loop_done = false;       // the loop has stopped (last status)

    // timing of the match kernel
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
    double match_ms = 0.0;
    int64_t match_launches = 0;
};

namespace {

thread_local std::string g_err;  // message of a failed standalone call (pmx_last_error(NULL))

int fail(pmx_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(ctx, PMX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define NCCLCHK(ctx, expr)                                                                     \
    do {                                                                                       \
        ncclResult_t r_ = (expr);                                                              \
        if (r_ != ncclSuccess)                                                                 \
            return fail(ctx, PMX_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

size_t tsize(const pmx_ctx* c) { return c->dtype == PMX_F64 ? 8 : 4; }

// the device loop's control word while iterations are being enqueued
const LoopCtl* loop_ctl(const pmx_ctx* c) { return c->loop_on ? c->d_ctl : nullptr; }

int ensure(pmx_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return PMX_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc(p, bytes > 0 ? bytes : 16));
    *cap = bytes;
    return PMX_OK;
}

// embed a rows x rows host transform (row-major T) into a 4x4 (see pmx_internal.h)
template <typename T>
Mat4<T> embed(const T* src, int rows) {
    Mat4<T> m{};
    if (rows == 4) {
        for (int i = 0; i < 16; ++i) m.m[i] = src[i];
    } else {
        const T a[16] = {src[0], src[1], 0, src[2], src[3], src[4], 0, src[5],
                         0,      0,      1, 0,      src[6], src[7], 0, src[8]};
        for (int i = 0; i < 16; ++i) m.m[i] = a[i];
    }
    return m;
}

template <typename T>
Mat4<T> step_mat(const pmx_ctx* c) {
    Mat4<T> m{};
    for (int i = 0; i < 16; ++i) m.m[i] = (T)c->Tstep[i];
    return m;
}

// ------------------------------------------------------------- collectives --
// A sharded ICP (reading split over ranks) exchanges, per
// iteration: the radix-select histograms (or the quantile window segments),
// VarTrimmed's distances, and the packed fp64 system.  All of them go through
// these two calls, on the context stream.
bool sharded(const pmx_ctx* c) { return c->comm != nullptr || c->host_ar != nullptr; }

size_t coll_size(int type) { return type == PMX_COLL_U32 ? 4 : 8; }

int stage_room(pmx_ctx* c, size_t bytes) {
    if (c->h_stage_cap >= bytes && c->h_stage) return PMX_OK;
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (a pending copy may still read the old stage)
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    const size_t cap = std::max<size_t>(bytes, 1 << 16);
    HIPCHK(c, hipHostMalloc(&c->h_stage, cap, hipHostMallocDefault));
    c->h_stage_cap = cap;
    return PMX_OK;
}

// in-place all-reduce of `count` elements of device memory
int coll_allreduce(pmx_ctx* c, void* dbuf, int64_t count, int type, int op) {
    if (!sharded(c) || count <= 0) return PMX_OK;
    ++c->n_allreduce;
    if (c->comm) {
        const ncclDataType_t dt = type == PMX_COLL_U32 ? ncclUint32 : type == PMX_COLL_U64 ? ncclUint64 : ncclFloat64;
        NCCLCHK(c, ncclAllReduce(dbuf, dbuf, (size_t)count, dt, op == PMX_COLL_MAX ? ncclMax : ncclSum, c->comm,
                                 c->stream));
        return PMX_OK;
    }
    const size_t bytes = (size_t)count * coll_size(type);
    int rc = stage_room(c, bytes);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->h_stage, dbuf, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = c->host_ar(c->host_user, c->h_stage, count, type, op)) != 0)
        return fail(c, PMX_E_RCCL, "host all-reduce callback failed (" + std::to_string(rc) + ")");
    HIPCHK(c, hipMemcpyAsync(dbuf, c->h_stage, bytes, hipMemcpyHostToDevice, c->stream));
    return PMX_OK;
}

// all-gather `bytes` per rank: recv holds nranks blocks in rank order
int coll_allgather(pmx_ctx* c, const void* dsend, void* drecv, size_t bytes) {
    if (!sharded(c)) {
        if (drecv != dsend) HIPCHK(c, hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, c->stream));
        return PMX_OK;
    }
    ++c->n_allgather;
    if (c->comm) {
        NCCLCHK(c, ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, c->stream));
        return PMX_OK;
    }
    const size_t total = bytes * (size_t)(c->nranks + 1);
    int rc = stage_room(c, total);
    if (rc) return rc;
    char* send = (char*)c->h_stage + bytes * (size_t)c->nranks;
    HIPCHK(c, hipMemcpyAsync(send, dsend, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = c->host_ag(c->host_user, send, c->h_stage, (int64_t)bytes)) != 0)
        return fail(c, PMX_E_RCCL, "host all-gather callback failed (" + std::to_string(rc) + ")");
    HIPCHK(c, hipMemcpyAsync(drecv, c->h_stage, bytes * (size_t)c->nranks, hipMemcpyHostToDevice, c->stream));
    return PMX_OK;
}

int allreduce_f64(pmx_ctx* c, double* buf, size_t n) { return coll_allreduce(c, buf, (int64_t)n, PMX_COLL_F64, PMX_COLL_SUM); }

void resolve_events(pmx_ctx* c) {
    for (auto& pr : c->ev_pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) {
            c->match_ms += ms;
            c->match_launches += 1;
        }
        c->ev_pool.push_back(pr.first);
        c->ev_pool.push_back(pr.second);
    }
    c->ev_pending.clear();
}

hipEvent_t get_event(pmx_ctx* c) {
    if (!c->ev_pool.empty()) {
        hipEvent_t e = c->ev_pool.back();
        c->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// -------------------------------------------------------------------- grid --
// Uniform grid of the (centred) reference for the exact shell search.  The
// cell size targets ~4 points per occupied cell: the occupied-cell count at
// two trial sizes gives the data's local dimension (surface ~2, volume ~3),
// from which the size for the target density follows.  Points are sorted by
// cell (x fastest, index order inside a cell) so every x-row of cells is one
// contiguous range.  The sizing runs on the host from three device counts;
// the build itself is pmx_setup.hip.
constexpr int64_t kMaxCells = (int64_t)1 << 26;

SetupShape grid_shape(const double lo[3], const double ext[3], double h) {
    SetupShape s;
    for (int a = 0; a < 3; ++a) {
        s.lo[a] = lo[a];
        const double gg = std::floor(ext[a] / h) + 1.0;
        s.g[a] = gg > 1e9 ? 1000000000 : (int)gg;
    }
    s.h = h;
    s.cells = (int64_t)s.g[0] * s.g[1] * s.g[2];
    return s;
}

// setup scratch for n points and grids of up to max_cells cells
int setup_room(pmx_ctx* c, int64_t n, int64_t max_cells) {
    n = std::max<int64_t>(n, 1);
    SetupScratch& sc = c->setup;
    if (c->setup_n < n) {
        for (void* p : {(void*)sc.keys64, (void*)sc.keys64_out, (void*)sc.idx, (void*)sc.idx_out})
            if (p) (void)hipFree(p);
        sc.keys64 = sc.keys64_out = nullptr;
        sc.idx = sc.idx_out = nullptr;
        c->setup_n = 0;
        HIPCHK(c, hipMalloc((void**)&sc.keys64, sizeof(unsigned long long) * n));
        HIPCHK(c, hipMalloc((void**)&sc.keys64_out, sizeof(unsigned long long) * n));
        HIPCHK(c, hipMalloc((void**)&sc.idx, sizeof(int32_t) * n));
        HIPCHK(c, hipMalloc((void**)&sc.idx_out, sizeof(int32_t) * n));
        sc.keys32 = (uint32_t*)sc.keys64;
        sc.keys32_out = (uint32_t*)sc.keys64_out;
        c->setup_n = n;
    }
    if (c->setup_cells < max_cells) {
        if (sc.counts) (void)hipFree(sc.counts);
        sc.counts = nullptr;
        c->setup_cells = 0;
        HIPCHK(c, hipMalloc((void**)&sc.counts, sizeof(uint32_t) * (size_t)(max_cells + 1)));
        c->setup_cells = max_cells;
    }
    const size_t tb = setup_temp_bytes(c->setup_n, c->setup_cells);
    if (sc.temp_bytes < tb) {
        if (sc.temp) (void)hipFree(sc.temp);
        sc.temp = nullptr;
        sc.temp_bytes = 0;
        HIPCHK(c, hipMalloc(&sc.temp, tb));
        sc.temp_bytes = tb;
    }
    return PMX_OK;
}

void setup_release(pmx_ctx* c) {
    SetupScratch& sc = c->setup;
    for (void* p : {(void*)sc.keys64, (void*)sc.keys64_out, (void*)sc.idx, (void*)sc.idx_out, (void*)sc.counts,
                    sc.temp})
        if (p) (void)hipFree(p);
    c->setup = SetupScratch{};
    c->setup_n = c->setup_cells = 0;
}

// host staging of one upload (the caller's cloud, pageable) into the raw buffer
int upload_raw(pmx_ctx* c, const void* src, size_t bytes) {
    int rc = ensure(c, &c->d_raw, &c->raw_bytes, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    if (bytes) HIPCHK(c, hipMemcpyAsync(c->d_raw, src, bytes, hipMemcpyHostToDevice, c->stream));
    return PMX_OK;
}

// the grid levels over the resident reference d_ref (M points) and d_nrm
template <typename T>
int build_grid(pmx_ctx* c, int64_t M) {
    const P4<T>* pts = (const P4<T>*)c->d_ref;
    const P4<T>* nrm = (const P4<T>*)c->d_nrm;
    // bounding box of the finite points (inf / NaN points can never be a neighbour)
    double* sb = nullptr;  // bbox partials, then 8 doubles of result
    size_t sbc = 0;
    int rc = ensure(c, (void**)&c->d_bbox, &c->bbox_bytes, bbox_scratch_bytes() + 16 * sizeof(double));
    if (rc) return rc;
    sb = (double*)c->d_bbox;
    (void)sbc;
    double* bb_out = sb + bbox_scratch_bytes() / sizeof(double);
    launch_bbox<T>(pts, M, sb, bb_out, c->stream);
    double bb[7];
    HIPCHK(c, hipMemcpyAsync(bb, bb_out, sizeof(bb), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    double lo[3] = {bb[0], bb[1], bb[2]}, hi[3] = {bb[3], bb[4], bb[5]};
    const int64_t valid = (int64_t)bb[6];
    if (valid == 0)
        for (int a = 0; a < 3; ++a) lo[a] = hi[a] = 0;
    double ext[3], maxe = 0;
    for (int a = 0; a < 3; ++a) {
        ext[a] = hi[a] - lo[a];
        maxe = std::max(maxe, ext[a]);
    }
    if (!(maxe > 0)) maxe = 1;
    // distinct occupied cells at a trial size (device bitmap)
    auto occupied = [&](double h, int64_t& occ) -> int {
        const SetupShape s = grid_shape(lo, ext, h);
        occ = -1;
        if (s.cells > ((int64_t)1 << 28)) return PMX_OK;
        // bitmap, then the 8-byte counter on its own aligned line (a 64-bit
        // atomic must be naturally aligned)
        const size_t words = (size_t)((s.cells + 31) / 32);
        const size_t cnt_off = (sizeof(uint32_t) * words + 255) & ~(size_t)255;
        int r = ensure(c, &c->d_occ, &c->occ_bytes, cnt_off + 256);
        if (r) return r;
        unsigned long long* cnt = (unsigned long long*)((char*)c->d_occ + cnt_off);
        HIPCHK(c, hipMemsetAsync(c->d_occ, 0, cnt_off + 8, c->stream));
        launch_occupancy<T>(pts, M, s, (uint32_t*)c->d_occ, cnt, c->stream);
        unsigned long long v = 0;
        HIPCHK(c, hipMemcpyAsync(&v, cnt, sizeof(v), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        occ = (int64_t)v;
        return PMX_OK;
    };
    double dim = 3.0, ppc1 = 1.0, h1 = maxe / 128.0;
    if (valid > 0) {
        const double h0 = maxe / 64.0;
        int64_t o0 = 0, o1 = 0;
        if ((rc = occupied(h0, o0)) || (rc = occupied(h1, o1))) return rc;
        o0 = std::max<int64_t>(1, o0);
        o1 = std::max<int64_t>(1, o1);
        dim = std::log2((double)o1 / (double)o0);
        dim = std::min(3.0, std::max(1.0, dim));
        ppc1 = (double)valid / (double)o1;
    }
    for (auto& L : c->levels) L.release();
    c->levels.clear();
    c->level = 0;
    c->match_count = 0;
    c->level_cells.assign(c->level_ppc.size(), 0.0);
    c->level_seen.assign(c->level_ppc.size(), 0);
    // the level shapes: cell size h (clamped to the 2^26-cell budget)
    std::vector<SetupShape> shapes;
    int64_t max_cells = 1;
    for (double target : c->level_ppc) {
        double h = valid > 0 ? h1 * std::pow(target / ppc1, 1.0 / dim) : maxe / 64.0;
        h = std::max(h, maxe / 4096.0);
        SetupShape s = grid_shape(lo, ext, h);
        while (s.cells > kMaxCells) {
            h *= 1.25;
            s = grid_shape(lo, ext, h);
        }
        shapes.push_back(s);
        max_cells = std::max(max_cells, s.cells);
    }
    if ((rc = setup_room(c, M, max_cells))) return rc;
    const int64_t np = std::max<int64_t>(valid, 1);
    for (size_t l = 0; l < shapes.size(); ++l) {
        const SetupShape& s = shapes[l];
        GridLevel L;
        auto bad = [&](int r) {
            L.release();
            return r;
        };
        if (hipMalloc(&L.gpts, sizeof(P4<T>) * np) != hipSuccess ||
            hipMalloc((void**)&L.gidx, sizeof(int32_t) * np) != hipSuccess ||
            hipMalloc((void**)&L.gstart, sizeof(uint32_t) * (size_t)(s.cells + 1)) != hipSuccess ||
            (nrm && hipMalloc(&L.gpn, 2 * sizeof(P4<T>) * np) != hipSuccess))
            return bad(fail(c, PMX_E_HIP, "grid level allocation failed"));
        const int r = build_level_device<T>(pts, M, nrm, s, valid, c->setup, (P4<T>*)L.gpts, (P4<T>*)L.gpn, L.gidx,
                                            L.gstart, c->stream);
        if (r) return bad(fail(c, PMX_E_HIP, "grid level build failed (" + std::to_string(r) + ")"));
        for (int a = 0; a < 3; ++a) {
            L.lo[a] = s.lo[a];
            L.dim[a] = s.g[a];
        }
        L.h = s.h;
        L.ppc = c->level_ppc[l];
        c->levels.push_back(L);
    }
    // the device table of levels (the device loop picks the level on the GPU)
    std::vector<GridDesc<T>> tab(c->levels.size());
    for (size_t l = 0; l < c->levels.size(); ++l) {
        const GridLevel& L = c->levels[l];
        GridDesc<T>& D = tab[l];
        D.gpts = (const P4<T>*)L.gpts;
        D.gpn = (const P4<T>*)L.gpn;
        D.gidx = L.gidx;
        D.start = L.gstart;
        for (int a = 0; a < 3; ++a) {
            D.G.lo[a] = L.lo[a];
            D.G.g[a] = L.dim[a];
        }
        D.G.h = L.h;
        D.G.inv_h = 1.0 / L.h;
    }
    if (c->d_gdesc) (void)hipFree(c->d_gdesc);
    c->d_gdesc = nullptr;
    HIPCHK(c, hipMalloc(&c->d_gdesc, sizeof(GridDesc<T>) * std::max<size_t>(tab.size(), 1)));
    HIPCHK(c, hipMemcpyAsync(c->d_gdesc, tab.data(), sizeof(GridDesc<T>) * tab.size(), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->grid_ready = true;
    return PMX_OK;
}

// Slot order of the reading: Morton order of the cell of the initially
// transformed point, so the 64 queries of a wave form a compact cluster
// (small shared LDS box in the tile kernel) and result writes are coalesced.
// Performance only: every kernel is order-independent up to fp64 summation
// order, and the mirrors undo the permutation.  Built on the device
// (pmx_setup.hip): the slot -> query order stays there (d_order) and is
// copied to the host only for a host mirror.
//
// Waves of the tile kernel (PMX_GRID_MODE=tile only): a wave takes up to 64
// consecutive slots but never crosses the boundary of an aligned Morton
// block of 2^L cells per side, so its queries never straddle two distant
// regions (a straddling wave would share one huge LDS box).  L is the
// smallest level whose wave count stays within `fill` (default 1.25,
// PMX_GRID_WAVE_FILL) of ceil(N / 64).
std::vector<uint32_t> tile_waves(const std::vector<unsigned long long>& key, int64_t N) {
    std::vector<uint32_t> waves;
    double fill = 1.25;
    if (const char* e = std::getenv("PMX_GRID_WAVE_FILL")) fill = std::max(1.0, std::atof(e));
    const int64_t full = (N + 63) / 64;
    auto cut = [&](int L, std::vector<uint32_t>* out) -> int64_t {
        int64_t W = 0;
        for (int64_t i = 0; i < N;) {
            const uint64_t blk = L >= 21 ? 0 : key[(size_t)i] >> (3 * L);
            int64_t j = i + 1;
            while (j < N && j - i < 64 && (L >= 21 ? 0 : key[(size_t)j] >> (3 * L)) == blk) ++j;
            if (out) out->push_back((uint32_t)i);
            ++W;
            i = j;
        }
        return W;
    };
    int L = 0;
    while (L < 21 && (double)cut(L, nullptr) > fill * (double)full) ++L;
    cut(L, &waves);
    waves.push_back((uint32_t)N);
    return waves;
}

// the host copy of the slot order (host mirrors only)
int host_order(pmx_ctx* c) {
    if (!c->has_order || (int64_t)c->slot_query.size() == c->N) return PMX_OK;
    c->slot_query.resize((size_t)c->N);
    HIPCHK(c, hipMemcpyAsync(c->slot_query.data(), c->d_order, sizeof(int32_t) * c->N, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PMX_OK;
}

// ------------------------------------------------------------------ clouds --
template <typename T>
int set_reference_impl(pmx_ctx* c, const T* feat, int rows, int64_t M, const T* normals) {
    if (rows != 3 && rows != 4) return fail(c, PMX_E_BAD_PARAM, "reference must have 3 (2-D) or 4 (3-D) rows");
    if (M <= 0) return fail(c, PMX_E_BAD_PARAM, "empty reference");
    if (M > (int64_t)0x7fffffff - kTile) return fail(c, PMX_E_BAD_PARAM, "reference larger than int32 ids");
    // the grid kernels address the reference with 32-bit byte offsets
    if ((M + kTile) * (int64_t)sizeof(P4<T>) >= ((int64_t)1 << 32))
        return fail(c, PMX_E_BAD_PARAM, "reference larger than 4 GiB of points (268M float / 134M double)");
    const int D = rows - 1;
    const int64_t M_pad = ((M + kTile - 1) / kTile) * kTile;
    int rc;
    if (c->d_ref) (void)hipFree(c->d_ref);
    c->d_ref = nullptr;
    HIPCHK(c, hipMalloc(&c->d_ref, sizeof(P4<T>) * M_pad));
    if ((rc = upload_raw(c, feat, sizeof(T) * (size_t)rows * M))) return rc;
    launch_pack_p4<T>((const T*)c->d_raw, rows, M, M_pad, (P4<T>*)c->d_ref, c->stream);
    if (c->d_nrm) (void)hipFree(c->d_nrm);
    c->d_nrm = nullptr;
    c->has_normals = normals != nullptr;
    if (normals) {
        HIPCHK(c, hipMalloc(&c->d_nrm, sizeof(P4<T>) * M));
        // (the raw buffer is reused: the copy is ordered after the pack on the stream)
        if ((rc = upload_raw(c, normals, sizeof(T) * (size_t)D * M))) return rc;
        launch_pack_nrm<T>((const T*)c->d_raw, D, M, (P4<T>*)c->d_nrm, c->stream);
    }
    HIPCHK(c, hipGetLastError());
    c->rows = rows;
    c->dim = D;
    c->M = M;
    c->M_pad = M_pad;
    c->have_match = false;
    c->grid_ready = false;
    // a resident reading keeps its slot order (any permutation is correct;
    // it was only chosen for the previous grid's locality)
    return build_grid<T>(c, M);
}

template <typename T>
int set_reading_impl(pmx_ctx* c, const T* feat, int rows, int64_t N, const T* T0) {
    if (c->rows == 0) return fail(c, PMX_E_STATE, "pmx_set_reference must be called first");
    if (rows != c->rows) return fail(c, PMX_E_BAD_PARAM, "reading and reference dimensions differ");
    if (N < 0) return fail(c, PMX_E_BAD_PARAM, "negative reading size");
    if (N > (int64_t)0x7fffffff) return fail(c, PMX_E_BAD_PARAM, "reading larger than int32 slots");
    const Mat4<T> M0 = embed<T>(T0, rows);
    int rc;
    const int64_t n1 = std::max<int64_t>(N, 1);
    c->has_radii = false;  // (a new reading: its radii, if any, follow)
    // raw P4 reading (pack), then the slot order, then T_refMean_dataIn
    void* d_p4 = nullptr;
    HIPCHK(c, hipMalloc(&d_p4, sizeof(P4<T>) * n1));
    std::unique_ptr<void, void (*)(void*)> free_p4(d_p4, [](void* p) { (void)hipFree(p); });
    if ((rc = upload_raw(c, feat, sizeof(T) * (size_t)rows * N))) return rc;
    launch_pack_p4<T>((const T*)c->d_raw, rows, N, N, (P4<T>*)d_p4, c->stream);
    if (c->d_rd) (void)hipFree(c->d_rd);
    c->d_rd = nullptr;
    HIPCHK(c, hipMalloc(&c->d_rd, sizeof(P4<T>) * n1));
    if (c->d_waves) (void)hipFree(c->d_waves);
    c->d_waves = nullptr;
    c->n_waves = 0;
    c->slot_query.clear();
    c->has_order = false;
    const bool order = c->grid_ready && N > 0 && !std::getenv("PMX_GRID_NOORDER");  // (knob: identity slot order)
    if (order) {
        // Morton order over the finest level's cells
        const GridLevel& L0 = c->lv(0);
        SetupShape s;
        for (int a = 0; a < 3; ++a) {
            s.lo[a] = L0.lo[a];
            s.g[a] = L0.dim[a];
        }
        s.h = L0.h;
        s.cells = (int64_t)s.g[0] * s.g[1] * s.g[2];
        const bool morton = s.g[0] <= (1 << 21) && s.g[1] <= (1 << 21) && s.g[2] <= (1 << 21);
        if ((rc = setup_room(c, N, std::max<int64_t>(c->setup_cells, 1)))) return rc;
        void* d_sorted = nullptr;
        HIPCHK(c, hipMalloc(&d_sorted, sizeof(P4<T>) * n1));
        std::unique_ptr<void, void (*)(void*)> free_sorted(d_sorted, [](void* p) { (void)hipFree(p); });
        const int r = reading_order_device<T>((const P4<T>*)d_p4, N, M0, s, morton, c->setup, (P4<T>*)d_sorted,
                                              c->stream);
        if (r) return fail(c, PMX_E_HIP, "reading order failed (" + std::to_string(r) + ")");
        size_t cap = c->order_bytes;
        if ((rc = ensure(c, (void**)&c->d_order, &cap, sizeof(int32_t) * n1))) return rc;
        c->order_bytes = cap;
        HIPCHK(c, hipMemcpyAsync(c->d_order, c->setup.idx_out, sizeof(int32_t) * N, hipMemcpyDeviceToDevice,
                                 c->stream));
        c->has_order = true;
        launch_transform<T>((const P4<T>*)d_sorted, (P4<T>*)c->d_rd, N, M0, c->stream);
        if (morton && c->grid_mode == 0) {  // the tile kernel's wave table (host, from the sorted keys)
            std::vector<unsigned long long> keys((size_t)N);
            HIPCHK(c, hipMemcpyAsync(keys.data(), c->setup.keys64_out, sizeof(unsigned long long) * N,
                                     hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            const std::vector<uint32_t> waves = tile_waves(keys, N);
            HIPCHK(c, hipMalloc((void**)&c->d_waves, sizeof(uint32_t) * waves.size()));
            HIPCHK(c, hipMemcpyAsync(c->d_waves, waves.data(), sizeof(uint32_t) * waves.size(),
                                     hipMemcpyHostToDevice, c->stream));
            c->n_waves = (int64_t)waves.size() - 1;
        }
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipStreamSynchronize(c->stream));  // (d_sorted is freed on return)
    } else if (N > 0) {
        launch_transform<T>((const P4<T>*)d_p4, (P4<T>*)c->d_rd, N, M0, c->stream);
        HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->N = N;
    c->N_total = N;
    c->N_max = N;
    // A new reading's first match has no previous match to adapt the level
    // from, and the initial pose is usually the worst aligned: a coarse level
    // walks few shells where the finest walks dozens (measured on MI355X, C3).
    // Any level answers exactly.
    if (c->adaptive && !c->levels.empty()) {
        int best = 0;
        for (int l = 0; l < (int)c->levels.size(); ++l)
            if (std::fabs(std::log(c->lv(l).ppc / c->first_ppc)) < std::fabs(std::log(c->lv(best).ppc / c->first_ppc)))
                best = l;
        c->level = best;
    }
    if (sharded(c)) {
        // global reading size and the largest shard (padding of all-gathers)
        double* tmp = c->d_result;
        double hv[2] = {(double)N, (double)N};
        HIPCHK(c, hipMemcpyAsync(tmp, hv, 2 * sizeof(double), hipMemcpyHostToDevice, c->stream));
        int rc2 = coll_allreduce(c, tmp, 1, PMX_COLL_F64, PMX_COLL_SUM);
        if (rc2 == PMX_OK) rc2 = coll_allreduce(c, tmp + 1, 1, PMX_COLL_F64, PMX_COLL_MAX);
        if (rc2) return rc2;
        HIPCHK(c, hipMemcpyAsync(hv, tmp, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        c->N_total = (int64_t)hv[0];
        c->N_max = (int64_t)hv[1];
    }
    c->have_match = false;
    return PMX_OK;
}

// ------------------------------------------------------------------- match --
template <typename T>
int match_impl(pmx_ctx* c, const T* Titer, int knn, double maxDist, uint64_t* visited) {
    if (!c->d_ref) return fail(c, PMX_E_STATE, "no reference (Matcher::init not called)");
    if (!c->d_rd && c->N > 0) return fail(c, PMX_E_STATE, "no reading");
    if (knn < 1 || knn > kMaxKnn) return fail(c, PMX_E_BAD_PARAM, "knn must be in [1, 256] on the GPU path");
    if (!(maxDist >= 0)) return fail(c, PMX_E_BAD_PARAM, "maxDist must be >= 0");
    const int64_t n = c->N * knn;
    size_t cap = (size_t)c->match_cap * tsize(c);
    if ((int64_t)c->match_cap < n || !c->d_dists) {
        size_t capd = 0, capi = 0, capw = 0;
        if (c->d_dists) (void)hipFree(c->d_dists);
        if (c->d_ids) (void)hipFree(c->d_ids);
        if (c->d_w) (void)hipFree(c->d_w);
        c->d_dists = nullptr;
        c->d_ids = nullptr;
        c->d_w = nullptr;
        int rc;
        if ((rc = ensure(c, &c->d_dists, &capd, sizeof(T) * (n > 0 ? n : 1)))) return rc;
        if ((rc = ensure(c, (void**)&c->d_ids, &capi, sizeof(int32_t) * (n > 0 ? n : 1)))) return rc;
        if ((rc = ensure(c, &c->d_w, &capw, sizeof(T) * (n > 0 ? n : 1)))) return rc;
        c->match_cap = n;
        c->safe_valid = false;
        (void)cap;
    }
    if (c->reuse_on && (c->safe_cap < c->N || !c->d_safe)) {
        if (c->d_safe) (void)hipFree(c->d_safe);
        c->d_safe = nullptr;
        size_t caps = 0;
        int rc;
        if ((rc = ensure(c, &c->d_safe, &caps, tsize(c) * (size_t)std::max<int64_t>(c->N, 1)))) return rc;
        c->safe_cap = std::max<int64_t>(c->N, 1);
        c->safe_valid = false;
    }
    const int64_t pe = match_part_elems<T>(c->N, c->M_pad, knn, c->cu_count);
    if (pe > c->part_cap) {
        size_t a = 0, b = 0;
        if (c->d_part_d) (void)hipFree(c->d_part_d);
        if (c->d_part_i) (void)hipFree(c->d_part_i);
        c->d_part_d = nullptr;
        c->d_part_i = nullptr;
        int rc;
        if ((rc = ensure(c, &c->d_part_d, &a, sizeof(T) * pe))) return rc;
        if ((rc = ensure(c, (void**)&c->d_part_i, &b, sizeof(int32_t) * pe))) return rc;
        c->part_cap = pe;
    }
    Mat4<T> Tm = embed<T>(Titer, c->rows);
    for (int i = 0; i < 16; ++i) {
        c->Tprev[i] = c->Tstep[i];  // (the previous match's: its warm start)
        c->Tstep[i] = (double)Tm.m[i];
    }
    const T md = (T)maxDist;
    const T maxR2 = md * md;  // libnabo squares the radius in T [ext]
    // reset the per-iteration error word and the pair / fallback counters
    // ([kBlkVisited, kBlkVisited + 16)); the grid match's counter-sum kernel
    // does both itself, which saves a fill launch per iteration
    const bool grid = !(c->search_type == 0 || !c->grid_ready);
    if (!grid)
        HIPCHK(c, hipMemsetAsync((char*)c->d_result + kBlkIterErr, 0, kBlkVisited + 16 - kBlkIterErr, c->stream));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->timing) {
        e0 = get_event(c);
        e1 = get_event(c);
    }
    if (c->search_type == 0 || !c->grid_ready) {
        if (knn > kLaneMaxK) {  // (the wave-per-query search over the whole reference, pmx_knn_wide.hip)
            if (e0) (void)hipEventRecord(e0, c->stream);
            launch_knn_wide<T>((const P4<T>*)c->d_ref, nullptr, nullptr, nullptr, c->M, (const P4<T>*)c->d_rd, c->N,
                               Tm, knn, maxR2, nullptr, (T*)c->d_dists, c->d_ids, nullptr, nullptr, nullptr, nullptr,
                               c->stream);
            if (e1) (void)hipEventRecord(e1, c->stream);
        } else {
            launch_match<T>((const P4<T>*)c->d_ref, c->M_pad, (const P4<T>*)c->d_rd, c->N, Tm, knn, maxR2,
                            (T*)c->d_dists, c->d_ids, (T*)c->d_part_d, c->d_part_i, c->part_cap, c->stream, e0, e1,
                            c->cu_count);
        }
        if (c->has_radii)
            launch_apply_radii<T>((T*)c->d_dists, c->d_ids, (const T*)c->d_radii, c->N, knn, c->stream);
        c->visited_host = (uint64_t)c->N * (uint64_t)c->M;
        c->ids_grid = false;
        c->safe_valid = false;
    } else {
        if (e0) (void)hipEventRecord(e0, c->stream);
        const GridLevel& L = c->lv(c->level);
        // warm start from the previous match of the same reading (same k):
        // its ids are positions in the level it ran on (in loop mode the
        // kernel takes that level from LoopCtl.hint_level)
        // temporal reuse: the output buffers hold this reading's previous
        // match (same k, same level) with its safe radii
        GridReuse<T> ru;
        const bool no_prev = !(c->safe_valid && c->have_match && c->ids_grid && c->knn == knn);
        if (c->reuse_on && c->grid_mode >= 1 && knn <= kLaneMaxK) {  // (the wide search keeps no safe radii)
            ru.mode = c->safe_valid && c->have_match && c->ids_grid && c->knn == knn && c->ids_level == c->level ? 2 : 1;
            ru.safe = (T*)c->d_safe;
            for (int i = 0; i < 16; ++i) ru.Tprev.m[i] = (T)c->Tprev[i];
        }
        // several ranks: the counter sum packs this rank's window segment,
        // the segments are all-gathered and every rank picks from the union
        SpecSel* spec = c->spec_now();
        c->spec_exchanged = false;
        unsigned long long* xseg = spec && sharded(c) ? c->d_specx : nullptr;
        launch_grid_match<T>(c->grid_mode, (const P4<T>*)L.gpts, L.gidx, L.gstart, L.lo, L.h, L.dim,
                             (const P4<T>*)c->d_rd, c->N, c->d_waves, c->n_waves, Tm, knn, maxR2, c->tile_max,
                             (T*)c->d_dists, c->d_ids, c->d_vpart, c->d_visited, c->d_iter_err, ru, loop_ctl(c),
                             (const GridDesc<T>*)c->d_gdesc, spec, c->d_sel, xseg,
                             c->has_radii ? (const T*)c->d_radii : nullptr, no_prev && c->reuse_on, e1, c->stream);
        if (xseg) {
            if (c->N <= 0)  // (no match kernel ran: an empty segment)
                HIPCHK(c, hipMemsetAsync(xseg, 0, kSpecXHdr * sizeof(unsigned long long), c->stream));
            int rc = coll_allgather(c, xseg, xseg + kSpecXStride, kSpecXStride * sizeof(unsigned long long));
            if (rc) return rc;
            launch_spec_pick<T>(xseg + kSpecXStride, c->nranks, spec, c->d_sel, loop_ctl(c), c->stream);
            c->spec_exchanged = true;
        }
        c->safe_valid = ru.mode != 0;
        c->visited_host = 0;
        c->ids_grid = true;
        c->ids_level = c->level;
    }
    HIPCHK(c, hipGetLastError());
    if (e0 && e1) c->ev_pending.emplace_back(e0, e1);
    c->knn = knn;
    c->have_match = true;
    c->chain_n = 0;  // new matches: the outlier chain starts over
    c->w_valid = false;
    if (visited) *visited = c->visited_host;
    return PMX_OK;
}

// ----------------------------------------------------------------- outliers --
// Several ranks, after the window segments were exchanged and picked from:
// 1 when the radix passes (and their histogram all-reduces) can be skipped —
// the window resolved the limit, or the device loop has converged (the pick
// then did not run).  Every rank picked from the same union and read the same
// all-reduced system, so every rank takes the same decision and the
// collective sequences stay matched.  Costs one stream synchronisation.
int sharded_window_resolved(pmx_ctx* c, SpecSel* spec) {
    if (!c->h_flags) HIPCHK(c, hipHostMalloc((void**)&c->h_flags, 64, hipHostMallocDefault));
    c->h_flags[0] = 0;
    c->h_flags[1] = 0;
    HIPCHK(c, hipMemcpyAsync(c->h_flags, &spec->hit, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    const LoopCtl* ctl = loop_ctl(c);
    if (ctl) HIPCHK(c, hipMemcpyAsync(c->h_flags + 1, &ctl->done, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (c->h_flags[1]) c->shard_done_seen = true;  // (the loop's later iterations are not enqueued)
    return c->h_flags[0] != 0 || c->h_flags[1] != 0 ? 1 : 0;
}

template <typename T>
int quantile_select(pmx_ctx* c, const T* d, int64_t n, double ratio, const double* ratio_dev, SelectState* st,
                    SpecSel* spec = nullptr) {
    // (no state reset: pass 0 starts a fresh select)
    const int passes = select_passes<T>();
    if (spec && c->spec_exchanged && sharded(c)) {
        c->spec_exchanged = false;
        const int r = sharded_window_resolved(c, spec);
        if (r < 0) return r;
        if (r == 1) return PMX_OK;  // (the pass kernels would return at spec->hit; no histogram exchange)
    }
    if (!sharded(c)) {
        // every pass in one launch (a no-op launch when the window resolved it)
        const int64_t g = select_all_blocks(n);
        if (g != c->selx_grid) {  // (the arrival generations assume a fixed block count)
            HIPCHK(c, hipMemsetAsync(c->d_selx, 0, selx_bytes(), c->stream));
            c->selx_grid = g;
        }
        launch_select_all<T>(d, n, c->d_selx, st, ratio, ratio_dev, c->d_iter_err, loop_ctl(c), spec, c->stream);
    } else {
        for (int p = 0; p < passes; ++p) {
            // the histogram is all-reduced between the two halves of a pass
            launch_select_hist<T>(d, n, c->d_hist, st, p, loop_ctl(c), spec, c->stream);
            int rc = coll_allreduce(c, c->d_hist, select_bins(p, 8 * (int)sizeof(T)), PMX_COLL_U32, PMX_COLL_SUM);
            if (rc) return rc;
            launch_select_pick<T>(c->d_hist, st, p, ratio, ratio_dev, c->d_iter_err, loop_ctl(c), spec, c->stream);
        }
    }
    HIPCHK(c, hipGetLastError());
    return PMX_OK;
}

int check_match(pmx_ctx* c) {
    if (!c->have_match) return fail(c, PMX_E_STATE, "pmx_match must be called first");
    return PMX_OK;
}

// the reference layout the current match ids index
const void* match_ref(const pmx_ctx* c) { return c->ids_grid ? c->lv(c->ids_level).gpts : c->d_ref; }
// the point-to-plane gather: a grid level's interleaved records (stride 2)
// or the reference and its normals (stride 1)
const void* match_pn(const pmx_ctx* c) { return c->ids_grid ? c->lv(c->ids_level).gpn : c->d_ref; }
const void* match_nrm(const pmx_ctx* c) {
    return c->ids_grid ? (const void*)((const char*)c->lv(c->ids_level).gpn + (c->dtype == PMX_F64 ? 32 : 16)) : c->d_nrm;
}
int match_rs(const pmx_ctx* c) { return c->ids_grid ? 2 : 1; }

// Adaptive grid level for the next match, from the pairs this match
// evaluated per query and per point-per-cell (~ occupied cells visited):
// beyond ~24 cells the search walked outer shells (misaligned clouds, large
// k) and the next coarser level is cheaper; below ~5 a finer one is.  Any
// level gives the identical exact result.
// With temporal reuse the level is judged on the full searches only (a
// certified query evaluates its k pairs whatever the level), and kept while
// fewer than 1/16 of the queries needed one: a level change restarts the
// reuse chain.
void choose_level(pmx_ctx* c, uint64_t visited, uint64_t full) {
    if (!c->adaptive || !c->ids_grid || c->levels.size() < 2 || c->N <= 0 || c->knn <= 0) return;
    const int l = c->ids_level;
    double q = (double)c->N, v = (double)visited;
    if (c->safe_valid) {
        if ((double)full * 16.0 < q) return;
        v -= (double)c->knn * (q - (double)full);
        q = (double)full;
    }
    const double cells = v / (q * c->lv(l).ppc);
    ++c->match_count;
    c->level_cells[(size_t)l] = cells;
    c->level_seen[(size_t)l] = c->match_count;
    int next = l;
    if (cells > 32.0 && l + 1 < (int)c->levels.size()) {
        next = l + 1;  // outer shells dominate: larger cells
    } else if (cells < 16.0 && l > 0) {
        // the 3x3x3 block sufficed: smaller cells evaluate fewer pairs, unless
        // the finer level was just seen walking shells (no ping-pong)
        const bool recent = c->level_seen[(size_t)l - 1] > 0 && c->match_count - c->level_seen[(size_t)l - 1] <= 3;
        if (!(recent && c->level_cells[(size_t)l - 1] > 32.0)) next = l - 1;
    }
    c->level = next;
}

// slot-major device array -> query-major host array (the reference's order)
template <typename V>
int unpermute(pmx_ctx* c, const std::vector<V>& src, V* dst, int k) {
    const int64_t N = c->N;
    if (!c->has_order) {
        std::memcpy(dst, src.data(), sizeof(V) * (size_t)(N * k));
        return PMX_OK;
    }
    const int rc = host_order(c);
    if (rc) return rc;
    for (int64_t s = 0; s < N; ++s) {
        const int64_t qi = c->slot_query[(size_t)s];
        for (int j = 0; j < k; ++j) dst[qi * k + j] = src[(size_t)(s * k + j)];
    }
    return PMX_OK;
}

// record predicate `pos` of the weight chain (position 0 starts a new chain)
void chain_set(pmx_ctx* c, int pos, int type, double thr) {
    if (pos == 0 || c->rb_pos >= pos) c->rb_pos = -1;  // (a new chain, or the robust filter's position rewritten)
    c->chain_n = pos + 1;
    c->chain_type[pos] = type;
    c->chain_thr[pos] = thr;
    c->w_valid = false;
}

template <typename T>
WChain<T> chain_of(const pmx_ctx* c) {
    WChain<T> w;
    if (c->chain_n == 0) {  // no filter applied: the empty chain's default (dist != inf)
        w.n = 1;
        w.type[0] = kWPDefault;
        return w;
    }
    w.n = c->chain_n;
    for (int i = 0; i < c->chain_n; ++i) {
        w.type[i] = c->chain_type[i];
        w.thr[i] = (T)c->chain_thr[i];
        w.st[i] = c->sel_slot(i);
    }
    if (c->rb_pos >= 0 && c->rb_pos < c->chain_n) {
        w.robust = 1;
        w.rb_fct = c->rb_fct;
        w.rb_k = (T)c->rb_k;
        w.rb_sqa = (T)c->rb_sqa;
        w.rb_scale = c->rob_scale(c->rb_pos);
        w.rb_p2pl = c->rb_p2pl;
    }
    return w;
}

// OutlierFilters::compute (OutlierFilter.cpp:63-103): filter `chain_pos` of
// the chain.  Quantile filters resolve their threshold on the device now;
// the 0/1 weights themselves are evaluated inline by the minimiser.
template <typename T>
int outlier_impl(pmx_ctx* c, int kind, int chain_pos, double p0, double p1, double p2) {
    int rc = check_match(c);
    if (rc) return rc;
    if (chain_pos < 0 || chain_pos >= kMaxChain) return fail(c, PMX_E_BAD_PARAM, "outlier chain longer than 8 filters");
    if (chain_pos > c->chain_n) return fail(c, PMX_E_BAD_PARAM, "outlier chain positions must be consecutive");
    const int64_t n = c->N * c->knn;
    const T* d = (const T*)c->d_dists;
    SelectState* slot = c->sel_slot(chain_pos);
    switch (kind) {
    case 0:  // default: empty chain, w = (dist != inf)
        chain_set(c, chain_pos, kWPDefault, 0.0);
        break;
    case 1:  // Null
        chain_set(c, chain_pos, kWPNull, 0.0);
        break;
    case 2: {  // MaxDist: w = d <= maxDist^2 (OutlierFiltersImpl.cpp:66-81)
        if (!(p0 >= 1e-7)) return fail(c, PMX_E_BAD_PARAM, "MaxDistOutlierFilter: maxDist < 1e-7");
        const T m = (T)p0;
        const T m2 = (T)std::pow((double)m, 2.0);
        chain_set(c, chain_pos, kWPLe, (double)m2);
        break;
    }
    case 3: {  // MinDist: w = d >= minDist^2 (OutlierFiltersImpl.cpp:87-100)
        if (!(p0 >= 1e-7)) return fail(c, PMX_E_BAD_PARAM, "MinDistOutlierFilter: minDist < 1e-7");
        const T m = (T)p0;
        const T m2 = (T)std::pow((double)m, 2.0);
        chain_set(c, chain_pos, kWPGe, (double)m2);
        break;
    }
    case 4: {  // MedianDist: limit = factor * quantile(0.5)
        if ((rc = quantile_select<T>(c, d, n, 0.5, nullptr, slot, chain_pos == 0 ? c->spec_now() : nullptr)))
            return rc;
        chain_set(c, chain_pos, kWPState, (double)(T)p0);
        break;
    }
    case 5: {  // TrimmedDist: limit = quantile(ratio)
        if (!(p0 >= 1e-7 && p0 <= 1.0)) return fail(c, PMX_E_BAD_PARAM, "TrimmedDistOutlierFilter: ratio out of [1e-7, 1]");
        if ((rc = quantile_select<T>(c, d, n, p0, nullptr, slot, chain_pos == 0 ? c->spec_now() : nullptr)))
            return rc;
        chain_set(c, chain_pos, kWPState, 1.0);
        break;
    }
    case 6: {  // VarTrimmedDist
        const T minR = (T)p0, maxR = (T)p1, lam = (T)p2;
        if (!(minR < maxR)) return fail(c, PMX_E_BAD_PARAM, "VarTrimmedDistOutlierFilter: minRatio should be smaller than maxRatio");
        const T* dsrc = d;
        int64_t nsrc = n;
        if (sharded(c)) {
            const int64_t per = c->N_max * c->knn;
            const size_t need = sizeof(T) * (size_t)per * (c->nranks + 1);
            if ((rc = ensure(c, &c->d_gather, &c->gather_bytes, need))) return rc;
            T* send = (T*)c->d_gather + (size_t)per * c->nranks;
            // local shard, padded with +inf (excluded by the filter) to the largest shard
            HIPCHK(c, hipMemcpyAsync(send, d, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));
            if (per > n) {
                std::vector<T> inf((size_t)(per - n), std::numeric_limits<T>::infinity());
                HIPCHK(c, hipMemcpyAsync(send + n, inf.data(), sizeof(T) * (per - n), hipMemcpyHostToDevice, c->stream));
                HIPCHK(c, hipStreamSynchronize(c->stream));
            }
            if ((rc = coll_allgather(c, send, c->d_gather, sizeof(T) * (size_t)per))) return rc;
            dsrc = (const T*)c->d_gather;
            nsrc = per * c->nranks;
        }
        const int points_nbr = (int)(c->N_total * c->knn);
        const int minEl = (int)std::floor(minR * (T)points_nbr);
        const int maxEl = (int)std::floor(maxR * (T)points_nbr);
        const int cnt = maxEl - minEl;
        if (cnt <= 0) return fail(c, PMX_E_BAD_PARAM, "VarTrimmedDistOutlierFilter: empty ratio range");
        if (c->deno_pts != points_nbr || c->deno_min != minEl || c->deno_max != maxEl ||
            !(c->deno_lambda == (double)lam)) {
            // pow(id / points_nbr, lambda) in T on the host: the same libm call
            // as the reference's Eigen array pow (OutlierFiltersImpl.cpp:209)
            std::vector<T> tab((size_t)cnt);
            for (int j = 0; j < cnt; ++j) {
                const T id = (T)(minEl + 1 + j);
                const T ratio = id / (T)points_nbr;
                tab[j] = std::pow(ratio, lam);
            }
            if ((rc = ensure(c, &c->d_deno, &c->deno_bytes, sizeof(T) * cnt))) return rc;
            HIPCHK(c, hipMemcpyAsync(c->d_deno, tab.data(), sizeof(T) * cnt, hipMemcpyHostToDevice, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            c->deno_pts = points_nbr;
            c->deno_min = minEl;
            c->deno_max = maxEl;
            c->deno_lambda = (double)lam;
        }
        const size_t need = vartrim_scratch_bytes<T>(nsrc);
        if ((rc = ensure(c, &c->d_vt, &c->vt_bytes, need))) return rc;
        launch_vartrim<T>(dsrc, nsrc, points_nbr, minR, maxR, (const T*)c->d_deno, c->d_vt, c->vt_bytes, c->d_ratio,
                          c->d_iter_err, loop_ctl(c), c->stream);
        HIPCHK(c, hipGetLastError());
        if ((rc = quantile_select<T>(c, d, n, 0.0, c->d_ratio, slot))) return rc;
        chain_set(c, chain_pos, kWPState, 1.0);
        break;
    }
    default:
        return fail(c, PMX_E_BAD_PARAM, "unknown outlier filter");
    }
    HIPCHK(c, hipGetLastError());
    return PMX_OK;
}

// RobustOutlierFilter::robustFiltering (OutlierFiltersImpl.cpp:494-598): the
// scale of this call on the device, then the filter joins the chain as its
// real-valued factor (evaluated inline by the weighted reductions)
template <typename T>
int outlier_robust_impl(pmx_ctx* c, int pos, int fct, double tuning, double approx, int mode, double target,
                        int p2pl) {
    int rc = check_match(c);
    if (rc) return rc;
    if (pos < 0 || pos >= kMaxChain) return fail(c, PMX_E_BAD_PARAM, "outlier chain longer than 8 filters");
    if (pos > c->chain_n) return fail(c, PMX_E_BAD_PARAM, "outlier chain positions must be consecutive");
    if (fct < kRFCauchy || fct > kRFStudent) return fail(c, PMX_E_BAD_PARAM, "Invalid robust function name.");
    if (mode < kRSNone || mode > kRSKeep) return fail(c, PMX_E_BAD_PARAM, "Invalid scale estimator name.");
    if (c->rb_pos >= 0 && c->rb_pos < pos && pos <= c->chain_n)
        return fail(c, PMX_E_BAD_PARAM, "one RobustOutlierFilter per outlier chain on this path");
    if (p2pl && !c->has_normals)
        return fail(c, PMX_E_BAD_PARAM, "RobustOutlierFilter point2plane requires \"normals\" on the reference");
    if (p2pl && c->dim != 3)  // (computePointToPlaneDistance reads 3 feature rows, :472-484)
        return fail(c, PMX_E_BAD_PARAM, "RobustOutlierFilter point2plane: 3-D clouds only");
    if (!c->d_rob) {
        HIPCHK(c, hipMalloc(&c->d_rob, 512));
        HIPCHK(c, hipMemsetAsync(c->d_rob, 0, 512, c->stream));
    }
    const int64_t n = c->N * c->knn;
    const T* d = (const T*)c->d_dists;
    SelectState* slot = c->sel_slot(pos);
    double* scale = c->rob_scale(pos);
    int smode = mode;
    switch (mode) {
    case kRSMad:  // Matches::getMedianAbsDeviation (Matches.cpp:88-122)
        if ((rc = quantile_select<T>(c, d, n, kRatioMedianIndex, nullptr, slot))) return rc;
        if ((rc = ensure(c, &c->d_rdev, &c->rdev_bytes, sizeof(T) * (size_t)(n > 0 ? n : 1)))) return rc;
        launch_abs_dev<T>(d, n, slot, (T*)c->d_rdev, c->stream);
        if ((rc = quantile_select<T>(c, (const T*)c->d_rdev, n, kRatioMedianIndex, nullptr, c->rob_sel()))) return rc;
        launch_robust_scale<T>(kRSMad, c->rob_sel(), nullptr, 0, 0.0, scale, c->stream);
        smode = -1;
        break;
    case kRSStd: {  // Matches::getStandardDeviation (Matches.cpp:124-129) over all k x N
        double* sums = c->rob_sums();
        const int64_t nt = c->N_total * c->knn;  // (the mean over every rank's distances)
        launch_moment<T>(d, n, 0, sums, c->d_partials, nt, c->stream);
        launch_finalize(c->d_partials, kRedBlocks, 1, sums, loop_ctl(c), c->stream);
        if ((rc = allreduce_f64(c, sums, 1))) return rc;
        launch_moment<T>(d, n, 1, sums, c->d_partials, nt, c->stream);
        launch_finalize(c->d_partials, kRedBlocks, 1, sums + 1, loop_ctl(c), c->stream);
        if ((rc = allreduce_f64(c, sums + 1, 1))) return rc;
        launch_robust_scale<T>(kRSStd, nullptr, sums, c->N_total * c->knn, 0.0, scale, c->stream);
        smode = -1;
        break;
    }
    case kRSBergFirst:  // 1.9 sqrt(getDistsQuantile(0.5))
        if ((rc = quantile_select<T>(c, d, n, 0.5, nullptr, slot))) return rc;
        launch_robust_scale<T>(kRSBergFirst, slot, nullptr, 0, 0.0, scale, c->stream);
        smode = -1;
        break;
    default: break;
    }
    if (smode >= 0) launch_robust_scale<T>(smode, nullptr, nullptr, 0, target, scale, c->stream);
    chain_set(c, pos, kWPRobust, 0.0);
    c->rb_pos = pos;
    c->rb_fct = fct;
    c->rb_k = (double)(T)tuning;
    // squaredApproximation = pow(approximation, 2) in T (:400)
    c->rb_sqa = std::isinf(approx) ? INFINITY : (double)(T)std::pow((double)(T)approx, 2.0);
    c->rb_p2pl = p2pl;
    HIPCHK(c, hipGetLastError());
    return PMX_OK;
}

template <typename T>
int set_radii_impl(pmx_ctx* c, const T* radii) {
    if (!radii) {
        c->has_radii = false;
        return PMX_OK;
    }
    if (!c->d_rd && c->N > 0) return fail(c, PMX_E_STATE, "pmx_set_reading must be called first");
    const int64_t n1 = std::max<int64_t>(c->N, 1);
    int rc;
    if ((rc = ensure(c, &c->d_radii, &c->radii_bytes, 2 * sizeof(T) * (size_t)n1))) return rc;
    T* raw = (T*)c->d_radii + n1;  // (upload half, then the slot-order half)
    HIPCHK(c, hipMemcpyAsync(raw, radii, sizeof(T) * (size_t)c->N, hipMemcpyHostToDevice, c->stream));
    launch_gather_scalar<T>(raw, c->has_order ? c->d_order : nullptr, c->N, (T*)c->d_radii, c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (the caller's buffer may go)
    c->has_radii = true;
    c->safe_valid = false;  // (the previous match used other radii)
    return PMX_OK;
}

template <typename T>
int robust_scale_impl(pmx_ctx* c, int pos, double* scale) {
    if (pos < 0 || pos >= kMaxChain || !c->d_rob) return fail(c, PMX_E_STATE, "no RobustOutlierFilter scale at this position");
    HIPCHK(c, hipMemcpyAsync(scale, c->rob_scale(pos), sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PMX_OK;
}

// -------------------------------------------------------------- minimizers --
// After a select_all wait timed out, some blocks left without arriving at the
// later passes: the arrival counters are off a multiple of the grid and some
// bins were never zeroed.  Start the next launch from zeroed state.
int select_reset(pmx_ctx* c) {
    HIPCHK(c, hipMemsetAsync(c->d_selx, 0, selx_bytes(), c->stream));
    c->selx_grid = 0;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PMX_OK;
}

// one D2H copy of the iteration block, then a stream sync
int readback(pmx_ctx* c) {
    HIPCHK(c, hipMemcpyAsync(c->h_result, c->d_result, kBlkCopy, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    return PMX_OK;
}
int host_iter_err(const pmx_ctx* c) {
    int e = 0;
    std::memcpy(&e, (const char*)c->h_result + kBlkIterErr, sizeof(int));
    return e;
}
double host_limit(const pmx_ctx* c) {
    double v = 0;
    std::memcpy(&v, (const char*)c->h_result + kBlkSel + offsetof(SelectState, limit), sizeof(double));
    return v;
}

void fill_stats(const pmx_ctx* c, pmx_stats* st, double kept, double nz, double rm, double rp, double sw,
                double limit) {
    if (!st) return;
    st->kept = (int64_t)kept;
    st->nonzero_weights = (int64_t)nz;
    st->rejected_matches = (int64_t)rm;
    st->rejected_points = (int64_t)rp;
    st->sum_w = sw;
    st->limit = limit;
    st->n_total = c->N_total * c->knn;
    unsigned long long v = 0;
    std::memcpy(&v, (const char*)c->h_result + kBlkVisited, sizeof(v));
    st->visited = c->visited_host ? (int64_t)c->visited_host : (int64_t)v;
    std::memcpy(&v, (const char*)c->h_result + kBlkVisited + 8, sizeof(v));
    st->fallback_queries = c->visited_host ? 0 : (int64_t)v;
}

// after a readback: adapt the grid level of the next match
void after_readback(pmx_ctx* c) {
    if (c->visited_host) return;
    unsigned long long v = 0, f = 0;
    std::memcpy(&v, (const char*)c->h_result + kBlkVisited, sizeof(v));
    std::memcpy(&f, (const char*)c->h_result + kBlkVisited + 8, sizeof(f));
    choose_level(c, v, f);
}

// the chain's weights into d_w (the host mirror; a point-to-plane robust
// distance under the point-to-point minimiser)
template <typename T>
int materialise_weights(pmx_ctx* c) {
    if (c->w_valid) return PMX_OK;
    launch_weights_chain<T>((const T*)c->d_dists, (T*)c->d_w, c->N * c->knn, chain_of<T>(c), (const P4<T>*)c->d_rd,
                            step_mat<T>(c), (const P4<T>*)match_pn(c), (const P4<T>*)match_nrm(c), match_rs(c),
                            c->d_ids, c->knn, c->stream);
    HIPCHK(c, hipGetLastError());
    c->w_valid = true;
    return PMX_OK;
}

// the point-to-plane system into the iteration block (no host sync)
template <typename T>
int p2plane_enqueue(pmx_ctx* c) {
    const WChain<T> chain = chain_of<T>(c);
    const int NV = chain.robust ? p2plane_nv_full(c->dim) : p2plane_nv(c->dim);
    Mat4<T> Tm = step_mat<T>(c);
    launch_p2plane_partial<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_pn(c), (const P4<T>*)match_nrm(c),
                              match_rs(c), (const T*)c->d_dists, c->d_ids, chain, c->knn, c->N, c->dim, c->d_partials,
                              loop_ctl(c), (const GridDesc<T>*)c->d_gdesc, c->stream);
    launch_finalize(c->d_partials, kRedBlocks, NV, c->d_result, loop_ctl(c), c->stream);
    HIPCHK(c, hipGetLastError());
    return allreduce_f64(c, c->d_result, NV);
}

// the point-to-point sums, means and cross-covariance (no host sync);
template <typename T>
int p2point_enqueue(pmx_ctx* c) {
    Mat4<T> Tm = step_mat<T>(c);
    WChain<T> chain = chain_of<T>(c);
    if (chain.robust && chain.rb_p2pl) {  // (the point-to-point kernels carry no normals)
        const int rc = materialise_weights<T>(c);
        if (rc) return rc;
        chain.w_arr = (const T*)c->d_w;
    }
    const GridDesc<T>* gd = (const GridDesc<T>*)c->d_gdesc;
    launch_p2point_pass1<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_ref(c), (const T*)c->d_dists, c->d_ids,
                            chain, c->knn, c->N, c->d_partials, loop_ctl(c), gd, c->stream);
    launch_finalize(c->d_partials, kRedBlocks, 11, c->d_result, loop_ctl(c), c->stream);
    int rc = allreduce_f64(c, c->d_result, 11);
    if (rc) return rc;
    launch_p2point_means<T>(c->d_result, (T*)c->d_means, c->dim, loop_ctl(c), c->stream);
    launch_p2point_pass2<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_ref(c), (const T*)c->d_dists, c->d_ids,
                            chain, c->knn, c->N, (const T*)c->d_means, c->d_partials, loop_ctl(c), gd, c->stream);
    launch_finalize(c->d_partials, kRedBlocks, 9, c->d_result + 16, loop_ctl(c), c->stream);
    HIPCHK(c, hipGetLastError());
    return allreduce_f64(c, c->d_result + 16, 9);
}

template <typename T>
int p2plane_impl(pmx_ctx* c, double* A, double* b, pmx_stats* st) {
    int rc = check_match(c);
    if (rc) return rc;
    if (!c->has_normals)
        return fail(c, PMX_E_BAD_PARAM, "PointToPlaneErrorMinimizer requires \"normals\" on the reference");
    const int NF = c->dim == 3 ? 6 : 3;
    const bool full = c->rb_pos >= 0 && c->rb_pos < c->chain_n;  // (the weighted layout, see p2plane_enqueue)
    const int NS = full ? NF * NF : NF * (NF + 1) / 2;
    if ((rc = p2plane_enqueue<T>(c))) return rc;
    if ((rc = readback(c))) return rc;
    after_readback(c);
    const double* r = c->h_result;
    const int ierr = host_iter_err(c);
    const int o = NS + NF;
    fill_stats(c, st, r[o + 0], r[o + 1], r[o + 2], r[o + 3], r[o + 4], host_limit(c));
    if (ierr == PMX_E_EMPTY_QUANTILE) return fail(c, PMX_E_EMPTY_QUANTILE, "no outlier to filter");
    if (ierr == kSelTimeout) {
        (void)select_reset(c);
        return fail(c, PMX_E_HIP, "radix select: device wait timed out");
    }
    if (ierr) return fail(c, ierr, "quantile must be between 0 and 1");
    if (r[o + 1] == 0.0) return fail(c, PMX_E_NO_POINTS, "ErrorMnimizer: no point to minimize");
    if (r[o + 0] == 0.0) return fail(c, PMX_E_NO_POINTS, "ErrorMnimizer: no point to minimize");
    if (full) {
        for (int i = 0; i < NF * NF; ++i) A[i] = r[i];
    } else {  // mirror the upper triangle (exactly symmetric with 0/1 weights, see pmx_reduce.hip)
        int a = 0;
        for (int i = 0; i < NF; ++i)
            for (int j = i; j < NF; ++j, ++a) A[i * NF + j] = A[j * NF + i] = r[a];
    }
    for (int i = 0; i < NF; ++i) b[i] = -r[NS + i];
    return PMX_OK;
}

template <typename T>
int p2point_impl(pmx_ctx* c, double* mean_p, double* mean_q, double* m, pmx_stats* st) {
    int rc = check_match(c);
    if (rc) return rc;
    if ((rc = p2point_enqueue<T>(c))) return rc;
    if ((rc = readback(c))) return rc;
    after_readback(c);
    const double* r = c->h_result;
    const int ierr = host_iter_err(c);
    fill_stats(c, st, r[7], r[8], r[9], r[10], r[0], host_limit(c));
    if (ierr == PMX_E_EMPTY_QUANTILE) return fail(c, PMX_E_EMPTY_QUANTILE, "no outlier to filter");
    if (ierr == kSelTimeout) {
        (void)select_reset(c);
        return fail(c, PMX_E_HIP, "radix select: device wait timed out");
    }
    if (ierr) return fail(c, ierr, "quantile must be between 0 and 1");
    if (r[8] == 0.0 || r[7] == 0.0) return fail(c, PMX_E_NO_POINTS, "ErrorMnimizer: no point to minimize");
    T means[6];
    std::memcpy(means, (const char*)c->h_result + kBlkMeans, sizeof(T) * 6);
    const int D = c->dim;
    for (int i = 0; i < D; ++i) {
        mean_p[i] = (double)means[i];
        mean_q[i] = (double)means[3 + i];
    }
    for (int i = 0; i < D; ++i)
        for (int j = 0; j < D; ++j) m[i * D + j] = r[16 + i * 3 + j];
    return PMX_OK;
}

template <typename T>
int get_matches_impl(pmx_ctx* c, void* dists, int32_t* ids) {
    int rc = check_match(c);
    if (rc) return rc;
    const int64_t n = c->N * c->knn;
    if (n <= 0) return PMX_OK;
    std::vector<T> hd;
    std::vector<int32_t> hi;
    if (dists) {
        hd.resize((size_t)n);
        HIPCHK(c, hipMemcpyAsync(hd.data(), c->d_dists, sizeof(T) * n, hipMemcpyDeviceToHost, c->stream));
    }
    int32_t* d_map = nullptr;
    if (ids) {
        hi.resize((size_t)n);
        const int32_t* src = c->d_ids;
        if (c->ids_grid) {  // grid positions -> reference indices
            HIPCHK(c, hipMalloc((void**)&d_map, sizeof(int32_t) * n));
            launch_pos_to_index(c->d_ids, c->lv(c->ids_level).gidx, d_map, n, c->stream);
            HIPCHK(c, hipGetLastError());
            src = d_map;
        }
        HIPCHK(c, hipMemcpyAsync(hi.data(), src, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
    }
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (d_map) (void)hipFree(d_map);
    HIPCHK(c, e);
    if (dists && (rc = unpermute<T>(c, hd, (T*)dists, c->knn))) return rc;
    if (ids && (rc = unpermute<int32_t>(c, hi, ids, c->knn))) return rc;
    return PMX_OK;
}

template <typename T>
int get_weights_impl(pmx_ctx* c, void* w) {
    int rc = check_match(c);
    if (rc) return rc;
    const int64_t n = c->N * c->knn;
    if (n <= 0) return PMX_OK;
    if ((rc = materialise_weights<T>(c))) return rc;
    std::vector<T> hw((size_t)n);
    HIPCHK(c, hipMemcpyAsync(hw.data(), c->d_w, sizeof(T) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if ((rc = unpermute<T>(c, hw, (T*)w, c->knn))) return rc;
    return PMX_OK;
}

// ------------------------------------------------------------ device loop --
// pmx_loop_*: whole ICP iterations enqueued back to back (pmx_loop.hip).  The
// host checks the stop flag once per batch of kLoopBatch iterations while the
// next batch is already queued, so the GPU never waits for the host; after a
// stop the queued iterations return at once (every kernel reads LoopCtl.done).
constexpr int kLoopBatch = 4;
// pinned status slot s (a copy of the device status block)
const char* stat_slot(const pmx_ctx* c, int s) { return (const char*)c->h_loop + (size_t)s * kStatBytes; }


template <typename T>
int loop_begin_impl(pmx_ctx* c, const pmx_loop_cfg* cfg, const T* T0) {
    if (!c->d_ref) return fail(c, PMX_E_STATE, "no reference (Matcher::init not called)");
    if (!c->d_rd && c->N > 0) return fail(c, PMX_E_STATE, "no reading");
    if (c->search_type == 0 || !c->grid_ready || c->grid_mode == 0)
        return fail(c, PMX_E_BAD_PARAM, "device loop: needs the per-lane grid matcher (searchType 1 or 2)");
    if (cfg->knn < 1 || cfg->knn > kMaxKnn) return fail(c, PMX_E_BAD_PARAM, "knn must be in [1, 256] on the GPU path");
    if (!(cfg->max_dist >= 0)) return fail(c, PMX_E_BAD_PARAM, "maxDist must be >= 0");
    if (cfg->n_filters < 0 || cfg->n_filters > kMaxChain)
        return fail(c, PMX_E_BAD_PARAM, "device loop: at most 8 outlier filters");
    for (int i = 0; i < cfg->n_filters; ++i) {
        const int k = cfg->filter_kind[i];
        const double* p = cfg->filter_p[i];
        if (k < PMX_FILTER_DEFAULT || k > PMX_FILTER_VARTRIMMED || (k == PMX_FILTER_DEFAULT && i != 0))
            return fail(c, PMX_E_BAD_PARAM, "device loop: unknown outlier filter");
        if ((k == PMX_FILTER_MAXDIST || k == PMX_FILTER_MINDIST) && !(p[0] >= 1e-7))
            return fail(c, PMX_E_BAD_PARAM, "device loop: distance threshold < 1e-7");
        if (k == PMX_FILTER_TRIMMED && !(p[0] >= 1e-7 && p[0] <= 1.0))
            return fail(c, PMX_E_BAD_PARAM, "TrimmedDistOutlierFilter: ratio out of [1e-7, 1]");
        if (k == PMX_FILTER_VARTRIMMED && !((T)p[0] < (T)p[1]))
            return fail(c, PMX_E_BAD_PARAM, "VarTrimmedDistOutlierFilter: minRatio should be smaller than maxRatio");
    }
    if (cfg->minimizer != 0 && cfg->minimizer != 1) return fail(c, PMX_E_BAD_PARAM, "device loop: unknown minimizer");
    if (cfg->minimizer == 0 && !c->has_normals)
        return fail(c, PMX_E_BAD_PARAM, "PointToPlaneErrorMinimizer requires \"normals\" on the reference");
    if (cfg->n_checkers < 0 || cfg->n_checkers > kMaxCheckers)
        return fail(c, PMX_E_BAD_PARAM, "device loop: at most 8 transformation checkers");
    for (int i = 0; i < cfg->n_checkers; ++i) {
        const int k = cfg->checker_kind[i];
        if (k < PMX_CHECK_COUNTER || k > PMX_CHECK_BOUND)
            return fail(c, PMX_E_BAD_PARAM, "device loop: unknown transformation checker");
        const double sl = cfg->checker_p[i][2];
        if (k == PMX_CHECK_DIFFERENTIAL && !(sl >= 0 && sl < kLoopHist && sl == std::floor(sl)))
            return fail(c, PMX_E_BAD_PARAM, "device loop: smoothLength must be an integer in [0, 63]");
    }
    if (c->levels.size() > (size_t)kMaxLevels) return fail(c, PMX_E_BAD_PARAM, "device loop: at most 8 grid levels");
    LoopCfg d{};
    d.rows = c->rows;
    d.minimizer = cfg->minimizer;
    d.n_checkers = cfg->n_checkers;
    for (int i = 0; i < cfg->n_checkers; ++i) {
        d.checker_kind[i] = cfg->checker_kind[i];
        for (int j = 0; j < 3; ++j) d.checker_p[i][j] = cfg->checker_p[i][j];
    }
    d.adaptive = c->adaptive ? 1 : 0;
    d.reuse = c->reuse_on && c->grid_mode >= 1 ? 1 : 0;
    d.knn = cfg->knn;
    d.n_levels = (int)c->levels.size();
    for (int l = 0; l < d.n_levels; ++l) d.level_ppc[l] = c->lv(l).ppc;
    d.n_local = c->N;
    int rc;
    size_t cap = 0;
    (void)cap;  // (LoopState lives in the status block)
    cap = 0;
    if (!c->d_loop_T0 && (rc = ensure(c, &c->d_loop_T0, &cap, 16 * sizeof(double)))) return rc;
    // pinned: two status-block slots (the batches in flight)
    if (!c->h_loop) HIPCHK(c, hipHostMalloc(&c->h_loop, 2 * kStatBytes, hipHostMallocDefault));
    for (hipEvent_t& e : c->loop_ev)
        if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->loop_cfg = *cfg;
    c->loop_dev = d;
    const int rr = c->rows * c->rows;
    HIPCHK(c, hipMemcpyAsync(c->d_loop_T0, T0, sizeof(T) * rr, hipMemcpyHostToDevice, c->stream));
    // the first loop match may reuse the last classic one
    const int prev_level =
        c->reuse_on && c->safe_valid && c->have_match && c->ids_grid && c->knn == cfg->knn ? c->ids_level : -1;
    launch_loop_init<T>(c->d_ctl, (LoopState<T>*)c->d_loop, d, (const T*)c->d_loop_T0, c->level, prev_level,
                        c->Tstep, c->stream);
    // quantile window: a fresh window each loop (the first iteration runs the
    // radix passes, which centre the window for the next)
    const int k0 = cfg->n_filters > 0 ? cfg->filter_kind[0] : -1;
    c->spec_on = c->spec_allowed &&
                 (k0 == PMX_FILTER_TRIMMED || k0 == PMX_FILTER_MEDIANDIST);
    if (c->spec_on) {
        if (!c->d_spec) {
            HIPCHK(c, hipMalloc((void**)&c->d_spec, sizeof(SpecSel)));
            HIPCHK(c, hipMalloc(&c->d_spec_keys, sizeof(unsigned long long) * kSpecCap));
        }
        if (sharded(c) && !c->d_specx)
            HIPCHK(c, hipMalloc((void**)&c->d_specx, sizeof(unsigned long long) * kSpecXStride * (c->nranks + 1)));
        SpecSel init{};
        init.keys = c->d_spec_keys;
        init.ratio = (double)(T)(k0 == PMX_FILTER_TRIMMED ? cfg->filter_p[0][0] : 0.5);
        c->spec_init = init;
        HIPCHK(c, hipMemcpyAsync(c->d_spec, &c->spec_init, sizeof(SpecSel), hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // (T0 may be a stack buffer of the caller)
    c->loop_issued = 0;
    c->loop_iters = 0;
    c->loop_done = false;
    c->shard_done_seen = false;
    c->loop_begun = true;
    return PMX_OK;
}

// trace room for `iters` iterations (the enqueued loop_step kernels hold the
// old pointer: drain the stream before the old buffer goes)
template <typename T>
int loop_trace_room(pmx_ctx* c, int64_t iters) {
    if (iters <= c->trace_cap && c->d_trace) return PMX_OK;
    const size_t rb = sizeof(T) * c->rows * c->rows;
    const int64_t cap = std::max<int64_t>({iters, 2 * c->trace_cap, 64});
    void* nb = nullptr;
    HIPCHK(c, hipMalloc(&nb, rb * (size_t)cap));
    if (c->d_trace) {
        HIPCHK(c, hipMemcpyAsync(nb, c->d_trace, rb * (size_t)c->trace_cap, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_trace);
    }
    c->d_trace = nb;
    c->trace_cap = cap;
    return PMX_OK;
}

// one ICP iteration, device-driven (transform and level from LoopCtl)
template <typename T>
int loop_enqueue_iteration(pmx_ctx* c) {
    const pmx_loop_cfg& cfg = c->loop_cfg;
    if (c->shard_done_seen) return PMX_OK;  // (every rank stops enqueuing at the same iteration)
    T Ir[16];  // (placeholder: in loop mode the kernels read the step transform from LoopCtl.T)
    for (int i = 0; i < c->rows * c->rows; ++i) Ir[i] = (i % (c->rows + 1) == 0) ? (T)1 : (T)0;
    int rc = match_impl<T>(c, Ir, cfg.knn, cfg.max_dist, nullptr);
    if (rc) return rc;
    if (cfg.n_filters == 0) {
        if ((rc = outlier_impl<T>(c, 0, 0, 0, 0, 0))) return rc;
    }
    for (int i = 0; i < cfg.n_filters; ++i) {
        const double* p = cfg.filter_p[i];
        if ((rc = outlier_impl<T>(c, cfg.filter_kind[i], i, p[0], p[1], p[2]))) return rc;
    }
    if ((rc = cfg.minimizer == 0 ? p2plane_enqueue<T>(c) : p2point_enqueue<T>(c))) return rc;
    launch_loop_step<T>(c->d_ctl, (LoopState<T>*)c->d_loop, c->d_result, c->d_iter_err, c->d_visited,
                        (const T*)c->d_means, c->loop_dev, cfg.keep_trace ? (T*)c->d_trace : nullptr, c->stream);
    HIPCHK(c, hipGetLastError());
    return PMX_OK;
}

template <typename T>
int loop_run_impl(pmx_ctx* c, int n, pmx_loop_status* st) {
    if (!c->loop_begun) return fail(c, PMX_E_STATE, "pmx_loop_begin must be called first");
    if (n < 0) return fail(c, PMX_E_BAD_PARAM, "negative iteration count");
    int rc = PMX_OK;
    int issued = 0, slot = 0, last_slot = -1;
    int fly[2], nfly = 0, head = 0;
    bool stop = c->loop_done;
    c->loop_on = true;
    while (!stop && rc == PMX_OK) {
        while (issued < n && nfly < 2 && rc == PMX_OK) {
            const int b = std::min(kLoopBatch, n - issued);
            if (c->loop_cfg.keep_trace && (rc = loop_trace_room<T>(c, c->loop_issued + b))) break;
            for (int i = 0; i < b && rc == PMX_OK; ++i) rc = loop_enqueue_iteration<T>(c);
            if (rc) break;
            c->loop_issued += b;
            issued += b;
            // the whole status block (state, control word, iteration block):
            // the stop flag of this batch, and the final status if it is the last
            hipError_t e = hipMemcpyAsync((char*)c->h_loop + (size_t)slot * kStatBytes, c->d_result, kStatBytes,
                                          hipMemcpyDeviceToHost, c->stream);
            if (e == hipSuccess) e = hipEventRecord(c->loop_ev[slot], c->stream);
            if (e != hipSuccess) {
                rc = fail(c, PMX_E_HIP, std::string("loop batch: ") + hipGetErrorString(e));
                break;
            }
            fly[(head + nfly) % 2] = slot;
            ++nfly;
            last_slot = slot;
            slot ^= 1;
        }
        if (rc || nfly == 0) break;
        const int s = fly[head];
        head = (head + 1) % 2;
        --nfly;
        const hipError_t e = hipEventSynchronize(c->loop_ev[s]);
        if (e != hipSuccess) rc = fail(c, PMX_E_HIP, std::string("loop batch: ") + hipGetErrorString(e));
        if (((const LoopState<T>*)(stat_slot(c, s) + kStatLoop))->done) stop = true;
    }
    // drain: the last issued batch's copy is the final status
    while (rc == PMX_OK && nfly > 0) {
        const hipError_t e = hipEventSynchronize(c->loop_ev[fly[head]]);
        if (e != hipSuccess) rc = fail(c, PMX_E_HIP, std::string("loop batch: ") + hipGetErrorString(e));
        head = (head + 1) % 2;
        --nfly;
    }
    c->loop_on = false;
    if (rc) {
        (void)hipStreamSynchronize(c->stream);
        return rc;
    }
    // the final state, the iteration block (limit, counters) and the control
    // word: the last batch's status copy (no batch issued: one copy now)
    if (last_slot < 0) {
        last_slot = 0;
        HIPCHK(c, hipMemcpyAsync(c->h_loop, c->d_result, kStatBytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    const char* fin = stat_slot(c, last_slot);
    std::memcpy(c->h_result, fin, kBlkCopy);
    resolve_events(c);
    LoopCtl ctl;
    std::memcpy(&ctl, fin + kStatCtl, sizeof(LoopCtl));
    const LoopState<T>& S = *(const LoopState<T>*)(fin + kStatLoop);
    c->loop_iters = S.iter;
    c->loop_done = S.done != 0;
    c->level = ctl.level;
    c->ids_level = S.last_level;
    if (S.iter > 0 || S.err)  // the last executed match's step transform (LoopCtl.T moved on)
        for (int i = 0; i < 16; ++i) c->Tstep[i] = ctl.Tprev[i];
    // map the device error to the reference's exception and message
    int err = 0;
    std::string msg;
    if (S.err) {
        const int e = S.err;
        if (e == kLoopNoPoints) {
            err = PMX_E_NO_POINTS;
            msg = "ErrorMnimizer: no point to minimize";
        } else if (e == PMX_E_EMPTY_QUANTILE) {
            err = PMX_E_EMPTY_QUANTILE;
            msg = "no outlier to filter";
        } else if (e == kSelTimeout) {
            (void)select_reset(c);
            err = PMX_E_HIP;
            msg = "radix select: a block waited too long for the pass before (device timeout)";
        } else if (e == kLoopNotRigid) {
            err = PMX_E_TRANSFORMATION;
            msg = "RigidTransformation: Error, rotation matrix is not orthogonal.";
        } else if (e == kLoopRotNaN) {
            err = PMX_E_CONVERGENCE;
            msg = "abs rotation norm not a number";
        } else if (e == kLoopTransNaN) {
            err = PMX_E_CONVERGENCE;
            msg = "abs translation norm not a number";
        } else if (e == kLoopBound) {
            err = PMX_E_CONVERGENCE;
            // TransformationCheckersImpl.cpp:215-222 (the first bound exceeded)
            for (int i = 0; i < c->loop_cfg.n_checkers; ++i) {
                if (c->loop_cfg.checker_kind[i] != PMX_CHECK_BOUND) continue;
                const T l0 = (T)c->loop_cfg.checker_p[i][0], l1 = (T)c->loop_cfg.checker_p[i][1];
                if (S.cond[i][0] > l0 || S.cond[i][1] > l1) {
                    std::ostringstream oss;
                    oss << "limit out of bounds: rot: " << S.cond[i][0] << "/" << l0 << " tr: " << S.cond[i][1] << "/"
                        << l1;
                    msg = oss.str();
                    break;
                }
            }
        } else {
            err = e;
            msg = "quantile must be between 0 and 1";
        }
        c->err = msg;
    }
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->iterations = S.iter;
        st->done = S.done;
        st->reason = S.reason;
        st->error = err;
        st->point_count_touched = (int64_t)S.touched;
        fill_stats(c, &st->last, S.kept, S.nz, S.rejM, S.rejP, S.sw, host_limit(c));
        st->last.visited = (int64_t)S.last_visited;
        const int rr = c->rows * c->rows;
        for (int i = 0; i < rr; ++i) st->T_iter[i] = (double)S.Titer[i];
        for (int i = 0; i < kMaxCheckers; ++i)
            for (int j = 0; j < 2; ++j) st->cond[i][j] = (double)S.cond[i][j];
    }
    return err;
}

template <typename T>
int loop_trace_impl(pmx_ctx* c, int first, int count, void* out) {
    if (!c->loop_begun || !c->loop_cfg.keep_trace) return fail(c, PMX_E_STATE, "no loop trace (keep_trace = 0)");
    if (first < 0 || count < 0 || first + count > c->loop_iters)
        return fail(c, PMX_E_BAD_PARAM, "trace range beyond the completed iterations");
    if (count == 0) return PMX_OK;
    const size_t rb = sizeof(T) * c->rows * c->rows;
    HIPCHK(c, hipMemcpyAsync(out, (const char*)c->d_trace + rb * first, rb * count, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PMX_OK;
}

// SurfaceNormalDataPointsFilter (DataPointsFilters/SurfaceNormal.cpp:80-290):
// self-match on a temporary context, the statistics kernel, and the
// smoothNormals pass on the host (the reference smooths in place, point by
// point: later points see the already smoothed normals of earlier ones,
// :256-283 — a sequential dependency kept as is).
template <typename T>
int surface_normals_impl(int device, const T* feat, int rows, int64_t n, int knn, double maxDist, unsigned flags,
                         T* o_nrm, T* o_dens, T* o_eval, T* o_evec, T* o_ids, T* o_mdist, int64_t* degenerate) {
    if (rows != 3 && rows != 4) {
        g_err = "SurfaceNormalDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    if (knn < 1 || knn > 16) {
        g_err = "SurfaceNormalDataPointsFilter: knn must be in [1, 16] on the GPU path";
        return PMX_E_BAD_PARAM;
    }
    if (degenerate) *degenerate = 0;
    if (n <= 0) return PMX_OK;
    pmx_ctx* c = nullptr;
    int rc = pmx_ctx_create(device, sizeof(T) == 8 ? PMX_F64 : PMX_F32, &c);
    if (rc) {
        g_err = "SurfaceNormalDataPointsFilter: no HIP device";
        return rc;
    }
    struct Guard {
        pmx_ctx* c;
        ~Guard() { pmx_ctx_destroy(c); }
    } guard{c};
    auto err = [&](int r) {
        g_err = c->err;
        return r;
    };
    c->reuse_on = false;
    c->search_type = 1;
    if (c->grid_mode == 0) c->grid_mode = 1;
    const int D = rows - 1;
    std::vector<T> I((size_t)rows * rows, (T)0);
    for (int i = 0; i < rows; ++i) I[(size_t)i * rows + i] = 1;
    if ((rc = set_reference_impl<T>(c, feat, rows, n, nullptr))) return err(rc);
    if ((rc = set_reading_impl<T>(c, feat, rows, n, I.data()))) return err(rc);
    if ((rc = match_impl<T>(c, I.data(), knn, maxDist, nullptr))) return err(rc);
    const int64_t per = D + 1 + D + D * D + 1;  // normals, density, eigen values, eigen vectors, mean distance
    T* d_out = nullptr;
    unsigned long long* d_deg = nullptr;
    HIPCHK(c, hipMalloc((void**)&d_out, sizeof(T) * (size_t)(n * per)));
    std::unique_ptr<void, void (*)(void*)> free_out(d_out, [](void* p) { (void)hipFree(p); });
    HIPCHK(c, hipMalloc((void**)&d_deg, sizeof(unsigned long long)));
    std::unique_ptr<void, void (*)(void*)> free_deg(d_deg, [](void* p) { (void)hipFree(p); });
    HIPCHK(c, hipMemsetAsync(d_deg, 0, sizeof(unsigned long long), c->stream));
    T* d_nrm = d_out;
    T* d_dens = d_nrm + n * D;
    T* d_eval = d_dens + n;
    T* d_evec = d_eval + n * D;
    T* d_md = d_evec + n * D * D;
    const GridLevel& L = c->lv(c->ids_level);
    launch_surface_normals<T>((const P4<T>*)c->d_rd, (const P4<T>*)L.gpts, c->d_ids, (const T*)c->d_dists, n, knn, D,
                              d_nrm, d_dens, d_eval, d_evec, d_md, d_deg, c->stream);
    HIPCHK(c, hipGetLastError());
    std::vector<T> h((size_t)(n * per));
    unsigned long long deg = 0;
    HIPCHK(c, hipMemcpyAsync(h.data(), d_out, sizeof(T) * h.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&deg, d_deg, sizeof(deg), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // slot order -> point order
    auto take = [&](int64_t off, int span, T* dst) {
        if (!dst) return;
        std::vector<T> src(h.begin() + off, h.begin() + off + n * span);
        (void)unpermute<T>(c, src, dst, span);  // (host_order below has run)
    };
    const bool smooth = (flags & PMX_SN_SMOOTH) && o_nrm;
    if ((rc = host_order(c))) return err(rc);
    take(0, D, o_nrm);
    take(n * D, 1, o_dens);
    take(n * (D + 1), D, o_eval);
    take(n * (2 * D + 1), D * D, o_evec);
    take(n * (2 * D + 1 + D * D), 1, o_mdist);
    if (o_ids || smooth) {
        std::vector<T> dd((size_t)(n * knn));
        std::vector<int32_t> ii((size_t)(n * knn));
        if ((rc = get_matches_impl<T>(c, dd.data(), ii.data()))) return err(rc);
        if (o_ids)  // matches.ids.cast<T>() (SurfaceNormal.cpp:250-253)
            for (size_t e = 0; e < ii.size(); ++e) o_ids[e] = (T)ii[e];
        if (smooth) {  // SurfaceNormal.cpp:256-283, in place, point order
            const T inf = std::numeric_limits<T>::infinity();
            for (int64_t i = 0; i < n; ++i) {
                T cur[3] = {0, 0, 0}, mean[3] = {0, 0, 0};
                for (int r = 0; r < D; ++r) cur[r] = o_nrm[i * D + r];
                int cnt = 0;
                for (int j = 0; j < knn; ++j) {
                    if (dd[(size_t)(i * knn + j)] == inf) continue;
                    const int64_t ref = ii[(size_t)(i * knn + j)];
                    const T* nb = o_nrm + ref * D;
                    T dot = 0;
                    for (int r = 0; r < D; ++r) dot = dot + cur[r] * nb[r];
                    for (int r = 0; r < D; ++r) mean[r] = dot > (T)0 ? mean[r] + nb[r] : mean[r] - nb[r];
                    ++cnt;
                }
                for (int r = 0; r < D; ++r) o_nrm[i * D + r] = mean[r] / (T)cnt;
            }
        }
    }
    if (degenerate) *degenerate = (int64_t)deg;
    return PMX_OK;
}

// SamplingSurfaceNormalDataPointsFilter::inPlaceFilter
// (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342): the split and the leaf
// statistics on the device (pmx_ssn.hip), the sampling and the output cloud
// here — fuseRange's draws in leaf order (:285-309), the output in index
// order (:145-164).
template <typename T>
int voxel_impl(int device, const T* feat, int rows, int64_t n, const T* desc, int desc_dim, const double* vsize,
               bool centroid, bool avg, T* feat_out, T* desc_out, int64_t* n_out) {
    if (rows != 3 && rows != 4) {
        g_err = "VoxelGridDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    *n_out = 0;
    if (n <= 0) return PMX_OK;
    if (hipSetDevice(device) != hipSuccess) {
        g_err = "VoxelGridDataPointsFilter: no HIP device";
        return PMX_E_HIP;
    }
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return PMX_E_HIP;
    std::unique_ptr<std::remove_pointer<hipStream_t>::type, void (*)(hipStream_t)> free_st(
        st, [](hipStream_t s) { (void)hipStreamDestroy(s); });
    const size_t fb = sizeof(T) * (size_t)rows * n, db = sizeof(T) * (size_t)desc_dim * n;
    char* buf = nullptr;
    if (hipMalloc(&buf, 2 * (fb + db) + 512) != hipSuccess) {
        g_err = "VoxelGridDataPointsFilter: device allocation failed";
        return PMX_E_HIP;
    }
    std::unique_ptr<void, void (*)(void*)> free_buf(buf, [](void* p) { (void)hipFree(p); });
    T* d_f = (T*)buf;
    T* d_d = (T*)(buf + ((fb + 255) & ~(size_t)255));
    T* d_of = (T*)((char*)d_d + ((db + 255) & ~(size_t)255));
    T* d_od = d_of + (size_t)rows * n;
    if (hipMemcpyAsync(d_f, feat, fb, hipMemcpyHostToDevice, st) != hipSuccess) return PMX_E_HIP;
    if (db && hipMemcpyAsync(d_d, desc, db, hipMemcpyHostToDevice, st) != hipSuccess) return PMX_E_HIP;
    std::string err;
    int64_t m = 0;
    const int rc = voxel_run<T>(d_f, rows, n, db ? d_d : nullptr, desc_dim, vsize, centroid, avg, d_of, d_od, &m, st,
                                err);
    if (rc) {
        g_err = err.empty() ? std::string("VoxelGridDataPointsFilter: HIP failure") : err;
        return rc;
    }
    if (hipMemcpyAsync(feat_out, d_of, sizeof(T) * (size_t)rows * m, hipMemcpyDeviceToHost, st) != hipSuccess)
        return PMX_E_HIP;
    if (db && desc_out &&
        hipMemcpyAsync(desc_out, d_od, sizeof(T) * (size_t)desc_dim * m, hipMemcpyDeviceToHost, st) != hipSuccess)
        return PMX_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return PMX_E_HIP;
    *n_out = m;
    return PMX_OK;
}

template <typename T>
int ssn_impl(int device, const T* feat, int rows, int64_t n, const T* desc, int desc_dim, int knn, int method,
             double ratio_d, double max_box_d, unsigned flags, T* feat_out, T* desc_out, T* o_nrm, T* o_dens,
             T* o_eval, T* o_evec, int64_t* n_out, int64_t* unfit_out) {
    if (rows != 3 && rows != 4) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    if (knn < 3) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: knn must be >= 3";
        return PMX_E_BAD_PARAM;
    }
    if (method != 0 && method != 1) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: samplingMethod must be 0 or 1";
        return PMX_E_BAD_PARAM;
    }
    if (n > (int64_t)0x7fffffff) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: more than 2^31 points";
        return PMX_E_BAD_PARAM;
    }
    if (n_out) *n_out = 0;
    if (unfit_out) *unfit_out = 0;
    if (n <= 0) return PMX_OK;
    pmx_ctx* c = nullptr;
    int rc = pmx_ctx_create(device, sizeof(T) == 8 ? PMX_F64 : PMX_F32, &c);
    if (rc) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: no HIP device";
        return rc;
    }
    struct Guard {
        pmx_ctx* c;
        ~Guard() { pmx_ctx_destroy(c); }
    } guard{c};
    const int D = rows - 1;
    void* d_pts = nullptr;
    if (hipMalloc(&d_pts, sizeof(P4<T>) * n) != hipSuccess) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: device allocation failed";
        return PMX_E_HIP;
    }
    std::unique_ptr<void, void (*)(void*)> free_pts(d_pts, [](void* p) { (void)hipFree(p); });
    if ((rc = upload_raw(c, feat, sizeof(T) * (size_t)rows * n))) {
        g_err = c->err;
        return rc;
    }
    launch_pack_p4<T>((const T*)c->d_raw, rows, n, n, (P4<T>*)d_pts, c->stream);
    const T ratio = (T)ratio_d, max_box = (T)max_box_d;
    const bool want_eig = (flags & (PMX_SSN_NORMALS | PMX_SSN_EIGVALUES | PMX_SSN_EIGVECTORS)) != 0;
    std::vector<int32_t> perm, lf, lc, fit;
    std::vector<T> rec;
    std::string err;
    if ((rc = ssn_run<T>((const P4<T>*)d_pts, D, n, knn, max_box, want_eig, c->stream, perm, lf, lc, fit, rec, err))) {
        g_err = err;
        return rc;
    }
    const int RS = D + D + 1 + D + D * D;
    // fuseRange's sampling, leaf by leaf in the recursion's order
    std::vector<int32_t> keep_leaf((size_t)n, -1);  // by point index: the leaf whose record it takes
    int64_t unfit = 0, kept = 0;
    for (size_t l = 0; l < lf.size(); ++l) {
        const int32_t f = lf[l], cnt = lc[l];
        if (!fit[l]) {
            unfit += cnt;
            continue;
        }
        if (method == 0) {
            for (int32_t i = 0; i < cnt; ++i) {
                const float r = (float)std::rand() / (float)RAND_MAX;
                if (r < ratio) {
                    keep_leaf[(size_t)perm[(size_t)(f + i)]] = (int32_t)l;
                    ++kept;
                }
            }
        } else {  // the smallest index of the leaf carries its mean
            keep_leaf[(size_t)perm[(size_t)f]] = (int32_t)l;
            ++kept;
        }
    }
    int64_t o = 0;
    for (int64_t k = 0; k < n; ++k) {
        const int32_t l = keep_leaf[(size_t)k];
        if (l < 0) continue;
        const T* R = rec.data() + (size_t)l * RS;
        if (feat_out) {
            if (method == 0) {
                for (int r = 0; r < rows; ++r) feat_out[o * rows + r] = feat[k * rows + r];
            } else {
                for (int r = 0; r < D; ++r) feat_out[o * rows + r] = R[r];
                feat_out[o * rows + D] = 1;
            }
        }
        if (desc_out && desc && desc_dim > 0) {
            if (method == 1 && (flags & PMX_SSN_AVERAGE)) {  // mergedDesc (:320-328)
                const int32_t f = lf[(size_t)l], cnt = lc[(size_t)l];
                for (int cc = 0; cc < desc_dim; ++cc) {
                    T s = 0;
                    for (int32_t i = 0; i < cnt; ++i) s = s + desc[(int64_t)perm[(size_t)(f + i)] * desc_dim + cc];
                    desc_out[o * desc_dim + cc] = s / (T)cnt;
                }
            } else {
                for (int cc = 0; cc < desc_dim; ++cc) desc_out[o * desc_dim + cc] = desc[k * desc_dim + cc];
            }
        }
        if (o_nrm)
            for (int r = 0; r < D; ++r) o_nrm[o * D + r] = R[D + r];
        if (o_dens) o_dens[o] = R[2 * D];
        if (o_eval)
            for (int r = 0; r < D; ++r) o_eval[o * D + r] = R[2 * D + 1 + r];
        if (o_evec)
            for (int e = 0; e < D * D; ++e) o_evec[o * D * D + e] = R[3 * D + 1 + e];
        ++o;
    }
    (void)kept;
    if (n_out) *n_out = o;
    if (unfit_out) *unfit_out = unfit;
    return PMX_OK;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char* pmx_version(void) { return "pmx 0.1 (HIP, gfx950)"; }

int pmx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* pmx_last_error(const pmx_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int pmx_ctx_create(int device, int dtype, pmx_ctx** out) {
    if (!out) return PMX_E_BAD_PARAM;
    *out = nullptr;
    if (dtype != PMX_F32 && dtype != PMX_F64) return PMX_E_BAD_PARAM;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return PMX_E_NO_DEVICE;
    if (device < 0 || device >= n) return PMX_E_BAD_PARAM;
    pmx_ctx* c = new pmx_ctx();
    c->device = device;
    c->dtype = dtype;
    // tuning knobs (defaults are the measured optimum on MI355X)
    if (const char* e = std::getenv("PMX_GRID_MODE"))
        c->grid_mode = std::strcmp(e, "tile") == 0 ? 0 : std::strcmp(e, "octant") == 0 ? 2 : 1;
    if (const char* e = std::getenv("PMX_GRID_TILE_MAX")) c->tile_max = (uint32_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("PMX_SPEC_SELECT")) c->spec_allowed = std::atoi(e) != 0;
    // grid levels: PMX_GRID_LEVELS="2,8,32" (points per occupied cell), or
    // PMX_GRID_PPC=x for a single fixed level; PMX_GRID_ADAPT=0 pins level 0
    if (const char* e = std::getenv("PMX_GRID_LEVELS")) {
        std::vector<double> v;
        for (const char* p = e; *p;) {
            char* end = nullptr;
            const double x = std::strtod(p, &end);
            if (end == p) break;
            if (x >= 0.25) v.push_back(x);
            p = *end == ',' ? end + 1 : end;
        }
        if (!v.empty()) c->level_ppc = v;
    }
    if (const char* e = std::getenv("PMX_GRID_PPC")) c->level_ppc = {std::max(0.25, std::atof(e))};
    if (const char* e = std::getenv("PMX_GRID_ADAPT")) c->adaptive = std::atoi(e) != 0;
    if (const char* e = std::getenv("PMX_GRID_REUSE")) c->reuse_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("PMX_GRID_FIRST_PPC")) c->first_ppc = std::max(0.25, std::atof(e));
    auto bad = [&](int code) {
        pmx_ctx_destroy(c);
        return code;
    };
    if (hipSetDevice(device) != hipSuccess) return bad(PMX_E_HIP);
    if (const char* e = std::getenv("PMX_SYNC")) {  // host wait policy for the per-iteration sync
        if (std::strcmp(e, "spin") == 0) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
        if (std::strcmp(e, "yield") == 0) (void)hipSetDeviceFlags(hipDeviceScheduleYield);
        if (std::strcmp(e, "block") == 0) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bad(PMX_E_HIP);
    static bool preloaded = false;  // (once per process; modules are per process)
    if (!preloaded) {
        preload_match();
        preload_grid();
        preload_select();
        preload_reduce();
        preload_loop();
        preload_normals();
        preload_setup();
        preload_ssn();
        preloaded = true;
    }
    // One small "iteration block" holds everything the host reads back per
    // iteration, so a single D2H copy returns it (see kBlk*):
    //   [0, 1024)     reduction results (128 doubles)
    //   [1024, ...)   SelectState, then the per-iteration error word
    //   [1152]        VarTrimmed ratio, [1216] pair-evaluation counter
    //   [1280, 1344)  point-to-point means (6 T)
    void* p = nullptr;
    if (hipMalloc(&p, kStatBytes) != hipSuccess) return bad(PMX_E_HIP);
    (void)hipMemset(p, 0, kStatBytes);
    c->d_result = (double*)p;
    c->d_ctl = (LoopCtl*)((char*)p + kStatCtl);  // (zero: done = 0, kernels given it run normally)
    c->d_loop = (char*)p + kStatLoop;
    c->d_sel = (SelectState*)((char*)p + kBlkSel);
    c->d_iter_err = (int*)(c->d_sel + 1);
    c->d_ratio = (double*)((char*)p + kBlkRatio);
    c->d_visited = (unsigned long long*)((char*)p + kBlkVisited);
    c->d_means = (char*)p + kBlkMeans;
    if (hipMalloc((void**)&c->d_sel_more, sizeof(SelectState) * (kMaxChain - 1)) != hipSuccess) return bad(PMX_E_HIP);
    (void)hipMemset(c->d_sel_more, 0, sizeof(SelectState) * (kMaxChain - 1));
    if (hipMalloc((void**)&c->d_vpart, grid_counter_bytes()) != hipSuccess) return bad(PMX_E_HIP);
    (void)hipMemset(c->d_vpart, 0, grid_counter_bytes());
    // 2048 histogram bins (the sharded select's per-pass histogram)
    if (hipMalloc((void**)&c->d_hist, 2048 * sizeof(uint32_t)) != hipSuccess) return bad(PMX_E_HIP);
    (void)hipMemset(c->d_hist, 0, 2048 * sizeof(uint32_t));
    if (hipMalloc(&c->d_selx, selx_bytes()) != hipSuccess) return bad(PMX_E_HIP);
    (void)hipMemset(c->d_selx, 0, selx_bytes());
    if (hipMalloc((void**)&c->d_partials, sizeof(double) * kRedBlocks * kNVMax) != hipSuccess) return bad(PMX_E_HIP);
    if (hipHostMalloc((void**)&c->h_result, kBlkBytes, hipHostMallocDefault) != hipSuccess) return bad(PMX_E_HIP);
    *out = c;
    return PMX_OK;
}

int pmx_ctx_destroy(pmx_ctx* c) {
    if (!c) return PMX_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->d_safe, c->d_ref,  c->d_nrm,      c->d_rd,     c->d_dists,  c->d_ids,   c->d_w,    c->d_part_d,
                    c->d_part_i, c->d_hist,   c->d_vt,     c->d_deno,  c->d_gather, c->d_partials,
                    c->d_result, c->d_waves, c->d_vpart,
                    c->d_sel_more, c->d_gdesc, c->d_loop_T0, c->d_trace,
                    c->d_spec, c->d_spec_keys, c->d_order, c->d_raw, c->d_bbox, c->d_occ, c->d_selx,
                    c->d_rob, c->d_rdev, c->d_radii};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& L : c->levels) L.release();
    setup_release(c);
    if (c->h_result) (void)hipHostFree(c->h_result);
    if (c->h_loop) (void)hipHostFree(c->h_loop);
    for (hipEvent_t e : c->loop_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& pr : c->ev_pending) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    if (c->d_specx) (void)hipFree(c->d_specx);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return PMX_OK;
}

int pmx_comm_unique_id(void* out128) {
    if (!out128) return PMX_E_BAD_PARAM;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return PMX_E_RCCL;
    std::memcpy(out128, &id, sizeof(id));
    return PMX_OK;
}

int pmx_comm_init(pmx_ctx* c, const void* uid128, int nranks, int rank) {
    if (!c || !uid128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(c, PMX_E_BAD_PARAM, "bad comm args");
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId id;
    std::memcpy(&id, uid128, sizeof(id));
    if (sharded(c)) return fail(c, PMX_E_STATE, "the context already has a communicator");
    NCCLCHK(c, ncclCommInitRank(&c->comm, nranks, id, rank));
    c->nranks = nranks;
    c->rank = rank;
    return PMX_OK;
}

int pmx_comm_init_host(pmx_ctx* c, int nranks, int rank, pmx_allreduce_fn allreduce, pmx_allgather_fn allgather,
                       void* user) {
    if (!c || !allreduce || !allgather || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(c, PMX_E_BAD_PARAM, "bad comm args");
    if (sharded(c)) return fail(c, PMX_E_STATE, "the context already has a communicator");
    c->host_ar = allreduce;
    c->host_ag = allgather;
    c->host_user = user;
    c->nranks = nranks;
    c->rank = rank;
    return PMX_OK;
}

int pmx_comm_stats(const pmx_ctx* c, uint64_t* allreduces, uint64_t* allgathers) {
    if (!c || !allreduces || !allgathers) return PMX_E_BAD_PARAM;
    *allreduces = c->n_allreduce;
    *allgathers = c->n_allgather;
    return PMX_OK;
}

int pmx_comm_size(const pmx_ctx* c, int* nranks, int* rank, int* kind) {
    if (!c) return PMX_E_BAD_PARAM;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (kind) *kind = c->comm ? 1 : c->host_ar ? 2 : 0;
    return PMX_OK;
}

#define DISPATCH(c, call_f, call_d) ((c)->dtype == PMX_F64 ? (call_d) : (call_f))

int pmx_set_reference(pmx_ctx* c, const void* feat, int rows, int64_t M, const void* normals) {
    if (!c || !feat) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c, set_reference_impl<float>(c, (const float*)feat, rows, M, (const float*)normals),
                    set_reference_impl<double>(c, (const double*)feat, rows, M, (const double*)normals));
}

int pmx_set_reading(pmx_ctx* c, const void* feat, int rows, int64_t N, const void* T0) {
    if (!c || (!feat && N > 0) || !T0) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c, set_reading_impl<float>(c, (const float*)feat, rows, N, (const float*)T0),
                    set_reading_impl<double>(c, (const double*)feat, rows, N, (const double*)T0));
}

int pmx_set_reading_radii(pmx_ctx* c, const void* radii) {
    if (!c) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c, set_radii_impl<float>(c, (const float*)radii), set_radii_impl<double>(c, (const double*)radii));
}

int pmx_match(pmx_ctx* c, const void* T_iter, int knn, double maxDist, double epsilon, uint64_t* visited) {
    if (!c || !T_iter) return fail(c, PMX_E_BAD_PARAM, "null argument");
    if (!(epsilon >= 0)) return fail(c, PMX_E_BAD_PARAM, "epsilon must be >= 0");
    return DISPATCH(c, match_impl<float>(c, (const float*)T_iter, knn, maxDist, visited),
                    match_impl<double>(c, (const double*)T_iter, knn, maxDist, visited));
}

#define OUTLIER(c, kind, pos, a, b, d)                                                     \
    ((c) ? DISPATCH(c, outlier_impl<float>(c, kind, pos, a, b, d), outlier_impl<double>(c, kind, pos, a, b, d)) \
         : PMX_E_BAD_PARAM)

int pmx_outlier_default(pmx_ctx* c) { return OUTLIER(c, 0, 0, 0, 0, 0); }
int pmx_outlier_null(pmx_ctx* c, int pos) { return OUTLIER(c, 1, pos, 0, 0, 0); }
int pmx_outlier_maxdist(pmx_ctx* c, int pos, double m) { return OUTLIER(c, 2, pos, m, 0, 0); }
int pmx_outlier_mindist(pmx_ctx* c, int pos, double m) { return OUTLIER(c, 3, pos, m, 0, 0); }
int pmx_outlier_mediandist(pmx_ctx* c, int pos, double f) { return OUTLIER(c, 4, pos, f, 0, 0); }
int pmx_outlier_trimmed(pmx_ctx* c, int pos, double r) { return OUTLIER(c, 5, pos, r, 0, 0); }
int pmx_outlier_vartrimmed(pmx_ctx* c, int pos, double a, double b, double l) { return OUTLIER(c, 6, pos, a, b, l); }

int pmx_p2plane_system(pmx_ctx* c, double* A, double* b, pmx_stats* st) {
    if (!c || !A || !b) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, p2plane_impl<float>(c, A, b, st), p2plane_impl<double>(c, A, b, st));
}

int pmx_p2point_system(pmx_ctx* c, double* mp, double* mq, double* m, pmx_stats* st) {
    if (!c || !mp || !mq || !m) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, p2point_impl<float>(c, mp, mq, m, st), p2point_impl<double>(c, mp, mq, m, st));
}

int pmx_get_matches(pmx_ctx* c, void* dists, int32_t* ids) {
    if (!c) return PMX_E_BAD_PARAM;
    return DISPATCH(c, get_matches_impl<float>(c, dists, ids), get_matches_impl<double>(c, dists, ids));
}

int pmx_outlier_robust(pmx_ctx* c, int pos, int fct, double tuning, double approx, int mode, double target,
                       int p2pl) {
    if (!c) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, outlier_robust_impl<float>(c, pos, fct, tuning, approx, mode, target, p2pl),
                    outlier_robust_impl<double>(c, pos, fct, tuning, approx, mode, target, p2pl));
}
int pmx_robust_scale(pmx_ctx* c, int pos, double* scale) {
    if (!c || !scale) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, robust_scale_impl<float>(c, pos, scale), robust_scale_impl<double>(c, pos, scale));
}
int pmx_get_weights(pmx_ctx* c, void* w) {
    if (!c || !w) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, get_weights_impl<float>(c, w), get_weights_impl<double>(c, w));
}

int pmx_get_shape(const pmx_ctx* c, int64_t* n_local, int* knn) {
    if (!c) return PMX_E_BAD_PARAM;
    if (n_local) *n_local = c->N;
    if (knn) *knn = c->knn;
    return PMX_OK;
}

int pmx_set_search(pmx_ctx* c, int search_type) {
    if (!c) return PMX_E_BAD_PARAM;
    if (search_type < 0 || search_type > 2) return fail(c, PMX_E_BAD_PARAM, "searchType must be 0, 1 or 2");
    c->search_type = search_type;
    return PMX_OK;
}

int pmx_timing_enable(pmx_ctx* c, int on) {
    if (!c) return PMX_E_BAD_PARAM;
    c->timing = on != 0;
    c->match_ms = 0.0;
    c->match_launches = 0;
    return PMX_OK;
}

int pmx_timing_read(pmx_ctx* c, double* match_ms, int64_t* launches, double* other_ms) {
    if (!c) return PMX_E_BAD_PARAM;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    resolve_events(c);
    if (match_ms) *match_ms = c->match_ms;
    if (launches) *launches = c->match_launches;
    if (other_ms) *other_ms = 0.0;
    return PMX_OK;
}

int pmx_sync(pmx_ctx* c) {
    if (!c) return PMX_E_BAD_PARAM;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PMX_OK;
}

int pmx_loop_begin(pmx_ctx* c, const pmx_loop_cfg* cfg, const void* T0) {
    if (!c || !cfg || !T0) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c, loop_begin_impl<float>(c, cfg, (const float*)T0), loop_begin_impl<double>(c, cfg, (const double*)T0));
}

int pmx_loop_run(pmx_ctx* c, int n, pmx_loop_status* st) {
    if (!c) return PMX_E_BAD_PARAM;
    (void)hipSetDevice(c->device);
    return DISPATCH(c, loop_run_impl<float>(c, n, st), loop_run_impl<double>(c, n, st));
}

int pmx_loop_trace(pmx_ctx* c, int first, int count, void* out) {
    if (!c || (!out && count > 0)) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, loop_trace_impl<float>(c, first, count, out), loop_trace_impl<double>(c, first, count, out));
}

int pmx_loop_select_stats(pmx_ctx* c, uint64_t* window_hits, uint64_t* window_misses) {
    if (!c || !window_hits || !window_misses) return fail(c, PMX_E_BAD_PARAM, "null argument");
    *window_hits = 0;
    *window_misses = 0;
    if (!c->d_spec) return PMX_OK;
    SpecSel h{};
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(&h, c->d_spec, sizeof(SpecSel), hipMemcpyDeviceToHost));
    *window_hits = h.n_hit;
    *window_misses = h.n_miss;
    return PMX_OK;
}

int pmx_sampling_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc,
                                 int desc_dim, int knn, int sampling_method, double ratio, double max_box_dim,
                                 unsigned flags, void* feat_out, void* desc_out, void* normals, void* densities,
                                 void* eig_values, void* eig_vectors, int64_t* n_out, int64_t* unfit) {
    if ((!feat && n > 0) || (desc_dim > 0 && !desc && n > 0)) {
        g_err = "null cloud";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return ssn_impl<float>(device, (const float*)feat, rows, n, (const float*)desc, desc_dim, knn, sampling_method,
                               ratio, max_box_dim, flags, (float*)feat_out, (float*)desc_out, (float*)normals,
                               (float*)densities, (float*)eig_values, (float*)eig_vectors, n_out, unfit);
    if (dtype == PMX_F64)
        return ssn_impl<double>(device, (const double*)feat, rows, n, (const double*)desc, desc_dim, knn,
                                sampling_method, ratio, max_box_dim, flags, (double*)feat_out, (double*)desc_out,
                                (double*)normals, (double*)densities, (double*)eig_values, (double*)eig_vectors,
                                n_out, unfit);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

int pmx_voxel_grid(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc, int desc_dim,
                   const double* vsize, int use_centroid, int average_desc, void* feat_out, void* desc_out,
                   int64_t* n_out) {
    if ((!feat && n > 0) || (desc_dim > 0 && !desc && n > 0) || !vsize || !n_out || (!feat_out && n > 0) ||
        desc_dim < 0) {
        g_err = "null argument";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return voxel_impl<float>(device, (const float*)feat, rows, n, (const float*)desc, desc_dim, vsize,
                                 use_centroid != 0, average_desc != 0, (float*)feat_out, (float*)desc_out, n_out);
    if (dtype == PMX_F64)
        return voxel_impl<double>(device, (const double*)feat, rows, n, (const double*)desc, desc_dim, vsize,
                                  use_centroid != 0, average_desc != 0, (double*)feat_out, (double*)desc_out, n_out);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

int pmx_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, int knn, double maxDist,
                        unsigned flags, void* normals, void* densities, void* eig_values, void* eig_vectors,
                        void* matched_ids, void* mean_dists, int64_t* degenerate) {
    if (!feat && n > 0) {
        g_err = "null cloud";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return surface_normals_impl<float>(device, (const float*)feat, rows, n, knn, maxDist, flags, (float*)normals,
                                           (float*)densities, (float*)eig_values, (float*)eig_vectors,
                                           (float*)matched_ids, (float*)mean_dists, degenerate);
    if (dtype == PMX_F64)
        return surface_normals_impl<double>(device, (const double*)feat, rows, n, knn, maxDist, flags,
                                            (double*)normals, (double*)densities, (double*)eig_values,
                                            (double*)eig_vectors, (double*)matched_ids, (double*)mean_dists,
                                            degenerate);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

}  // extern "C"
