// pmx_ctx.h — the per-ICP-object device state behind the C ABI of
// include/pmx.h (struct pmx_ctx) and the host-side helpers the ABI's
// translation units share:
//   pmx_capi.hip          context lifecycle, collectives, timing
//   pmx_chain.hip         clouds and grid (Matcher::init), match, outlier
//                         filters, minimisers, host mirrors
//   pmx_loop_capi.hip     the device-resident ICP loop (pmx_loop_*)
//   pmx_filters_capi.hip  the stand-alone data filters (normals, SSN, voxel)
// One HIP stream per context sequences the kernels; the host reads one small
// status block per iteration (per batch of iterations in the device loop).
#pragma once

#include "pmx_internal.h"
#include "pmx_p2plane.h"
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
    // allocated capacities (a new reference reuses the buffers when it fits:
    // hipMalloc / hipFree of 4 buffers x 6 levels was a large part of setup)
    size_t cap_pts = 0, cap_gpn = 0, cap_idx = 0, cap_start = 0;
    void release() {
        for (void* b : {gpts, gpn, (void*)gidx, (void*)gstart})
            if (b) (void)hipFree(b);
        gpts = gpn = nullptr;
        gidx = nullptr;
        gstart = nullptr;
        cap_pts = cap_gpn = cap_idx = cap_start = 0;
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
    size_t ref_bytes = 0, nrm_bytes = 0;  // (capacities: kept across references)
    bool has_normals = false;

    // uniform grid over the reference (exact shell search, pmx_grid.hip)
    int search_type = 1;
    int grid_mode = 1;            // 1 = per-lane shell search (default), 0 = LDS tiles (option grid_mode=tile)
    uint32_t tile_max = 4096;     // largest per-wave box scanned from LDS (option tile_max)
    // Grid levels of increasing cell size (points per occupied cell:
    // level_ppc, option grid_levels).  Every level answers exactly; the level of
    // the next match is chosen from the last match's pair count (adaptive:
    // converged iterations want small cells, misaligned ones or large k want
    // large cells, see choose_level).
    std::vector<GridLevel> levels;
    std::vector<double> level_ppc{2.0, 4.0, 8.0, 16.0, 32.0, 64.0};
    // Levels are built lazily: Matcher::init builds the finest ones up to
    // the cold level (first_ppc), the coarser ones on the first match that
    // wants one (ensure_level).  levels[0, levels_built) are built.
    int levels_built = 0;
    std::vector<SetupShape> level_shapes;
    int64_t grid_valid = 0;   // finite reference points (the levels' size)
    int level = 0;      // level of the next grid match
    double first_ppc = 8.0;   // level of a new reading's first (cold) match (option first_ppc)
    int ids_level = 0;  // level whose positions the current match ids are
    std::vector<double> level_cells;   // last cells-per-query seen at each level
    std::vector<int64_t> level_seen;   // match count when it was seen (0: never)
    int64_t match_count = 0;
    bool adaptive = true;
    // developer options (PMX_OPTS / pmx_ctx_set_option, README "Options"):
    // A/B switches of measured alternatives and test hooks, per context
    bool fuse_step = true;        // fuse_step: the last finalize and the step in one launch (device loop, one rank)
    bool step_counter_on = true;  // step_counter: the match's counter phase folded into that launch (no window)
    bool p2p_onepass = true;      // p2p_onepass: device-loop point-to-point in one moments pass (the step centres)
    bool side_levels = true;      // side_levels: the levels finer than the cold one on a side stream
    bool reading_copy = true;     // reading_copy: the reading's upload on the copy stream
    bool reading_order = true;    // reading_order: the reading in slot (Morton) order
    int loop_batch = 0;           // loop_batch: one status batch size for the device loop (0: 4, then 8)
    double wave_fill = 1.25;      // wave_fill: the tile mode's wave table fill
    int setup_trace = 0;          // setup_trace: setup timeline on stderr (1: stream-synchronised marks, 2: host)
    bool tile_prof = false;       // tile_prof: the cold tile form's per-wave profile on stderr
    bool tile_prof_raw = false;   // (tile_prof=2: and the raw words to tile_prof.bin)
    bool reuse_on = true;         // temporal reuse of the grid match (pmx_grid.hip; option grid_reuse=0: off)
    bool safe_valid = false;      // d_safe holds the safe radii of the match in d_dists / d_ids
    void* d_safe = nullptr;       // T[N]: safe radius per query
    int64_t safe_cap = 0;
    int tile_dispatch_req = -1;   // tile dispatch in the device loop: -1 auto (reading >= 4x the reference), 0 off, 1 on (option tile_dispatch)
    int coop_max = 4;             // wave-cooperative full searches for blocks with <= this many misses (option coop_max)
    // k = 1 neighbour records (GridReuse::nbr): P4<T>[N]; nbr_prev: the last
    // match wrote them (option nbr_cache=0: off)
    void* d_nbr = nullptr;
    size_t nbr_bytes = 0;
    bool nbr_prev = false;
    bool nbr_normals = false;  // (the last match's records carry the normals, at d_nbr + N)
    bool nbr_on = true;
    bool grid_ready = false;
    const GridLevel& lv(int i) const { return levels[(size_t)i]; }
    std::vector<int32_t> slot_query;  // host copy of d_order (host mirrors only; filled on demand)
    int32_t* d_order = nullptr;       // slot -> reading index (has_order; else identity)
    size_t order_bytes = 0;
    bool has_order = false;
    // once-per-compute setup on the device (pmx_setup.hip)
    SetupScratch setup;
    int64_t setup_n = 0, setup_cells = 0;
    // the levels finer than the cold one, built on a side stream while the
    // reading is set and the cold match runs (own scratch); every later match
    // waits for side_ev on the context stream (side_join)
    hipStream_t side = nullptr;
    hipEvent_t side_ev = nullptr;
    hipEvent_t side_start_ev = nullptr;  // the context stream's packs (points, normals) before the side builds
    bool side_pending = false;
    SetupScratch setup_side;
    int64_t setup_side_n = 0, setup_side_cells = 0;
    // the level table's pinned staging (its copy is asynchronous: table_ev
    // guards the rewrite), and the reading's upload stream: the caller's
    // cloud crosses PCIe while the context stream builds the cold level
    // (raw_ev: the last pack that read d_raw; copy_ev: the upload done)
    void* h_table = nullptr;
    hipEvent_t table_ev = nullptr;
    hipStream_t copy = nullptr;
    hipEvent_t raw_ev = nullptr, copy_ev = nullptr;
    void* d_raw2 = nullptr;  // the reference normals' upload staging (copy stream, beside d_raw's points)
    size_t raw2_bytes = 0;
    hipEvent_t nrm_ev = nullptr;
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
    size_t rd_bytes = 0;
    void* d_rd_p4 = nullptr;       // set_reading scratch: the packed reading before / after the slot sort
    void* d_rd_sorted = nullptr;
    size_t rd_p4_bytes = 0, rd_sorted_bytes = 0;
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
    int64_t vt_n = -1;  // distances the last VarTrimmed launch sorted (its scratch layout; -1: none)
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
    // Stall-and-replay of a sharded device loop (pmx_loop_capi.hip): the host
    // reads the window verdict back (a stream synchronisation per iteration)
    // only until kAsyncAfterHits hits in a row; after that it enqueues whole
    // iterations without reading it, a miss stalls the loop on the device
    // (kCtlStalled) and the batch check replays the stalled iteration.
    int shard_hit_streak = 0;
    bool shard_async = false;     // the iteration being enqueued does not read its verdict back
    bool shard_replay = false;    // the iteration being enqueued replays a stalled one (its match ran)
    bool spec_fresh = false;      // the window is empty (a loop's first iteration): a known miss
    int64_t enq_iter = -1;        // loop iteration being enqueued (-1: not in a loop)
    uint64_t n_verdict_sync = 0, n_async = 0, n_stall = 0;  // pmx_comm_loop_stats
    std::vector<int64_t> debug_force_miss;  // option force_miss: loop iterations whose window pick misses
    size_t h_stage_cap = 0;
    unsigned long long* d_specx = nullptr;  // quantile window exchange: own segment, then nranks gathered

    // device-resident loop (pmx_loop.hip)
    LoopCtl* d_ctl = nullptr;     // control word read by every kernel in loop mode
    void* d_gdesc = nullptr;      // GridDesc<T>[levels]
    void* d_loop = nullptr;       // LoopState<T>
    void* d_loop_T0 = nullptr;    // initial T_iter (upload)
    void* d_trace = nullptr;      // T_iter per iteration (keep_trace)
    long long* d_diag = nullptr;  // per-iteration diagnostics ring (kDiagCap x kDiagWords, pmx_loop_diag)
    unsigned int* d_ticket = nullptr;  // finalize_step_kernel's arrival ticket (0 between launches)
    // device loop, one rank: the minimiser's last finalize is left to the
    // fused finalize + step launch (final_out / final_nv: its accumulators)
    bool fuse_final = false;
    double* final_out = nullptr;
    int final_nv = 0;
    int64_t trace_cap = 0;        // iterations
    bool loop_on = false;         // enqueueing loop iterations
    // quantile window fused into the grid match (pmx_spec.h): device loop,
    // single rank, quantile filter at chain position 0 (option spec_select=0: off)
    SpecSel* d_spec = nullptr;
    void* d_spec_keys = nullptr;
    bool spec_allowed = true;
    bool spec_on = false;
    // device loop, single rank, window on, quantile at chain position 0: the
    // match's counter phase runs inside the select launch (every block folds
    // the counters, pmx_selectall.h counter_merged), one launch fewer per
    // iteration; the point-to-plane launch then zeroes the spread counters
    bool merge_counter = false;  // (set for the match being enqueued)
    bool step_counter = false;   // (the match's counter phase runs in the fused finalize + step launch)
    bool vpart_dirty = false;    // (the merged counter phase read them: the next reduction zeroes them)
    SpecSel spec_init{};  // (host staging of the reset)
    SpecSel* spec_now() const { return spec_on && loop_on ? d_spec : nullptr; }
    bool loop_begun = false;
    pmx_loop_cfg loop_cfg{};
    LoopCfg loop_dev{};
    void* h_loop = nullptr;       // pinned: two copies of the status block (the batches in flight)
    hipEvent_t loop_ev[2] = {nullptr, nullptr};  // end of the batches in flight
    hipEvent_t loop_stage_ev = nullptr;          // pmx_loop_begin's uploads have left the pinned staging
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

namespace pmxc {

extern thread_local std::string g_err;  // message of a failed standalone call (pmx_last_error(NULL))
int fail(pmx_ctx* c, int code, const std::string& msg);

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

size_t tsize(const pmx_ctx* c);
// the device loop's control word while iterations are being enqueued
const LoopCtl* loop_ctl(const pmx_ctx* c);
LoopCtl* loop_on_ctl(pmx_ctx* c);  // (the same, writable: the kernels that stop the loop)
int ensure(pmx_ctx* c, void** p, size_t* cap, size_t bytes);

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

// collectives of a sharded ICP (pmx_capi.hip)
bool sharded(const pmx_ctx* c);
int coll_allreduce(pmx_ctx* c, void* dbuf, int64_t count, int type, int op);
int coll_allgather(pmx_ctx* c, const void* dsend, void* drecv, size_t bytes);
int allreduce_f64(pmx_ctx* c, double* buf, size_t n);
// match timing events
void resolve_events(pmx_ctx* c);
hipEvent_t get_event(pmx_ctx* c);

// pmx_chain.hip (instantiated for float and double)
void setup_release(pmx_ctx* c);
int upload_raw(pmx_ctx* c, const void* src, size_t bytes);
int host_order(pmx_ctx* c);
int select_reset(pmx_ctx* c);
int ensure_level(pmx_ctx* c, int l);     // grid level l built (pmx_chain.hip)
double host_limit(const pmx_ctx* c);
void fill_stats(const pmx_ctx* c, pmx_stats* st, double kept, double nz, double rm, double rp, double sw,
                double limit);
void side_join(pmx_ctx* c);
void side_finish(pmx_ctx* c);
template <typename T>
int set_reference_impl(pmx_ctx* c, const T* feat, int rows, int64_t M, const T* normals, const T* offset = nullptr,
                       T* mean_out = nullptr);
template <typename T>
int set_reading_impl(pmx_ctx* c, const T* feat, int rows, int64_t N, const T* T0);
template <typename T>
int match_impl(pmx_ctx* c, const T* Titer, int knn, double maxDist, uint64_t* visited);
template <typename T>
int outlier_impl(pmx_ctx* c, int kind, int chain_pos, double p0, double p1, double p2);
template <typename T>
int outlier_robust_impl(pmx_ctx* c, int pos, int fct, double tuning, double approx, int mode, double target,
                        int p2pl);
template <typename T>
int p2plane_enqueue(pmx_ctx* c);
template <typename T>
int p2point_enqueue(pmx_ctx* c);
template <typename T>
int get_matches_impl(pmx_ctx* c, void* dists, int32_t* ids);
template <typename V>
int unpermute(pmx_ctx* c, const std::vector<V>& src, V* dst, int k);

}  // namespace pmxc

#define DISPATCH(c, call_f, call_d) ((c)->dtype == PMX_F64 ? (call_d) : (call_f))
