// pmx_chain.hip — the module-level C ABI of include/pmx.h on a context:
// the clouds and the grid levels (Matcher::init, MatchersImpl.cpp:77-83),
// the match (findClosests, :85-101), the outlier chain
// (OutlierFilter.cpp:63-103), the minimisers' systems (PointToPlane.cpp:
// 171-243, PointToPoint.cpp:61-101) and the host mirrors.  Host
// synchronisation happens once per ICP iteration, in pmx_p2plane_system /
// pmx_p2point_system, when the ~400-byte system is copied back for the host
// solve (PointToPlane.cpp:108-161).
#include "pmx_ctx.h"

#include <chrono>
#include <functional>
#include <thread>

namespace pmxc {

// -------------------------------------------------------------------- grid --
// Uniform grid of the (centred) reference for the exact shell search.  The
// cell size targets ~4 points per occupied cell: the occupied-cell count at
// two trial sizes gives the data's local dimension (surface ~2, volume ~3),
// from which the size for the target density follows.  Points are sorted by
// cell (x fastest, index order inside a cell) so every x-row of cells is one
// contiguous range.  The sizing runs on the host from three device counts;
// the build itself is pmx_setup.hip.
constexpr int64_t kMaxCells = (int64_t)1 << 26;
int cold_level(const pmx_ctx* c);
template <typename T>
int build_levels(pmx_ctx* c, int upto);
template <typename T>
int build_levels_cold(pmx_ctx* c, int cold);

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

// setup scratch for n points and grids of up to max_cells cells (the
// context's, or the side stream's)
int setup_room(pmx_ctx* c, int64_t n, int64_t max_cells, bool side = false) {
    n = std::max<int64_t>(n, 1);
    SetupScratch& sc = side ? c->setup_side : c->setup;
    int64_t& setup_n = side ? c->setup_side_n : c->setup_n;
    int64_t& setup_cells = side ? c->setup_side_cells : c->setup_cells;
    if (setup_n < n) {
        for (void* p : {(void*)sc.keys64, (void*)sc.keys64_out, (void*)sc.idx, (void*)sc.idx_out})
            if (p) (void)hipFree(p);
        sc.keys64 = sc.keys64_out = nullptr;
        sc.idx = sc.idx_out = nullptr;
        setup_n = 0;
        HIPCHK(c, hipMalloc((void**)&sc.keys64, sizeof(unsigned long long) * n));
        HIPCHK(c, hipMalloc((void**)&sc.keys64_out, sizeof(unsigned long long) * n));
        HIPCHK(c, hipMalloc((void**)&sc.idx, sizeof(int32_t) * n));
        HIPCHK(c, hipMalloc((void**)&sc.idx_out, sizeof(int32_t) * n));
        sc.keys32 = (uint32_t*)sc.keys64;
        sc.keys32_out = (uint32_t*)sc.keys64_out;
        setup_n = n;
    }
    if (setup_cells < max_cells) {
        if (sc.counts) (void)hipFree(sc.counts);
        sc.counts = nullptr;
        setup_cells = 0;
        HIPCHK(c, hipMalloc((void**)&sc.counts, sizeof(uint32_t) * (size_t)(max_cells + 1)));
        setup_cells = max_cells;
    }
    const size_t tb = setup_temp_bytes(setup_n, setup_cells);
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
    side_finish(c);
    for (SetupScratch* sc : {&c->setup, &c->setup_side})
        for (void* p : {(void*)sc->keys64, (void*)sc->keys64_out, (void*)sc->idx, (void*)sc->idx_out,
                        (void*)sc->counts, sc->temp})
            if (p) (void)hipFree(p);
    c->setup = SetupScratch{};
    c->setup_side = SetupScratch{};
    c->setup_n = c->setup_cells = 0;
    c->setup_side_n = c->setup_side_cells = 0;
}

// the side stream's level builds, ordered before everything enqueued next on
// the context stream (a device-side wait: no host synchronisation)
void side_join(pmx_ctx* c) {
    if (!c->side_pending) return;
    (void)hipStreamWaitEvent(c->stream, c->side_ev, 0);
    c->side_pending = false;
}
// ... and finished on the host (before the level buffers are freed or reused)
void side_finish(pmx_ctx* c) {
    if (c->side) (void)hipStreamSynchronize(c->side);
    c->side_pending = false;
}

// Setup timeline (development trace, option setup_trace=1): each mark waits
// for the stream and prints the wall time since the previous mark to stderr
// (setup_trace=2: host wall time only, no stream synchronisation).
struct SetupTrace {
    pmx_ctx* c;
    int on;
    std::chrono::steady_clock::time_point t;
    explicit SetupTrace(pmx_ctx* cc)
        : c(cc), on(cc->setup_trace), t(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        if (on == 1) (void)hipStreamSynchronize(c->stream);
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "setup_trace %-22s %8.3f ms\n", what, std::chrono::duration<double>(n - t).count() * 1e3);
        t = n;
    }
};

// host staging of one upload (the caller's cloud, pageable) into the raw buffer
int upload_raw(pmx_ctx* c, const void* src, size_t bytes) {
    int rc = ensure(c, &c->d_raw, &c->raw_bytes, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    if (bytes) HIPCHK(c, hipMemcpyAsync(c->d_raw, src, bytes, hipMemcpyHostToDevice, c->stream));
    return PMX_OK;
}

// upload_raw on the copy stream: after the last pack that read d_raw, but
// not after the rest of the context stream (the level builds), which then
// waits for the copy on the device
int copy_stream(pmx_ctx* c) {
    if (!c->copy) {
        HIPCHK(c, hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
        HIPCHK(c, hipEventCreateWithFlags(&c->raw_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->copy_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->nrm_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->raw_ev, c->stream));
        HIPCHK(c, hipEventRecord(c->nrm_ev, c->stream));
    }
    return PMX_OK;
}

int upload_raw_async(pmx_ctx* c, const void* src, size_t bytes) {
    if (int r = copy_stream(c)) return r;
    // (ensure may free and reallocate d_raw: hipFree waits for the device)
    int rc = ensure(c, &c->d_raw, &c->raw_bytes, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    if (bytes) {
        HIPCHK(c, hipStreamWaitEvent(c->copy, c->raw_ev, 0));
        HIPCHK(c, hipMemcpyAsync(c->d_raw, src, bytes, hipMemcpyHostToDevice, c->copy));
        HIPCHK(c, hipEventRecord(c->copy_ev, c->copy));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->copy_ev, 0));
    }
    return PMX_OK;
}

// the grid levels over the resident reference d_ref (M points) and d_nrm
template <typename T>
int build_grid(pmx_ctx* c, int64_t M, const std::function<int()>& before_levels = {}) {
    SetupTrace gt(c);
    side_finish(c);  // (a previous reference's side builds write level buffers kept below)
    gt.mark("side finish");
    const P4<T>* pts = (const P4<T>*)c->d_ref;
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
    gt.mark("bbox");
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
    // distinct occupied cells at two trial sizes (device bitmaps; one host sync)
    auto occupied = [&](double ha, double hb, int64_t& oa, int64_t& ob) -> int {
        const SetupShape sa = grid_shape(lo, ext, ha), sb = grid_shape(lo, ext, hb);
        // (the count, then the per-slice bitmaps: pmx_setup.hip)
        if (sa.cells > kOccMaxCells || sb.cells > kOccMaxCells)
            return fail(c, PMX_E_BAD_PARAM, "grid sizing: trial grid beyond 129^3 cells");
        const size_t ba = (occupancy_bytes(sa.cells) + 255) & ~(size_t)255;
        int r = ensure(c, &c->d_occ, &c->occ_bytes, ba + occupancy_bytes(sb.cells));
        if (r) return r;
        char* base = (char*)c->d_occ;
        HIPCHK(c, hipMemsetAsync(base, 0, 8, c->stream));
        HIPCHK(c, hipMemsetAsync(base + ba, 0, 8, c->stream));
        launch_occupancy<T>(pts, M, sa, base, c->stream);
        launch_occupancy<T>(pts, M, sb, base + ba, c->stream);
        unsigned long long v[2] = {0, 0};
        HIPCHK(c, hipMemcpyAsync(&v[0], base, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(&v[1], base + ba, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        oa = (int64_t)v[0];
        ob = (int64_t)v[1];
        return PMX_OK;
    };
    double dim = 3.0, ppc1 = 1.0, h1 = maxe / 128.0;
    if (valid > 0) {
        const double h0 = maxe / 64.0;
        int64_t o0 = 0, o1 = 0;
        if ((rc = occupied(h0, h1, o0, o1))) return rc;
        o0 = std::max<int64_t>(1, o0);
        o1 = std::max<int64_t>(1, o1);
        gt.mark("occupancy");
        dim = std::log2((double)o1 / (double)o0);
        dim = std::min(3.0, std::max(1.0, dim));
        ppc1 = (double)valid / (double)o1;
    }
    // (the level buffers are kept: reused when the new shapes fit)
    if (c->levels.size() > c->level_ppc.size()) {
        for (size_t l = c->level_ppc.size(); l < c->levels.size(); ++l) c->levels[l].release();
        c->levels.resize(c->level_ppc.size());
    }
    std::vector<GridLevel> keep;
    keep.swap(c->levels);
    keep.resize(c->level_ppc.size());
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
    c->level_shapes = shapes;
    c->grid_valid = valid;
    c->levels_built = 0;
    // every level entry exists (kept buffers reused); the finest ones up to
    // the cold level are built now, the coarser ones on demand
    for (size_t l = 0; l < shapes.size(); ++l) {
        GridLevel L = keep[l];
        keep[l] = GridLevel{};
        L.ppc = c->level_ppc[l];
        c->levels.push_back(L);
    }
    gt.mark("sizing");
    if (before_levels && (rc = before_levels())) return rc;
    gt.mark("normals join+pack");
    return build_levels_cold<T>(c, c->adaptive ? cold_level(c) : 0);
}

// the level a new reading's first match runs on: the ppc nearest first_ppc
int cold_level(const pmx_ctx* c) {
    int best = 0;
    for (int l = 0; l < (int)c->level_ppc.size(); ++l)
        if (std::fabs(std::log(c->level_ppc[(size_t)l] / c->first_ppc)) <
            std::fabs(std::log(c->level_ppc[(size_t)best] / c->first_ppc)))
            best = l;
    return best;
}

// one level of the current reference: buffers, the build enqueued on `st`
// with scratch `sc`, the host's copy of its geometry
template <typename T>
int build_one_level(pmx_ctx* c, int l, const SetupScratch& sc, hipStream_t st) {
    const P4<T>* pts = (const P4<T>*)c->d_ref;
    const P4<T>* nrm = c->has_normals ? (const P4<T>*)c->d_nrm : nullptr;
    const int64_t M = c->M, valid = c->grid_valid;
    const int64_t np = std::max<int64_t>(valid, 1);
    auto room = [](void** p, size_t* cap, size_t bytes) -> bool {
        if (*p && *cap >= bytes) return true;
        if (*p) (void)hipFree(*p);
        *p = nullptr;
        *cap = 0;
        if (hipMalloc(p, bytes) != hipSuccess) return false;
        *cap = bytes;
        return true;
    };
    const SetupShape& s = c->level_shapes[(size_t)l];
    GridLevel& L = c->levels[(size_t)l];
    if (!nrm && L.gpn) {  // (no normals: no interleaved records, so nothing stale can be gathered)
        (void)hipFree(L.gpn);
        L.gpn = nullptr;
        L.cap_gpn = 0;
    }
    if (!room(&L.gpts, &L.cap_pts, sizeof(P4<T>) * np) || !room((void**)&L.gidx, &L.cap_idx, sizeof(int32_t) * np) ||
        !room((void**)&L.gstart, &L.cap_start, sizeof(uint32_t) * (size_t)(s.cells + 1)) ||
        (nrm && !room(&L.gpn, &L.cap_gpn, 2 * sizeof(P4<T>) * np))) {
        c->grid_ready = false;
        return fail(c, PMX_E_HIP, "grid level allocation failed");
    }
    const int r = build_level_device<T>(pts, M, nrm, s, valid, sc, (P4<T>*)L.gpts, (P4<T>*)L.gpn, L.gidx, L.gstart, st);
    if (r) {
        c->grid_ready = false;
        return fail(c, PMX_E_HIP, "grid level build failed (" + std::to_string(r) + ")");
    }

    for (int a = 0; a < 3; ++a) {
        L.lo[a] = s.lo[a];
        L.dim[a] = s.g[a];
    }
    L.h = s.h;
    return PMX_OK;
}

// the device table of levels [0, levels_built) (the device loop picks the
// level on the GPU, among the built ones)
template <typename T>
int publish_levels(pmx_ctx* c) {
    if (c->levels_built > kMaxLevels) return fail(c, PMX_E_BAD_PARAM, "at most 8 grid levels");
    if (!c->h_table) {
        HIPCHK(c, hipHostMalloc(&c->h_table, sizeof(GridDesc<double>) * kMaxLevels, hipHostMallocDefault));
        HIPCHK(c, hipEventCreateWithFlags(&c->table_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->table_ev, c->stream));
    }
    HIPCHK(c, hipEventSynchronize(c->table_ev));  // (the previous table's copy has read the staging)
    GridDesc<T>* tab = (GridDesc<T>*)c->h_table;
    for (size_t l = 0; l < (size_t)c->levels_built; ++l) {
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
    if (!c->d_gdesc) HIPCHK(c, hipMalloc(&c->d_gdesc, sizeof(GridDesc<T>) * kMaxLevels));
    // (stream-ordered and asynchronous: the host goes on — the reading's
    // upload overlaps the level builds still running)
    HIPCHK(c, hipMemcpyAsync(c->d_gdesc, tab, sizeof(GridDesc<T>) * (size_t)c->levels_built, hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->table_ev, c->stream));
    c->grid_ready = true;
    return PMX_OK;
}

// build levels [levels_built, upto] of the current reference (stream order:
// after whatever was enqueued before) and publish the device level table
template <typename T>
int build_levels(pmx_ctx* c, int upto) {
    upto = std::min(upto, (int)c->levels.size() - 1);
    if (upto < c->levels_built) return PMX_OK;
    SetupTrace tr(c);
    for (int l = c->levels_built; l <= upto; ++l) {
        int rc = build_one_level<T>(c, l, c->setup, c->stream);
        if (rc) return rc;
        c->levels_built = l + 1;
        tr.mark(l == 0 ? "level 0" : l == 1 ? "level 1" : l == 2 ? "level 2" : l == 3 ? "level 3" : "level 4+");
    }
    return publish_levels<T>(c);
}

// Matcher::init's levels: the cold one (a new reading's first match) on the
// context stream; the finer ones, which the matches after it move to, on the
// side stream with their own scratch, overlapping the reading's setup and the
// cold match (every match after a reading's first waits for them on the
// device, side_join).  Option side_levels=0: all on the context stream.
template <typename T>
int build_levels_cold(pmx_ctx* c, int cold) {
    cold = std::min(cold, (int)c->levels.size() - 1);
    if (cold <= 0 || !c->side_levels || c->levels_built > 0) return build_levels<T>(c, cold);
    if (!c->side) {
        // (the lowest priority: the context stream's cold level, reading
        // order and first match go first when both have work)
        int least = 0, greatest = 0;
        HIPCHK(c, hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCHK(c, hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, least));
        HIPCHK(c, hipEventCreateWithFlags(&c->side_ev, hipEventDisableTiming));
        HIPCHK(c, hipEventCreateWithFlags(&c->side_start_ev, hipEventDisableTiming));
    }
    int64_t cells = 1;
    for (int l = 0; l < cold; ++l) cells = std::max(cells, c->level_shapes[(size_t)l].cells);
    int rc = setup_room(c, c->M, cells, true);
    if (rc) return rc;
    // The side builds read d_ref and d_nrm: the points' pack completed before
    // build_grid read the sizing counts back, but the normals' pack was
    // enqueued on the context stream after that (before_levels) and may still
    // be waiting for its upload.  A device-side wait on everything enqueued
    // so far orders both (no host synchronisation).
    HIPCHK(c, hipEventRecord(c->side_start_ev, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->side, c->side_start_ev, 0));
    for (int l = 0; l < cold; ++l)
        if ((rc = build_one_level<T>(c, l, c->setup_side, c->side))) return rc;
    HIPCHK(c, hipEventRecord(c->side_ev, c->side));
    c->side_pending = true;
    SetupTrace tr(c);
    tr.mark("side levels enqueued");
    if ((rc = build_one_level<T>(c, cold, c->setup, c->stream))) return rc;
    tr.mark("cold level");
    c->levels_built = cold + 1;
    rc = publish_levels<T>(c);
    tr.mark("publish");
    return rc;
}

// Slot order of the reading: Morton order of the cell of the initially
// transformed point, so the 64 queries of a wave form a compact cluster
// (small shared LDS box in the tile kernel) and result writes are coalesced.
// Performance only: every kernel is order-independent up to fp64 summation
// order, and the mirrors undo the permutation.  Built on the device
// (pmx_setup.hip): the slot -> query order stays there (d_order) and is
// copied to the host only for a host mirror.
//
// Waves of the tile kernel (option grid_mode=tile only): a wave takes up to 64
// consecutive slots but never crosses the boundary of an aligned Morton
// block of 2^L cells per side, so its queries never straddle two distant
// regions (a straddling wave would share one huge LDS box).  L is the
// smallest level whose wave count stays within `fill` (default 1.25, option
// wave_fill) of ceil(N / 64).
std::vector<uint32_t> tile_waves(const std::vector<unsigned long long>& key, int64_t N, double fill) {
    std::vector<uint32_t> waves;
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
// the reference mean in T, ICP.cpp:291-292: each coordinate's sum sequential
// in point order (the sums in one pass), divided by M
template <typename T>
void reference_mean(const T* f, int rows, int64_t M, T* mean) {
    T sum[3] = {0, 0, 0};
    if (rows == 4) {
        for (int64_t j = 0; j < M; ++j) {
            sum[0] = sum[0] + f[j * 4];
            sum[1] = sum[1] + f[j * 4 + 1];
            sum[2] = sum[2] + f[j * 4 + 2];
        }
    } else {
        for (int64_t j = 0; j < M; ++j) {
            sum[0] = sum[0] + f[j * 3];
            sum[1] = sum[1] + f[j * 3 + 1];
        }
    }
    for (int r = 0; r < rows - 1; ++r) mean[r] = sum[r] / (T)M;
}

template <typename T>
int set_reference_impl(pmx_ctx* c, const T* feat, int rows, int64_t M, const T* normals, const T* offset,
                       T* mean_out) {
    if (rows != 3 && rows != 4) return fail(c, PMX_E_BAD_PARAM, "reference must have 3 (2-D) or 4 (3-D) rows");
    if (M <= 0) return fail(c, PMX_E_BAD_PARAM, "empty reference");
    if (M > (int64_t)0x7fffffff - kTile) return fail(c, PMX_E_BAD_PARAM, "reference larger than int32 ids");
    // the grid kernels address the reference with 32-bit byte offsets
    if ((M + kTile) * (int64_t)sizeof(P4<T>) >= ((int64_t)1 << 32))
        return fail(c, PMX_E_BAD_PARAM, "reference larger than 4 GiB of points (268M float / 134M double)");
    const int D = rows - 1;
    const int64_t M_pad = ((M + kTile - 1) / kTile) * kTile;
    int rc;
    SetupTrace tr(c);
    // mean_out: the mean on a host thread while the normals, then the points
    // upload (a sequential sum, ~0.4 ms per 1M points: it hides behind the
    // ~0.5 ms of PCIe copies instead of preceding them)
    std::thread mean_thread;
    if (mean_out) {
        mean_thread = std::thread([=] { reference_mean<T>(feat, rows, M, mean_out); });
        offset = mean_out;
    }
    struct Join {
        std::thread& t;
        ~Join() {
            if (t.joinable()) t.join();
        }
    } join{mean_thread};
    // The normals cross PCIe on the copy stream, uploaded by a host thread
    // (a pageable copy blocks its caller) while this one uploads the points,
    // packs them and sizes the grid; they are packed just before the level
    // builds, which interleave them (before_levels).
    c->has_normals = normals != nullptr;
    std::thread nrm_thread;
    int nrm_rc = PMX_OK;
    const size_t nrm_bytes = sizeof(T) * (size_t)D * M;
    if (normals) {
        if ((rc = ensure(c, &c->d_nrm, &c->nrm_bytes, sizeof(P4<T>) * M))) return rc;
        if ((rc = ensure(c, &c->d_raw2, &c->raw2_bytes, std::max<size_t>(nrm_bytes, 16)))) return rc;
        if ((rc = copy_stream(c))) return rc;
        // (after the previous normals' pack, which read d_raw2)
        HIPCHK(c, hipStreamWaitEvent(c->copy, c->nrm_ev, 0));
        nrm_thread = std::thread([c, normals, nrm_bytes, &nrm_rc] {
            (void)hipSetDevice(c->device);
            hipError_t e = hipMemcpyAsync(c->d_raw2, normals, nrm_bytes, hipMemcpyHostToDevice, c->copy);
            if (e == hipSuccess) e = hipEventRecord(c->nrm_ev, c->copy);
            if (e != hipSuccess) nrm_rc = PMX_E_HIP;
        });
    }
    struct JoinN {
        std::thread& t;
        ~JoinN() {
            if (t.joinable()) t.join();
        }
    } join_n{nrm_thread};
    // (buffers kept across references; the stream orders a previous user's reads first)
    if ((rc = ensure(c, &c->d_ref, &c->ref_bytes, sizeof(P4<T>) * M_pad))) return rc;
    if ((rc = upload_raw(c, feat, sizeof(T) * (size_t)rows * M))) return rc;
    if (mean_thread.joinable()) mean_thread.join();  // (the pack reads the offset on the host)
    launch_pack_p4<T>((const T*)c->d_raw, rows, M, M_pad, (P4<T>*)c->d_ref, c->stream, offset);
    tr.mark("reference upload+pack");
    auto pack_normals = [&]() -> int {
        if (!normals) return PMX_OK;
        nrm_thread.join();
        if (nrm_rc) return fail(c, PMX_E_HIP, "normals upload failed");
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->nrm_ev, 0));
        launch_pack_nrm<T>((const T*)c->d_raw2, D, M, (P4<T>*)c->d_nrm, c->stream);
        HIPCHK(c, hipEventRecord(c->nrm_ev, c->stream));  // (d_raw2 free again after this pack)
        tr.mark("normals upload+pack");
        return PMX_OK;
    };
    HIPCHK(c, hipGetLastError());
    c->rows = rows;
    c->dim = D;
    c->M = M;
    c->M_pad = M_pad;
    c->have_match = false;
    c->grid_ready = false;
    // a resident reading keeps its slot order (any permutation is correct;
    // it was only chosen for the previous grid's locality)
    return build_grid<T>(c, M, pack_normals);
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
    SetupTrace tr(c);
    c->has_radii = false;  // (a new reading: its radii, if any, follow)
    // raw P4 reading (pack), then the slot order, then T_refMean_dataIn
    // (scratch and the resident reading kept across readings: ICPSequence
    // scans pay no allocation)
    if ((rc = ensure(c, &c->d_rd_p4, &c->rd_p4_bytes, sizeof(P4<T>) * n1))) return rc;
    void* d_p4 = c->d_rd_p4;
    // (option reading_copy=0: the reading's upload on the context stream)
    if ((rc = c->reading_copy ? upload_raw_async(c, feat, sizeof(T) * (size_t)rows * N)
                       : upload_raw(c, feat, sizeof(T) * (size_t)rows * N)))
        return rc;
    launch_pack_p4<T>((const T*)c->d_raw, rows, N, N, (P4<T>*)d_p4, c->stream);
    HIPCHK(c, hipEventRecord(c->raw_ev, c->stream));
    if ((rc = ensure(c, &c->d_rd, &c->rd_bytes, sizeof(P4<T>) * n1))) return rc;
    if (c->d_waves) (void)hipFree(c->d_waves);
    c->d_waves = nullptr;
    c->n_waves = 0;
    c->slot_query.clear();
    c->has_order = false;
    const bool order = c->grid_ready && N > 0 && c->reading_order;  // (option reading_order=0: identity slot order)
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
        if ((rc = ensure(c, &c->d_rd_sorted, &c->rd_sorted_bytes, sizeof(P4<T>) * n1))) return rc;
        void* d_sorted = c->d_rd_sorted;
        tr.mark("reading upload+pack");
        const int r = reading_order_device<T>((const P4<T>*)d_p4, N, M0, s, morton, c->setup, (P4<T>*)d_sorted,
                                              c->stream);
        if (r) return fail(c, PMX_E_HIP, "reading order failed (" + std::to_string(r) + ")");
        tr.mark("reading order");
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
            const std::vector<uint32_t> waves = tile_waves(keys, N, c->wave_fill);
            HIPCHK(c, hipMalloc((void**)&c->d_waves, sizeof(uint32_t) * waves.size()));
            HIPCHK(c, hipMemcpyAsync(c->d_waves, waves.data(), sizeof(uint32_t) * waves.size(),
                                     hipMemcpyHostToDevice, c->stream));
            c->n_waves = (int64_t)waves.size() - 1;
            tr.mark("tile wave table");
        }
        HIPCHK(c, hipGetLastError());
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
        c->level = std::min(cold_level(c), c->levels_built - 1);  // (built with the reference)
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
    if (knn < 1) return fail(c, PMX_E_BAD_PARAM, "knn must be >= 1");
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
        // a reading's first match runs on the cold level; any other match
        // may use the finer levels the side stream builds
        if (c->side_pending && (c->have_match || c->level != cold_level(c))) side_join(c);
        const GridLevel& L = c->lv(c->level);
        // warm start from the previous match of the same reading (same k):
        // its ids are positions in the level it ran on (in loop mode the
        // kernel takes that level from LoopCtl.hint_level)
        // temporal reuse: the output buffers hold this reading's previous
        // match (same k, same level) with its safe radii
        GridReuse<T> ru;
        const bool no_prev = !(c->safe_valid && c->have_match && c->ids_grid && c->knn == knn);
        if (c->reuse_on && c->grid_mode >= 1 && knn <= kLaneMaxK) {  // (the wide search keeps no safe radii)
            ru.mode = !no_prev && c->ids_level == c->level ? 2 : 1;
            ru.safe = (T*)c->d_safe;
            ru.coop_max = c->coop_max;
            for (int i = 0; i < 16; ++i) ru.Tprev.m[i] = (T)c->Tprev[i];
            if (knn == 1 && c->nbr_on && (ru.mode != 2 || c->nbr_prev || c->loop_on) &&
                       !(c->loop_on && c->loop_dev.tile_dispatch)) {
                // (a reuse match reads the records only if the last match
                // wrote them; a device-loop match decides reuse on the device,
                // where every match of the loop writes them.  Not for dense
                // readings, tile dispatch: most queries miss there, and the
                // records' writes cost more than the certificate saves, C5
                // 1.51 vs 1.47 ms/iteration)
                int rc = ensure(c, &c->d_nbr, &c->nbr_bytes, 2 * sizeof(P4<T>) * (size_t)std::max<int64_t>(c->N, 1));
                if (rc) return rc;
                ru.nbr = (P4<T>*)c->d_nbr;
                ru.gpn = (const P4<T>*)L.gpn;
            }
        }
        c->nbr_prev = ru.nbr != nullptr;
        c->nbr_normals = ru.gpn != nullptr;
        // several ranks: the counter sum packs this rank's window segment,
        // the segments are all-gathered and every rank picks from the union
        SpecSel* spec = c->spec_now();
        c->spec_exchanged = false;
        // (this rank's segment is its block of the gathered array: an in-place all-gather)
        // (d_specx is allocated by a loop_begin on a sharded context: a window
        // switched on before the context became sharded has none)
        if (spec && sharded(c) && !c->d_specx)
            HIPCHK(c, hipMalloc((void**)&c->d_specx, sizeof(unsigned long long) * kSpecXStride * c->nranks));
        unsigned long long* xseg = spec && sharded(c) ? c->d_specx + (size_t)kSpecXStride * c->rank : nullptr;
        const bool cold_now = no_prev && c->reuse_on;
        // (development profile of the cold form's waves, option tile_prof=1:
        // per wave duration, rounds and points copied, summarised on stderr)
        const bool tile_prof = c->tile_prof;
        unsigned long long* prof_buf = nullptr;
        const int64_t nw = (c->N + 63) / 64;
        if (tile_prof && cold_now) {
            HIPCHK(c, hipMalloc((void**)&prof_buf, sizeof(unsigned long long) * 4 * std::max<int64_t>(nw, 1)));
            set_tile_prof(prof_buf);
        }
        launch_grid_match<T>(c->grid_mode, (const P4<T>*)L.gpts, L.gidx, L.gstart, L.lo, L.h, L.dim,
                             (const P4<T>*)c->d_rd, c->N, c->d_waves, c->n_waves, Tm, knn, maxR2, c->tile_max,
                             (T*)c->d_dists, c->d_ids, c->d_vpart, c->merge_counter || c->step_counter ? nullptr : c->d_visited,
                             c->d_iter_err, ru, loop_ctl(c),
                             (const GridDesc<T>*)c->d_gdesc, spec, c->d_sel, xseg,
                             c->has_radii ? (const T*)c->d_radii : nullptr, cold_now,
                             c->loop_on && c->loop_dev.tile_dispatch, e0, e1, c->stream);
        if (prof_buf) {
            std::vector<unsigned long long> h((size_t)(4 * nw));
            HIPCHK(c, hipMemcpyAsync(h.data(), prof_buf, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            set_tile_prof(nullptr);
            (void)hipFree(prof_buf);
            std::vector<double> dur((size_t)nw);
            unsigned long long t0 = ~0ull, t1 = 0;
            double rsum = 0, csum = 0, fb = 0;
            for (int64_t w = 0; w < nw; ++w) {
                dur[(size_t)w] = (double)(h[4 * w + 1] - h[4 * w]) * 0.01;  // (100 MHz: us)
                t0 = std::min(t0, h[4 * w]);
                t1 = std::max(t1, h[4 * w + 1]);
                rsum += (double)(h[4 * w + 2] & 0xffffffffull);
                fb += (double)(h[4 * w + 2] >> 32);
                csum += (double)(h[4 * w + 3] & 0xffffffffull);
            }
            std::vector<double> sd = dur;
            std::sort(sd.begin(), sd.end());
            auto q = [&](double f) { return sd[(size_t)std::min<double>((double)(nw - 1), f * (double)nw)]; };
            double tot = 0;
            for (double d : dur) tot += d;
            // the last-started waves: how long after the kernel's start they began and ran
            int64_t last = 0;
            for (int64_t w = 0; w < nw; ++w)
                if (h[4 * w] > h[4 * last]) last = w;
            std::fprintf(stderr,
                         "tile_prof waves %lld span %.1f us  wave us: mean %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f"
                         "  sum %.0f us  rounds/wave %.2f  points copied/wave %.0f  fallback lanes %.0f"
                         "  last-started wave at %.1f us ran %.1f us\n",
                         (long long)nw, (double)(t1 - t0) * 0.01, tot / (double)nw, q(0.5), q(0.9), q(0.99),
                         sd.back(), tot, rsum / (double)nw, csum / (double)nw, fb, (double)(h[4 * last] - t0) * 0.01,
                         dur[(size_t)last]);
            // the waves that handed lanes to the per-lane fallback walk
            {
                double fsum = 0, fmax = 0, nmax = 0;
                int64_t fcnt = 0;
                for (int64_t w = 0; w < nw; ++w) {
                    if ((h[4 * w + 2] >> 32) > 0) {
                        ++fcnt;
                        fsum += dur[(size_t)w];
                        fmax = std::max(fmax, dur[(size_t)w]);
                    } else {
                        nmax = std::max(nmax, dur[(size_t)w]);
                    }
                }
                int64_t over = 0;  // waves over 150 us, and how many of them fell back
                int64_t over_fb = 0;
                for (int64_t w = 0; w < nw; ++w)
                    if (dur[(size_t)w] > 150.0) {
                        ++over;
                        over_fb += (h[4 * w + 2] >> 32) > 0 ? 1 : 0;
                    }
                std::fprintf(stderr,
                             "tile_prof fallback waves %lld mean %.1f us max %.1f us; other waves max %.1f us; "
                             "waves over 150 us %lld (%lld with fallback)\n",
                             (long long)fcnt, fcnt ? fsum / (double)fcnt : 0.0, fmax, nmax, (long long)over,
                             (long long)over_fb);
            }
            // (tile_prof=2: the raw per-wave words to tile_prof.bin in the working directory)
            if (c->tile_prof_raw) {
                if (FILE* f = std::fopen("tile_prof.bin", "wb")) {
                    std::fwrite(h.data(), 8, h.size(), f);
                    std::fclose(f);
                }
            }
            // duration by dispatch decile
            for (int dcl = 0; dcl < 10; ++dcl) {
                double s2 = 0;
                int64_t a = nw * dcl / 10, b = nw * (dcl + 1) / 10;
                for (int64_t w = a; w < b; ++w) s2 += dur[(size_t)w];
                std::fprintf(stderr, "tile_prof decile %d mean %.1f us\n", dcl, s2 / (double)std::max<int64_t>(b - a, 1));
            }
        }
        if (xseg) {
            if (c->N <= 0)  // (no match kernel ran: an empty segment)
                HIPCHK(c, hipMemsetAsync(xseg, 0, kSpecXHdr * sizeof(unsigned long long), c->stream));
            int rc = coll_allgather(c, xseg, c->d_specx, kSpecXStride * sizeof(unsigned long long));
            if (rc) return rc;
            const bool force = c->enq_iter >= 0 && std::find(c->debug_force_miss.begin(), c->debug_force_miss.end(),
                                                             c->enq_iter) != c->debug_force_miss.end();
            launch_spec_pick<T>(c->d_specx, c->nranks, spec, c->d_sel, loop_on_ctl(c), c->shard_async ? 1 : 0,
                                force ? 1 : 0, c->stream);
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
    ++c->n_verdict_sync;
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
        if (c->shard_replay || c->spec_fresh) {
            // a known miss (the stalled pick missed, or the window is still
            // empty): the passes below, no verdict to read
            c->spec_fresh = false;
            c->shard_hit_streak = 0;
        } else if (c->shard_async) {
            // verdict not read back: on a miss spec_pick_kernel stalled the
            // loop, and the host replays this iteration (pmx_loop_capi.hip)
            return PMX_OK;
        } else {
            const int r = sharded_window_resolved(c, spec);
            if (r < 0) return r;
            c->shard_hit_streak = r == 1 ? c->shard_hit_streak + 1 : 0;
            if (r == 1) return PMX_OK;  // (the pass kernels would return at spec->hit; no histogram exchange)
        }
    }
    if (!sharded(c)) {
        // every pass in one launch (a no-op launch when the window resolved it)
        const int64_t g = select_all_blocks(n);
        if (g != c->selx_grid) {  // (the arrival generations assume a fixed block count)
            HIPCHK(c, hipMemsetAsync(c->d_selx, 0, selx_bytes(), c->stream));
            c->selx_grid = g;
        }
        // (merged: this launch also runs the match's counter phase)
        const bool merged = c->merge_counter && spec;
        launch_select_all<T>(d, n, c->d_selx, st, ratio, ratio_dev, c->d_iter_err, loop_ctl(c), spec,
                             merged ? c->d_vpart : nullptr, merged ? c->d_visited : nullptr, c->stream);
        if (merged) c->vpart_dirty = true;
        c->merge_counter = false;
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
    if (cells > 32.0 && l + 1 < (int)c->levels.size() && ensure_level(c, l + 1) == PMX_OK) {
        next = l + 1;  // outer shells dominate: larger cells
    } else if (cells < 16.0 && l > 0) {
        // the 3x3x3 block sufficed: smaller cells evaluate fewer pairs, unless
        // the finer level was just seen walking shells (no ping-pong)
        const bool recent = c->level_seen[(size_t)l - 1] > 0 && c->match_count - c->level_seen[(size_t)l - 1] <= 3;
        if (!(recent && c->level_cells[(size_t)l - 1] > 32.0)) next = l - 1;
    }
    c->level = next;
}

// level l built (a coarser level on its first use)
// A coarser level that fails to build (allocation) leaves the grid as it was:
// the built levels stay valid and published (grid_ready kept, levels_built
// unchanged), the failed level's buffers are released, and the error is
// returned (choose_level then keeps the current level: exact, only slower).
int ensure_level(pmx_ctx* c, int l) {
    if (l < c->levels_built) return PMX_OK;
    const int built = c->levels_built;
    const bool ready = c->grid_ready;
    const int rc = c->dtype == PMX_F64 ? build_levels<double>(c, l) : build_levels<float>(c, l);
    if (rc != PMX_OK && built > 0) {
        (void)hipStreamSynchronize(c->stream);  // (the failed builds' kernels may read the buffers)
        // (levels built before the failing one were not published either)
        for (int i = built; i < (int)c->levels.size() && i <= l; ++i) c->levels[(size_t)i].release();
        c->levels_built = built;
        c->grid_ready = ready;
    }
    return rc;
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
        const bool vt_new = !c->d_vt || c->vt_bytes < need;
        if ((rc = ensure(c, &c->d_vt, &c->vt_bytes, need))) return rc;
        if (vt_new)  // (a new allocation: the radix sort's counters start at zero)
            HIPCHK(c, hipMemsetAsync(c->d_vt, 0, vartrim_scratch_head(), c->stream));
        c->vt_n = nsrc;
        // (the quantile at the optimised ratio from the sorted keys: no radix
        // passes, and on several ranks no histogram all-reduces — the sort
        // covers the gathered distances)
        launch_vartrim<T>(dsrc, nsrc, points_nbr, minR, maxR, (const T*)c->d_deno, c->d_vt, c->vt_bytes, c->d_ratio,
                          c->d_iter_err, slot, loop_ctl(c), c->stream);
        HIPCHK(c, hipGetLastError());
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
        launch_abs_dev<T>(d, n, slot, (T*)c->d_rdev, loop_ctl(c), c->stream);
        if ((rc = quantile_select<T>(c, (const T*)c->d_rdev, n, kRatioMedianIndex, nullptr, c->rob_sel()))) return rc;
        launch_robust_scale<T>(kRSMad, c->rob_sel(), nullptr, 0, 0.0, scale, loop_ctl(c), c->stream);
        smode = -1;
        break;
    case kRSStd: {  // Matches::getStandardDeviation (Matches.cpp:124-129) over all k x N
        double* sums = c->rob_sums();
        const int64_t nt = c->N_total * c->knn;  // (the mean over every rank's distances)
        launch_moment<T>(d, n, 0, sums, c->d_partials, nt, loop_ctl(c), c->stream);
        launch_finalize(c->d_partials, kRedBlocks, 1, sums, loop_ctl(c), c->stream);
        if ((rc = allreduce_f64(c, sums, 1))) return rc;
        launch_moment<T>(d, n, 1, sums, c->d_partials, nt, loop_ctl(c), c->stream);
        launch_finalize(c->d_partials, kRedBlocks, 1, sums + 1, loop_ctl(c), c->stream);
        if ((rc = allreduce_f64(c, sums + 1, 1))) return rc;
        launch_robust_scale<T>(kRSStd, nullptr, sums, c->N_total * c->knn, 0.0, scale, loop_ctl(c), c->stream);
        smode = -1;
        break;
    }
    case kRSBergFirst:  // 1.9 sqrt(getDistsQuantile(0.5))
        if ((rc = quantile_select<T>(c, d, n, 0.5, nullptr, slot))) return rc;
        launch_robust_scale<T>(kRSBergFirst, slot, nullptr, 0, 0.0, scale, loop_ctl(c), c->stream);
        smode = -1;
        break;
    default: break;
    }
    if (smode >= 0) launch_robust_scale<T>(smode, nullptr, nullptr, 0, target, scale, loop_ctl(c), c->stream);
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
    // (k = 1 after a match that left its neighbour records with normals:
    // the reduction reads them in slot order instead of gathering by id)
    const bool nbr = c->nbr_prev && c->nbr_normals && c->knn == 1 && c->ids_grid && !chain.robust;
    launch_p2plane_partial<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_pn(c), (const P4<T>*)match_nrm(c),
                              match_rs(c), (const T*)c->d_dists, c->d_ids, chain, c->knn, c->N, c->dim, c->d_partials,
                              loop_ctl(c), (const GridDesc<T>*)c->d_gdesc, c->vpart_dirty ? c->d_vpart : nullptr,
                              c->stream, nbr ? (const P4<T>*)c->d_nbr : nullptr);
    c->vpart_dirty = false;
    if (c->fuse_final) {  // (summed by the fused finalize + step launch)
        c->final_out = c->d_result;
        c->final_nv = NV;
        HIPCHK(c, hipGetLastError());
        return PMX_OK;
    }
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
    if (c->loop_on && c->loop_dev.p2p_onepass) {
        // device loop: both passes' sums in one read of the matches, the
        // step centres the moments (LoopCfg.p2p_onepass)
        launch_p2point_moments<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_ref(c), (const T*)c->d_dists,
                                  c->d_ids, chain, c->knn, c->N, c->d_partials, loop_ctl(c), gd, c->stream);
        if (c->fuse_final) {  // (summed by the fused finalize + step launch)
            c->final_out = c->d_result;
            c->final_nv = 20;
            HIPCHK(c, hipGetLastError());
            return PMX_OK;
        }
        launch_finalize(c->d_partials, kRedBlocks, 20, c->d_result, loop_ctl(c), c->stream);
        HIPCHK(c, hipGetLastError());
        return allreduce_f64(c, c->d_result, 20);
    }
    launch_p2point_pass1<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_ref(c), (const T*)c->d_dists, c->d_ids,
                            chain, c->knn, c->N, c->d_partials, loop_ctl(c), gd, c->stream);
    launch_finalize(c->d_partials, kRedBlocks, 11, c->d_result, loop_ctl(c), c->stream);
    int rc = allreduce_f64(c, c->d_result, 11);
    if (rc) return rc;
    launch_p2point_means<T>(c->d_result, (T*)c->d_means, c->dim, loop_ctl(c), c->stream);
    launch_p2point_pass2<T>((const P4<T>*)c->d_rd, Tm, (const P4<T>*)match_ref(c), (const T*)c->d_dists, c->d_ids,
                            chain, c->knn, c->N, (const T*)c->d_means, c->d_partials, loop_ctl(c), gd, c->stream);
    if (c->fuse_final) {  // (summed by the fused finalize + step launch)
        c->final_out = c->d_result + 16;
        c->final_nv = 9;
        HIPCHK(c, hipGetLastError());
        return PMX_OK;
    }
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

// ---- instantiations used by the other translation units (pmx_ctx.h) ----
#define PMX_INST(T)                                                                          \
    template int set_reference_impl<T>(pmx_ctx*, const T*, int, int64_t, const T*, const T*, T*); \
    template int set_reading_impl<T>(pmx_ctx*, const T*, int, int64_t, const T*);            \
    template int match_impl<T>(pmx_ctx*, const T*, int, double, uint64_t*);                  \
    template int outlier_impl<T>(pmx_ctx*, int, int, double, double, double);               \
    template int outlier_robust_impl<T>(pmx_ctx*, int, int, double, double, int, double, int); \
    template int p2plane_enqueue<T>(pmx_ctx*);                                              \
    template int p2point_enqueue<T>(pmx_ctx*);                                              \
    template int get_matches_impl<T>(pmx_ctx*, void*, int32_t*);                            \
    template int unpermute<T>(pmx_ctx*, const std::vector<T>&, T*, int);
PMX_INST(float)
PMX_INST(double)
#undef PMX_INST

}  // namespace pmxc

using namespace pmxc;

extern "C" {

#define DISPATCH(c, call_f, call_d) ((c)->dtype == PMX_F64 ? (call_d) : (call_f))

int pmx_set_reference(pmx_ctx* c, const void* feat, int rows, int64_t M, const void* normals) {
    if (!c || !feat) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c, set_reference_impl<float>(c, (const float*)feat, rows, M, (const float*)normals),
                    set_reference_impl<double>(c, (const double*)feat, rows, M, (const double*)normals));
}

int pmx_set_reference_centred(pmx_ctx* c, const void* feat, int rows, int64_t M, const void* normals,
                              const void* offset) {
    if (!c || !feat || !offset) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c,
                    set_reference_impl<float>(c, (const float*)feat, rows, M, (const float*)normals,
                                              (const float*)offset),
                    set_reference_impl<double>(c, (const double*)feat, rows, M, (const double*)normals,
                                               (const double*)offset));
}

int pmx_set_reference_mean_centred(pmx_ctx* c, const void* feat, int rows, int64_t M, const void* normals,
                                   void* mean_out) {
    if (!c || !feat || !mean_out) return fail(c, PMX_E_BAD_PARAM, "null argument");
    (void)hipSetDevice(c->device);
    return DISPATCH(c,
                    set_reference_impl<float>(c, (const float*)feat, rows, M, (const float*)normals, nullptr,
                                              (float*)mean_out),
                    set_reference_impl<double>(c, (const double*)feat, rows, M, (const double*)normals, nullptr,
                                               (double*)mean_out));
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
int pmx_vartrim_partial_sums(pmx_ctx* c, void* out, int64_t capacity, int64_t* count) {
    if (!c || !count) return fail(c, PMX_E_BAD_PARAM, "null argument");
    if (c->vt_n < 0 || !c->d_vt) return fail(c, PMX_E_STATE, "no VarTrimmedDist filter has run");
    // scratch layout of launch_vartrim: the 256-byte header (count), the
    // radix sort's counters (vartrim_scratch_head), two key arrays, then the
    // partial sums
    const size_t ksz = c->dtype == PMX_F64 ? 8 : 4;
    const auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    int cnt = 0;
    HIPCHK(c, hipMemcpyAsync(&cnt, (const int*)c->d_vt + vartrim_hdr_copy(), sizeof(int), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    *count = cnt;
    if (!out) return PMX_OK;
    if (capacity < cnt) return fail(c, PMX_E_BAD_PARAM, "capacity below the partial-sum count");
    const char* cum = (const char*)c->d_vt + vartrim_scratch_head() + 2 * al(ksz * (size_t)c->vt_n);
    HIPCHK(c, hipMemcpyAsync(out, cum, ksz * (size_t)cnt, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (g_vt_trace) {  // (development trace of the last walk, PMX_VT_TRACE)
        const int mx = vartrim_trace_max();
        std::vector<unsigned long long> tr(2 * (size_t)mx + 1);
        const size_t off = c->dtype == PMX_F64 ? vartrim_trace_offset<double>(c->vt_n) : vartrim_trace_offset<float>(c->vt_n);
        HIPCHK(c, hipMemcpy(tr.data(), (const char*)c->d_vt + off, 8 * tr.size(), hipMemcpyDeviceToHost));
        const int nm = (int)std::min<unsigned long long>(tr[2 * (size_t)mx], (unsigned long long)mx);
        for (int i = 0; i < nm; ++i)
            std::fprintf(stderr, "vt_trace %d t=%.2fus type=%llu chunk=%llu detail=%llu\n", i,
                         (double)(tr[2 * i] - tr[0]) * 0.01, tr[2 * i + 1] >> 56, (tr[2 * i + 1] >> 24) & 0xffffffffull,
                         tr[2 * i + 1] & 0xffffffull);
    }
    return PMX_OK;
}

int pmx_get_weights(pmx_ctx* c, void* w) {
    if (!c || !w) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return DISPATCH(c, get_weights_impl<float>(c, w), get_weights_impl<double>(c, w));
}

}  // extern "C"
