// pmx_capi.hip — the C ABI of include/pmx.h: context lifecycle (device,
// stream, the iteration / status block, the select and reduction scratch),
// collectives (RCCL over xGMI or caller callbacks), timing.  The module and
// loop entry points are in pmx_chain.hip / pmx_loop_capi.hip, the data
// filters in pmx_filters_capi.hip (pmx_ctx.h lists them).
#include "pmx_ctx.h"

#include <chrono>

namespace pmxc {

thread_local std::string g_err;  // message of a failed standalone call (pmx_last_error(NULL))

int fail(pmx_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

size_t tsize(const pmx_ctx* c) { return c->dtype == PMX_F64 ? 8 : 4; }

// the device loop's control word while iterations are being enqueued
const LoopCtl* loop_ctl(const pmx_ctx* c) { return c->loop_on ? c->d_ctl : nullptr; }
LoopCtl* loop_on_ctl(pmx_ctx* c) { return c->loop_on ? c->d_ctl : nullptr; }

int ensure(pmx_ctx* c, void** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes && *p) return PMX_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCHK(c, hipMalloc(p, bytes > 0 ? bytes : 16));
    *cap = bytes;
    return PMX_OK;
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

// all-gather `bytes` per rank: recv holds nranks blocks in rank order (send
// may be this rank's block of recv: in place)
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

// ---------------------------------------------------------------- options --
// The developer options of a context (README "Options"): switches between
// measured alternatives and test hooks, set from PMX_OPTS="name=value,..." at
// pmx_ctx_create or one at a time by pmx_ctx_set_option.  Lists (grid_levels,
// force_miss) are ':'-separated.  An unknown name or a malformed value is an
// error (PMX_E_BAD_PARAM), never silently ignored.
int set_option(pmx_ctx* c, const std::string& key, const std::string& val) {
    auto num = [&](double& out) -> bool {
        if (val.empty()) return false;
        char* end = nullptr;
        out = std::strtod(val.c_str(), &end);
        return end && *end == 0 && out == out;
    };
    auto list = [&](std::vector<double>& out) -> bool {
        out.clear();
        size_t p = 0;
        while (p <= val.size()) {
            const size_t q = std::min(val.find(':', p), val.size());
            const std::string t = val.substr(p, q - p);
            char* end = nullptr;
            const double x = std::strtod(t.c_str(), &end);
            if (t.empty() || !end || *end != 0 || x != x) return false;
            out.push_back(x);
            p = q + 1;
        }
        return !out.empty();
    };
    double v = 0;
    std::vector<double> xs;
    bool ok = true;
    if (key == "grid_mode") {
        ok = val == "tile" || val == "lane";
        if (ok) c->grid_mode = val == "tile" ? 0 : 1;
    } else if (key == "grid_levels") {  // points per occupied cell of each level, e.g. 2:8:32 (one value: one level)
        ok = list(xs);
        for (double x : xs) ok = ok && x >= 0.25;
        if (ok) c->level_ppc = xs;
    } else if (key == "first_ppc") {
        ok = num(v) && v >= 0.25;
        if (ok) c->first_ppc = v;
    } else if (key == "force_miss") {  // test hook: device-loop iterations whose sharded window pick misses
        ok = list(xs);
        if (ok) {
            c->debug_force_miss.clear();
            for (double x : xs) c->debug_force_miss.push_back((int64_t)x);
        }
    } else if ((ok = num(v))) {
        const bool b = v != 0;
        if (key == "tile_max") c->tile_max = (uint32_t)std::max(0.0, v);
        else if (key == "nbr_cache") c->nbr_on = b;
        else if (key == "spec_select") c->spec_allowed = b;
        else if (key == "grid_adapt") c->adaptive = b;
        else if (key == "grid_reuse") c->reuse_on = b;
        else if (key == "tile_dispatch") c->tile_dispatch_req = v < 0 ? -1 : (b ? 1 : 0);
        else if (key == "coop_max") c->coop_max = (int)std::max(0.0, std::min(256.0, v));
        else if (key == "fuse_step") c->fuse_step = b;
        else if (key == "step_counter") c->step_counter_on = b;
        else if (key == "p2p_onepass") c->p2p_onepass = b;
        else if (key == "side_levels") c->side_levels = b;
        else if (key == "reading_copy") c->reading_copy = b;
        else if (key == "reading_order") c->reading_order = b;
        else if (key == "loop_batch") c->loop_batch = (int)std::max(0.0, v);
        else if (key == "wave_fill") c->wave_fill = std::max(1.0, v);
        else if (key == "setup_trace") c->setup_trace = (int)v;
        else if (key == "tile_prof") {
            c->tile_prof = b;
            c->tile_prof_raw = v >= 2;
        }
        else if (key == "vt_trace") g_vt_trace = (int)v;
        else ok = false;
    }
    if (!ok) return fail(c, PMX_E_BAD_PARAM, "unknown option or bad value: " + key + "=" + val);
    return PMX_OK;
}

int set_options(pmx_ctx* c, const char* s) {
    const std::string all(s);
    size_t p = 0;
    while (p < all.size()) {
        const size_t q = std::min(all.find(',', p), all.size());
        const std::string item = all.substr(p, q - p);
        p = q + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) return fail(c, PMX_E_BAD_PARAM, "option without a value: " + item);
        if (int rc = set_option(c, item.substr(0, eq), item.substr(eq + 1))) return rc;
    }
    return PMX_OK;
}

}  // namespace pmxc

using namespace pmxc;

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
    // developer options (defaults are the measured optimum on MI355X)
    if (const char* e = std::getenv("PMX_OPTS")) {
        if (set_options(c, e) != PMX_OK) {
            g_err = c->err;
            delete c;
            return PMX_E_BAD_PARAM;
        }
    }
    auto bad = [&](int code) {
        pmx_ctx_destroy(c);
        return code;
    };
    if (hipSetDevice(device) != hipSuccess) return bad(PMX_E_HIP);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->cu_count = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bad(PMX_E_HIP);
    static bool preloaded = false;  // (once per process; modules are per process)
    if (!preloaded) {
        // (option setup_trace: each module's load time on stderr)
        auto timed = [&](const char* name, void (*f)()) {
            const auto t0 = std::chrono::steady_clock::now();
            f();
            if (c->setup_trace)
                std::fprintf(stderr, "preload %s %.2f ms\n", name,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        };
        timed("match", preload_match);
        timed("grid", preload_grid);
        timed("select", preload_select);
        timed("reduce", preload_reduce);
        timed("loop", preload_loop);
        timed("normals", preload_normals);
        timed("setup", preload_setup);
        timed("ssn", preload_ssn);
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

int pmx_ctx_set_option(pmx_ctx* c, const char* name, const char* value) {
    if (!c || !name || !value) return fail(c, PMX_E_BAD_PARAM, "null argument");
    return set_option(c, name, value);
}

int pmx_ctx_destroy(pmx_ctx* c) {
    if (!c) return PMX_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void* bufs[] = {c->d_safe, c->d_ref,  c->d_nrm,      c->d_rd,     c->d_dists,  c->d_ids,   c->d_w,    c->d_part_d,
                    c->d_part_i, c->d_hist,   c->d_vt,     c->d_deno,  c->d_gather, c->d_partials,
                    c->d_result, c->d_waves, c->d_vpart,
                    c->d_sel_more, c->d_gdesc, c->d_loop_T0, c->d_trace, c->d_diag, c->d_ticket, c->d_nbr,
                    c->d_spec, c->d_spec_keys, c->d_order, c->d_raw, c->d_bbox, c->d_occ, c->d_selx,
                    c->d_rob, c->d_rdev, c->d_radii, c->d_rd_p4, c->d_rd_sorted};
    side_finish(c);  // (the side stream may still be building levels)
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    for (auto& L : c->levels) L.release();
    setup_release(c);
    if (c->h_result) (void)hipHostFree(c->h_result);
    if (c->h_loop) (void)hipHostFree(c->h_loop);
    for (hipEvent_t e : c->loop_ev)
        if (e) (void)hipEventDestroy(e);
    if (c->loop_stage_ev) (void)hipEventDestroy(c->loop_stage_ev);
    for (auto& pr : c->ev_pending) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    if (c->d_specx) (void)hipFree(c->d_specx);
    if (c->side_ev) (void)hipEventDestroy(c->side_ev);
    if (c->side_start_ev) (void)hipEventDestroy(c->side_start_ev);
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->d_raw2) (void)hipFree(c->d_raw2);
    for (hipEvent_t e : {c->table_ev, c->raw_ev, c->copy_ev, c->nrm_ev})
        if (e) (void)hipEventDestroy(e);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->h_table) (void)hipHostFree(c->h_table);
    if (c->side) (void)hipStreamDestroy(c->side);
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

int pmx_comm_loop_stats(const pmx_ctx* c, uint64_t* verdict_syncs, uint64_t* async_iterations, uint64_t* stalls) {
    if (!c || !verdict_syncs || !async_iterations || !stalls) return PMX_E_BAD_PARAM;
    *verdict_syncs = c->n_verdict_sync;
    *async_iterations = c->n_async;
    *stalls = c->n_stall;
    return PMX_OK;
}

int pmx_comm_size(const pmx_ctx* c, int* nranks, int* rank, int* kind) {
    if (!c) return PMX_E_BAD_PARAM;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (kind) *kind = c->comm ? 1 : c->host_ar ? 2 : 0;
    return PMX_OK;
}

int pmx_get_shape(const pmx_ctx* c, int64_t* n_local, int* knn) {
    if (!c) return PMX_E_BAD_PARAM;
    if (n_local) *n_local = c->N;
    if (knn) *knn = c->knn;
    return PMX_OK;
}

int pmx_grid_level_records(pmx_ctx* c, int level, int64_t* count, int32_t* ids, void* points, void* normals) {
    if (!c || !count) return fail(c, PMX_E_BAD_PARAM, "null argument");
    if (!c->grid_ready || level < 0 || level >= (int)c->levels.size())
        return fail(c, PMX_E_BAD_PARAM, "pmx_grid_level_records: no such grid level");
    HIPCHK(c, hipSetDevice(c->device));
    side_join(c);  // (the finer levels build on the side stream)
    int rc = ensure_level(c, level);
    if (rc) return rc;
    const GridLevel& L = c->lv(level);
    const int64_t n = c->grid_valid;
    *count = n;
    if (normals && !L.gpn) return fail(c, PMX_E_STATE, "pmx_grid_level_records: the reference has no normals");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t rec = 4 * (c->dtype == PMX_F64 ? sizeof(double) : sizeof(float));
    if (ids) HIPCHK(c, hipMemcpy(ids, L.gidx, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost));
    if (points) HIPCHK(c, hipMemcpy(points, L.gpts, rec * (size_t)n, hipMemcpyDeviceToHost));
    if (normals) {  // (the interleaved point / normal records: every second one)
        HIPCHK(c, hipMemcpy2D(normals, rec, (const char*)L.gpn + rec, 2 * rec, rec, (size_t)n, hipMemcpyDeviceToHost));
    }
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

}  // extern "C"
