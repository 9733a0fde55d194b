// pmx_loop_capi.hip — pmx_loop_begin / _run / _trace (include/pmx.h): whole
// ICP iterations (ICP.cpp:371-430) enqueued back to back on the context
// stream, transform, level and stop flag kept on the device (pmx_loop.hip).
#include "pmx_ctx.h"

#include <cstdlib>

namespace pmxc {

// ------------------------------------------------------------ device loop --
// pmx_loop_*: whole ICP iterations enqueued back to back (pmx_loop.hip).  The
// host checks the stop flag once per batch of iterations while the next batch
// is already queued, so the GPU never waits for the host; after a stop the
// queued iterations return at once (every kernel reads LoopCtl.done).  Batches
// of kLoopBatch while an ICP is young (one that stops early runs few no-op
// iterations), of kLoopBatchLong from iteration kLoopBatchAfter on: one status
// copy per 8 iterations.  Same-box means of four runs at C3: driver 0.06728 vs
// 0.06775 ms/iteration with 4 throughout (8 throughout 0.0673), whole ICP
// 0.0932 vs 0.0939 — small; 2 throughout is slower (0.068-0.071).
// Option loop_batch fixes one size (A/Bs).
constexpr int kLoopBatch = 4;
constexpr int kLoopBatchLong = 8;
constexpr int kLoopBatchAfter = 8;
// pinned status slot s (a copy of the device status block)
const char* stat_slot(const pmx_ctx* c, int s) { return (const char*)c->h_loop + (size_t)s * kStatBytes; }
// pinned staging of pmx_loop_begin's uploads, after the two status slots
constexpr size_t kLoopStage = 256 + ((sizeof(SpecSel) + 255) & ~(size_t)255);


template <typename T>
int loop_begin_impl(pmx_ctx* c, const pmx_loop_cfg* cfg, const T* T0) {
    if (!c->d_ref) return fail(c, PMX_E_STATE, "no reference (Matcher::init not called)");
    if (!c->d_rd && c->N > 0) return fail(c, PMX_E_STATE, "no reading");
    if (c->search_type == 0 || !c->grid_ready || c->grid_mode == 0)
        return fail(c, PMX_E_BAD_PARAM, "device loop: needs the per-lane grid matcher (searchType 1 or 2)");
    if (cfg->knn < 1) return fail(c, PMX_E_BAD_PARAM, "knn must be >= 1");
    if (!(cfg->max_dist >= 0)) return fail(c, PMX_E_BAD_PARAM, "maxDist must be >= 0");
    if (cfg->n_filters < 0 || cfg->n_filters > kMaxChain)
        return fail(c, PMX_E_BAD_PARAM, "device loop: at most 8 outlier filters");
    int n_robust = 0;
    for (int i = 0; i < cfg->n_filters; ++i) {
        const int k = cfg->filter_kind[i];
        const double* p = cfg->filter_p[i];
        if (k < PMX_FILTER_DEFAULT || k > PMX_FILTER_ROBUST || (k == PMX_FILTER_DEFAULT && i != 0))
            return fail(c, PMX_E_BAD_PARAM, "device loop: unknown outlier filter");
        if (k == PMX_FILTER_ROBUST) {
            ++n_robust;
            if (cfg->robust_fct < PMX_RF_CAUCHY || cfg->robust_fct > PMX_RF_STUDENT ||
                cfg->robust_estimator < PMX_RSE_NONE || cfg->robust_estimator > PMX_RSE_BERG)
                return fail(c, PMX_E_BAD_PARAM, "device loop: bad RobustOutlierFilter parameters");
            // (the point-to-point kernels carry no normals: the point2plane
            // distance's weights are materialised on the module path)
            if (cfg->robust_p2pl && (cfg->minimizer != 0 || c->dim != 3))
                return fail(c, PMX_E_BAD_PARAM, "device loop: RobustOutlierFilter point2plane needs PointToPlane, 3-D");
        }
        if ((k == PMX_FILTER_MAXDIST || k == PMX_FILTER_MINDIST) && !(p[0] >= 1e-7))
            return fail(c, PMX_E_BAD_PARAM, "device loop: distance threshold < 1e-7");
        if (k == PMX_FILTER_TRIMMED && !(p[0] >= 1e-7 && p[0] <= 1.0))
            return fail(c, PMX_E_BAD_PARAM, "TrimmedDistOutlierFilter: ratio out of [1e-7, 1]");
        if (k == PMX_FILTER_VARTRIMMED && !((T)p[0] < (T)p[1]))
            return fail(c, PMX_E_BAD_PARAM, "VarTrimmedDistOutlierFilter: minRatio should be smaller than maxRatio");
    }
    if (n_robust > 1) return fail(c, PMX_E_BAD_PARAM, "device loop: one RobustOutlierFilter per chain");
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
    d.full = n_robust > 0 ? 1 : 0;  // (point-to-plane: the weighted system's full A layout)
    d.n_checkers = cfg->n_checkers;
    for (int i = 0; i < cfg->n_checkers; ++i) {
        d.checker_kind[i] = cfg->checker_kind[i];
        for (int j = 0; j < 3; ++j) d.checker_p[i][j] = cfg->checker_p[i][j];
    }
    d.adaptive = c->adaptive ? 1 : 0;
    d.reuse = c->reuse_on && c->grid_mode >= 1 ? 1 : 0;
    d.knn = cfg->knn;  // (pairs a certified query evaluates)
    // tile dispatch: a reading much denser than the reference (the tile
    // kernel's wave-shared boxes serve 64 nearby queries with one load);
    // the per-lane kernel's temporal reuse must be on (the step judges its
    // certificate failures), no reuse candidates, k within the lane lists
    {
        const bool dense = c->N >= 4 * std::max<int64_t>(c->grid_valid, 1);
        const bool want = c->tile_dispatch_req > 0 || (c->tile_dispatch_req < 0 && dense);
        d.tile_dispatch = want && d.reuse && cfg->knn < kLaneMaxK ? 1 : 0;
    }
    d.n_levels = c->levels_built;
    d.n_levels_all = (int)c->levels.size();
    for (int l = 0; l < d.n_levels_all; ++l) d.level_ppc[l] = c->lv(l).ppc;
    d.n_local = c->N;
    // (double only: in float the reference centres in T before its products,
    // and the one-pass form drifted 1.05e-5 from the per-module path over 25
    // iterations, past the 1e-5 bar; in double both are far inside 1e-12)
    d.p2p_onepass = cfg->minimizer == 1 && c->p2p_onepass && c->dtype == PMX_F64 ? 1 : 0;
    int rc;
    size_t cap = 0;
    (void)cap;  // (LoopState lives in the status block)
    cap = 0;
    if (!c->d_loop_T0 && (rc = ensure(c, &c->d_loop_T0, &cap, 16 * sizeof(double)))) return rc;
    if (!c->d_ticket) {
        HIPCHK(c, hipMalloc((void**)&c->d_ticket, 64));
        HIPCHK(c, hipMemsetAsync(c->d_ticket, 0, 64, c->stream));
    }
    if (!c->d_diag) {
        HIPCHK(c, hipMalloc((void**)&c->d_diag, sizeof(long long) * kDiagCap * kDiagWords));
        HIPCHK(c, hipMemsetAsync(c->d_diag, 0, sizeof(long long) * kDiagCap * kDiagWords, c->stream));
    }
    // pinned: two status-block slots (the batches in flight), then the
    // staging of this call's uploads (T0, the window reset): the uploads are
    // asynchronous, so the caller's T0 may go away and no host sync is needed
    if (!c->h_loop) HIPCHK(c, hipHostMalloc(&c->h_loop, 2 * kStatBytes + kLoopStage, hipHostMallocDefault));
    for (hipEvent_t& e : c->loop_ev)
        if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!c->loop_stage_ev) HIPCHK(c, hipEventCreateWithFlags(&c->loop_stage_ev, hipEventDisableTiming));
    HIPCHK(c, hipEventSynchronize(c->loop_stage_ev));  // (the last call's uploads have left the staging)
    char* stage = (char*)c->h_loop + 2 * kStatBytes;
    c->loop_cfg = *cfg;
    c->loop_dev = d;
    const int rr = c->rows * c->rows;
    std::memcpy(stage, T0, sizeof(T) * rr);
    HIPCHK(c, hipMemcpyAsync(c->d_loop_T0, stage, sizeof(T) * rr, hipMemcpyHostToDevice, c->stream));
    // the first loop match may reuse the last classic one
    // (k = 1: only if that match left its neighbour records, which the
    // loop's reuse reads)
    const bool nbr_ok = !(cfg->knn == 1 && c->nbr_on) || c->nbr_prev;
    const int prev_level = c->reuse_on && c->safe_valid && c->have_match && c->ids_grid && c->knn == cfg->knn && nbr_ok
                               ? c->ids_level
                               : -1;
    launch_loop_init<T>(c->d_ctl, (LoopState<T>*)c->d_loop, d, (const T*)c->d_loop_T0, c->level, prev_level,
                        c->Tstep, c->d_iter_err, c->stream);
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
            HIPCHK(c, hipMalloc((void**)&c->d_specx, sizeof(unsigned long long) * kSpecXStride * c->nranks));
        SpecSel init{};
        init.keys = c->d_spec_keys;
        init.ratio = (double)(T)(k0 == PMX_FILTER_TRIMMED ? cfg->filter_p[0][0] : 0.5);
        init.wide = sharded(c) ? 1 : 0;
        c->spec_init = init;
        std::memcpy(stage + 256, &c->spec_init, sizeof(SpecSel));
        HIPCHK(c, hipMemcpyAsync(c->d_spec, stage + 256, sizeof(SpecSel), hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(c, hipEventRecord(c->loop_stage_ev, c->stream));
    HIPCHK(c, hipGetLastError());
    c->loop_issued = 0;
    c->loop_iters = 0;
    c->loop_done = false;
    c->shard_done_seen = false;
    c->shard_hit_streak = 0;
    c->shard_replay = false;
    c->spec_fresh = c->spec_on && sharded(c);  // (the first pick of an empty window misses)
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

// Sharded loops read the window verdict back (one stream synchronisation per
// iteration) while the quantile is still moving: after a miss, until this
// many hits in a row.  Past that the iterations are enqueued blind (stall and
// replay, loop_run_impl).
// 0: every iteration after the loop's first is enqueued blind; a miss
// costs its stall and replay only (C3 dist at world size 1: 0.0726 with 2,
// 0.0711 with 1, 0.0694 ms with 0 — the same stalls;
// profiles/r06/scale/async_after_hits.txt)
constexpr int kAsyncAfterHits = 0;

// one ICP iteration, device-driven (transform and level from LoopCtl)
template <typename T>
int loop_enqueue_iteration(pmx_ctx* c) {
    const pmx_loop_cfg& cfg = c->loop_cfg;
    if (c->shard_done_seen) return PMX_OK;  // (every rank stops enqueuing at the same iteration)
    T Ir[16];  // (placeholder: in loop mode the kernels read the step transform from LoopCtl.T)
    for (int i = 0; i < c->rows * c->rows; ++i) Ir[i] = (i % (c->rows + 1) == 0) ? (T)1 : (T)0;
    // the match's counter phase merged into the quantile's select launch
    // (point-to-plane: its reduction zeroes the spread counters afterwards).
    // Sharded: the counter phase packs the window segment the all-gather
    // sends, so it stays a launch of its own before the collective.
    const int k0 = cfg.n_filters > 0 ? cfg.filter_kind[0] : -1;
    c->merge_counter = c->spec_on && !sharded(c) && cfg.minimizer == 0 && c->grid_mode >= 1 && c->N > 0 &&
                       cfg.knn <= kLaneMaxK && (k0 == PMX_FILTER_TRIMMED || k0 == PMX_FILTER_MEDIANDIST);
    // no quantile window (a MaxDist chain, or none): the counter phase runs
    // in the fused finalize + step launch instead (one launch fewer; the
    // step is the first reader of the counters).  Not with a robust filter:
    // its replayed iterations return before the step.
    const bool fuse_env = c->fuse_step, step_counter_env = c->step_counter_on;  // (options fuse_step, step_counter)
    bool robust = false;
    for (int i = 0; i < cfg.n_filters; ++i) robust = robust || cfg.filter_kind[i] == PMX_FILTER_ROBUST;
    c->step_counter = step_counter_env && fuse_env && !c->spec_on && !sharded(c) && !robust && c->grid_mode >= 1 &&
                      c->N > 0;
    c->vpart_dirty = false;
    c->shard_async = c->spec_on && sharded(c) && !c->shard_replay && !c->spec_fresh &&
                     c->shard_hit_streak >= kAsyncAfterHits;
    int rc;
    if (c->shard_replay) {
        // the stalled iteration: its match and window exchange ran (the
        // outputs are intact: every kernel enqueued after the stall returned
        // at once); its quantile from the radix passes, then the rest
        c->spec_exchanged = true;
        c->chain_n = 0;
        c->w_valid = false;
    } else {
        if (c->shard_async) ++c->n_async;
        rc = match_impl<T>(c, Ir, cfg.knn, cfg.max_dist, nullptr);
        if (rc) return rc;
    }
    if (cfg.n_filters == 0) {
        if ((rc = outlier_impl<T>(c, 0, 0, 0, 0, 0))) return rc;
    }
    for (int i = 0; i < cfg.n_filters; ++i) {
        const double* p = cfg.filter_p[i];
        if (cfg.filter_kind[i] == PMX_FILTER_ROBUST) {
            // RobustOutlierFilter::robustFiltering's scale schedule for this
            // loop iteration (OutlierFiltersImpl.cpp:500-531; the host module
            // counts the iterations that ran, pm_icp.cpp RobustOF)
            const int64_t call = (int64_t)cfg.robust_first_call + c->enq_iter;
            const bool recompute = cfg.robust_nb_iter_for_scale == 0 || call <= cfg.robust_nb_iter_for_scale;
            int mode = PMX_RS_NONE;
            if (cfg.robust_estimator == PMX_RSE_MAD) mode = recompute ? PMX_RS_MAD : PMX_RS_KEEP;
            else if (cfg.robust_estimator == PMX_RSE_STD) mode = recompute ? PMX_RS_STD : PMX_RS_KEEP;
            else if (cfg.robust_estimator == PMX_RSE_BERG)
                mode = !recompute ? PMX_RS_KEEP : (call == 1 ? PMX_RS_BERG_FIRST : PMX_RS_BERG_NEXT);
            if ((rc = outlier_robust_impl<T>(c, i, cfg.robust_fct, cfg.robust_tuning, cfg.robust_approx, mode,
                                             cfg.robust_berg_target, cfg.robust_p2pl)))
                return rc;
            continue;
        }
        if ((rc = outlier_impl<T>(c, cfg.filter_kind[i], i, p[0], p[1], p[2]))) return rc;
    }
    // one rank: the minimiser's last finalize and the step in one launch
    c->fuse_final = fuse_env && !sharded(c);
    c->final_out = nullptr;
    rc = cfg.minimizer == 0 ? p2plane_enqueue<T>(c) : p2point_enqueue<T>(c);
    const bool fused = c->fuse_final && c->final_out;
    c->fuse_final = false;
    const bool step_counter = c->step_counter;
    c->step_counter = false;
    if (rc) return rc;
    if (step_counter && !fused) return fail(c, PMX_E_STATE, "device loop: counter phase left unfolded");
    const int* hitp = c->spec_on && c->d_spec ? &c->d_spec->hit : nullptr;
    T* trace = cfg.keep_trace ? (T*)c->d_trace : nullptr;
    if (fused)
        launch_finalize_step<T>(c->d_partials, kRedBlocks, c->final_nv, c->final_out, c->d_result, c->d_ticket,
                                c->d_ctl, (LoopState<T>*)c->d_loop, c->d_iter_err, c->d_visited, (const T*)c->d_means,
                                c->loop_dev, trace, hitp, c->d_diag, step_counter ? c->d_vpart : nullptr, c->stream);
    else
        launch_loop_step<T>(c->d_ctl, (LoopState<T>*)c->d_loop, c->d_result, c->d_iter_err, c->d_visited,
                            (const T*)c->d_means, c->loop_dev, trace, hitp, c->d_diag, c->stream);
    HIPCHK(c, hipGetLastError());
    c->shard_replay = false;
    return PMX_OK;
}

template <typename T>
int loop_run_impl(pmx_ctx* c, int n, pmx_loop_status* st) {
    if (!c->loop_begun) return fail(c, PMX_E_STATE, "pmx_loop_begin must be called first");
    if (n < 0) return fail(c, PMX_E_BAD_PARAM, "negative iteration count");
    int rc = PMX_OK;
    // (iterations issued by this call: c->loop_issued - start; a stall
    // winds loop_issued back to the stalled iteration)
    const int64_t start = c->loop_issued;
    int slot = 0, last_slot = -1;
    int fly[2], nfly = 0, head = 0;
    bool stop = c->loop_done;
    c->loop_on = true;
    while (!stop && rc == PMX_OK) {
        while (c->loop_issued - start < n && nfly < 2 && rc == PMX_OK) {
            const int fixed = c->loop_batch;  // (option loop_batch)
            // (sharded loops keep batches of 4: a stall replays from the stalled
            // iteration, and the rest of its batch ran as no-ops; world size 1
            // over RCCL 0.0812 with 8 vs 0.077 ms/iteration)
            const int kb = fixed                                                   ? fixed
                           : !sharded(c) && c->loop_issued >= kLoopBatchAfter ? kLoopBatchLong
                                                                               : kLoopBatch;
            const int b = (int)std::min<int64_t>(kb, n - (c->loop_issued - start));
            if (c->loop_cfg.keep_trace && (rc = loop_trace_room<T>(c, c->loop_issued + b))) break;
            for (int i = 0; i < b && rc == PMX_OK; ++i) {
                c->enq_iter = c->loop_issued + i;
                rc = loop_enqueue_iteration<T>(c);
            }
            c->enq_iter = -1;
            if (rc) break;
            c->loop_issued += b;
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
        if (e != hipSuccess) {
            rc = fail(c, PMX_E_HIP, std::string("loop batch: ") + hipGetErrorString(e));
            break;
        }
        const LoopState<T>* Sb = (const LoopState<T>*)(stat_slot(c, s) + kStatLoop);
        if (!Sb->done && Sb->want_level >= c->levels_built) {
            // a coarser grid level wanted: built now (enqueued after the
            // batch in flight), offered to the step kernels enqueued next
            if ((rc = ensure_level(c, Sb->want_level)) != PMX_OK) break;
            c->loop_dev.n_levels = c->levels_built;
        }
        if (Sb->done) {
            stop = true;
        } else if (((const LoopCtl*)(stat_slot(c, s) + kStatCtl))->done == kCtlStalled) {
            // A sharded window pick missed in an iteration whose verdict was
            // not read: every kernel after it returned at once (the
            // collectives were still issued, identically on every rank).  Let
            // the later batch drain, then replay from the stalled iteration:
            // its radix passes and the rest of it (loop_enqueue_iteration),
            // then the iterations that were skipped.
            while (rc == PMX_OK && nfly > 0) {
                const hipError_t e2 = hipEventSynchronize(c->loop_ev[fly[head]]);
                if (e2 != hipSuccess) rc = fail(c, PMX_E_HIP, std::string("loop batch: ") + hipGetErrorString(e2));
                head = (head + 1) % 2;
                --nfly;
            }
            if (rc) break;
            c->loop_issued = Sb->iter;  // (the stalled iteration: matched, not yet filtered / minimised)
            c->shard_replay = true;
            c->shard_hit_streak = 0;
            ++c->n_stall;
            hipError_t e3 = hipMemsetAsync(&c->d_ctl->done, 0, sizeof(int), c->stream);
            if (e3 != hipSuccess) rc = fail(c, PMX_E_HIP, std::string("loop replay: ") + hipGetErrorString(e3));
        }
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

}  // namespace pmxc

using namespace pmxc;

extern "C" {

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

int pmx_loop_diag(pmx_ctx* c, int first, int count, int64_t* out) {
    if (!c || (!out && count > 0)) return fail(c, PMX_E_BAD_PARAM, "null argument");
    if (!c->loop_begun || !c->d_diag) return fail(c, PMX_E_STATE, "no device loop");
    if (first < 0 || count < 0 || first + count > c->loop_iters || count > kDiagCap ||
        (int64_t)c->loop_iters - first > kDiagCap)
        return fail(c, PMX_E_BAD_PARAM, "diagnostics range beyond the completed iterations or the ring");
    (void)hipSetDevice(c->device);
    std::vector<long long> ring((size_t)kDiagCap * kDiagWords);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(ring.data(), c->d_diag, sizeof(long long) * ring.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < count; ++i)
        for (int w = 0; w < kDiagWords; ++w)
            out[(size_t)i * kDiagWords + w] = (int64_t)ring[(size_t)((first + i) % kDiagCap) * kDiagWords + w];
    return PMX_OK;
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

}  // extern "C"
