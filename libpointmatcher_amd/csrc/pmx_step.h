// pmx_step.h — the device form of the host's per-iteration work after the
// minimiser (pmx_loop.hip's step kernel and pmx_post.hip's fused launch):
//   * quantile / empty-match errors of the iteration (ConvergenceError),
//   * PointToPlane: solvePossiblyUnderdetermined on the 6x6 / 3x3 system and
//     the rigid step (PointToPlane.cpp:108-161, 245-312); PointToPoint: the
//     SVD of the cross-covariance (PointToPoint.cpp:61-101),
//   * T_iter = dT * T_iter (ICP.cpp:419),
//   * the checkers in chain order: Counter, Differential, Bound
//     (TransformationCheckersImpl.cpp:45-225), with the reference's stop /
//     exception semantics,
//   * the next iteration's grid level (the rule of choose_level, pmx_capi.hip),
// publishing the next step transform and level in the LoopCtl word every
// kernel of the next iteration reads.  One lane runs it.
#pragma once

#include "pmx_internal.h"

#include "common/pmx_dense.h"
#include "pmx_loop.h"

namespace pmx {

using namespace pmx_dense;

template <typename T>
__device__ void loop_fail(LoopCtl* ctl, LoopState<T>* S, int code, int reason) {
    S->err = code;
    S->reason = reason;
    S->done = 1;
    ctl->done = 1;
}

template <typename T>
__device__ void loop_publish(LoopCtl* ctl, const T* m, int rows) {
    // the next step transform, embedded in 4x4 as the kernels expect
    if (rows == 4) {
        for (int i = 0; i < 16; ++i) ctl->T[i] = (double)m[i];
    } else {
        const double e[16] = {m[0], m[1], 0, m[2], m[3], m[4], 0, m[5], 0, 0, 1, 0, m[6], m[7], 0, m[8]};
        for (int i = 0; i < 16; ++i) ctl->T[i] = e[i];
    }
}

template <typename T>
__device__ void quat_of(const T* M, int rows, bool init2d, T* q) {
    T m3[9];
    if (init2d) {  // TransformationCheckersImpl.cpp:107-110: 2-D init uses [R 0; 0 1]
        for (int i = 0; i < 9; ++i) m3[i] = (i % 4 == 0) ? (T)1 : (T)0;
        m3[0] = M[0];
        m3[1] = M[1];
        m3[3] = M[3];
        m3[4] = M[4];
    } else {
        // topLeftCorner(3,3): in 2-D the whole homogeneous 3x3
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) m3[r * 3 + c] = M[r * rows + c];
    }
    quat_from_matrix(m3, q);
}

// The normal equations of the point-to-plane step as T (PointToPlane.cpp:230, 243)
template <typename T, int NF>
__device__ __forceinline__ void p2plane_system_of(const double* __restrict__ res, T* A, T* b) {
    constexpr int NS = NF * (NF + 1) / 2;
    int a = 0;
    for (int i = 0; i < NF; ++i)
        for (int j = i; j < NF; ++j, ++a) A[i * NF + j] = A[j * NF + i] = (T)res[a];
    for (int i = 0; i < NF; ++i) b[i] = (T)(-res[NS + i]);
}

// Rank-deficient point-to-plane system: rare, kept out of line so that its
// dynamically indexed work arrays do not push the hot path's into scratch.
template <typename T, int NF>
__device__ __noinline__ void loop_solve_rank_deficient(const double* __restrict__ res, int full, T* __restrict__ xout) {
    T A[36], b[6], x[6];
    if (full) {
        for (int i = 0; i < NF * NF; ++i) A[i] = (T)res[i];
        for (int i = 0; i < NF; ++i) b[i] = (T)(-res[NF * NF + i]);
    } else {
        p2plane_system_of<T, NF>(res, A, b);
    }
    solve_rank_deficient(A, b, NF, x);
    for (int i = 0; i < NF; ++i) xout[i] = x[i];
}

// A sufficient condition for FullPivHouseholderQR(A).isInvertible() of the
// SPD point-to-plane system, from its LLT factor: lambda_min(A) >=
// 1 / ||L^-1||_F^2 and sigma_max(A) <= ||A||_F, so the ratio below bounds
// sigma_min / sigma_max from below.  At QR step k the trailing block B_k of
// [R11 R12; 0 B_k] has sigma_min(B_k) >= sigma_min(A) (B_k^-1 is a block of
// R^-1) and ||B_k|| <= ||A||; the pivot is B_k's largest entry, so |R_kk|
// (its column's norm) >= max|B_k| >= sigma_min(A) / n, and every pivot and
// |R_kk| <= sigma_max(A).  The rank threshold is max|R_kk| * n * eps (7.2e-7
// in float, 1.3e-15 in double): a ratio of 1e-3 (float) / 1e-9 (double)
// clears it by a factor of 230 / 1e5, far beyond the rounding of every
// quantity involved (backward error ~n^2 eps ||A||).  Below the ratio (or with a failed / non-finite
// factor) the QR decides, as before.
template <typename T, int NF>
__device__ __forceinline__ bool well_conditioned(const T* A, const T* L) {
    T inv[NF * NF], rd[NF];  // L^-1 (lower), column by column; 1 / diag (a bound: no exact division needed)
    T s = 0, fa = 0;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        ok = ok && L[k * NF + k] > (T)0;
        rd[k] = (T)1 / L[k * NF + k];
    }
#pragma unroll
    for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            if (i < j) continue;
            T v = i == j ? (T)1 : (T)0;
#pragma unroll
            for (int k = 0; k < NF; ++k)
                if (k >= j && k < i) v = v - L[i * NF + k] * inv[k * NF + j];
            v = v * rd[i];
            inv[i * NF + j] = v;
            s = s + v * v;
        }
#pragma unroll
    for (int i = 0; i < NF * NF; ++i) fa = fa + A[i] * A[i];
    const T ratio = sizeof(T) == 4 ? (T)1e-3 : (T)1e-9;
    // (NaN / inf fail every comparison below)
    return ok && s > (T)0 && s < (T)__builtin_huge_val() && fa < (T)__builtin_huge_val() &&
           (T)1 / s >= ratio * sqrt(fa);
}

// One lane: res = the minimiser's sums (point-to-plane layout, or
// point-to-point's two passes at 0 and 16), e = the iteration's error word,
// vis0 / vis1 = the match's pair evaluations and full searches.
// ROWS is the homogeneous dimension (4 in 3-D, 3 in 2-D): with every size a
// compile-time constant the dense kit's arrays live in VGPRs, not scratch
// (a single lane walking scratch took ~75 us per iteration at C3).
// MIN: the minimiser (0 point-to-plane, 1 point-to-point) as a template
// parameter, so each kernel holds one minimiser's dense code (registers).
template <typename T, int ROWS, int MIN>
__device__ __forceinline__ void step_body(LoopCtl* __restrict__ ctl, LoopState<T>* __restrict__ S,
                                       const double* __restrict__ res, int e, unsigned long long vis0,
                                       unsigned long long vis1, const T* __restrict__ means, const LoopCfg& cfg,
                                       T* __restrict__ trace) {
    constexpr int rows = ROWS, D = ROWS - 1;
    // Every global read of the step first, together: the data was written
    // by other XCDs' kernels, so each read is a memory round trip, and in
    // use order they were serialised (~1.5 us of the kernel, clock64
    // timestamps per phase on MI355X)
    const int level_now = ctl->level;
    T Tit[ROWS * ROWS];
#pragma unroll
    for (int i = 0; i < ROWS * ROWS; ++i) Tit[i] = S->Titer[i];
    T cnt[kMaxCheckers];
#pragma unroll
    for (int ci = 0; ci < kMaxCheckers; ++ci) cnt[ci] = S->cond[ci][0];
    // statistics of the iteration (ErrorElements, ErrorMinimizer.cpp:133-192)
    double kept, nz, rejM, rejP, sw;
    if (MIN == 0) {
        const int NF = D == 3 ? 6 : 3, o = (cfg.full ? NF * NF : NF * (NF + 1) / 2) + NF;
        kept = res[o];
        nz = res[o + 1];
        rejM = res[o + 2];
        rejP = res[o + 3];
        sw = res[o + 4];
    } else {
        kept = res[7];
        nz = res[8];
        rejM = res[9];
        rejP = res[10];
        sw = res[0];
    }
    S->last_level = level_now;  // the level whose positions this iteration's ids are
    // the next match may reuse this one's output (pmx_grid.hip temporal reuse)
    for (int i = 0; i < 16; ++i) ctl->Tprev[i] = ctl->T[i];
    ctl->prev_level = level_now;
    if (e) {
        loop_fail(ctl, S, e, kLoopError);
        return;
    }
    if (nz == 0.0 || kept == 0.0) {
        loop_fail(ctl, S, kLoopNoPoints, kLoopError);  // "ErrorMnimizer: no point to minimize"
        return;
    }
    // the minimiser returned: its statistics and the matcher's visit counter
    // (ICP.cpp:406-416, MatchersImpl.cpp:98)
    S->kept = kept;
    S->nz = nz;
    S->rejM = rejM;
    S->rejP = rejP;
    S->sw = sw;
    S->last_visited = vis0;
    S->touched += vis0;
    // the step transform
    T dT[16];
    if constexpr (MIN == 0) {
        constexpr int NF = D == 3 ? 6 : 3;
        T A[NF * NF], b[NF], x[NF], L[NF * NF];
        if (cfg.full) {  // (a robust chain: (w F_r) F_c in T, the reference's asymmetric wF * F^T)
#pragma unroll
            for (int i = 0; i < NF * NF; ++i) A[i] = (T)res[i];
#pragma unroll
            for (int i = 0; i < NF; ++i) b[i] = (T)(-res[NF * NF + i]);
        } else {
            p2plane_system_of<T, NF>(res, A, b);
        }
        // solve_full_rank: FullPivQR(A).isInvertible() -> LLT solve.  The
        // QR's rank test is skipped when the LLT factor proves A far from
        // rank-deficient (well_conditioned below): its answer is then known.
        llt(A, NF, L);
        bool full = well_conditioned<T, NF>(A, L);
        if (!full) {
            FullPivQR<T> qr;
            qr.compute(A, NF);
            full = qr.rank() == NF;
        }
        if (full) {
            llt_solve(L, NF, b, x);
        } else {
            loop_solve_rank_deficient<T, NF>(res, cfg.full, S->xsolve);
            for (int i = 0; i < NF; ++i) x[i] = S->xsolve[i];
        }
        p2plane_transform(rows, x, dT);
    } else {
        T m[9], mp[3], mq[3];
        if (cfg.p2p_onepass) {
            // one moments pass (launch_p2point_moments): the weighted means in
            // T (p2point_means_kernel's arithmetic), the moments centred in fp64
            const T winv = (T)1 / (T)res[0];
            for (int i = 0; i < D; ++i) {
                mp[i] = (T)res[1 + i] * winv;
                mq[i] = (T)res[4 + i] * winv;
            }
            for (int i = 0; i < D; ++i)
                for (int j = 0; j < D; ++j) {
                    const double a = (double)mq[i], bb = (double)mp[j];
                    m[i * D + j] = (T)(((res[11 + i * 3 + j] - a * res[1 + j]) - res[4 + i] * bb) + res[0] * a * bb);
                }
        } else {
            for (int i = 0; i < D; ++i) {
                mp[i] = means[i];
                mq[i] = means[3 + i];
                for (int j = 0; j < D; ++j) m[i * D + j] = (T)res[16 + i * 3 + j];
            }
        }
        p2point_transform(rows, m, mp, mq, dT);
    }
    matmul(dT, Tit, rows, Tit);
#pragma unroll
    for (int i = 0; i < ROWS * ROWS; ++i) S->Titer[i] = Tit[i];
    // transformation checkers, in chain order (TransformationCheckers::check)
    bool stop = false;
    for (int ci = 0; ci < cfg.n_checkers; ++ci) {
        const int kind = cfg.checker_kind[ci];
        if (kind == kCheckCounter) {
            T cv = cnt[0];  // (cnt[ci] by static indices: registers)
#pragma unroll
            for (int u = 1; u < kMaxCheckers; ++u)
                if (u == ci) cv = cnt[u];
            cv = cv + (T)1;
            S->cond[ci][0] = cv;
            if (cv >= (T)cfg.checker_p[ci][0]) {  // MaxNumIterationsReached: ends the loop
                stop = true;
                S->reason = kLoopCounter;
                break;  // (the exception skips the remaining checkers)
            }
        } else if (kind == kCheckDifferential) {
            const int sl = (int)cfg.checker_p[ci][2];
            T q[4];
            quat_of(Tit, rows, false, q);
            const int slot = S->nhist % kLoopHist;
            for (int i = 0; i < 4; ++i) S->qhist[slot][i] = q[i];
            for (int r = 0; r < 3; ++r) S->thist[slot][r] = r < D ? Tit[r * rows + D] : (T)0;
            ++S->nhist;
            T cv0 = 0, cv1 = 0;
            if (S->nhist > sl) {
                for (int i = S->nhist - 1; i >= S->nhist - sl; --i) {
                    const int a0 = i % kLoopHist, a1 = (i - 1) % kLoopHist;
                    cv0 = cv0 + fabs(angular_distance(S->qhist[a0], S->qhist[a1]));
                    T nn = 0;
                    for (int r = 0; r < D; ++r) {
                        const T d = S->thist[a0][r] - S->thist[a1][r];
                        nn = nn + d * d;
                    }
                    cv1 = cv1 + fabs(sqrt(nn));
                }
                cv0 = cv0 / (T)sl;
                cv1 = cv1 / (T)sl;
                if (cv0 < (T)cfg.checker_p[ci][0] && cv1 < (T)cfg.checker_p[ci][1]) {
                    stop = true;
                    S->reason = kLoopDifferential;
                }
            }
            S->cond[ci][0] = cv0;
            S->cond[ci][1] = cv1;
            if (cv0 != cv0 || cv1 != cv1) {
                loop_fail(ctl, S, cv0 != cv0 ? kLoopRotNaN : kLoopTransNaN, kLoopError);
                return;
            }
        } else {  // kCheckBound
            T cv0;
            if (rows == 4) {
                T q[4];
                quat_of(Tit, rows, false, q);
                cv0 = angular_distance(q, S->bq0);
            } else {
                T v = acos(Tit[0]) - S->brot2d0;
                while (v > (T)3.14159265358979323846) v -= (T)(2 * 3.14159265358979323846);
                while (v < (T)-3.14159265358979323846) v += (T)(2 * 3.14159265358979323846);
                cv0 = v;
            }
            T nn = 0;
            for (int r = 0; r < D; ++r) {
                const T d = Tit[r * rows + D] - S->bt0[r];
                nn = nn + d * d;
            }
            const T cv1 = sqrt(nn);
            S->cond[ci][0] = cv0;
            S->cond[ci][1] = cv1;
            if (cv0 > (T)cfg.checker_p[ci][0] || cv1 > (T)cfg.checker_p[ci][1]) {
                loop_fail(ctl, S, kLoopBound, kLoopError);
                return;
            }
        }
    }
    if (trace) {
        T* t = trace + (size_t)S->iter * rows * rows;
        for (int i = 0; i < rows * rows; ++i) t[i] = Tit[i];
    }
    ++S->iter;
    if (stop) {
        S->done = 1;
        ctl->done = 1;
        return;
    }
    // the next step starts with RigidTransformation::compute's check
    // (TransformationsImpl.cpp:62-63)
    if (fabs((T)1 - det_rot(Tit, rows)) > (T)0.001) {
        loop_fail(ctl, S, kLoopNotRigid, kLoopError);
        return;
    }
    // grid level of the next match (pmx_capi.hip choose_level)
    // (with reuse: judged on the full searches only, kept while fewer than
    // 1/16 of the queries needed one — the rule of choose_level)
    double q = (double)cfg.n_local, v = (double)vis0;
    bool adapt = cfg.adaptive && cfg.n_levels_all > 1 && cfg.n_local > 0;
    if (adapt && cfg.reuse) {
        const double full = (double)vis1;
        adapt = full * 16.0 >= q;
        v -= (double)cfg.knn * (q - full);
        q = full;
    }
    if (adapt) {
        const int l = level_now;
        const double cells = v / (q * cfg.level_ppc[l]);
        ++S->match_count;
        S->level_cells[l] = cells;
        S->level_seen[l] = S->match_count;
        int next = l;
        if (cells > 32.0 && l + 1 < cfg.n_levels) {
            next = l + 1;
        } else if (cells > 32.0 && l + 1 < cfg.n_levels_all) {
            S->want_level = l + 1;  // (built by the host at its next batch check; this level meanwhile)
        } else if (cells < 16.0 && l > 0) {
            const bool recent = S->level_seen[l - 1] > 0 && S->match_count - S->level_seen[l - 1] <= 3;
            if (!(recent && S->level_cells[l - 1] > 32.0)) next = l - 1;
        }
        ctl->level = next;
    }
    // Tile dispatch (dense readings, LoopCfg.tile_dispatch): while almost
    // every query fails the reuse certificate, the tile kernel's warm form
    // (LDS boxes shared by a wave's 64 queries) is cheaper than 64 per-lane
    // full searches.  Both forms report the queries that fail the per-lane
    // certificate (the tile form evaluates its bound without using it); the
    // tile form runs the next match while that is >= 85 % of the queries
    // (MI355X, C5: round 5 set 94 %, where the per-lane match costs about
    // what the warm tile form costs; round 6 A/B of 80 / 85 / 90 / 94 / 97 %:
    // 1.274 / 1.270 / 1.272 / 1.279 / 1.315 ms per timed iteration,
    // profiles/r06/c5/tile_dispatch_threshold.txt).
    if (cfg.tile_dispatch)
        ctl->use_tile = cfg.n_local > 0 && (double)vis1 >= 0.85 * (double)cfg.n_local ? 1 : 0;
    loop_publish(ctl, Tit, rows);
}

}  // namespace pmx
