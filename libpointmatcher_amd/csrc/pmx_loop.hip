// pmx_loop.hip — the device-resident ICP iteration (ICP.cpp:371-430 with the
// host solve moved onto the GPU).
//
// The classic path syncs once per iteration: the host reads the normal
// equations back, solves them, updates T_iter, runs the transformation
// checkers and launches the next match — the GPU idles for the round trip
// (~25-30 us at C3, 15 % of an iteration).  In loop mode the host enqueues
// whole iterations back to back; the last kernel of each iteration is
// loop_step_kernel (one lane) which does what the host did:
//   * quantile / empty-match errors of the iteration (ConvergenceError),
//   * PointToPlane: solvePossiblyUnderdetermined on the 6x6 / 3x3 system and
//     the rigid step (PointToPlane.cpp:108-161, 245-312); PointToPoint: the
//     SVD of the cross-covariance (PointToPoint.cpp:61-101),
//   * T_iter = dT * T_iter (ICP.cpp:419),
//   * the checkers in chain order: Counter, Differential, Bound
//     (TransformationCheckersImpl.cpp:45-225), with the reference's stop /
//     exception semantics,
//   * the next iteration's grid level (same rule as choose_level),
// and publishes the next step transform and level in the LoopCtl word every
// kernel of the next iteration reads.  Once a checker stops the loop (or an
// error is raised) the remaining enqueued iterations return at once.  The
// same dense code (common/pmx_dense.h) runs on the host in classic mode.
#include "pmx_internal.h"

#include "pmx_step.h"

namespace pmx {

// The minimiser's last finalize, fused (single rank: no all-reduce between
// the reduction and the step).  Every kernel boundary costs ~4.5 us on
// MI355X (the release / acquire of the dispatch across 8 XCD L2s, measured
// in the kernel trace), so the block sums of finalize_kernel are done here,
// by the step kernel's 256 threads, in finalize_kernel's exact order (thread
// t adds blocks t, t + 256, ...; wave butterflies; (w0 + w1) + (w2 + w3)):
// the system is bit-identical to the unfused path.  fin: kNVMax doubles of
// LDS; the sums are also stored to out (the host's iteration block).
__device__ __forceinline__ double step_wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
// NVC values per block; every thread's loads issued together (the two
// blocks it adds at kRedBlocks = 512), then the butterflies
template <int NVC>
__device__ void fused_finalize_n(const double* __restrict__ partials, int nblocks, double* __restrict__ out,
                                 double* fin) {
    __shared__ double red[4][NVC];
    const int t = threadIdx.x;
    double s[NVC];
#pragma unroll
    for (int v = 0; v < NVC; ++v) s[v] = 0.0;
    int b = t;
    for (; b + 256 < nblocks; b += 512) {
        double x0[NVC], x1[NVC];
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            x0[v] = partials[(int64_t)v * nblocks + b];
            x1[v] = partials[(int64_t)v * nblocks + b + 256];
        }
#pragma unroll
        for (int v = 0; v < NVC; ++v) {
            s[v] += x0[v];
            s[v] += x1[v];
        }
    }
    for (; b < nblocks; b += 256) {
#pragma unroll
        for (int v = 0; v < NVC; ++v) s[v] += partials[(int64_t)v * nblocks + b];
    }
#pragma unroll
    for (int v = 0; v < NVC; ++v) {
        const double w = step_wave_sum(s[v]);
        if ((t & 63) == 0) red[t >> 6][v] = w;
    }
    __syncthreads();
    for (int v = t; v < NVC; v += blockDim.x) {
        const double r = (red[0][v] + red[1][v]) + (red[2][v] + red[3][v]);
        fin[v] = r;
        out[v] = r;
    }
    __syncthreads();
}
__device__ void fused_finalize(const double* __restrict__ partials, int nblocks, int nv, double* __restrict__ out,
                               double* fin) {
    switch (nv) {  // (uniform) the value counts of the minimisers' last reductions
    case 32: fused_finalize_n<32>(partials, nblocks, out, fin); break;  // point-to-plane 3-D
    case 14: fused_finalize_n<14>(partials, nblocks, out, fin); break;  // point-to-plane 2-D
    default: fused_finalize_n<9>(partials, nblocks, out, fin); break;   // point-to-point pass 2
    }
}

// The step after the minimiser (pmx_step.h).  partials != null: the fused
// finalize above (256 threads), the system then read from LDS; otherwise res
// holds it (64 threads).
template <typename T, int ROWS, int MIN>
__global__ __launch_bounds__(256) void loop_step_kernel(LoopCtl* __restrict__ ctl, LoopState<T>* __restrict__ S,
                                 const double* __restrict__ res_g, const int* __restrict__ iter_err,
                                 const unsigned long long* __restrict__ visited, const T* __restrict__ means,
                                 LoopCfg cfg, T* __restrict__ trace, const double* __restrict__ partials,
                                 int nblocks, int nv, double* __restrict__ res_out) {
    // LDS view of the iteration block's result area: the fused sums land at
    // their place (point-to-point: the second pass at +16, after the first
    // pass's sums, which are copied from res_g)
    __shared__ double fin[64];
    if (ctl->done) return;  // (uniform)
    const double* res = res_g;
    if (partials) {
        const int off = cfg.minimizer == 0 ? 0 : 16;
        if ((int)threadIdx.x < off) fin[threadIdx.x] = res_g[threadIdx.x];
        fused_finalize(partials, nblocks, nv, res_out, fin + off);
        res = fin;
    }
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    // (every global read of the step first, together: each is a memory round trip)
    const int e = *iter_err;
    const unsigned long long vis0 = visited[0], vis1 = visited[1];
    step_body<T, ROWS, MIN>(ctl, S, res, e, vis0, vis1, means, cfg, trace);
}

// reset the loop state for a new ICP (checkers' init, ICP.cpp:368-369)
template <typename T>
__global__ void loop_init_kernel(LoopCtl* __restrict__ ctl, LoopState<T>* __restrict__ S, LoopCfg cfg,
                                 const T* __restrict__ T0, int level, int prev_level, Mat4d Tprev) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int rows = cfg.rows, D = rows - 1;
    LoopState<T> z = {};
    *S = z;
    for (int i = 0; i < rows * rows; ++i) S->Titer[i] = T0[i];
    for (int ci = 0; ci < cfg.n_checkers; ++ci) {
        if (cfg.checker_kind[ci] == kCheckDifferential) {
            T q[4];
            quat_of(S->Titer, rows, rows != 4, q);
            for (int i = 0; i < 4; ++i) S->qhist[0][i] = q[i];
            for (int r = 0; r < 3; ++r) S->thist[0][r] = r < D ? S->Titer[r * rows + D] : (T)0;
            S->nhist = 1;
        } else if (cfg.checker_kind[ci] == kCheckBound) {
            if (rows == 4) {
                quat_of(S->Titer, rows, false, S->bq0);
            } else {
                S->brot2d0 = acos(S->Titer[0]);
            }
            for (int r = 0; r < 3; ++r) S->bt0[r] = r < D ? S->Titer[r * rows + D] : (T)0;
        }
    }
    ctl->done = 0;
    ctl->level = level;
    ctl->prev_level = prev_level;
    for (int i = 0; i < 16; ++i) ctl->Tprev[i] = Tprev.m[i];
    loop_publish(ctl, S->Titer, rows);
}

template <typename T>
void launch_loop_init(LoopCtl* ctl, LoopState<T>* S, const LoopCfg& cfg, const T* T0, int level, int prev_level,
                      const double* Tprev, hipStream_t s) {
    Mat4d tp;
    for (int i = 0; i < 16; ++i) tp.m[i] = Tprev[i];
    hipLaunchKernelGGL(loop_init_kernel<T>, dim3(1), dim3(64), 0, s, ctl, S, cfg, T0, level, prev_level, tp);
}
template <typename T>
void launch_loop_step(LoopCtl* ctl, LoopState<T>* S, const double* res, const int* iter_err,
                      const unsigned long long* visited, const T* means, const LoopCfg& cfg, T* trace,
                      const double* partials, int nblocks, int nv, double* res_out, hipStream_t s) {
    const unsigned th = partials ? 256 : 64;
#define PMX_STEP(R, M)                                                                                            \
    hipLaunchKernelGGL((loop_step_kernel<T, R, M>), dim3(1), dim3(th), 0, s, ctl, S, res, iter_err, visited, means, \
                       cfg, trace, partials, nblocks, nv, res_out)
    if (cfg.rows == 4) {
        if (cfg.minimizer == 0)
            PMX_STEP(4, 0);
        else
            PMX_STEP(4, 1);
    } else {
        if (cfg.minimizer == 0)
            PMX_STEP(3, 0);
        else
            PMX_STEP(3, 1);
    }
#undef PMX_STEP
}

template void launch_loop_init<float>(LoopCtl*, LoopState<float>*, const LoopCfg&, const float*, int, int,
                                      const double*, hipStream_t);
template void launch_loop_init<double>(LoopCtl*, LoopState<double>*, const LoopCfg&, const double*, int, int,
                                       const double*, hipStream_t);
template void launch_loop_step<float>(LoopCtl*, LoopState<float>*, const double*, const int*,
                                      const unsigned long long*, const float*, const LoopCfg&, float*,
                                      const double*, int, int, double*, hipStream_t);
template void launch_loop_step<double>(LoopCtl*, LoopState<double>*, const double*, const int*,
                                       const unsigned long long*, const double*, const LoopCfg&, double*,
                                       const double*, int, int, double*, hipStream_t);


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_loop() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&loop_step_kernel<float, 4, 0>));
}

}  // namespace pmx
