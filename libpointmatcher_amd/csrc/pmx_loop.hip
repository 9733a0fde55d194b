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

#include "pmx_p2plane.h"
#include "pmx_spec.h"
#include "pmx_step.h"

namespace pmx {

// The step after the minimiser (pmx_step.h); res holds the system (one lane
// runs it; folding the last finalize into this launch measured slower: the
// 256-thread step launch costs more than the finalize kernel it saves,
// 0.0821 vs 0.0910 ms per iteration at C3).
template <typename T, int ROWS, int MIN>
__global__ __launch_bounds__(64) void loop_step_kernel(LoopCtl* __restrict__ ctl, LoopState<T>* __restrict__ S,
                                 const double* __restrict__ res, const int* __restrict__ iter_err,
                                 const unsigned long long* __restrict__ visited, const T* __restrict__ means,
                                 LoopCfg cfg, T* __restrict__ trace, const int* __restrict__ spec_hit,
                                 long long* __restrict__ diag) {
    if (ctl->done) return;  // (uniform)
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    // (every global read of the step first, together: each is a memory round trip)
    const int e = *iter_err;
    const unsigned long long vis0 = visited[0], vis1 = visited[1];
    const int hit = spec_hit ? *spec_hit : -1;
    if (diag) {
        long long* r = diag + (size_t)(S->iter % kDiagCap) * kDiagWords;
        r[0] = ctl->level;
        r[1] = hit;
        r[2] = (long long)vis0;
        r[3] = (long long)vis1;
    }
    step_body<T, ROWS, MIN>(ctl, S, res, e, vis0, vis1, means, cfg, trace);
}

// The minimiser's last finalize and the step in one launch (device loop, one
// rank): block v sums accumulator v exactly as finalize_kernel does
// (pmx_reduce.hip) and publishes it write-through; the last block to take a
// ticket reads the whole result block back coherently and runs the step.  It
// saves the step's own launch (a dependent kernel boundary costs ~4.6 us in
// the kernel trace here, an empty launch included: profiles/r05/anatomy).
template <typename T, int ROWS, int MIN>
__global__ __launch_bounds__(256) void finalize_step_kernel(const double* __restrict__ partials, int nblocks, int nv,
                                                            double* __restrict__ out, double* __restrict__ res,
                                                            unsigned int* __restrict__ ticket, LoopCtl* __restrict__ ctl,
                                                            LoopState<T>* __restrict__ S,
                                                            int* __restrict__ iter_err,
                                                            unsigned long long* __restrict__ visited,
                                                            const T* __restrict__ means, LoopCfg cfg,
                                                            T* __restrict__ trace, const int* __restrict__ spec_hit,
                                                            long long* __restrict__ diag,
                                                            unsigned long long* __restrict__ vpart) {
    __shared__ double red[4];
    __shared__ unsigned long long vred[2][4];
    __shared__ int s_last;
    __shared__ double sres[kStepRes];
    if (ctl->done) return;  // (uniform)
    const int v = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += 256) s += partials[(int64_t)v * nblocks + b];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        // publish (write-through), then the ticket behind a release
        __hip_atomic_store(&out[v], (red[0] + red[1]) + (red[2] + red[3]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == (unsigned)(nv - 1) ? 1 : 0;
    }
    __syncthreads();
    if (!s_last) return;  // (block-uniform)
    if (threadIdx.x < kStepRes) {
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        sres[threadIdx.x] = __hip_atomic_load(&res[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (vpart) {
        static_assert(kVSlots == 256, "one spread slot per thread");
        // the match's counter phase (counter_phase, pmx_spec.h) folded in
        // here, no window in the loop: the pair / fallback counters summed
        // and zeroed for the next match
        unsigned long long v[2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned long long* p = vpart + (size_t)(q * kVSlots + threadIdx.x) * kVStride;
            if (q < 2) v[q] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int off = 32; off > 0; off >>= 1) {
            v[0] += __shfl_xor(v[0], off);
            v[1] += __shfl_xor(v[1], off);
        }
        if ((threadIdx.x & 63) == 0) {
            vred[0][threadIdx.x >> 6] = v[0];
            vred[1][threadIdx.x >> 6] = v[1];
        }
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (the next launch starts at 0)
    const int e = *iter_err;
    unsigned long long vis0, vis1;
    if (vpart) {
        vis0 = (vred[0][0] + vred[0][1]) + (vred[0][2] + vred[0][3]);
        vis1 = (vred[1][0] + vred[1][1]) + (vred[1][2] + vred[1][3]);
        visited[0] = vis0;
        visited[1] = vis1;
        *iter_err = 0;  // (the next iteration's filters start clean; counter_phase's reset)
    } else {
        vis0 = visited[0];
        vis1 = visited[1];
    }
    const int hit = spec_hit ? *spec_hit : -1;
    if (diag) {
        long long* r = diag + (size_t)(S->iter % kDiagCap) * kDiagWords;
        r[0] = ctl->level;
        r[1] = hit;
        r[2] = (long long)vis0;
        r[3] = (long long)vis1;
    }
    step_body<T, ROWS, MIN>(ctl, S, sres, e, vis0, vis1, means, cfg, trace);
}

template <typename T>
void launch_finalize_step(const double* partials, int nblocks, int nv, double* out, double* res, unsigned int* ticket,
                          LoopCtl* ctl, LoopState<T>* S, int* iter_err, unsigned long long* visited,
                          const T* means, const LoopCfg& cfg, T* trace, const int* spec_hit, long long* diag,
                          unsigned long long* vpart, hipStream_t s) {
#define PMX_FSTEP(R, M)                                                                                          \
    hipLaunchKernelGGL((finalize_step_kernel<T, R, M>), dim3(nv), dim3(256), 0, s, partials, nblocks, nv, out, res, \
                       ticket, ctl, S, iter_err, visited, means, cfg, trace, spec_hit, diag, vpart)
    if (cfg.rows == 4) {
        if (cfg.minimizer == 0)
            PMX_FSTEP(4, 0);
        else
            PMX_FSTEP(4, 1);
    } else {
        if (cfg.minimizer == 0)
            PMX_FSTEP(3, 0);
        else
            PMX_FSTEP(3, 1);
    }
#undef PMX_FSTEP
}
template void launch_finalize_step<float>(const double*, int, int, double*, double*, unsigned int*, LoopCtl*,
                                          LoopState<float>*, int*, unsigned long long*, const float*,
                                          const LoopCfg&, float*, const int*, long long*, unsigned long long*,
                                          hipStream_t);
template void launch_finalize_step<double>(const double*, int, int, double*, double*, unsigned int*, LoopCtl*,
                                           LoopState<double>*, int*, unsigned long long*, const double*,
                                           const LoopCfg&, double*, const int*, long long*, unsigned long long*,
                                           hipStream_t);

// reset the loop state for a new ICP (checkers' init, ICP.cpp:368-369)
template <typename T>
__global__ void loop_init_kernel(LoopCtl* __restrict__ ctl, LoopState<T>* __restrict__ S, LoopCfg cfg,
                                 const T* __restrict__ T0, int level, int prev_level, Mat4d Tprev,
                                 int* __restrict__ iter_err) {
    // (the state zeroed by the whole wave, word by word: a LoopState<T> z = {}
    // copied by one lane went through scratch, ~60 us)
    static_assert(sizeof(LoopState<T>) % 4 == 0, "LoopState: whole words");
    uint32_t* sw = reinterpret_cast<uint32_t*>(S);
    for (int i = threadIdx.x; i < (int)(sizeof(LoopState<T>) / 4); i += blockDim.x) sw[i] = 0u;
    __syncthreads();
    if (threadIdx.x != 0) return;
    *iter_err = 0;  // (a loop whose counter phase runs in the step resets it after each step only)
    const int rows = cfg.rows, D = rows - 1;
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
    ctl->use_tile = 0;
    ctl->level = level;
    ctl->prev_level = prev_level;
    for (int i = 0; i < 16; ++i) ctl->Tprev[i] = Tprev.m[i];
    loop_publish(ctl, S->Titer, rows);
}

template <typename T>
void launch_loop_init(LoopCtl* ctl, LoopState<T>* S, const LoopCfg& cfg, const T* T0, int level, int prev_level,
                      const double* Tprev, int* iter_err, hipStream_t s) {
    Mat4d tp;
    for (int i = 0; i < 16; ++i) tp.m[i] = Tprev[i];
    hipLaunchKernelGGL(loop_init_kernel<T>, dim3(1), dim3(64), 0, s, ctl, S, cfg, T0, level, prev_level, tp, iter_err);
}
template <typename T>
void launch_loop_step(LoopCtl* ctl, LoopState<T>* S, const double* res, const int* iter_err,
                      const unsigned long long* visited, const T* means, const LoopCfg& cfg, T* trace,
                      const int* spec_hit, long long* diag, hipStream_t s) {
#define PMX_STEP(R, M)                                                                                            \
    hipLaunchKernelGGL((loop_step_kernel<T, R, M>), dim3(1), dim3(64), 0, s, ctl, S, res, iter_err, visited, means, \
                       cfg, trace, spec_hit, diag)
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
                                      const double*, int*, hipStream_t);
template void launch_loop_init<double>(LoopCtl*, LoopState<double>*, const LoopCfg&, const double*, int, int,
                                       const double*, int*, hipStream_t);
template void launch_loop_step<float>(LoopCtl*, LoopState<float>*, const double*, const int*,
                                      const unsigned long long*, const float*, const LoopCfg&, float*, const int*,
                                      long long*, hipStream_t);
template void launch_loop_step<double>(LoopCtl*, LoopState<double>*, const double*, const int*,
                                       const unsigned long long*, const double*, const LoopCfg&, double*,
                                       const int*, long long*, hipStream_t);


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_loop() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&loop_step_kernel<float, 4, 0>));
}

}  // namespace pmx
