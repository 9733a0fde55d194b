// pmx_reduce.hip — error-minimiser reductions (normal equations) on the device.
//
// Replaces ErrorElements (pointmatcher/ErrorMinimizer.cpp:58-193: compaction
// of the kept pairs + gather of the matched reference points) and the dense
// parts of PointToPlaneErrorMinimizer::compute_in_place
// (ErrorMinimizers/PointToPlane.cpp:171-243, crossProduct
// ErrorMinimizer.cpp:281-315) and PointToPointErrorMinimizer::compute_in_place
// (ErrorMinimizers/PointToPoint.cpp:61-81).  Nothing is compacted: each lane
// walks its slots, evaluates the outlier chain on the distance (weights are
// 0/1, see WChain), skips dist == inf, counts weight 0 as a rejected match,
// and for kept pairs gathers q = ref[id], n = normal[id] (grid order after a
// grid match: coherent) and adds the T-precision products of the reference's
// formulas into fp64 accumulators:
//   F = [p x n ; n]  (3-D),  F = [p_x n_y - p_y n_x ; n]  (2-D)
//   A_rc += (w F_r) F_c,   b_r += (w F_r) dot,   dot = ((dx n_x + dy n_y) + dz n_z)
// With w = 1, (w F_r) F_c == F_r F_c == F_c F_r bit for bit, so Eigen's
// wF * F^T is exactly symmetric: only the upper triangle (21 / 6 terms) is
// accumulated and the host mirrors it.  Per-block partials (fixed 1024-block
// grid, fixed lane order) are summed by finalize_kernel in block order, so
// results are deterministic.  ~56 B per pair (reading 16, dist 4, id 4,
// gathered point 16, gathered normal 16).
#include "pmx_internal.h"
#include "pmx_p2plane.h"
#include "pmx_spec.h"

namespace pmx {

// The chain's weight of one match when it holds a RobustOutlierFilter:
// (predicates' 0/1) * robust(e^2), e^2 = dist / scale^2 in T
// (OutlierFiltersImpl.cpp:537-540); dist = the match distance, or for
// distanceType point2plane (n^ . (p - q))^2 with the normalised reference
// normal (computePointToPlaneDistance, :460-489: 0 for an invalid match)
template <typename T>
__device__ __forceinline__ T robust_chain_weight(const WChain<T>& c, const WRange<T>& wr, T dist, int64_t e) {
    if (c.w_arr) return c.w_arr[e];
    const T pred = chain_keep(wr, dist) ? (T)1 : (T)0;
    const T s = (T)*c.rb_scale;
    const T e2 = dist / (s * s);
    return pred * robust_weight<T>(c.rb_fct, c.rb_k, c.rb_sqa, e2);
}
template <typename T>
__device__ __forceinline__ T p2pl_distance(T px, T py, T pz, const P4<T>& q, const P4<T>& n) {
    // Eigen normalized(): v / sqrt(squaredNorm), v itself when the norm is 0
    const T sq = (n.x * n.x + n.y * n.y) + n.z * n.z;
    const T nn = sq > (T)0 ? sqrt(sq) : (T)1;
    const T dot = ((n.x / nn) * (px - q.x) + (n.y / nn) * (py - q.y)) + (n.z / nn) * (pz - q.z);
    return dot * dot;  // (pow(dot, 2) rounds to the same T)
}

// result layout: [0, NS) upper triangle of A row-major (r <= c), [NS, NS+NF) b,
// then kept, nonzero weights, rejected matches, rejected points
template <typename T, int DIM>
__global__ __launch_bounds__(256) void p2plane_partial_kernel(const P4<T>* __restrict__ rd, Mat4<T> Tm,
                                                              const P4<T>* __restrict__ ref,
                                                              const P4<T>* __restrict__ nrm, int rs,
                                                              const T* __restrict__ d,
                                                              const int32_t* __restrict__ ids, WChain<T> chain,
                                                              int k, int64_t N, double* __restrict__ partials,
                                                              const LoopCtl* __restrict__ ctl,
                                                              const GridDesc<T>* __restrict__ gd,
                                                              unsigned long long* __restrict__ vzero,
                                                              const P4<T>* __restrict__ nbr) {
    if (ctl) {  // device loop
        if (ctl->done) return;
        ctl_transform(ctl, Tm);
        ref = gd[ctl->level].gpn;
        nrm = ref + 1;
        rs = 2;
    }
    if (vzero && blockIdx.x == 0)  // (the spread counters the merged counter phase read, for the next match)
        for (int c = 0; c < 4; ++c) vzero[(size_t)(c * kVSlots + threadIdx.x) * kVStride] = 0ull;
    p2plane_body<T, DIM>(rd, Tm, ref, nrm, rs, d, ids, chain, k, N, partials, nbr);
}

// Real-valued weights (a RobustOutlierFilter in the chain; per-module path):
// the ErrorElements counts on w != 0, sum of w in the fifth counter.  A is
// accumulated in full: (w F_r) F_c and (w F_c) F_r round differently, and the
// reference's wF * F^T keeps that asymmetry (PointToPlane.cpp:218-227).
template <typename T, int DIM, int NV>
__device__ __forceinline__ void p2plane_add_full(double (&acc)[NV], T px, T py, T pz, const P4<T>& q,
                                                 const P4<T>& n, T w) {
    constexpr int NF = DIM == 3 ? 6 : 3;
    T F[NF];
    T dot;
    if (DIM == 3) {
        F[0] = py * n.z - pz * n.y;
        F[1] = pz * n.x - px * n.z;
        F[2] = px * n.y - py * n.x;
        F[3] = n.x;
        F[4] = n.y;
        F[5] = n.z;
        dot = ((px - q.x) * n.x + (py - q.y) * n.y) + (pz - q.z) * n.z;
    } else {
        F[0] = px * n.y - py * n.x;
        F[1] = n.x;
        F[2] = n.y;
        dot = (px - q.x) * n.x + (py - q.y) * n.y;
    }
#pragma unroll
    for (int r = 0; r < NF; ++r) {
        const T wF = w * F[r];
#pragma unroll
        for (int c = 0; c < NF; ++c) acc[r * NF + c] += (double)(wF * F[c]);
        acc[NF * NF + r] += (double)(wF * dot);
    }
}
template <typename T, int DIM>
__global__ __launch_bounds__(256) void p2plane_weighted_kernel(const P4<T>* __restrict__ rd, Mat4<T> Tm,
                                                               const P4<T>* __restrict__ ref,
                                                               const P4<T>* __restrict__ nrm, int rs,
                                                               const T* __restrict__ d,
                                                               const int32_t* __restrict__ ids, WChain<T> chain,
                                                               int k, int64_t N, double* __restrict__ partials,
                                                               const LoopCtl* __restrict__ ctl,
                                                               const GridDesc<T>* __restrict__ gd) {
    if (ctl) {  // device loop (a robust chain): transform and level from the device
        if (ctl->done) return;
        ctl_transform(ctl, Tm);
        ref = gd[ctl->level].gpn;
        nrm = ref + 1;
        rs = 2;
    }
    constexpr int NF = DIM == 3 ? 6 : 3;
    constexpr int NS = NF * NF;  // (full A)
    constexpr int NV = NS + NF + 5;
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    const WRange<T> wr = chain_resolve(chain);
    const T inf = (T)__builtin_huge_val();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        T px, py, pz;
        xform3(Tm, rd[i], px, py, pz);
        bool exist = false;
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            const T dv = d[e];
            const int32_t id = ids[e];
            P4<T> q{}, n{};
            if (id >= 0) {
                q = gld(ref, (int64_t)id * rs);
                n = gld(nrm, (int64_t)id * rs);
            }
            const T dist = chain.rb_p2pl ? (id >= 0 ? p2pl_distance(px, py, pz, q, n) : (T)0) : dv;
            // (the predicates judge the match distance; the robust function the chosen one)
            const T pred = chain_keep(wr, dv) ? (T)1 : (T)0;
            const T sc = (T)*chain.rb_scale;
            const T w = pred * robust_weight<T>(chain.rb_fct, chain.rb_k, chain.rb_sqa, dist / (sc * sc));
            if (w != (T)0) acc[NS + NF + 1] += 1.0;  // (w != 0).count()
            if (dv == inf) continue;
            if (w == (T)0) {
                acc[NS + NF + 2] += 1.0;  // rejected match
                continue;
            }
            exist = true;
            acc[NS + NF + 0] += 1.0;
            acc[NS + NF + 4] += (double)w;
            p2plane_add_full<T, DIM, NV>(acc, px, py, pz, q, n, w);
        }
        if (!exist) acc[NS + NF + 3] += 1.0;
    }
    block_store<NV>(acc, partials);
}

template <typename T>
void launch_p2plane_partial(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const P4<T>* nrm, int rs,
                            const T* d, const int32_t* ids, const WChain<T>& chain, int k, int64_t N, int dim,
                            double* partials, const LoopCtl* ctl, const GridDesc<T>* gd, unsigned long long* vzero,
                            hipStream_t s, const P4<T>* nbr) {
    if (chain.robust) {  // real-valued weights: the full asymmetric A
        if (dim == 3)
            hipLaunchKernelGGL((p2plane_weighted_kernel<T, 3>), dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, nrm,
                               rs, d, ids, chain, k, N, partials, ctl, gd);
        else
            hipLaunchKernelGGL((p2plane_weighted_kernel<T, 2>), dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, nrm,
                               rs, d, ids, chain, k, N, partials, ctl, gd);
        return;
    }
    if (dim == 3)
        hipLaunchKernelGGL((p2plane_partial_kernel<T, 3>), dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, nrm, rs,
                           d, ids, chain, k, N, partials, ctl, gd, vzero, nbr);
    else
        hipLaunchKernelGGL((p2plane_partial_kernel<T, 2>), dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, nrm, rs,
                           d, ids, chain, k, N, partials, ctl, gd, vzero, nbr);
}

// Sum the per-block partials: one block per accumulator, each thread adds a
// fixed strided subset in order, then a fixed-shape tree — the summation
// order never changes, so results are bitwise reproducible.
__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ partials, int nblocks, int nv,
                                                       double* __restrict__ out, const LoopCtl* __restrict__ ctl) {
    __shared__ double red[4];
    if (ctl && ctl->done) return;
    const int v = blockIdx.x;
    double s = 0.0;
    for (int b = threadIdx.x; b < nblocks; b += 256) s += partials[(int64_t)v * nblocks + b];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[v] = (red[0] + red[1]) + (red[2] + red[3]);
}

void launch_finalize(const double* partials, int nblocks, int nv, double* out, const LoopCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(finalize_kernel, dim3(nv), dim3(256), 0, s, partials, nblocks, nv, out, ctl);
}

// ------------------------------------------------------------ point-to-point --
// pass 1: sum w, sum p*w, sum q*w (PointToPoint.cpp:67-72) + ErrorElements counts
// layout: [0] sw, [1..3] sp, [4..6] sq, [7] kept, [8] nz, [9] rejM, [10] rejP
template <typename T>
__global__ __launch_bounds__(256) void p2point_pass1_kernel(const P4<T>* __restrict__ rd, Mat4<T> Tm,
                                                            const P4<T>* __restrict__ ref, const T* __restrict__ d,
                                                            const int32_t* __restrict__ ids, WChain<T> chain, int k,
                                                            int64_t N, double* __restrict__ partials,
                                                            const LoopCtl* __restrict__ ctl,
                                                            const GridDesc<T>* __restrict__ gd) {
    constexpr int NV = 11;
    if (ctl) {  // device loop
        if (ctl->done) return;
        ctl_transform(ctl, Tm);
        ref = gd[ctl->level].gpts;
    }
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    const WRange<T> wr = chain_resolve(chain);
    const T inf = (T)__builtin_huge_val();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        T px, py, pz;
        xform3(Tm, rd[i], px, py, pz);
        bool exist = false;
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            const T dv = d[e];
            // 0/1 weights, or a robust chain's real weight (point2point distance)
            const T w = chain.robust ? robust_chain_weight(chain, wr, dv, e) : (chain_keep(wr, dv) ? (T)1 : (T)0);
            if (w != (T)0) acc[8] += 1.0;
            if (dv == inf) continue;
            if (w == (T)0) {
                acc[9] += 1.0;
                continue;
            }
            exist = true;
            acc[7] += 1.0;
            const P4<T> q = gld(ref, ids[e]);
            // (with w = 1, p * w == p exactly)
            acc[0] += (double)w;
            acc[1] += (double)(px * w);
            acc[2] += (double)(py * w);
            acc[3] += (double)(pz * w);
            acc[4] += (double)(q.x * w);
            acc[5] += (double)(q.y * w);
            acc[6] += (double)(q.z * w);
        }
        if (!exist) acc[10] += 1.0;
    }
    block_store<NV>(acc, partials);
}

template <typename T>
void launch_p2point_pass1(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d, const int32_t* ids,
                          const WChain<T>& chain, int k, int64_t N, double* partials, const LoopCtl* ctl,
                          const GridDesc<T>* gd, hipStream_t s) {
    hipLaunchKernelGGL(p2point_pass1_kernel<T>, dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, d, ids, chain, k, N,
                       partials, ctl, gd);
}

// means in T: w_sum_inv = 1 / w.sum(); mean = sum * w_sum_inv (PointToPoint.cpp:67-72)
template <typename T>
__global__ void p2point_means_kernel(const double* __restrict__ sums, T* __restrict__ means, int dim,
                                     const LoopCtl* __restrict__ ctl) {
    if (threadIdx.x != 0 || (ctl && ctl->done)) return;
    const T winv = (T)1 / (T)sums[0];
    for (int r = 0; r < 3; ++r) {
        means[r] = r < dim ? (T)sums[1 + r] * winv : (T)0;
        means[3 + r] = r < dim ? (T)sums[4 + r] * winv : (T)0;
    }
}

template <typename T>
void launch_p2point_means(const double* sums, T* means_dev, int dim, const LoopCtl* ctl, hipStream_t s) {
    hipLaunchKernelGGL(p2point_means_kernel<T>, dim3(1), dim3(64), 0, s, sums, means_dev, dim, ctl);
}

// pass 2: m = sum (qc * w) pc^T  (PointToPoint.cpp:76-81), 3x3 (2-D uses the
// top-left 2x2; z terms are exactly zero)
template <typename T>
__global__ __launch_bounds__(256) void p2point_pass2_kernel(const P4<T>* __restrict__ rd, Mat4<T> Tm,
                                                            const P4<T>* __restrict__ ref, const T* __restrict__ d,
                                                            const int32_t* __restrict__ ids, WChain<T> chain, int k,
                                                            int64_t N, const T* __restrict__ means,
                                                            double* __restrict__ partials,
                                                            const LoopCtl* __restrict__ ctl,
                                                            const GridDesc<T>* __restrict__ gd) {
    constexpr int NV = 9;
    if (ctl) {  // device loop
        if (ctl->done) return;
        ctl_transform(ctl, Tm);
        ref = gd[ctl->level].gpts;
    }
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    const WRange<T> wr = chain_resolve(chain);
    const T inf = (T)__builtin_huge_val();
    const T mp[3] = {means[0], means[1], means[2]};
    const T mq[3] = {means[3], means[4], means[5]};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        T p[3];
        xform3(Tm, rd[i], p[0], p[1], p[2]);
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            const T dv = d[e];
            const T w = chain.robust ? robust_chain_weight(chain, wr, dv, e) : (chain_keep(wr, dv) ? (T)1 : (T)0);
            if (dv == inf || w == (T)0) continue;
            const P4<T> q4 = gld(ref, ids[e]);
            const T q[3] = {q4.x, q4.y, q4.z};
            T pc[3], qc[3];
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                pc[r] = p[r] - mp[r];
                qc[r] = q[r] - mq[r];
            }
#pragma unroll
            for (int r = 0; r < 3; ++r) {
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[r * 3 + c] += (double)((qc[r] * w) * pc[c]);  // (qc * w) pc
            }
        }
    }
    block_store<NV>(acc, partials);
}

template <typename T>
void launch_p2point_pass2(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d, const int32_t* ids,
                          const WChain<T>& chain, int k, int64_t N, const T* means_dev, double* partials,
                          const LoopCtl* ctl, const GridDesc<T>* gd, hipStream_t s) {
    hipLaunchKernelGGL(p2point_pass2_kernel<T>, dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, d, ids, chain, k, N,
                       means_dev, partials, ctl, gd);
}

// Point-to-point in one pass (device loop): the sums both of the reference's
// passes need — sum w, sum w p, sum w q, the ErrorElements counters and the
// raw moments sum (w q) p^T — in one read of the matches.  The step forms the
// weighted means in T as p2point_means_kernel does and centres the moments in
// fp64: sum w (q - mq)(p - mp)^T = sum (w q) p^T - mq (sum w p)^T
// - (sum w q) mp^T + (sum w) mq mp^T (PointToPoint.cpp:67-81 by the same
// identity; the two-pass kernels above are the per-module path's).
// Layout: [0] sum w, [1, 4) sum w p, [4, 7) sum w q, [7, 11) kept, nonzero
// weights, rejected matches, rejected points, [11, 20) sum (w q_r) p_c.
template <typename T>
__global__ __launch_bounds__(256) void p2point_moments_kernel(const P4<T>* __restrict__ rd, Mat4<T> Tm,
                                                              const P4<T>* __restrict__ ref, const T* __restrict__ d,
                                                              const int32_t* __restrict__ ids, WChain<T> chain, int k,
                                                              int64_t N, double* __restrict__ partials,
                                                              const LoopCtl* __restrict__ ctl,
                                                              const GridDesc<T>* __restrict__ gd) {
    constexpr int NV = 20;
    if (ctl) {  // device loop
        if (ctl->done) return;
        ctl_transform(ctl, Tm);
        ref = gd[ctl->level].gpts;
    }
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    const WRange<T> wr = chain_resolve(chain);
    const T inf = (T)__builtin_huge_val();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)xcd_block() * blockDim.x + threadIdx.x; i < N; i += stride) {
        T px, py, pz;
        xform3(Tm, rd[i], px, py, pz);
        bool exist = false;
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            const T dv = d[e];
            const T w = chain.robust ? robust_chain_weight(chain, wr, dv, e) : (chain_keep(wr, dv) ? (T)1 : (T)0);
            if (w != (T)0) acc[8] += 1.0;
            if (dv == inf) continue;
            if (w == (T)0) {
                acc[9] += 1.0;
                continue;
            }
            exist = true;
            acc[7] += 1.0;
            const P4<T> q = gld(ref, ids[e]);
            const T wq[3] = {q.x * w, q.y * w, q.z * w};
            const double p[3] = {(double)px, (double)py, (double)pz};
            acc[0] += (double)w;
            acc[1] += (double)(px * w);
            acc[2] += (double)(py * w);
            acc[3] += (double)(pz * w);
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                acc[4 + r] += (double)wq[r];
#pragma unroll
                for (int c = 0; c < 3; ++c) acc[11 + r * 3 + c] += (double)wq[r] * p[c];
            }
        }
        if (!exist) acc[10] += 1.0;
    }
    block_store<NV>(acc, partials);
}

template <typename T>
void launch_p2point_moments(const P4<T>* rd, const Mat4<T>& Tm, const P4<T>* ref, const T* d, const int32_t* ids,
                            const WChain<T>& chain, int k, int64_t N, double* partials, const LoopCtl* ctl,
                            const GridDesc<T>* gd, hipStream_t s) {
    hipLaunchKernelGGL(p2point_moments_kernel<T>, dim3(kRedBlocks), dim3(256), 0, s, rd, Tm, ref, d, ids, chain, k,
                       N, partials, ctl, gd);
}

// materialise the chain's weights (host mirror only); point-to-plane robust
// distances need the step reading, the match ids and the reference records
template <typename T>
__global__ void weights_chain_kernel(const T* __restrict__ d, T* __restrict__ w, int64_t n, WChain<T> chain,
                                     const P4<T>* __restrict__ rd, Mat4<T> Tm, const P4<T>* __restrict__ ref,
                                     const P4<T>* __restrict__ nrm, int rs, const int32_t* __restrict__ ids, int k) {
    const WRange<T> wr = chain_resolve(chain);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (!chain.robust) {
            w[i] = chain_keep(wr, d[i]) ? (T)1 : (T)0;
            continue;
        }
        T dist = d[i];
        if (chain.rb_p2pl) {
            const int32_t id = ids[i];
            dist = 0;
            if (id >= 0) {
                T px, py, pz;
                xform3(Tm, rd[i / k], px, py, pz);
                dist = p2pl_distance(px, py, pz, gld(ref, (int64_t)id * rs), gld(nrm, (int64_t)id * rs));
            }
        }
        const T pred = chain_keep(wr, d[i]) ? (T)1 : (T)0;
        const T sc = (T)*chain.rb_scale;
        w[i] = pred * robust_weight<T>(chain.rb_fct, chain.rb_k, chain.rb_sqa, dist / (sc * sc));
    }
}
template <typename T>
void launch_weights_chain(const T* d, T* w, int64_t n, const WChain<T>& chain, const P4<T>* rd, const Mat4<T>& Tm,
                          const P4<T>* ref, const P4<T>* nrm, int rs, const int32_t* ids, int k, hipStream_t s) {
    if (n <= 0) return;
    int64_t g = (n + 1023) / 1024;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(weights_chain_kernel<T>, dim3((unsigned)g), dim3(256), 0, s, d, w, n, chain, rd, Tm, ref, nrm,
                       rs, ids, k);
}

#define PMX_INST(T)                                                                                                  \
    template void launch_p2plane_partial<T>(const P4<T>*, const Mat4<T>&, const P4<T>*, const P4<T>*, int, const T*, \
                                            const int32_t*, const WChain<T>&, int, int64_t, int, double*,           \
                                            const LoopCtl*, const GridDesc<T>*, unsigned long long*, hipStream_t,     \
                                            const P4<T>*);                                                            \
    template void launch_p2point_pass1<T>(const P4<T>*, const Mat4<T>&, const P4<T>*, const T*, const int32_t*,     \
                                          const WChain<T>&, int, int64_t, double*, const LoopCtl*,                   \
                                          const GridDesc<T>*, hipStream_t);                                          \
    template void launch_p2point_means<T>(const double*, T*, int, const LoopCtl*, hipStream_t);                      \
    template void launch_p2point_moments<T>(const P4<T>*, const Mat4<T>&, const P4<T>*, const T*, const int32_t*,   \
                                            const WChain<T>&, int, int64_t, double*, const LoopCtl*,              \
                                            const GridDesc<T>*, hipStream_t);                                      \
    template void launch_p2point_pass2<T>(const P4<T>*, const Mat4<T>&, const P4<T>*, const T*, const int32_t*,     \
                                          const WChain<T>&, int, int64_t, const T*, double*, const LoopCtl*,         \
                                          const GridDesc<T>*, hipStream_t);                                          \
    template void launch_weights_chain<T>(const T*, T*, int64_t, const WChain<T>&, const P4<T>*, const Mat4<T>&,     \
                                          const P4<T>*, const P4<T>*, int, const int32_t*, int, hipStream_t);
PMX_INST(float)
PMX_INST(double)
#undef PMX_INST


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_reduce() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&finalize_kernel));
}

}  // namespace pmx
