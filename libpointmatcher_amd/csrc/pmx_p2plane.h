// pmx_p2plane.h — the point-to-plane accumulation of the reduction kernel
// (pmx_reduce.hip).
#pragma once

#include "pmx_internal.h"

namespace pmx {

template <typename T>
__device__ __forceinline__ void xform3(const Mat4<T>& M, const P4<T>& p, T& x, T& y, T& z) {
    x = ((M.m[0] * p.x + M.m[1] * p.y) + M.m[2] * p.z) + M.m[3] * p.w;
    y = ((M.m[4] * p.x + M.m[5] * p.y) + M.m[6] * p.z) + M.m[7] * p.w;
    z = ((M.m[8] * p.x + M.m[9] * p.y) + M.m[10] * p.z) + M.m[11] * p.w;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// The wave sums of V per-lane values (V a power of two, <= 64) by a
// butterfly that halves the values at every step: V - 1 + log2(64 / V)
// shuffles instead of V * 6 for V separate wave_sums.  On return lane L holds
// the sum of value idx = (L >> log2(64 / V)) ... in a fixed order (every
// lane of a group of 64 / V lanes holds the same sum); deterministic.
template <int V>
__device__ __forceinline__ double wave_transpose_sum(double (&v)[V], int& idx) {
    static_assert(V >= 1 && V <= 64 && (V & (V - 1)) == 0, "power of two <= 64");
    const int lane = threadIdx.x & 63;
    idx = 0;
    int d = 32;
#pragma unroll
    for (int h = V / 2; h >= 1; h >>= 1, d >>= 1) {
        const bool up = (lane & d) != 0;
        // (the halves are exchanged with bit masks: a select between two
        // elements would become a dynamically indexed load of the array,
        // which moves the whole array to scratch)
        const long long m = up ? -1ll : 0ll;
#pragma unroll
        for (int i = 0; i < h; ++i) {
            const long long a = __double_as_longlong(v[i]), b = __double_as_longlong(v[i + h]);
            const double send = __longlong_as_double((a & m) | (b & ~m));
            const double keep = __longlong_as_double((b & m) | (a & ~m));
            v[i] = keep + __shfl_xor(send, d);
        }
        idx += up ? h : 0;
    }
    double s = v[0];
#pragma unroll
    for (; d >= 1; d >>= 1) s += __shfl_xor(s, d);
    return s;
}
// the lane that writes value idx of a wave_transpose_sum<V>
template <int V>
__device__ __forceinline__ bool transpose_writer() {
    return ((threadIdx.x & 63) & (64 / V - 1)) == 0;
}

// block reduction of NV accumulators; writes partials[v * gridDim.x + blockIdx.x]
// (value-major: the finalize reads each value's block partials contiguously)
// kCoherent: agent-scope atomic stores (another block of the same launch sums
// the partials: pmx_post.hip's last-block finalize)
template <int NV, bool kCoherent = false>
__device__ __forceinline__ void block_store(double (&acc)[NV], double* __restrict__ partials) {
    // (the power of two the transposed wave sum takes)
    constexpr int V = NV <= 8 ? 8 : NV <= 16 ? 16 : NV <= 32 ? 32 : 64;
    static_assert(NV <= 64, "block_store: at most 64 values");
    __shared__ double red[4][V];
    const int wave = threadIdx.x >> 6;
    double x[V];
#pragma unroll
    for (int v = 0; v < V; ++v) x[v] = v < NV ? acc[v] : 0.0;
    int idx;
    const double s = wave_transpose_sum<V>(x, idx);
    if (transpose_writer<V>()) red[wave][idx] = s;
    __syncthreads();
    for (int v = threadIdx.x; v < NV; v += blockDim.x) {
        const double r = ((red[0][v] + red[1][v]) + red[2][v]) + red[3][v];
        double* dst = &partials[(int64_t)v * gridDim.x + blockIdx.x];
        if (kCoherent)
            __hip_atomic_store(dst, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            *dst = r;
    }
}


// one kept pair: F and dot in T exactly as PointToPlane.cpp:171-243, the
// upper triangle of F F^T and F dot added in fp64
template <typename T, int DIM, int NV>
__device__ __forceinline__ void p2plane_add(double (&acc)[NV], T px, T py, T pz, const P4<T>& q, const P4<T>& n,
                                            T w = (T)1) {
    constexpr int NF = DIM == 3 ? 6 : 3;
    constexpr int NS = NF * (NF + 1) / 2;
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
    // wF = w * F (PointToPlane.cpp:218-227); with the 0/1 weights w = 1 and
    // wF is F exactly
    int a = 0;
#pragma unroll
    for (int r = 0; r < NF; ++r) {
        const T wF = w * F[r];
#pragma unroll
        for (int c = r; c < NF; ++c) acc[a++] += (double)(wF * F[c]);
        acc[NS + r] += (double)(wF * dot);
    }
}

// result layout: [0, NS) upper triangle of A row-major (r <= c), [NS, NS+NF) b,
// then kept, nonzero weights, rejected matches, rejected points, sum of weights;
// one block's sums to partials[v * gridDim.x + blockIdx.x]
// k up to this: the reduction issues a query's k gathers together
constexpr int kGatherK = 4;
template <typename T, int DIM, bool kCoherent = false>
__device__ __forceinline__ void p2plane_body(const P4<T>* __restrict__ rd, const Mat4<T>& Tm,
                                             const P4<T>* __restrict__ ref, const P4<T>* __restrict__ nrm, int rs,
                                             const T* __restrict__ d, const int32_t* __restrict__ ids,
                                             const WChain<T>& chain, int k, int64_t N,
                                             double* __restrict__ partials, const P4<T>* __restrict__ nbr = nullptr) {
    constexpr int NF = DIM == 3 ? 6 : 3;
    constexpr int NS = NF * (NF + 1) / 2;
    constexpr int NV = NS + NF + 5;  // (the fifth counter, sum of w, is the kept count with 0/1 weights)
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.0;
    const WRange<T> wr = chain_resolve(chain);
    const T inf = (T)__builtin_huge_val();
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // XCD-aware block order (pmx_internal.h): the blocks of one XCD take
    // adjacent slot ranges, so the gathered point/normal records of
    // neighbouring queries meet in one L2 (the partial slot stays blockIdx.x)
    int64_t i0 = (int64_t)xcd_block() * blockDim.x + threadIdx.x;
    if (k == 1) {
        // k = 1: U slots per round with every load issued up front (the
        // reduction is latency-bound: slot -> id -> gathered point / normal;
        // with the match's neighbour records, nbr, the point and the normal
        // come in slot order with the query, no dependent gather)
        constexpr int U = 4;
        for (; i0 < N; i0 += U * stride) {
            P4<T> r[U];
            T dv[U];
            int32_t id[U];
            P4<T> q[U], n[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t ii = i0 + u * stride;
                const int64_t jj = ii < N ? ii : i0;
                r[u] = rd[jj];
                dv[u] = d[jj];
                if (nbr) {
                    q[u] = nbr[jj];
                    n[u] = nbr[N + jj];
                } else {
                    id[u] = ids[jj];
                }
            }
            bool kp[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                kp[u] = i0 + u * stride < N && dv[u] != inf && chain_keep(wr, dv[u]);
                if (!nbr) {
                    const int64_t g = (int64_t)(kp[u] ? id[u] : 0) * rs;  // (position 0 always exists)
                    q[u] = gld(ref, g);
                    n[u] = gld(nrm, g);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (i0 + u * stride >= N) continue;
                const bool keep = chain_keep(wr, dv[u]);
                if (keep) acc[NS + NF + 1] += 1.0;                 // (w != 0).count()
                if (dv[u] != inf && !keep) acc[NS + NF + 2] += 1.0;  // rejected match
                if (!kp[u]) {
                    acc[NS + NF + 3] += 1.0;  // rejected point
                    continue;
                }
                acc[NS + NF + 0] += 1.0;
                acc[NS + NF + 4] += 1.0;
                T px, py, pz;
                xform3(Tm, r[u], px, py, pz);
                p2plane_add<T, DIM, NV>(acc, px, py, pz, q[u], n[u]);
            }
        }
    }
    if (k > 1 && k <= kGatherK) {
        // 1 < k <= kGatherK: the query's k distances and ids first, then every
        // kept entry's point and normal gathers in flight together, then the
        // sums in rank order (the loop below, one dependent gather at a time,
        // took 45 us for C4's 4 M pairs)
        for (; i0 < N; i0 += stride) {
            const int64_t i = i0;
            const P4<T> rp = rd[i];
            T dv[kGatherK];
            int32_t id[kGatherK];
#pragma unroll
            for (int s = 0; s < kGatherK; ++s) {
                dv[s] = s < k ? d[i * k + s] : inf;
                id[s] = s < k ? ids[i * k + s] : -1;
            }
            P4<T> q[kGatherK], n[kGatherK];
#pragma unroll
            for (int s = 0; s < kGatherK; ++s) {
                const bool kp = s < k && dv[s] != inf && chain_keep(wr, dv[s]);
                const int64_t g = (int64_t)(kp ? id[s] : 0) * rs;  // (position 0 always exists)
                q[s] = gld(ref, g);
                n[s] = gld(nrm, g);
            }
            T px, py, pz;
            xform3(Tm, rp, px, py, pz);
            bool exist = false;
#pragma unroll
            for (int s = 0; s < kGatherK; ++s) {
                if (s >= k) continue;
                const bool keep = chain_keep(wr, dv[s]);
                if (keep) acc[NS + NF + 1] += 1.0;  // (w != 0).count()
                if (dv[s] == inf) continue;
                if (!keep) {
                    acc[NS + NF + 2] += 1.0;  // rejected match
                    continue;
                }
                exist = true;
                acc[NS + NF + 0] += 1.0;  // kept
                acc[NS + NF + 4] += 1.0;  // sum of the 0/1 weights
                p2plane_add<T, DIM, NV>(acc, px, py, pz, q[s], n[s]);
            }
            if (!exist) acc[NS + NF + 3] += 1.0;  // rejected point
        }
    }
    for (int64_t i = i0; k != 1 && i < N; i += stride) {
        T px, py, pz;
        xform3(Tm, rd[i], px, py, pz);
        bool exist = false;
        for (int s = 0; s < k; ++s) {
            const int64_t e = i * k + s;
            const T dv = d[e];
            const bool keep = chain_keep(wr,dv);
            if (keep) acc[NS + NF + 1] += 1.0;  // (w != 0).count()
            if (dv == inf) continue;
            if (!keep) {
                acc[NS + NF + 2] += 1.0;  // rejected match
                continue;
            }
            exist = true;
            acc[NS + NF + 0] += 1.0;  // kept
            acc[NS + NF + 4] += 1.0;  // sum of the 0/1 weights
            const int32_t id = ids[e];
            p2plane_add<T, DIM, NV>(acc, px, py, pz, gld(ref, (int64_t)id * rs), gld(nrm, (int64_t)id * rs));
        }
        if (!exist) acc[NS + NF + 3] += 1.0;  // rejected point
    }
    block_store<NV, kCoherent>(acc, partials);
}

}  // namespace pmx
