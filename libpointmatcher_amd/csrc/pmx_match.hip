// pmx_match.hip — exact brute-force k-NN with the rigid transform fused in.
//
// Replaces KDTreeMatcher::findClosests (pointmatcher/MatchersImpl.cpp:85-101,
// libnabo knn [ext]) and the per-iteration transformations.apply of
// pointmatcher/ICP.cpp:381 (RigidTransformation::compute,
// TransformationsImpl.cpp:66-69): the step reading is never materialised —
// each query is transformed in registers from the resident reading.
//
// Arithmetic contract (parity with the CPU path, bit for bit):
//   query  q_r = ((T_r0 x + T_r1 y) + T_r2 z) + T_r3 h        (no FMA)
//   dist   d   = ((dx*dx + dy*dy) + dz*dz), dx = r.x - q.x     (libnabo's
//                sequential "dist += diff*diff", no FMA)
//   ties   lowest reference index wins; k-lists sorted ascending.
// The file is compiled with -ffp-contract=off so no multiply-add is fused.
//
// Kernel shape (gfx950, wave64): a block of 256 threads owns 256*QPT queries
// held in registers (QPT per lane) and streams one chunk of the reference
// through a 1024-point LDS tile; every reference point is an LDS broadcast
// read (ds_read_b128, conflict-free) amortised over QPT queries.  k = 1 uses
// min-then-rescan: the inner loop keeps only a running min per 32-point
// sub-block (v_min3: 0.5 op/pair) and remembers the sub-block that improved
// the best; the winning index is recovered after the scan by re-evaluating
// that one sub-block.  When N is too small to fill the 256 CUs the reference
// is split into chunks whose per-query partials a merge kernel combines
// (lexicographic (dist, index)).
#include "pmx_internal.h"

#include <algorithm>
#include <cmath>
#include <limits>

namespace pmx {

template <typename T>
__device__ __forceinline__ T tmin(T a, T b) {
    return a < b ? a : b;
}
template <>
__device__ __forceinline__ float tmin<float>(float a, float b) {
    return __builtin_fminf(a, b);
}
template <>
__device__ __forceinline__ double tmin<double>(double a, double b) {
    return __builtin_fmin(a, b);
}

template <typename T>
__device__ __forceinline__ T tinf() {
    return __builtin_huge_val();
}
template <>
__device__ __forceinline__ float tinf<float>() {
    return __builtin_huge_valf();
}

template <typename T>
__device__ __forceinline__ void xform(const Mat4<T>& M, const P4<T>& p, T& x, T& y, T& z) {
    x = ((M.m[0] * p.x + M.m[1] * p.y) + M.m[2] * p.z) + M.m[3] * p.w;
    y = ((M.m[4] * p.x + M.m[5] * p.y) + M.m[6] * p.z) + M.m[7] * p.w;
    z = ((M.m[8] * p.x + M.m[9] * p.y) + M.m[10] * p.z) + M.m[11] * p.w;
}

// Read a whole P4 from LDS.  The w lane is unused by the distance; keeping
// it alive makes the compiler issue one ds_read_b128 (4 LDS cycles per
// broadcast wave-instruction) instead of ds_read_b96 (8 cycles).
template <typename T>
__device__ __forceinline__ P4<T> lds_load(const P4<T>* p) {
    P4<T> v = *p;
    asm volatile("" ::"v"(v.w));
    return v;
}

template <typename T>
__device__ __forceinline__ T sqd(T qx, T qy, T qz, const P4<T>& r) {
    const T dx = r.x - qx;
    const T dy = r.y - qy;
    const T dz = r.z - qz;
    T d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// ------------------------------------------------------------------ k = 1 --
template <typename T, int QPT, bool FINAL>
__global__ __launch_bounds__(kBlock) void match1_kernel(const P4<T>* __restrict__ ref, int64_t chunk_len,
                                                        int64_t M_pad, const P4<T>* __restrict__ rd,
                                                        int64_t N, Mat4<T> Tm, T maxR2,
                                                        T* __restrict__ out_d,
                                                        int32_t* __restrict__ out_i) {
    __shared__ P4<T> tile[kTile];
    const int tid = threadIdx.x;
    const int64_t qbase = (int64_t)blockIdx.x * (kBlock * QPT);
    const int64_t r0 = (int64_t)blockIdx.y * chunk_len;
    const int64_t r1 = r0 + chunk_len < M_pad ? r0 + chunk_len : M_pad;

    T qx[QPT], qy[QPT], qz[QPT], best[QPT];
    int bsb[QPT];
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int64_t qi = qbase + j * kBlock + tid;
        P4<T> p = {0, 0, 0, 1};
        if (qi < N) p = rd[qi];
        xform(Tm, p, qx[j], qy[j], qz[j]);
        best[j] = tinf<T>();
        bsb[j] = -1;
    }

    for (int64_t t0 = r0; t0 < r1; t0 += kTile) {
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kTile / kBlock; ++s) tile[s * kBlock + tid] = ref[t0 + s * kBlock + tid];
        __syncthreads();
        const int gsb0 = (int)(t0 / kSub);
        for (int sb = 0; sb < kTile / kSub; ++sb) {
            T m[QPT];
#pragma unroll
            for (int j = 0; j < QPT; ++j) m[j] = tinf<T>();
#pragma unroll
            for (int r = 0; r < kSub; r += 2) {
                const P4<T> a = lds_load(&tile[sb * kSub + r]);
                const P4<T> b = lds_load(&tile[sb * kSub + r + 1]);
#pragma unroll
                for (int j = 0; j < QPT; ++j) {
                    const T da = sqd(qx[j], qy[j], qz[j], a);
                    const T db = sqd(qx[j], qy[j], qz[j], b);
                    m[j] = tmin(tmin(m[j], da), db);  // -> v_min3(m, da, db)
                }
            }
#pragma unroll
            for (int j = 0; j < QPT; ++j) {
                if (m[j] < best[j]) {
                    best[j] = m[j];
                    bsb[j] = gsb0 + sb;
                }
            }
        }
    }

    // rescan the winning sub-block: first index reproducing the best value
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int64_t qi = qbase + j * kBlock + tid;
        if (qi >= N) continue;
        T bd = best[j];
        int32_t id = -1;
        if (bsb[j] >= 0) {
            const int64_t base = (int64_t)bsb[j] * kSub;
            for (int r = 0; r < kSub; ++r) {
                const T d = sqd(qx[j], qy[j], qz[j], ref[base + r]);
                if (d == bd) {
                    id = (int32_t)(base + r);
                    break;
                }
            }
        }
        if (FINAL) {
            if (!(bd <= maxR2)) {
                bd = tinf<T>();
                id = -1;
            }
            out_d[qi] = bd;
            out_i[qi] = id;
        } else {
            out_d[(int64_t)blockIdx.y * N + qi] = bd;
            out_i[(int64_t)blockIdx.y * N + qi] = id;
        }
    }
}

template <typename T>
__global__ void merge1_kernel(const T* __restrict__ pd, const int32_t* __restrict__ pi, int S, int64_t N,
                              T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i) {
    const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= N) return;
    T bd = tinf<T>();
    int32_t bi = -1;
    for (int c = 0; c < S; ++c) {
        const T d = pd[(int64_t)c * N + qi];
        if (d < bd) {
            bd = d;
            bi = pi[(int64_t)c * N + qi];
        }
    }
    if (!(bd <= maxR2)) {
        bd = tinf<T>();
        bi = -1;
    }
    out_d[qi] = bd;
    out_i[qi] = bi;
}

// ------------------------------------------------------------------ k > 1 --
// sorted insertion (ascending, stable: a later index never passes an equal
// distance), fully unrolled so the lists stay in registers
template <typename T, int KT>
__device__ __forceinline__ void kinsert(T (&kd)[KT], int32_t (&ki)[KT], T d, int32_t id) {
    kd[KT - 1] = d;
    ki[KT - 1] = id;
#pragma unroll
    for (int s = KT - 1; s > 0; --s) {
        const bool sw = kd[s] < kd[s - 1];
        const T td = sw ? kd[s - 1] : kd[s];
        const int32_t ti = sw ? ki[s - 1] : ki[s];
        kd[s - 1] = sw ? kd[s] : kd[s - 1];
        ki[s - 1] = sw ? ki[s] : ki[s - 1];
        kd[s] = td;
        ki[s] = ti;
    }
}

template <typename T, int QPT, int KT, bool FINAL>
__global__ __launch_bounds__(kBlock) void matchk_kernel(const P4<T>* __restrict__ ref, int64_t chunk_len,
                                                        int64_t M_pad, const P4<T>* __restrict__ rd,
                                                        int64_t N, Mat4<T> Tm, int k, T maxR2,
                                                        T* __restrict__ out_d,
                                                        int32_t* __restrict__ out_i) {
    __shared__ P4<T> tile[kTile];
    const int tid = threadIdx.x;
    const int64_t qbase = (int64_t)blockIdx.x * (kBlock * QPT);
    const int64_t r0 = (int64_t)blockIdx.y * chunk_len;
    const int64_t r1 = r0 + chunk_len < M_pad ? r0 + chunk_len : M_pad;

    T qx[QPT], qy[QPT], qz[QPT];
    T kd[QPT][KT];
    int32_t ki[QPT][KT];
#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int64_t qi = qbase + j * kBlock + tid;
        P4<T> p = {0, 0, 0, 1};
        if (qi < N) p = rd[qi];
        xform(Tm, p, qx[j], qy[j], qz[j]);
#pragma unroll
        for (int s = 0; s < KT; ++s) {
            kd[j][s] = tinf<T>();
            ki[j][s] = -1;
        }
    }

    for (int64_t t0 = r0; t0 < r1; t0 += kTile) {
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kTile / kBlock; ++s) tile[s * kBlock + tid] = ref[t0 + s * kBlock + tid];
        __syncthreads();
        for (int sb = 0; sb < kTile / kSub; ++sb) {
            T m[QPT];
#pragma unroll
            for (int j = 0; j < QPT; ++j) m[j] = tinf<T>();
#pragma unroll
            for (int r = 0; r < kSub; r += 2) {
                const P4<T> a = lds_load(&tile[sb * kSub + r]);
                const P4<T> b = lds_load(&tile[sb * kSub + r + 1]);
#pragma unroll
                for (int j = 0; j < QPT; ++j) {
                    const T da = sqd(qx[j], qy[j], qz[j], a);
                    const T db = sqd(qx[j], qy[j], qz[j], b);
                    m[j] = tmin(tmin(m[j], da), db);  // -> v_min3(m, da, db)
                }
            }
            bool need = false;
#pragma unroll
            for (int j = 0; j < QPT; ++j) need |= m[j] < kd[j][KT - 1];
            if (need) {
                const int32_t gbase = (int32_t)(t0 + sb * kSub);
                for (int r = 0; r < kSub; ++r) {
                    const P4<T> a = tile[sb * kSub + r];
#pragma unroll
                    for (int j = 0; j < QPT; ++j) {
                        const T d = sqd(qx[j], qy[j], qz[j], a);
                        if (d < kd[j][KT - 1]) kinsert<T, KT>(kd[j], ki[j], d, gbase + r);
                    }
                }
            }
        }
    }

#pragma unroll
    for (int j = 0; j < QPT; ++j) {
        const int64_t qi = qbase + j * kBlock + tid;
        if (qi >= N) continue;
        for (int s = 0; s < k; ++s) {
            T d = kd[j][s];
            int32_t id = ki[j][s];
            if (FINAL) {
                if (!(d <= maxR2)) {
                    d = tinf<T>();
                    id = -1;
                }
                out_d[qi * k + s] = d;
                out_i[qi * k + s] = id;
            } else {
                out_d[((int64_t)blockIdx.y * N + qi) * k + s] = d;
                out_i[((int64_t)blockIdx.y * N + qi) * k + s] = id;
            }
        }
    }
}

template <typename T, int KT>
__global__ void mergek_kernel(const T* __restrict__ pd, const int32_t* __restrict__ pi, int S, int64_t N,
                              int k, T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i) {
    const int64_t qi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (qi >= N) return;
    T kd[KT];
    int32_t ki[KT];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        kd[s] = tinf<T>();
        ki[s] = -1;
    }
    // chunks are visited in index order, so a strict '<' keeps the lower
    // index among equal distances (lexicographic (dist, index))
    for (int c = 0; c < S; ++c)
        for (int s = 0; s < k; ++s) {
            const T d = pd[((int64_t)c * N + qi) * k + s];
            if (d < kd[KT - 1]) kinsert<T, KT>(kd, ki, d, pi[((int64_t)c * N + qi) * k + s]);
        }
    for (int s = 0; s < k; ++s) {
        T d = kd[s];
        int32_t id = ki[s];
        if (!(d <= maxR2)) {
            d = tinf<T>();
            id = -1;
        }
        out_d[qi * k + s] = d;
        out_i[qi * k + s] = id;
    }
}

// ------------------------------------------------------------ transform ---
template <typename T>
__global__ void transform_kernel(const P4<T>* __restrict__ in, P4<T>* __restrict__ out, int64_t N, Mat4<T> M) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const P4<T> p = in[i];
    P4<T> o;
    xform(M, p, o.x, o.y, o.z);
    o.w = ((M.m[12] * p.x + M.m[13] * p.y) + M.m[14] * p.z) + M.m[15] * p.w;
    out[i] = o;
}

template <typename T>
void launch_transform(const P4<T>* in, P4<T>* out, int64_t N, const Mat4<T>& Tm, hipStream_t s) {
    if (N <= 0) return;
    const int64_t g = (N + 255) / 256;
    hipLaunchKernelGGL(transform_kernel<T>, dim3((unsigned)g), dim3(256), 0, s, in, out, N, Tm);
}

// ------------------------------------------------------------- dispatch ---
// queries per lane: more ILP / fewer LDS reads per pair with larger QPT;
// k-lists cost registers, so QPT shrinks as KT grows
template <typename T>
constexpr int qpt_k1() {
    return sizeof(T) == 4 ? 4 : 2;
}

static int kt_for(int k) {
    if (k <= 2) return 2;
    if (k <= 4) return 4;
    if (k <= 8) return 8;
    return 16;
}
template <typename T>
static int qpt_for(int k) {
    if (k == 1) return qpt_k1<T>();
    const int kt = kt_for(k);
    if (kt <= 4) return 2;
    return 1;
}

// Split the reference into S chunks so that nqb*S blocks fill the chip with
// little quantisation loss (blocks of equal work; "slots" = resident blocks).
static int choose_chunks(int64_t nqb, int64_t ntiles, int cu_count) {
    const int64_t slots = (int64_t)cu_count * 8;
    int best = 1;
    double bestc = 1e300;
    for (int S = 1; S <= 64 && S <= ntiles; ++S) {
        const int64_t blocks = nqb * S;
        const int64_t rounds = (blocks + slots - 1) / slots;
        const double cost = (double)rounds / (double)S + 0.002 * S;  // merge / re-read overhead
        if (cost < bestc - 1e-12) {
            bestc = cost;
            best = S;
        }
    }
    return best;
}

template <typename T>
int64_t match_part_elems(int64_t N, int64_t M_pad, int knn, int cu_count) {
    const int qpt = qpt_for<T>(knn);
    const int64_t nqb = (N + (int64_t)kBlock * qpt - 1) / ((int64_t)kBlock * qpt);
    const int S = choose_chunks(nqb, M_pad / kTile, cu_count);
    return S > 1 ? (int64_t)S * N * knn : 0;
}

template <typename T, int QPT>
static void run1(const P4<T>* ref, int64_t M_pad, const P4<T>* rd, int64_t N, const Mat4<T>& Tm,
                 T maxR2, T* dists, int32_t* ids, T* pd, int32_t* pi, hipStream_t s, hipEvent_t ev0,
                 hipEvent_t ev1, int cu_count) {
    const int64_t nqb = (N + (int64_t)kBlock * QPT - 1) / ((int64_t)kBlock * QPT);
    const int64_t ntiles = M_pad / kTile;
    const int S = choose_chunks(nqb, ntiles, cu_count);
    const int64_t chunk = ((ntiles + S - 1) / S) * kTile;
    const int Sx = (int)((M_pad + chunk - 1) / chunk);
    dim3 grid((unsigned)nqb, (unsigned)Sx);
    if (ev0) (void)hipEventRecord(ev0, s);
    if (Sx == 1)
        hipLaunchKernelGGL((match1_kernel<T, QPT, true>), grid, dim3(kBlock), 0, s, ref, chunk, M_pad, rd, N,
                           Tm, maxR2, dists, ids);
    else
        hipLaunchKernelGGL((match1_kernel<T, QPT, false>), grid, dim3(kBlock), 0, s, ref, chunk, M_pad, rd,
                           N, Tm, maxR2, pd, pi);
    if (ev1) (void)hipEventRecord(ev1, s);
    if (Sx > 1)
        hipLaunchKernelGGL(merge1_kernel<T>, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, pd, pi, Sx, N,
                           maxR2, dists, ids);
}

template <typename T, int QPT, int KT>
static void runk(const P4<T>* ref, int64_t M_pad, const P4<T>* rd, int64_t N, const Mat4<T>& Tm, int k,
                 T maxR2, T* dists, int32_t* ids, T* pd, int32_t* pi, hipStream_t s, hipEvent_t ev0,
                 hipEvent_t ev1, int cu_count) {
    const int64_t nqb = (N + (int64_t)kBlock * QPT - 1) / ((int64_t)kBlock * QPT);
    const int64_t ntiles = M_pad / kTile;
    const int S = choose_chunks(nqb, ntiles, cu_count);
    const int64_t chunk = ((ntiles + S - 1) / S) * kTile;
    const int Sx = (int)((M_pad + chunk - 1) / chunk);
    dim3 grid((unsigned)nqb, (unsigned)Sx);
    if (ev0) (void)hipEventRecord(ev0, s);
    if (Sx == 1)
        hipLaunchKernelGGL((matchk_kernel<T, QPT, KT, true>), grid, dim3(kBlock), 0, s, ref, chunk, M_pad, rd,
                           N, Tm, k, maxR2, dists, ids);
    else
        hipLaunchKernelGGL((matchk_kernel<T, QPT, KT, false>), grid, dim3(kBlock), 0, s, ref, chunk, M_pad,
                           rd, N, Tm, k, maxR2, pd, pi);
    if (ev1) (void)hipEventRecord(ev1, s);
    if (Sx > 1)
        hipLaunchKernelGGL((mergek_kernel<T, KT>), dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, pd, pi,
                           Sx, N, k, maxR2, dists, ids);
}

template <typename T>
void launch_match(const P4<T>* ref, int64_t M_pad, const P4<T>* rd, int64_t N, const Mat4<T>& Tm, int knn,
                  T maxR2, T* dists, int32_t* ids, T* part_d, int32_t* part_i, int64_t part_cap,
                  hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, int cu_count) {
    (void)part_cap;
    if (N <= 0) return;
    constexpr int Q1 = qpt_k1<T>();
    if (knn == 1) {
        run1<T, Q1>(ref, M_pad, rd, N, Tm, maxR2, dists, ids, part_d, part_i, s, ev0, ev1, cu_count);
        return;
    }
    switch (kt_for(knn)) {
    case 2: runk<T, 2, 2>(ref, M_pad, rd, N, Tm, knn, maxR2, dists, ids, part_d, part_i, s, ev0, ev1, cu_count); break;
    case 4: runk<T, 2, 4>(ref, M_pad, rd, N, Tm, knn, maxR2, dists, ids, part_d, part_i, s, ev0, ev1, cu_count); break;
    case 8: runk<T, 1, 8>(ref, M_pad, rd, N, Tm, knn, maxR2, dists, ids, part_d, part_i, s, ev0, ev1, cu_count); break;
    default: runk<T, 1, 16>(ref, M_pad, rd, N, Tm, knn, maxR2, dists, ids, part_d, part_i, s, ev0, ev1, cu_count); break;
    }
}

template void launch_match<float>(const P4<float>*, int64_t, const P4<float>*, int64_t, const Mat4<float>&, int,
                                  float, float*, int32_t*, float*, int32_t*, int64_t, hipStream_t, hipEvent_t,
                                  hipEvent_t, int);
template void launch_match<double>(const P4<double>*, int64_t, const P4<double>*, int64_t, const Mat4<double>&,
                                   int, double, double*, int32_t*, double*, int32_t*, int64_t, hipStream_t,
                                   hipEvent_t, hipEvent_t, int);
template int64_t match_part_elems<float>(int64_t, int64_t, int, int);
template int64_t match_part_elems<double>(int64_t, int64_t, int, int);
template void launch_transform<float>(const P4<float>*, P4<float>*, int64_t, const Mat4<float>&, hipStream_t);
template void launch_transform<double>(const P4<double>*, P4<double>*, int64_t, const Mat4<double>&,
                                       hipStream_t);


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_match() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&transform_kernel<float>));
}

}  // namespace pmx
