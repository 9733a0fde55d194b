// pmx_grid.hip — exact k-NN over a uniform grid of the reference.
//
// Same contract as pmx_match.hip (KDTreeMatcher::findClosests,
// MatchersImpl.cpp:85-101 with libnabo's exact search): distances are the
// bit-identical ((dx*dx + dy*dy) + dz*dz) in T without FMA, candidates are
// ordered by (distance, original index) so ties resolve to the lowest index,
// k-lists are sorted ascending.  Only the set of pairs evaluated changes:
// instead of all N*M pairs, each query visits the cells of growing cubic
// shells around its own cell and stops once the k-th best distance is
// provably below every unvisited point:
//
//   LB_R = min over axes and existing sides of the distance from q to the
//          faces of the (2R+1)^3 block of visited cells (computed in double);
//   stop when  d_k < LB_R^2 * (1 - 1e-5)   (and the list is full).
//
// The 1e-5 relative margin dominates every rounding involved (T distances
// carry a few ulp; cell assignment is done in double), so an unvisited point
// can never produce a distance <= d_k: the result equals the brute-force one
// exactly, ties included.  With a finite radius the search also stops once
// LB_R^2 (1 - 1e-5) > maxDist^2.
//
// Layout (built once per Matcher::init on the host, pmx_capi.hip):
//   gpts  P4<T>[M]        reference points sorted by cell (x fastest)
//   gidx  int32[M]        their original indices
//   start uint32[C + 1]   first point of each cell (C = gx * gy * gz)
// Each x-row of cells is one contiguous point range, so a shell is walked as
// a handful of contiguous scans.  Queries are visited in the order of their
// initial cell (a permutation computed at pmx_set_reading) so neighbouring
// lanes walk neighbouring cells.
#include "pmx_internal.h"

namespace pmx {

template <typename T>
__device__ __forceinline__ void gxform(const Mat4<T>& M, const P4<T>& p, T& x, T& y, T& z) {
    x = ((M.m[0] * p.x + M.m[1] * p.y) + M.m[2] * p.z) + M.m[3] * p.w;
    y = ((M.m[4] * p.x + M.m[5] * p.y) + M.m[6] * p.z) + M.m[7] * p.w;
    z = ((M.m[8] * p.x + M.m[9] * p.y) + M.m[10] * p.z) + M.m[11] * p.w;
}

template <typename T>
__device__ __forceinline__ T gsqd(T qx, T qy, T qz, const P4<T>& r) {
    const T dx = r.x - qx;
    const T dy = r.y - qy;
    const T dz = r.z - qz;
    T d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

template <typename T, int KT>
__device__ __forceinline__ void ginsert(T (&kd)[KT], int32_t (&ki)[KT], T d, int32_t id) {
    // lexicographic (d, id) insertion; candidates arrive in arbitrary index order
    kd[KT - 1] = d;
    ki[KT - 1] = id;
#pragma unroll
    for (int s = KT - 1; s > 0; --s) {
        const bool sw = kd[s] < kd[s - 1] || (kd[s] == kd[s - 1] && ki[s] < ki[s - 1]);
        const T td = sw ? kd[s - 1] : kd[s];
        const int32_t ti = sw ? ki[s - 1] : ki[s];
        kd[s - 1] = sw ? kd[s] : kd[s - 1];
        ki[s - 1] = sw ? ki[s] : ki[s - 1];
        kd[s] = td;
        ki[s] = ti;
    }
}

template <typename T, int KT>
__device__ __forceinline__ void consider(const int32_t* __restrict__ gidx, uint32_t j, T d, T (&kd)[KT],
                                         int32_t (&ki)[KT]) {
    if (d <= kd[KT - 1]) {
        const int32_t id = gidx[j];
        if (d < kd[KT - 1] || id < ki[KT - 1]) ginsert<T, KT>(kd, ki, d, id);
    }
}

// Scan one contiguous point range.  The scan is latency-bound (each lane
// walks its own cells), so points are fetched eight at a time with
// independent loads before any of them is used.
template <typename T, int KT>
__device__ __forceinline__ void scan_range(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                           uint32_t a, uint32_t b, T qx, T qy, T qz, T (&kd)[KT],
                                           int32_t (&ki)[KT], uint32_t& visits) {
    visits += b - a;
    uint32_t j = a;
    constexpr int U = 8;
    for (; j + U <= b; j += U) {
        P4<T> p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = gpts[j + u];
        T d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = gsqd(qx, qy, qz, p[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) consider<T, KT>(gidx, j + u, d[u], kd, ki);
    }
    for (; j < b; ++j) consider<T, KT>(gidx, j, gsqd(qx, qy, qz, gpts[j]), kd, ki);
}

struct GridGeom {
    double lo[3];
    double h, inv_h;
    int g[3];
};

template <typename T, int KT>
__global__ __launch_bounds__(256) void grid_match_kernel(const P4<T>* __restrict__ gpts,
                                                         const int32_t* __restrict__ gidx,
                                                         const uint32_t* __restrict__ start, GridGeom G,
                                                         const P4<T>* __restrict__ rd,
                                                         const int32_t* __restrict__ order, int64_t N,
                                                         Mat4<T> Tm, int k, T maxR2, T* __restrict__ out_d,
                                                         int32_t* __restrict__ out_i,
                                                         unsigned long long* __restrict__ visited) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t visits = 0;
    if (j < N) {
        const int64_t qi = order ? (int64_t)order[j] : j;
        T qx, qy, qz;
        gxform(Tm, rd[qi], qx, qy, qz);
        T kd[KT];
        int32_t ki[KT];
#pragma unroll
        for (int s = 0; s < KT; ++s) {
            kd[s] = (T)__builtin_huge_val();
            ki[s] = 0x7fffffff;
        }
        const double q[3] = {(double)qx, (double)qy, (double)qz};
        int c[3];
        bool qnan = false;
        for (int a = 0; a < 3; ++a) {
            const double f = (q[a] - G.lo[a]) * G.inv_h;
            if (!(f == f)) qnan = true;
            int ci = f < 0.0 ? 0 : (f >= (double)G.g[a] ? G.g[a] - 1 : (int)f);
            c[a] = ci;
        }
        if (!qnan) {
            const double margin = 1.0 - 1e-5;
            {
                // phase 1: the whole 3x3x3 block (R = 0 and 1).  The nine row
                // bounds are loaded together from always-valid (clamped)
                // addresses and masked afterwards, then the rows are scanned.
                uint32_t ra[9], rb[9];
                const int x0 = max(c[0] - 1, 0), x1 = min(c[0] + 1, G.g[0] - 1);
#pragma unroll
                for (int r = 0; r < 9; ++r) {
                    const int z = c[2] + r / 3 - 1, y = c[1] + r % 3 - 1;
                    const bool ok = z >= 0 && z < G.g[2] && y >= 0 && y < G.g[1];
                    const int zc = min(max(z, 0), G.g[2] - 1), yc = min(max(y, 0), G.g[1] - 1);
                    const int64_t row = ((int64_t)zc * G.g[1] + yc) * G.g[0];
                    const uint32_t va = start[row + x0];
                    const uint32_t vb = start[row + x1 + 1];
                    ra[r] = ok ? va : 0u;
                    rb[r] = ok ? vb : 0u;
                }
#pragma unroll
                for (int r = 0; r < 9; ++r) scan_range<T, KT>(gpts, gidx, ra[r], rb[r], qx, qy, qz, kd, ki, visits);
            }
            for (int R = 1;; ++R) {
              if (R >= 2) {
                // walk the shell at Chebyshev radius R
                const int y0 = max(c[1] - R, 0), y1 = min(c[1] + R, G.g[1] - 1);
                const int z0 = max(c[2] - R, 0), z1 = min(c[2] + R, G.g[2] - 1);
                const int x0 = max(c[0] - R, 0), x1 = min(c[0] + R, G.g[0] - 1);
                for (int z = z0; z <= z1; ++z) {
                    const bool zface = (z == c[2] - R) || (z == c[2] + R);
                    for (int y = y0; y <= y1; ++y) {
                        const bool yface = (y == c[1] - R) || (y == c[1] + R);
                        const int64_t row = ((int64_t)z * G.g[1] + y) * G.g[0];
                        if (zface || yface) {
                            scan_range<T, KT>(gpts, gidx, start[row + x0], start[row + x1 + 1], qx, qy, qz, kd, ki,
                                              visits);
                        } else {
                            if (c[0] - R >= 0)
                                scan_range<T, KT>(gpts, gidx, start[row + c[0] - R], start[row + c[0] - R + 1], qx,
                                                  qy, qz, kd, ki, visits);
                            if (c[0] + R <= G.g[0] - 1)
                                scan_range<T, KT>(gpts, gidx, start[row + c[0] + R], start[row + c[0] + R + 1], qx,
                                                  qy, qz, kd, ki, visits);
                        }
                    }
                }
              }
                // lower bound on the distance to any unvisited cell
                double lb = 1e300;
                bool any = false;
                for (int a = 0; a < 3; ++a) {
                    if (c[a] - R - 1 >= 0) {
                        const double face = G.lo[a] + (double)(c[a] - R) * G.h;
                        lb = fmin(lb, q[a] - face);
                        any = true;
                    }
                    if (c[a] + R + 1 <= G.g[a] - 1) {
                        const double face = G.lo[a] + (double)(c[a] + R + 1) * G.h;
                        lb = fmin(lb, face - q[a]);
                        any = true;
                    }
                }
                if (!any) break;  // the whole grid has been visited
                if (lb > 0.0) {
                    const double lb2 = lb * lb * margin;
                    if ((double)kd[KT - 1] < lb2 && ki[KT - 1] != 0x7fffffff) break;
                    if (lb2 > (double)maxR2) break;
                }
            }
        }
        for (int s = 0; s < k; ++s) {
            T d = kd[s];
            int32_t id = ki[s];
            if (id == 0x7fffffff || !(d <= maxR2)) {
                d = (T)__builtin_huge_val();
                id = -1;
            }
            out_d[qi * k + s] = d;
            out_i[qi * k + s] = id;
        }
    }
    // PointCountTouched: one atomic per wave
    unsigned long long v = visits;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && visited) atomicAdd(visited, v);
}

template <typename T>
void launch_grid_match(const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const double* lo, double h,
                       const int* g, const P4<T>* rd, const int32_t* order, int64_t N, const Mat4<T>& Tm, int knn,
                       T maxR2, T* dists, int32_t* ids, unsigned long long* visited, hipStream_t s) {
    if (N <= 0) return;
    GridGeom G;
    for (int a = 0; a < 3; ++a) {
        G.lo[a] = lo[a];
        G.g[a] = g[a];
    }
    G.h = h;
    G.inv_h = 1.0 / h;
    const dim3 grid((unsigned)((N + 255) / 256));
    if (knn == 1)
        hipLaunchKernelGGL((grid_match_kernel<T, 1>), grid, dim3(256), 0, s, gpts, gidx, start, G, rd, order, N, Tm,
                           knn, maxR2, dists, ids, visited);
    else if (knn <= 2)
        hipLaunchKernelGGL((grid_match_kernel<T, 2>), grid, dim3(256), 0, s, gpts, gidx, start, G, rd, order, N, Tm,
                           knn, maxR2, dists, ids, visited);
    else if (knn <= 4)
        hipLaunchKernelGGL((grid_match_kernel<T, 4>), grid, dim3(256), 0, s, gpts, gidx, start, G, rd, order, N, Tm,
                           knn, maxR2, dists, ids, visited);
    else if (knn <= 8)
        hipLaunchKernelGGL((grid_match_kernel<T, 8>), grid, dim3(256), 0, s, gpts, gidx, start, G, rd, order, N, Tm,
                           knn, maxR2, dists, ids, visited);
    else
        hipLaunchKernelGGL((grid_match_kernel<T, 16>), grid, dim3(256), 0, s, gpts, gidx, start, G, rd, order, N,
                           Tm, knn, maxR2, dists, ids, visited);
}

template void launch_grid_match<float>(const P4<float>*, const int32_t*, const uint32_t*, const double*, double,
                                       const int*, const P4<float>*, const int32_t*, int64_t, const Mat4<float>&, int,
                                       float, float*, int32_t*, unsigned long long*, hipStream_t);
template void launch_grid_match<double>(const P4<double>*, const int32_t*, const uint32_t*, const double*, double,
                                        const int*, const P4<double>*, const int32_t*, int64_t, const Mat4<double>&,
                                        int, double, double*, int32_t*, unsigned long long*, hipStream_t);

}  // namespace pmx
