// pmx_knn_wide.hip — exact k-NN for k > 16 (KDTreeMatcher knn: any k >= 1,
// MatchersImpl.h:83; lists past 1024 entries in chunks of 1024).
//
// Same contract as pmx_grid.hip / pmx_match.hip (MatchersImpl.cpp:85-101
// with libnabo's exact search): distances are ((dx*dx + dy*dy) + dz*dz) in T
// without FMA, the k-list is sorted by (distance, original index), entries
// beyond maxDist (or a per-query radius) come out as (+inf, -1).
//
// The per-lane searches keep a query's k-list in registers, which stops at
// k = 16.  Here ONE WAVE owns one query and the list is spread over the
// wave: entry s lives in lane s % 64, slot s / 64 (E slots per lane, k <=
// 64 E).  The search walks the same cubic shells of grid cells as the
// per-lane shell search (the 3x3x3 block, then shell R = 2, 3, ...), with the
// same row pruning against the k-th distance and the same certificate
//   stop when  d_k < LB^2 (1 - 1e-5)  or  LB^2 (1 - 1e-5) > maxDist^2
// (LB = distance from the query to the unvisited cells), but a shell's point
// ranges are flattened over the wave: the lanes decode their rows' ranges,
// an inclusive scan numbers the points, and every batch of 64 points is
// evaluated one per lane.  Points that beat the current k-th entry are
// inserted in lane order, one at a time (a broadcast, a compare per slot and
// a shift up by one entry through the lanes), so the result never depends on
// the evaluation order: the list is the k smallest (distance, index) pairs.
//
// Brute force (no grid, or pmx_set_search(brute)): the same kernel with one
// range, the whole reference; ids are then reference indices.
#include "pmx_internal.h"
#include "pmx_spec.h"

namespace pmx {

namespace {

constexpr int32_t kNone = 0x7fffffff;  // empty entry (sorts after every real index)
constexpr int kWideChunk = 1024;       // the largest k-list one wave holds (16 entries per lane)

template <typename T>
__device__ __forceinline__ T wsqd(T qx, T qy, T qz, const P4<T>& r) {
    const T dx = r.x - qx;
    const T dy = r.y - qy;
    const T dz = r.z - qz;
    T d = dx * dx;
    d = d + dy * dy;
    d = d + dz * dz;
    return d;
}

// (d, o) sorts before (wd, wo)
template <typename T>
__device__ __forceinline__ bool before(T d, int32_t o, T wd, int32_t wo) {
    return d < wd || (d == wd && o < wo);
}

template <typename T, int E>
struct WideList {
    T d[E];
    int32_t o[E];  // original reference index (the tie rule)
    int32_t p[E];  // position in the searched array (the id written out)
};

template <typename T, int E>
__device__ __forceinline__ void wl_clear(WideList<T, E>& L) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
        L.d[e] = (T)__builtin_huge_val();
        L.o[e] = kNone;
        L.p[e] = kNone;
    }
}

// entry s of the list (uniform s), broadcast to every lane
template <typename T, int E>
__device__ __forceinline__ void wl_at(const WideList<T, E>& L, int s, T& d, int32_t& o) {
    T dv = L.d[0];
    int32_t ov = L.o[0];
#pragma unroll
    for (int e = 1; e < E; ++e)
        if ((s >> 6) == e) {
            dv = L.d[e];
            ov = L.o[e];
        }
    d = __shfl(dv, s & 63);
    o = __shfl(ov, s & 63);
}

// insert (d, o, p) (uniform; it sorts before entry k - 1): every entry after
// it moves up by one
template <typename T, int E>
__device__ __forceinline__ void wl_insert(WideList<T, E>& L, T d, int32_t o, int32_t p) {
    const int lane = threadIdx.x & 63;
    int gt[E];
#pragma unroll
    for (int e = 0; e < E; ++e) gt[e] = before(d, o, L.d[e], L.o[e]) ? 1 : 0;
    T pd[E];
    int32_t po[E], pp[E];
    int pg[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {  // the entry before each one (lane 0: slot e - 1 of lane 63)
        pd[e] = __shfl_up(L.d[e], 1);
        po[e] = __shfl_up(L.o[e], 1);
        pp[e] = __shfl_up(L.p[e], 1);
        pg[e] = __shfl_up(gt[e], 1);
        if (e > 0) {
            const T wd = __shfl(L.d[e - 1], 63);
            const int32_t wo = __shfl(L.o[e - 1], 63), wp = __shfl(L.p[e - 1], 63);
            const int wg = __shfl(gt[e - 1], 63);
            if (lane == 0) {
                pd[e] = wd;
                po[e] = wo;
                pp[e] = wp;
                pg[e] = wg;
            }
        } else if (lane == 0) {
            pg[e] = 0;
        }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (!gt[e]) continue;
        L.d[e] = pg[e] ? pd[e] : d;
        L.o[e] = pg[e] ? po[e] : o;
        L.p[e] = pg[e] ? pp[e] : p;
    }
}

// Evaluate the points of the lanes' ranges [a0, b0) + [a1, b1) against the
// list; wd / wo: the current entry k - 1 (updated).  ld / lo: the chunk's
// lower bound — only points sorting after (ld, lo) compete (chunked k-lists)
template <typename T, int E>
__device__ __forceinline__ void wl_scan(const P4<T>* __restrict__ pts, const int32_t* __restrict__ gidx, uint32_t a0,
                                        uint32_t b0, uint32_t a1, uint32_t b1, T qx, T qy, T qz, int k,
                                        WideList<T, E>& L, T& wd, int32_t& wo, uint32_t& visits, T ld,
                                        int32_t lo) {
    const int lane = threadIdx.x & 63;
    const uint32_t l0 = b0 - a0, len = l0 + (b1 - a1);
    uint32_t inc = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(inc, off);
        if (lane >= off) inc += v;
    }
    const uint32_t total = __shfl(inc, 63);
    for (uint32_t base = 0; base < total; base += 64) {  // (uniform)
        const uint32_t f = base + (uint32_t)lane;
        // the range owner: the first lane whose inclusive count exceeds f
        int own = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
            const uint32_t v = __shfl(inc, own + step - 1);
            if (v <= f) own += step;
        }
        own = own > 63 ? 63 : own;
        const uint32_t o_inc = __shfl(inc, own), o_len = __shfl(len, own), o_a0 = __shfl(a0, own),
                       o_l0 = __shfl(l0, own), o_a1 = __shfl(a1, own);
        const bool act = f < total;
        const uint32_t off = f - (o_inc - o_len);
        const uint32_t pos = act ? (off < o_l0 ? o_a0 + off : o_a1 + (off - o_l0)) : 0u;
        T d = (T)__builtin_huge_val();
        if (act) {
            d = wsqd(qx, qy, qz, gld32(pts, pos));
            ++visits;
        }
        bool pass = act && d <= wd && d >= ld;
        int32_t o = kNone;
        if (pass) {
            o = gidx ? gld32(gidx, pos) : (int32_t)pos;
            pass = before(d, o, wd, wo) && before(ld, lo, d, o);
        }
        unsigned long long m = __ballot(pass);
        while (m) {  // (uniform) in lane order; each re-checked against the moved k-th entry
            const int src = __ffsll((long long)m) - 1;
            m &= m - 1;
            const T cd = __shfl(d, src);
            const int32_t co = __shfl(o, src), cp = __shfl((int32_t)pos, src);
            if (before(cd, co, wd, wo)) {
                wl_insert<T, E>(L, cd, co, cp);
                wl_at<T, E>(L, k - 1, wd, wo);
            }
        }
    }
}

__device__ __forceinline__ double wgap(const GridGeom& G, int a, int c, double v) {
    const double lo = G.lo[a] + (double)c * G.h, hi = lo + G.h;
    return v < lo ? lo - v : (v > hi ? v - hi : 0.0);
}
__device__ __forceinline__ int wcell_x(const GridGeom& G, double v) {
    const double f = (v - G.lo[0]) * G.inv_h;
    return f < 0.0 ? 0 : (f >= (double)G.g[0] ? G.g[0] - 1 : (int)f);
}

}  // namespace

// One wave per query (4 per block).  gidx / start null: brute force over
// pts[0, M) (ids are indices).  Loop mode (ctl): transform and level from the
// device, as the per-lane kernel.
// Chunked k-lists (k > 64 E: KDTreeMatcher's knn is bounded only by int,
// MatchersImpl.h:83): this launch finds entries [c0, c0 + k) of the query's
// list of kstride entries — the k smallest (distance, index) pairs after
// entry c0 - 1, which the previous launch wrote — with the same search and
// certificate; the launches run in stream order.
template <typename T, int E>
__global__ __launch_bounds__(256) void knn_wide_kernel(const P4<T>* __restrict__ pts, const int32_t* __restrict__ gidx,
                                                       const uint32_t* __restrict__ start, GridGeom G, int64_t M,
                                                       const P4<T>* __restrict__ rd, int64_t N, Mat4<T> Tm, int k,
                                                       int c0, int kstride, T maxR2, const T* __restrict__ radii,
                                                       T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                                       unsigned long long* __restrict__ visited,
                                                       const LoopCtl* __restrict__ ctl,
                                                       const GridDesc<T>* __restrict__ gd, SpecSel* __restrict__ spec) {
    if (ctl) {
        if (ctl->done) return;
        const GridDesc<T>& D = gd[ctl->level];
        pts = D.gpts;
        gidx = D.gidx;
        start = D.start;
        G = D.G;
        ctl_transform(ctl, Tm);
    }
    const int lane = threadIdx.x & 63;
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= N) return;  // (whole wave)
    const T r2 = radii ? radii[j] * radii[j] : maxR2;
    // the chunk's lower bound: the previous chunk's last entry
    T ld = -(T)__builtin_huge_val();
    int32_t lo = -1;
    bool none = false;  // (the previous chunk already ran out of points: padding only)
    if (c0 > 0) {
        const int32_t pp = out_i[j * kstride + c0 - 1];
        ld = out_d[j * kstride + c0 - 1];
        none = pp < 0;
        lo = none ? -1 : (gidx ? gld32(gidx, (uint32_t)pp) : (int32_t)pp);
    }
    T qx, qy, qz;
    {
        const P4<T> p = gld(rd, j);
        qx = ((Tm.m[0] * p.x + Tm.m[1] * p.y) + Tm.m[2] * p.z) + Tm.m[3] * p.w;
        qy = ((Tm.m[4] * p.x + Tm.m[5] * p.y) + Tm.m[6] * p.z) + Tm.m[7] * p.w;
        qz = ((Tm.m[8] * p.x + Tm.m[9] * p.y) + Tm.m[10] * p.z) + Tm.m[11] * p.w;
    }
    WideList<T, E> L;
    wl_clear<T, E>(L);
    T wd = (T)__builtin_huge_val();
    int32_t wo = kNone;
    uint32_t visits = 0;
    const double q[3] = {(double)qx, (double)qy, (double)qz};
    bool qnan = !(q[0] == q[0]) || !(q[1] == q[1]) || !(q[2] == q[2]) || none;
    if (!start) {
        // brute force: lane 0 holds the one range
        if (!qnan)
            wl_scan<T, E>(pts, nullptr, 0u, lane == 0 ? (uint32_t)M : 0u, 0u, 0u, qx, qy, qz, k, L, wd, wo, visits,
                          ld, lo);
    } else if (!qnan) {
        const double margin = 1.0 - 1e-5;
        int c[3];
        for (int a = 0; a < 3; ++a) {
            const double f = (q[a] - G.lo[a]) * G.inv_h;
            c[a] = f < 0.0 ? 0 : (f >= (double)G.g[a] ? G.g[a] - 1 : (int)f);
        }
        for (int R = 1;; ++R) {
            // rows of this step: R = 1 the 3x3 rows of the whole block, else the
            // (2R + 1)^2 rows of shell R (face rows: an x-range, others: the two end cells)
            const int side = 2 * R + 1;
            const int nrows = side * side;
            const double lim = wo == kNone ? 1e300 : (double)wd / margin;
            for (int r0 = 0; r0 < nrows; r0 += 64) {  // (uniform)
                const int r = r0 + lane;
                uint32_t a0 = 0, b0 = 0, a1 = 0, b1 = 0;
                if (r < nrows) {
                    const int z = c[2] - R + r / side, y = c[1] - R + r % side;
                    if (z >= 0 && z < G.g[2] && y >= 0 && y < G.g[1]) {
                        const uint32_t row = ((uint32_t)z * (uint32_t)G.g[1] + (uint32_t)y) * (uint32_t)G.g[0];
                        const int x0 = max(c[0] - R, 0), x1 = min(c[0] + R, G.g[0] - 1);
                        if (R == 1) {
                            a0 = gld32(start, row + x0);
                            b0 = gld32(start, row + x1 + 1);
                        } else {
                            // pruned: every point of a skipped cell is farther than the k-th entry
                            const double gz = wgap(G, 2, z, q[2]), gy = wgap(G, 1, y, q[1]);
                            const double g2 = gz * gz + gy * gy;
                            const bool face = z == c[2] - R || z == c[2] + R || y == c[1] - R || y == c[1] + R;
                            if (g2 <= lim) {
                                if (face) {
                                    int xa = x0, xb = x1;
                                    if (lim < 1e300) {
                                        const double rem = sqrt(lim - g2);
                                        xa = max(x0, wcell_x(G, q[0] - rem) - 1);
                                        xb = min(x1, wcell_x(G, q[0] + rem) + 1);
                                    }
                                    if (xa <= xb) {
                                        a0 = gld32(start, row + xa);
                                        b0 = gld32(start, row + xb + 1);
                                    }
                                } else {
                                    const int xl = c[0] - R, xr = c[0] + R;
                                    if (xl >= 0) {
                                        const double gx = wgap(G, 0, xl, q[0]);
                                        if (g2 + gx * gx <= lim) {
                                            a0 = gld32(start, row + xl);
                                            b0 = gld32(start, row + xl + 1);
                                        }
                                    }
                                    if (xr <= G.g[0] - 1) {
                                        const double gx = wgap(G, 0, xr, q[0]);
                                        if (g2 + gx * gx <= lim) {
                                            a1 = gld32(start, row + xr);
                                            b1 = gld32(start, row + xr + 1);
                                        }
                                    }
                                }
                            }
                        }
                    }
                }
                wl_scan<T, E>(pts, gidx, a0, b0, a1, b1, qx, qy, qz, k, L, wd, wo, visits, ld, lo);
            }
            // the lower bound on every unvisited cell (uniform)
            double lb = 1e300;
            bool any = false;
            for (int a = 0; a < 3; ++a) {
                if (c[a] - R - 1 >= 0) {
                    lb = fmin(lb, q[a] - (G.lo[a] + (double)(c[a] - R) * G.h));
                    any = true;
                }
                if (c[a] + R + 1 <= G.g[a] - 1) {
                    lb = fmin(lb, (G.lo[a] + (double)(c[a] + R + 1) * G.h) - q[a]);
                    any = true;
                }
            }
            if (!any) break;  // the whole grid has been visited
            if (lb > 0.0) {
                const double lb2 = lb * lb * margin;
                if ((double)wd < lb2 && wo != kNone) break;
                if (lb2 > (double)r2) break;
            }
        }
    }
    // the list, coalesced: entry s of query j at j * k + s
    SpecAcc<T> sa;
    spec_acc_init<T>(sa, spec);
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int s = e * 64 + lane;
        if (s < k) {
            T d = L.d[e];
            int32_t id = L.p[e];
            if (id == kNone || !(d <= r2)) {
                d = (T)__builtin_huge_val();
                id = -1;
            }
            out_d[j * kstride + c0 + s] = d;
            out_i[j * kstride + c0 + s] = id;
            if (sa.on) spec_acc<T>(sa, d);
        }
    }
    if (visited) {
        unsigned long long v = visits;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0 && v) {
            const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6);
            atomicAdd(visited + (size_t)(wave & (kVSlots - 1)) * kVStride, v);
        }
        if (sa.on) {
            const unsigned wave = blockIdx.x * 4 + (threadIdx.x >> 6);
            spec_acc_flush<T>(sa, visited + ((size_t)2 * kVSlots + (wave & (kVSlots - 1))) * kVStride,
                              visited + ((size_t)3 * kVSlots + (wave & (kVSlots - 1))) * kVStride);
        }
    }
}

template <typename T>
void launch_knn_wide(const P4<T>* pts, const int32_t* gidx, const uint32_t* start, const GridGeom* G, int64_t M,
                     const P4<T>* rd, int64_t N, const Mat4<T>& Tm, int k, T maxR2, const T* radii, T* out_d,
                     int32_t* out_i, unsigned long long* visited, const LoopCtl* ctl, const GridDesc<T>* gd,
                     SpecSel* spec, hipStream_t s) {
    if (N <= 0) return;
    GridGeom g{};
    if (G) g = *G;
    const dim3 grid((unsigned)((N + 3) / 4));
#define PMX_WIDE(E, KC, C0)                                                                                          \
    hipLaunchKernelGGL((knn_wide_kernel<T, E>), grid, dim3(256), 0, s, pts, gidx, start, g, M, rd, N, Tm, KC, C0, k, \
                       maxR2, radii, out_d, out_i, visited, ctl, gd, spec)
    if (k <= 64)
        PMX_WIDE(1, k, 0);
    else if (k <= 128)
        PMX_WIDE(2, k, 0);
    else if (k <= 256)
        PMX_WIDE(4, k, 0);
    else if (k <= 512)
        PMX_WIDE(8, k, 0);
    else
        for (int c0 = 0; c0 < k; c0 += kWideChunk) PMX_WIDE(16, std::min(kWideChunk, k - c0), c0);
#undef PMX_WIDE
}

template void launch_knn_wide<float>(const P4<float>*, const int32_t*, const uint32_t*, const GridGeom*, int64_t,
                                     const P4<float>*, int64_t, const Mat4<float>&, int, float, const float*, float*,
                                     int32_t*, unsigned long long*, const LoopCtl*, const GridDesc<float>*, SpecSel*,
                                     hipStream_t);
template void launch_knn_wide<double>(const P4<double>*, const int32_t*, const uint32_t*, const GridGeom*, int64_t,
                                      const P4<double>*, int64_t, const Mat4<double>&, int, double, const double*,
                                      double*, int32_t*, unsigned long long*, const LoopCtl*,
                                      const GridDesc<double>*, SpecSel*, hipStream_t);

}  // namespace pmx
