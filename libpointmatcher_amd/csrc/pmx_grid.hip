// pmx_grid.hip — exact k-NN over a uniform grid of the reference.
//
// Same contract as pmx_match.hip (KDTreeMatcher::findClosests,
// MatchersImpl.cpp:85-101 with libnabo's exact search): distances are the
// bit-identical ((dx*dx + dy*dy) + dz*dz) in T without FMA, candidates are
// ordered by (distance, original index) so ties resolve to the lowest index,
// k-lists are sorted ascending.  Only the set of pairs evaluated changes.
//
// Layout (built once per Matcher::init on the host, pmx_capi.hip):
//   gpts  P4<T>[M]        reference points sorted by cell (x fastest)
//   gidx  int32[M]        their original indices
//   start uint32[C + 1]   first point of each cell (C = gx * gy * gz)
// Each x-row of cells is one contiguous point range.  Match ids produced
// here are POSITIONS in gpts (the reductions gather gpts / sorted normals
// coherently); gidx maps them back to reference indices for ties and for
// the host mirror.  The reading arrives in slot order (Morton order of the
// initial cell, pmx_set_reading), so consecutive lanes hold nearby queries
// and every output write is coalesced.
//
// Per-lane shell search (default): each lane visits the cells of growing
// cubic shells around its query's cell (the 3x3x3 block first, its nine row
// bounds prefetched together) and stops at the LB test below with the box of
// visited cells.  Measured best at ~2-4 points per occupied cell (C3:
// 0.106 ms per 1M queries); it is bound by the dependent gather latency of
// the row scans, not by pair evaluation.
//
// Tile kernel (option grid_mode=tile, pmx_grid_tile.inc).  One wave = up to 64
// queries inside one aligned Morton block (the wave table of
// pmx_set_reading).  The wave takes the bounding box of its queries' cells, grows it
// by one cell, copies the box's reference points (ny * nz contiguous row
// ranges) into LDS, and every lane scans the whole LDS list (broadcast reads,
// no divergence); the box grows by one cell per round until every lane is
// certified.  A lane's result is exact when its k-th distance is below the
// squared distance to the nearest box face that is not a grid boundary:
//
//   LB = min over interior box faces of |q - face|   (in double)
//   certified when  d_k < LB^2 (1 - 1e-5)   or  LB^2 (1 - 1e-5) > maxDist^2.
//
// The 1e-5 relative margin dominates every rounding involved (T distances
// carry a few ulp; cell assignment is done in double), so no point outside
// the box can produce a distance <= d_k.  Lanes of waves whose box grows too
// large run the per-lane shell search.  It evaluates 5x more pairs than the
// per-lane search from LDS (broadcast reads) and measures 0.187 ms at C3: a
// candidate for QPT > 1 and for very dense references.
#include "pmx_internal.h"

#include <hip/hip_ext.h>

#include "pmx_spec.h"

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

// position <-> the w lane of an LDS point (bit pattern, never used as a number)
__device__ __forceinline__ float pos_w(uint32_t p, float) { return __uint_as_float(p); }
__device__ __forceinline__ double pos_w(uint32_t p, double) { return __longlong_as_double((long long)p); }
__device__ __forceinline__ uint32_t w_pos(float w) { return __float_as_uint(w); }
__device__ __forceinline__ uint32_t w_pos(double w) { return (uint32_t)__double_as_longlong(w); }

constexpr int32_t kNoPos = 0x7fffffff;

__device__ __forceinline__ float vmin(float a, float b) { return fminf(a, b); }
__device__ __forceinline__ double vmin(double a, double b) { return fmin(a, b); }

// (equal distance) does candidate position a come before the held position b?
// Ties are broken on the ORIGINAL reference index, as the brute force does.
__device__ __forceinline__ bool tie_first(const int32_t* __restrict__ gidx, int32_t a, int32_t b) {
    if (b == kNoPos) return true;
    if (a == kNoPos) return false;
    return gld32(gidx, (uint32_t)a) < gld32(gidx, (uint32_t)b);
}

template <typename T, int KT>
__device__ __forceinline__ void ginsert(const int32_t* __restrict__ gidx, T (&kd)[KT], int32_t (&ki)[KT], T d,
                                        int32_t pos) {
    // lexicographic (d, original index) insertion
    kd[KT - 1] = d;
    ki[KT - 1] = pos;
#pragma unroll
    for (int s = KT - 1; s > 0; --s) {
        bool sw = kd[s] < kd[s - 1];
        if (!sw && kd[s] == kd[s - 1]) sw = tie_first(gidx, ki[s], ki[s - 1]);
        const T td = sw ? kd[s - 1] : kd[s];
        const int32_t ti = sw ? ki[s - 1] : ki[s];
        kd[s - 1] = sw ? kd[s] : kd[s - 1];
        ki[s - 1] = sw ? ki[s] : ki[s - 1];
        kd[s] = td;
        ki[s] = ti;
    }
}

template <typename T, int KT>
__device__ __forceinline__ void consider(const int32_t* __restrict__ gidx, int32_t pos, T d, T (&kd)[KT],
                                         int32_t (&ki)[KT]) {
    if (d <= kd[KT - 1]) {
        if (d < kd[KT - 1] || tie_first(gidx, pos, ki[KT - 1])) ginsert<T, KT>(gidx, kd, ki, d, pos);
    }
}

// the k-th entry of a k-list (k <= KT; static indexing keeps the list in
// registers)
template <typename T, int KT>
__device__ __forceinline__ void kth(const T (&kd)[KT], const int32_t (&ki)[KT], int k, T& dk, int32_t& ik) {
    dk = kd[0];
    ik = ki[0];
#pragma unroll
    for (int s = 1; s < KT; ++s)
        if (s == k - 1) {
            dk = kd[s];
            ik = ki[s];
        }
}

// Scan one contiguous point range of gpts (per-lane search).  Latency-bound:
// points are fetched kScanU at a time with independent loads; a short row
// (a few points at the default density) is one masked chunk — a scalar tail
// loop would make every point its own dependent round trip.
constexpr int kScanU = 4;
// phase-1 row grouping of the per-lane search (rows per group, points per row)
constexpr int kP1G = 3;
constexpr int kP1U = 4;
static_assert(9 % kP1G == 0, "phase-1 groups must tile the nine rows");
template <typename T, int KT>
__device__ __forceinline__ void scan_range(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                           uint32_t a, uint32_t b, T qx, T qy, T qz, T (&kd)[KT],
                                           int32_t (&ki)[KT], uint32_t& visits) {
    visits += b - a;
    constexpr int U = kScanU;
    for (uint32_t j = a; j < b; j += U) {
        P4<T> p[U];
#pragma unroll
        for (int u = 0; u < U; ++u) p[u] = gld32(gpts, j + u < b ? j + u : a);  // in-range address either way
        T d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = gsqd(qx, qy, qz, p[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (j + u < b) consider<T, KT>(gidx, (int32_t)(j + u), d[u], kd, ki);
    }
}

__device__ __forceinline__ void cell_of_q(const GridGeom& G, const double q[3], int c[3], bool& qnan) {
    qnan = false;
    for (int a = 0; a < 3; ++a) {
        const double f = (q[a] - G.lo[a]) * G.inv_h;
        if (!(f == f)) qnan = true;
        c[a] = f < 0.0 ? 0 : (f >= (double)G.g[a] ? G.g[a] - 1 : (int)f);
    }
}

// distance from coordinate v to the slab of cell c along axis a (0 inside)
__device__ __forceinline__ double axis_gap(const GridGeom& G, int a, int c, double v) {
    const double lo = G.lo[a] + (double)c * G.h, hi = lo + G.h;
    return v < lo ? lo - v : (v > hi ? v - hi : 0.0);
}
// x cell of a coordinate, clamped to the grid
__device__ __forceinline__ int cell_x(const GridGeom& G, double v) {
    const double f = (v - G.lo[0]) * G.inv_h;
    return f < 0.0 ? 0 : (f >= (double)G.g[0] ? G.g[0] - 1 : (int)f);
}

// Exact shell search for one query (from scratch); kd/ki must be
// initialised.  Certified on the k-th entry of the list (entries past k, when
// KT > k, are the next-nearest points visited).  lb_exit: the distance from
// the query to the unvisited region at exit (1e300: the whole grid).
// kp: the list entry (1-based) cells are pruned against — the one the safe
// radius of the temporal reuse takes as a bound on every point not kept;
// 0: k + 1 when the list has room.
template <typename T, int KT>
__device__ __forceinline__ void lane_search(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                            const uint32_t* __restrict__ start, const GridGeom& G, T qx, T qy, T qz,
                            const double q[3], const int c[3], T maxR2, int k, T (&kd)[KT], int32_t (&ki)[KT],
                            uint32_t& visits, double& lb_exit, int kp = 0) {
    if (kp <= 0) kp = k < KT ? k + 1 : k;
    const double margin = 1.0 - 1e-5;
    lb_exit = 1e300;
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
            const uint32_t row = ((uint32_t)zc * (uint32_t)G.g[1] + (uint32_t)yc) * (uint32_t)G.g[0];
            const uint32_t va = gld32(start, row + x0);
            const uint32_t vb = gld32(start, row + x1 + 1);
            ra[r] = ok ? va : 0u;
            rb[r] = ok ? vb : 0u;
        }
        // The rows are scanned in groups of kP1G: the first kP1U points of
        // every row of a group are loaded together (one round trip per group
        // instead of one per row), longer rows finish with chunked scans.
        constexpr int GR = kP1G, U = kP1U;
#pragma unroll
        for (int g = 0; g < 9; g += GR) {
            P4<T> p[GR][U];
#pragma unroll
            for (int rr = 0; rr < GR; ++rr)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t j = ra[g + rr] + u;
                    p[rr][u] = gld32(gpts, j < rb[g + rr] ? j : 0u);  // masked: any in-range address
                }
#pragma unroll
            for (int rr = 0; rr < GR; ++rr) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t j = ra[g + rr] + u;
                    if (j < rb[g + rr]) consider<T, KT>(gidx, (int32_t)j, gsqd(qx, qy, qz, p[rr][u]), kd, ki);
                }
                visits += rb[g + rr] - ra[g + rr];
                uint32_t rest = ra[g + rr] + U;
                if (rest < rb[g + rr]) {
                    uint32_t v0 = 0;
                    scan_range<T, KT>(gpts, gidx, rest, rb[g + rr], qx, qy, qz, kd, ki, v0);
                }
            }
        }
    }
    for (int R = 1;; ++R) {
        if (R >= 2) {
            // walk the shell at Chebyshev radius R.  Rows (and the x-range of
            // a face row) whose cells are all farther than the current k-th
            // (k+1-th) distance are skipped: every point there has d > d_k, so it can
            // neither enter the list nor tie (1e-5 relative margin on the
            // gap, far above the T rounding of d and the host's cell
            // assignment; one extra cell each side of an x-range for the
            // latter).  The certificate below is unchanged: skipped cells hold
            // no candidate.
            const int y0 = max(c[1] - R, 0), y1 = min(c[1] + R, G.g[1] - 1);
            const int z0 = max(c[2] - R, 0), z1 = min(c[2] + R, G.g[2] - 1);
            const int x0 = max(c[0] - R, 0), x1 = min(c[0] + R, G.g[0] - 1);
            for (int z = z0; z <= z1; ++z) {
                // (pruned against list entry k + 1 when the list has room for
                // it: the safe radius of the temporal reuse takes that entry
                // as a bound on every non-neighbour, so no cell holding a
                // point closer than it may be skipped)
                T dkT;
                int32_t ikT;
                kth(kd, ki, kp, dkT, ikT);
                const double lim = ikT == kNoPos ? 1e300 : (double)dkT / margin;
                const double gz = axis_gap(G, 2, z, q[2]), gz2 = gz * gz;
                if (gz2 > lim) continue;
                const bool zface = (z == c[2] - R) || (z == c[2] + R);
                for (int y = y0; y <= y1; ++y) {
                    const double gy = axis_gap(G, 1, y, q[1]), g2 = gz2 + gy * gy;
                    if (g2 > lim) continue;
                    const bool yface = (y == c[1] - R) || (y == c[1] + R);
                    const uint32_t row = ((uint32_t)z * (uint32_t)G.g[1] + (uint32_t)y) * (uint32_t)G.g[0];
                    if (zface || yface) {
                        int xa = x0, xb = x1;
                        if (lim < 1e300) {
                            const double rem = sqrt(lim - g2);
                            xa = max(x0, cell_x(G, q[0] - rem) - 1);
                            xb = min(x1, cell_x(G, q[0] + rem) + 1);
                        }
                        if (xa <= xb)
                            scan_range<T, KT>(gpts, gidx, gld32(start, row + xa), gld32(start, row + xb + 1), qx, qy,
                                              qz, kd, ki, visits);
                    } else {
                        const int xl = c[0] - R, xr = c[0] + R;
                        if (xl >= 0) {
                            const double gx = axis_gap(G, 0, xl, q[0]);
                            if (g2 + gx * gx <= lim)
                                scan_range<T, KT>(gpts, gidx, gld32(start, row + xl), gld32(start, row + xl + 1), qx,
                                                  qy, qz, kd, ki, visits);
                        }
                        if (xr <= G.g[0] - 1) {
                            const double gx = axis_gap(G, 0, xr, q[0]);
                            if (g2 + gx * gx <= lim)
                                scan_range<T, KT>(gpts, gidx, gld32(start, row + xr), gld32(start, row + xr + 1), qx,
                                                  qy, qz, kd, ki, visits);
                        }
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
        lb_exit = any ? lb : 1e300;
        if (!any) break;  // the whole grid has been visited
        if (lb > 0.0) {
            const double lb2 = lb * lb * margin;
            T dk;
            int32_t ik;
            kth(kd, ki, k, dk, ik);
            if ((double)dk < lb2 && ik != kNoPos) break;
            if (lb2 > (double)maxR2) break;
        }
    }
}

template <typename T, int KT>
__device__ __forceinline__ void write_out(int64_t j, int k, T maxR2, const T (&kd)[KT], const int32_t (&ki)[KT],
                                          T* __restrict__ out_d, int32_t* __restrict__ out_i, SpecAcc<T>& sa) {
#pragma unroll
    for (int s = 0; s < KT; ++s) {  // static indexing keeps kd/ki in registers
        if (s < k) {
            T d = kd[s];
            int32_t id = ki[s];
            if (id == kNoPos || !(d <= maxR2)) {
                d = (T)__builtin_huge_val();
                id = -1;
            }
            st_out(&out_d[j * k + s], d);
            st_out(&out_i[j * k + s], id);
            if (sa.on) spec_acc<T>(sa, d);
        }
    }
}

// k = 1 neighbour record (GridReuse::nbr): the point the k-list holds, with
// the id write_out stores (-1: none, or beyond the radius) in w
// (gpn: the level's interleaved point / normal records — the normal then
// goes to nbr[N + j], what the point-to-plane reduction reads)
template <typename T, int KT>
__device__ __forceinline__ void write_nbr(P4<T>* __restrict__ nbr, const P4<T>* __restrict__ gpts,
                                          const P4<T>* __restrict__ gpn, int64_t N, int64_t j, T maxR2,
                                          const T (&kd)[KT], const int32_t (&ki)[KT]) {
    if (!nbr) return;
    int32_t id = ki[0];
    if (id == kNoPos || !(kd[0] <= maxR2)) id = -1;
    const uint32_t g = id >= 0 ? (uint32_t)id : 0u;
    P4<T> r = gpn ? gpn[2 * (size_t)g] : gld32(gpts, g);
    if (gpn) nbr[N + j] = gpn[2 * (size_t)g + 1];
    r.w = pos_w((uint32_t)id, T(0));
    nbr[j] = r;
}

template <typename T, int KT>
__device__ __forceinline__ void write_out(int64_t j, int k, T maxR2, const T (&kd)[KT], const int32_t (&ki)[KT],
                                          T* __restrict__ out_d, int32_t* __restrict__ out_i) {
    SpecAcc<T> none;
    none.on = false;
    write_out<T, KT>(j, k, maxR2, kd, ki, out_d, out_i, none);
}

// Pair / fallback counters.  One device-scope atomic per wave on a single
// address serialises (~110 us for 16K waves at C3), so every wave adds into
// one of kVSlots counters, each on its own 128-byte line; counter_sum_kernel
// folds them into the iteration block after the match.
__device__ __forceinline__ unsigned long long* vslot(unsigned long long* vpart, int which) {
    const unsigned wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    return vpart + ((size_t)which * kVSlots + (wave & (kVSlots - 1))) * kVStride;
}
__device__ __forceinline__ void add_visits(uint32_t visits, unsigned long long* vpart) {
    unsigned long long v = visits;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && vpart && v) atomicAdd(vslot(vpart, 0), v);
}

template <typename T>
__global__ __launch_bounds__(kVSlots) void counter_sum_kernel(unsigned long long* __restrict__ vpart,
                                                              unsigned long long* __restrict__ out,
                                                              int* __restrict__ iter_err,
                                                              const LoopCtl* __restrict__ ctl,
                                                              SpecSel* __restrict__ spec,
                                                              SelectState* __restrict__ st,
                                                              unsigned long long* __restrict__ xseg) {
    if (ctl && ctl->done) return;
    counter_phase<T>(vpart, out, iter_err, spec, st, xseg);
}

// Several ranks: resolve the quantile from the all-gathered window segments
// (pmx_spec.h).  Every rank runs it on the same segments and writes the same
// limit; a miss leaves the radix passes (with their histogram all-reduce) to
// resolve it.
// stall (the host enqueued the rest of the iteration without reading the
// verdict): a miss stops the loop with done = kCtlStalled, so every kernel
// enqueued after it returns at once, until the host replays the iteration's
// radix passes (pmx_loop_capi.hip).  Every rank picks from the same union, so
// every rank stalls at the same iteration.
template <typename T>
__global__ __launch_bounds__(kVSlots) void spec_pick_kernel(const unsigned long long* __restrict__ segs, int nseg,
                                                            SpecSel* __restrict__ spec,
                                                            SelectState* __restrict__ st,
                                                            LoopCtl* __restrict__ ctl, int stall, int force_miss) {
    __shared__ uint32_t lh[2048];
    __shared__ unsigned long long part[kVSlots];
    __shared__ unsigned long long bc[2];
    if (ctl && ctl->done) return;
    unsigned long long fin = 0, below = 0, nk = 0;
    bool overflow = force_miss != 0;  // (an overflowing segment makes the pick miss)
    for (int s = 0; s < nseg; ++s) {  // (uniform; a handful of segments)
        const unsigned long long* g = segs + (size_t)s * kSpecXStride;
        fin += g[0];
        below += g[1];
        nk += g[2];
        overflow = overflow || g[2] > kSpecXCap;
    }
    SpecKeys<T> src;
    src.segs = segs;
    src.nseg = nseg;
    // the union's keys into LDS once when they fit (every radix round of the
    // pick reads them all; the segments are global memory)
    using K = typename KeyOf<T>::K;
    constexpr unsigned kPickLds = 4096;
    __shared__ K lkeys[kPickLds];
    if (!overflow && nk <= kPickLds && spec->valid) {
        unsigned o = 0;
        for (int s = 0; s < nseg; ++s) {  // (uniform)
            const unsigned ns = src.n(s);
            for (unsigned i = threadIdx.x; i < ns; i += kVSlots) lkeys[o + i] = (K)segs[(size_t)s * kSpecXStride + kSpecXHdr + i];
            o += ns;
        }
        __syncthreads();
        src = SpecKeys<T>();
        src.local = lkeys;
        src.n_local = o;
        src.lds = lkeys;
    }
    const bool hit = spec_pick<T, kVSlots>(spec, st, fin, below, nk, overflow, src, lh, part, bc);
    if (!hit && stall && ctl && threadIdx.x == 0) ctl->done = kCtlStalled;
}

template <typename T>
void launch_spec_pick(const unsigned long long* segs, int nseg, SpecSel* spec, SelectState* st, LoopCtl* ctl,
                      int stall, int force_miss, hipStream_t s) {
    hipLaunchKernelGGL(spec_pick_kernel<T>, dim3(1), dim3(kVSlots), 0, s, segs, nseg, spec, st, ctl, stall,
                       force_miss);
}
template void launch_spec_pick<float>(const unsigned long long*, int, SpecSel*, SelectState*, LoopCtl*, int, int,
                                      hipStream_t);
template void launch_spec_pick<double>(const unsigned long long*, int, SpecSel*, SelectState*, LoopCtl*, int, int,
                                       hipStream_t);

// counters: 0 pairs, 1 full-search fallbacks, 2 finite distances, 3 below the quantile window
// (+ the fold tickets: kTicketGroups + 1 counters, 128 bytes apart)
size_t grid_counter_bytes() { return sizeof(unsigned long long) * 4 * kVSlots * kVStride; }

// ---------------------------------------------------- temporal reuse --
// ICP matches the same reading every iteration under a slowly changing
// transform.  A full search of query q' (previous position) leaves two
// facts: its k-list, whose k-th squared distance is dk', and a safe radius
// rs' — every reference point outside the k-list is at least rs' from q'
// (rs' = min(distance to the unvisited region at exit, distance of the
// (k+1)-th point visited)).  At the new position q = q' + delta:
//   the k-list points are within  a = sqrt(dk') + |delta|,
//   every other point is beyond   b = rs' - |delta|,
// so when a < b (with 1e-5 relative margins, far above the T rounding of
// any distance involved) the k nearest neighbours of q are exactly the
// previous k-list.  Their distances are recomputed in T (the same arithmetic
// a full search uses) and re-sorted with the (distance, original index)
// rule, so the output is bit-identical to a full search; the new safe radius
// is b.  Queries that fail the test (moved too far, previous list
// incomplete, grid level changed) take the full search.  Only the certificate
// decides the result: no cached answer is ever returned unverified.
//
// reuse: 0 = off, 1 = store safe radii only (no usable previous match),
//        2 = store and try the certificate (out_d/out_i/safe hold the
//            previous match of this reading at this level, made at Tprev).
constexpr double kReuseMargin = 1e-5;

// safe radius of a full search: the unvisited region and the (k+1)-th
// visited point (list entry k, when KT > k) bound every non-neighbour
template <typename T, int KT>
__device__ __forceinline__ T safe_radius(const T (&kd)[KT], const int32_t (&ki)[KT], int k, double lb_exit) {
    double r = lb_exit;
    T dn = (T)__builtin_huge_val();
#pragma unroll
    for (int s = 1; s < KT; ++s)
        if (s == k) dn = kd[s];
    if (k >= KT) r = -1.0;  // (no room for the next point: never certify)
    r = fmin(r, sqrt((double)dn));
    T dk;
    int32_t ik;
    kth(kd, ki, k, dk, ik);
    if (ik == kNoPos || !(r > 0.0)) return (T)0;
    return (T)(r * (1.0 - 1e-6));  // (rounded down into T)
}

// the squared search radius of query j: the per-point radii of
// KDTreeVarDistMatcher (MatchersImpl.cpp:131-146; libnabo squares each in T),
// else the matcher's maxDist^2
template <typename T>
__device__ __forceinline__ T qr2(const T* __restrict__ radii, int64_t j, T maxR2) {
    if (!radii) return maxR2;
    const T r = radii[j];
    return r * r;
}

// one query from scratch: the shell search; its k-list, the neighbour record
// (k = 1) and its safe radius
template <typename T, int KT>
__device__ __forceinline__ void full_query(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                           const uint32_t* __restrict__ start, const GridGeom& G,
                                           const P4<T>* __restrict__ rd, int64_t j, const Mat4<T>& Tm, int k,
                                           T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                           T* __restrict__ safe, uint32_t& visits, SpecAcc<T>& sa,
                                           P4<T>* __restrict__ nbr = nullptr, const P4<T>* __restrict__ gpn = nullptr,
                                           int64_t N = 0) {
    T qx, qy, qz;
    gxform(Tm, gld(rd, j), qx, qy, qz);
    T kd[KT];
    int32_t ki[KT];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        kd[s] = (T)__builtin_huge_val();
        ki[s] = kNoPos;
    }
    const double q[3] = {(double)qx, (double)qy, (double)qz};
    int c[3];
    bool qnan;
    cell_of_q(G, q, c, qnan);
    double lb_exit = -1.0;
    if (!qnan) lane_search<T, KT>(gpts, gidx, start, G, qx, qy, qz, q, c, maxR2, k, kd, ki, visits, lb_exit);
    write_out<T, KT>(j, k, maxR2, kd, ki, out_d, out_i, sa);
    write_nbr<T, KT>(nbr, gpts, gpn, N, j, maxR2, kd, ki);
    if (safe) st_out(&safe[j], safe_radius<T, KT>(kd, ki, k, lb_exit));
}

// ---------------------------------------------- wave-cooperative search --
// One query searched by a whole wave: the rows of each cubic ring are split
// over the lanes (one round trip for their bounds, one for their points),
// every lane keeps a private (distance, original index) list of the points it
// evaluated, and the wave merges the lists after each ring.  A per-lane
// search walks the same rings as a chain of dependent row gathers (tens of
// round trips for a query whose certificate failed); here a ring costs two.
// Used for the few queries of a wave that miss the reuse certificate in a
// converged match (the per-lane kernel's phase 2).  The result is the exact
// k-list of the per-lane search: the same (distance, original index) order,
// the same certificate on the interior faces of the visited box.
constexpr int kCoopU = 4;  // ring points each lane has in flight
template <typename T>
struct CoopEnt {
    T d;
    int32_t g;    // original reference index (ties)
    int32_t pos;  // grid position (the match id)
};
template <typename T>
__device__ __forceinline__ bool coop_less(T da, int32_t ga, T db, int32_t gb) {
    return da < db || (da == db && ga < gb);
}
template <typename T, int KT>
__device__ __forceinline__ void coop_insert(T (&ld)[KT], int32_t (&lg)[KT], int32_t (&lp)[KT], T d, int32_t g,
                                            int32_t pos) {
    if (!coop_less(d, g, ld[KT - 1], lg[KT - 1])) return;
    ld[KT - 1] = d;
    lg[KT - 1] = g;
    lp[KT - 1] = pos;
#pragma unroll
    for (int s = KT - 1; s > 0; --s) {
        const bool sw = coop_less(ld[s], lg[s], ld[s - 1], lg[s - 1]);
        const T td = sw ? ld[s - 1] : ld[s];
        const int32_t tg = sw ? lg[s - 1] : lg[s], tp = sw ? lp[s - 1] : lp[s];
        ld[s - 1] = sw ? ld[s] : ld[s - 1];
        lg[s - 1] = sw ? lg[s] : lg[s - 1];
        lp[s - 1] = sw ? lp[s] : lp[s - 1];
        ld[s] = td;
        lg[s] = tg;
        lp[s] = tp;
    }
}
__device__ __forceinline__ float shfl_x(float v, int m) { return __shfl_xor(v, m); }
__device__ __forceinline__ double shfl_x(double v, int m) { return __shfl_xor(v, m); }

// Merge the wave's private lists into the KT smallest (uniform in kd / kg /
// kp); afterwards lane 0 holds the merged list and every other lane an empty
// one (no point is counted twice by a later merge).
template <typename T, int KT>
__device__ __forceinline__ void coop_merge(T (&ld)[KT], int32_t (&lg)[KT], int32_t (&lp)[KT], T (&kd)[KT],
                                           int32_t (&kg)[KT], int32_t (&kp)[KT]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        T md = ld[0];
        int32_t mg = lg[0], mp = lp[0];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const T od = shfl_x(md, off);
            const int32_t og = __shfl_xor(mg, off), op = __shfl_xor(mp, off);
            if (coop_less(od, og, md, mg)) {
                md = od;
                mg = og;
                mp = op;
            }
        }
        kd[s] = md;
        kg[s] = mg;
        kp[s] = mp;
        // the owner pops its head (an empty head, +inf / kNoPos, pops nothing real)
        if (ld[0] == md && lg[0] == mg && mp != kNoPos) {
#pragma unroll
            for (int u = 0; u < KT - 1; ++u) {
                ld[u] = ld[u + 1];
                lg[u] = lg[u + 1];
                lp[u] = lp[u + 1];
            }
            ld[KT - 1] = (T)__builtin_huge_val();
            lg[KT - 1] = kNoPos;
            lp[KT - 1] = kNoPos;
        }
    }
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        ld[s] = lane == 0 ? kd[s] : (T)__builtin_huge_val();
        lg[s] = lane == 0 ? kg[s] : kNoPos;
        lp[s] = lane == 0 ? kp[s] : kNoPos;
    }
}

// The search of one query (uniform arguments), every lane of the wave
// calling.  ks: the rank the exit certifies (k).
// Returns the merged list (uniform, kd / kp as lane_search leaves them:
// positions, kNoPos for an empty entry), lb_exit and the points evaluated
// (lane 0 adds them to its visit count).
template <typename T, int KT>
__device__ __forceinline__ void coop_search(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                         const uint32_t* __restrict__ start, const GridGeom& G, T qx, T qy, T qz,
                                         int ks, T maxR2, T (&kd)[KT], int32_t (&kp)[KT], double& lb_exit,
                                         uint32_t& visits) {
    const int lane = threadIdx.x & 63;
    const double q[3] = {(double)qx, (double)qy, (double)qz};
    int c[3];
    bool qnan;
    cell_of_q(G, q, c, qnan);
    T ld[KT];
    int32_t lg[KT], lp[KT];
    int32_t kg[KT];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        ld[s] = kd[s] = (T)__builtin_huge_val();
        lg[s] = lp[s] = kg[s] = kp[s] = kNoPos;
    }
    lb_exit = -1.0;
    if (qnan) return;  // (uniform: no neighbour, radius 0)
    const double margin = 1.0 - 1e-5;
    uint32_t evals = 0;
    for (int R = 1;; ++R) {
        // ring R: rows (y, z) in [c - R, c + R]^2; R = 1 takes the whole
        // 3x3x3 block, later rings the cells at Chebyshev distance R only
        const int side = 2 * R + 1, nrows = side * side;
        for (int rb = 0; rb < nrows; rb += 64) {
            uint32_t a1 = 0, l1 = 0, a2 = 0, l2 = 0;
            const int r = rb + lane;
            if (r < nrows) {
                const int y = c[1] - R + r % side, z = c[2] - R + r / side;
                if (y >= 0 && y < G.g[1] && z >= 0 && z < G.g[2]) {
                    const uint32_t row = ((uint32_t)z * (uint32_t)G.g[1] + (uint32_t)y) * (uint32_t)G.g[0];
                    const bool face = R == 1 || y == c[1] - R || y == c[1] + R || z == c[2] - R || z == c[2] + R;
                    if (face) {
                        const int xa = max(c[0] - R, 0), xb = min(c[0] + R, G.g[0] - 1);
                        a1 = gld32(start, row + xa);
                        l1 = gld32(start, row + xb + 1) - a1;
                    } else {
                        if (c[0] - R >= 0) {
                            a1 = gld32(start, row + c[0] - R);
                            l1 = gld32(start, row + c[0] - R + 1) - a1;
                        }
                        if (c[0] + R <= G.g[0] - 1) {
                            a2 = gld32(start, row + c[0] + R);
                            l2 = gld32(start, row + c[0] + R + 1) - a2;
                        }
                    }
                }
            }
            // the segments' prefix over the wave
            uint32_t incl = l1 + l2;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t v = __shfl_up(incl, off);
                if (lane >= off) incl += v;
            }
            const uint32_t total = __shfl(incl, 63);
            const uint32_t excl = incl - (l1 + l2);
            evals += total;
            // point t of the ring: the lane whose [excl, incl) holds it
            for (uint32_t b0 = 0; b0 < total; b0 += 64 * kCoopU) {
                int32_t pos[kCoopU];
#pragma unroll
                for (int u = 0; u < kCoopU; ++u) {
                    const uint32_t t = b0 + (uint32_t)(u * 64 + lane);
                    // binary search over the lanes' exclusive prefixes (uniform steps)
                    int lo = 0;
#pragma unroll
                    for (int st = 32; st > 0; st >>= 1) {
                        const uint32_t e = __shfl(excl, lo + st);
                        if (lo + st < 64 && e <= t) lo += st;
                    }
                    const uint32_t e0 = __shfl(excl, lo), s1 = __shfl(a1, lo), n1 = __shfl(l1, lo),
                                   s2 = __shfl(a2, lo);
                    const uint32_t loc = t - e0;
                    pos[u] = t < total ? (int32_t)(loc < n1 ? s1 + loc : s2 + (loc - n1)) : kNoPos;
                }
                P4<T> p[kCoopU];
                int32_t g[kCoopU];
#pragma unroll
                for (int u = 0; u < kCoopU; ++u) {
                    const uint32_t pa = pos[u] == kNoPos ? 0u : (uint32_t)pos[u];  // (in-range dummy)
                    p[u] = gld32(gpts, pa);
                    g[u] = gld32(gidx, pa);
                }
#pragma unroll
                for (int u = 0; u < kCoopU; ++u)
                    if (pos[u] != kNoPos) coop_insert<T, KT>(ld, lg, lp, gsqd(qx, qy, qz, p[u]), g[u], pos[u]);
            }
        }
        coop_merge<T, KT>(ld, lg, lp, kd, kg, kp);
        // lower bound on the distance to any unvisited cell (lane_search's rule)
        double lb = 1e300;
        bool any = false;
#pragma unroll
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
        lb_exit = any ? lb : 1e300;
        if (!any) break;
        if (lb > 0.0) {
            const double lb2 = lb * lb * margin;
            T dk = kd[0];
            int32_t pk = kp[0];
#pragma unroll
            for (int s = 1; s < KT; ++s)
                if (s == ks - 1) {
                    dk = kd[s];
                    pk = kp[s];
                }
            if ((double)dk < lb2 && pk != kNoPos) break;
            if (lb2 > (double)maxR2) break;
        }
    }
    if (lane == 0) visits += evals;
}

// ------------------------------------------------------- per-lane kernel --
// Phase 1 (the reuse certificate) takes LaneQ slots per thread, its loads
// staged so that a thread keeps every slot's chain in flight; phase 2 (full
// searches) takes the block's misses 256 at a time.  One slot per thread:
// measured at C3 with 4 (blocks of 1024 slots) the converged match went
// 25-27 -> 23-26 us, but the first match after the cold one (every query a
// full search) 217 -> 349 us — a block's four rounds of full searches run
// back to back instead of being spread over the CUs as separate blocks.
template <int KT>
struct LaneQ {
    static constexpr int value = 1;
};

// XCD-aware block order of the per-lane kernel (pmx_internal.h xcd_block:
// adjacent slot ranges gather through one L2; match HBM traffic 75.3 -> 66.5
// MB per launch at C3)
// waves per SIMD the per-lane and tile kernels are built for (their VGPR
// budget: 512 / waves).  The double forms spill at 128 VGPRs (C5: 78 VGPRs to
// scratch inside the shell walk), so they are built for 2 (the compiler then
// takes 133-220 VGPRs, 2-3 waves, no spills): C5 1.79 -> 1.62 ms/iteration.
// The float KT = 8 form spills 26 at 128 but measured faster that way than
// unspilled at 3 waves (C4 0.202 vs 0.217 ms/iteration).
template <typename T, int KT>
struct LaneWaves {
    static constexpr int value = sizeof(T) == 8 ? 2 : 4;
};
template <typename T, int KT>
struct TileWaves {
    static constexpr int value = sizeof(T) == 8 ? 2 : 4;
};

template <typename T, int KT, int Q>
__global__ __launch_bounds__(256, (LaneWaves<T, KT>::value)) void grid_lane_kernel(const P4<T>* __restrict__ gpts,
                                                        const int32_t* __restrict__ gidx,
                                                        const uint32_t* __restrict__ start, GridGeom G,
                                                        const P4<T>* __restrict__ rd, int64_t N, Mat4<T> Tm, int k,
                                                        T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                                        unsigned long long* __restrict__ visited, int reuse,
                                                        T* __restrict__ safe, Mat4<T> Tprev,
                                                        const LoopCtl* __restrict__ ctl,
                                                        const GridDesc<T>* __restrict__ gd,
                                                        SpecSel* __restrict__ spec, const T* __restrict__ radii,
                                                        int coop_max, P4<T>* __restrict__ nbr,
                                                        const P4<T>* __restrict__ nbr_gpn) {
    if (ctl) {  // device loop: transform, level and reuse state from the device
        if (ctl->done) return;
        if (ctl->use_tile) return;  // (tile dispatch: the tile kernel's warm form runs this match)
        const GridDesc<T>& D = gd[ctl->level];
        gpts = D.gpts;
        gidx = D.gidx;
        start = D.start;
        G = D.G;
        if (nbr_gpn) nbr_gpn = D.gpn;
        ctl_transform(ctl, Tm);
        if (reuse) {
            reuse = ctl->prev_level == ctl->level ? 2 : 1;
#pragma unroll
            for (int i = 0; i < 16; ++i) Tprev.m[i] = (T)ctl->Tprev[i];
        }
    }
    if (!reuse) safe = nullptr;
    if (!safe || k != 1 || KT < 2) nbr = nullptr;  // (the record serves the k = 1 certificate)
    uint32_t visits = 0;
    // quantile window (pmx_spec.h): every written distance is classified
    SpecAcc<T> sa;
    spec_acc_init<T>(sa, spec);
    constexpr int B = 256 * Q;  // slots of the block
    __shared__ int miss[B];
    __shared__ int wave_cnt[Q][4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)xcd_block() * B;
    bool missed[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) missed[q] = base + q * 256 + threadIdx.x < N;
    if (reuse == 2) {
        // the certificate (see the temporal reuse notes above) for the
        // thread's Q slots, in stages so that each stage's loads are in flight
        // together.  A list kept for reuse holds k <= KT - 1 entries (room for
        // the (k+1)-th: the safe radius); KT = 16 keeps no room and never
        // certifies.  The bound a uses the previous k-th distance, so a query
        // that cannot pass costs no gather.
        constexpr int KR = KT > 1 ? KT - 1 : 1;
        P4<T> p[Q];
        T rs[Q], dkp[Q];
        int32_t id[Q][KR];
        P4<T> r[Q][KR];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int64_t j = missed[q] ? base + q * 256 + threadIdx.x : base;  // (base < N: an in-range slot)
            p[q] = gld(rd, j);
            rs[q] = safe[j];
            dkp[q] = out_d[j * k + k - 1];
            if (nbr) {  // (k = 1: the neighbour's record with the query, no dependent gather)
                r[q][0] = nbr[j];
                id[q][0] = (int32_t)w_pos(r[q][0].w);
            } else {
#pragma unroll
                for (int s = 0; s < KR; ++s) id[q][s] = s < k ? out_i[j * k + s] : 0;
            }
        }
        bool ok[Q];
        double bq[Q];
        T qx[Q], qy[Q], qz[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            gxform(Tm, p[q], qx[q], qy[q], qz[q]);
            bool o = missed[q] && k <= KR && rs[q] > (T)0 && dkp[q] < (T)__builtin_huge_val();
#pragma unroll
            for (int s = 0; s < KR; ++s) o = o && id[q][s] >= 0;
            T ox, oy, oz;
            gxform(Tprev, p[q], ox, oy, oz);
            const double ex = (double)qx[q] - (double)ox, ey = (double)qy[q] - (double)oy,
                         ez = (double)qz[q] - (double)oz;
            const double delta = sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + kReuseMargin);
            const double av = sqrt((double)dkp[q]) * (1.0 + kReuseMargin) + delta;
            bq[q] = (double)rs[q] * (1.0 - kReuseMargin) - delta;
            ok[q] = o && av < bq[q];
        }
        if (!nbr) {
#pragma unroll
            for (int q = 0; q < Q; ++q)
#pragma unroll
                for (int s = 0; s < KR; ++s) r[q][s] = gld32(gpts, ok[q] && s < k ? (uint32_t)id[q][s] : 0u);
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            if (!ok[q]) continue;
            // the same points: new distances, sorted as a full search sorts them
            const int64_t j = base + q * 256 + threadIdx.x;
            T kd[KT];
            int32_t ki[KT];
#pragma unroll
            for (int s = 0; s < KT; ++s) {
                kd[s] = (T)__builtin_huge_val();
                ki[s] = kNoPos;
            }
#pragma unroll
            for (int s = 0; s < KR; ++s)
                if (s < k) ginsert<T, KT>(gidx, kd, ki, gsqd(qx[q], qy[q], qz[q], r[q][s]), id[q][s]);
            visits += (uint32_t)k;
            write_out<T, KT>(j, k, qr2(radii, j, maxR2), kd, ki, out_d, out_i, sa);
            st_out(&safe[j], (T)(bq[q] * (1.0 - 1e-6)));
            missed[q] = false;
        }
    }
    // the block's misses, compacted in slot order
    unsigned long long mq[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        mq[q] = __ballot(missed[q]);
        if (lane == 0) wave_cnt[q][wave] = __popcll(mq[q]);
    }
    __syncthreads();
    int total = 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        int off = total;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int cw = wave_cnt[q][w];
            off += w < wave ? cw : 0;
            total += cw;
        }
        if (missed[q]) miss[off + __popcll(mq[q] & ((1ull << lane) - 1))] = q * 256 + threadIdx.x;
    }
    __syncthreads();
    if (total <= coop_max) {
        // few misses (a converged match): each is searched by a whole wave
        // (wave w takes misses w, w + 4, ...), two round trips per ring
        // instead of a lane's chain of dependent row gathers
        for (int t = wave; t < total; t += 4) {  // (wave-uniform)
            const int64_t j2 = base + miss[t];
            T qx, qy, qz;
            gxform(Tm, gld(rd, j2), qx, qy, qz);
            const T r2 = qr2(radii, j2, maxR2);
            T kd[KT];
            int32_t kp[KT];
            double lbx;
            coop_search<T, KT>(gpts, gidx, start, G, qx, qy, qz, k, r2, kd, kp, lbx, visits);
            if (lane == 0) {
                write_out<T, KT>(j2, k, r2, kd, kp, out_d, out_i, sa);
                write_nbr<T, KT>(nbr, gpts, nbr_gpn, N, j2, r2, kd, kp);
                if (safe) st_out(&safe[j2], safe_radius<T, KT>(kd, kp, k, lbx));
            }
        }
    } else {
        for (int t = threadIdx.x; t < (Q == 1 ? min(total, 256) : total); t += 256) {  // (Q = 1: at most once)
            const int64_t j2 = base + miss[t];
            full_query<T, KT>(gpts, gidx, start, G, rd, j2, Tm, k, qr2(radii, j2, maxR2), out_d, out_i, safe, visits,
                              sa, nbr, nbr_gpn, N);
            if (Q == 1) break;
        }
    }
    add_visits(visits, visited);
    // queries that took the full search (the "fallback" counter the level choice reads)
    if (threadIdx.x == 0 && visited && total && reuse) atomicAdd(vslot(visited, 1), (unsigned long long)total);
    if (sa.on) spec_acc_flush<T>(sa, vslot(visited, 2), vslot(visited, 3));
}

// ------------------------------------------------------------ tile kernel --
#include "pmx_grid_tile.inc"

template <typename T, int KT>
static void launch_kt(int mode, const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const GridGeom& G,
                      const P4<T>* rd, int64_t N, const uint32_t* waves, int64_t n_waves, const Mat4<T>& Tm, int knn,
                      T maxR2, uint32_t max_pts, T* dists, int32_t* ids, unsigned long long* visited,
                      const GridReuse<T>& ru, const LoopCtl* ctl, const GridDesc<T>* gd, SpecSel* spec,
                      const T* radii, bool cold, bool tile_disp, hipEvent_t e0, hipEvent_t e1, hipStream_t s) {
    // (timing: e0 / e1 are recorded by the dispatch itself — the first
    // launch's start, the last launch's end — hipExtLaunchKernelGGL, the
    // kernel's own execution as a rocprofv3 kernel trace counts it; null
    // events record nothing)
    if (cold) {  // a new reading's first match: the tile kernel's cold form (pmx_grid_tile.inc)
        hipExtLaunchKernelGGL((grid_tile_kernel<T, KT>), dim3((unsigned)((N + 63) / 64)), dim3(64), 0, s, e0, e1, 0,
                              gpts, gidx, start, G, rd, N, (const uint32_t*)nullptr, Tm, knn, maxR2, max_pts, dists,
                              ids, visited, radii, 1, ctl, gd, spec, ru.safe, ru.nbr, ru.gpn);
    } else if (mode >= 1) {  // the per-lane shell search
        const bool both = tile_disp && ctl && ru.mode;
        if (both)  // (device loop: the step picks one of the two forms)
            hipExtLaunchKernelGGL((grid_tile_kernel<T, KT>), dim3((unsigned)((N + 63) / 64)), dim3(64), 0, s, e0,
                                  (hipEvent_t) nullptr, 0, gpts, gidx, start, G, rd, N, (const uint32_t*)nullptr, Tm,
                                  knn, maxR2, max_pts, dists, ids, visited, radii, 2, ctl, gd, spec, ru.safe,
                                  ru.nbr, ru.gpn);
        constexpr int Q = LaneQ<KT>::value;
        const int64_t grid = (N + 256 * Q - 1) / (256 * Q);
        hipExtLaunchKernelGGL((grid_lane_kernel<T, KT, Q>), dim3((unsigned)grid), dim3(256), 0, s,
                              both ? (hipEvent_t) nullptr : e0, e1, 0, gpts, gidx, start, G, rd, N, Tm, knn, maxR2,
                              dists, ids, visited, ru.mode, ru.safe, ru.Tprev, ctl, gd, spec, radii, ru.coop_max,
                              ru.nbr, ru.gpn);
    } else {
        const int64_t W = waves ? n_waves : (N + 63) / 64;
        hipExtLaunchKernelGGL((grid_tile_kernel<T, KT>), dim3((unsigned)W), dim3(64), 0, s, e0, e1, 0, gpts, gidx,
                              start, G, rd, N, waves, Tm, knn, maxR2, max_pts, dists, ids, visited, radii, 0,
                              (const LoopCtl*)nullptr, (const GridDesc<T>*)nullptr, (SpecSel*)nullptr, (T*)nullptr,
                              (P4<T>*)nullptr, (const P4<T>*)nullptr);
    }
}

// option tile_prof: the cold form's per-wave profile into buf (4 words per wave)
void set_tile_prof(unsigned long long* buf) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tile_prof), &buf, sizeof(buf)); }

template <typename T>
void launch_grid_match(int mode, const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const double* lo,
                       double h, const int* g, const P4<T>* rd, int64_t N, const uint32_t* waves, int64_t n_waves,
                       const Mat4<T>& Tm, int knn, T maxR2, uint32_t max_pts, T* dists, int32_t* ids,
                       unsigned long long* visited, unsigned long long* vout, int* iter_err,
                       const GridReuse<T>& ru, const LoopCtl* ctl, const GridDesc<T>* gd, SpecSel* spec,
                       SelectState* spec_st, unsigned long long* xseg, const T* radii, bool cold, bool tile_disp,
                       hipEvent_t ev_start, hipEvent_t ev_end, hipStream_t s) {
    if (N <= 0) return;
    cold = cold && mode >= 1;
    if (mode < 1 || !visited) spec = nullptr;  // (the window needs the per-lane kernel and the counters)
    GridGeom G;
    for (int a = 0; a < 3; ++a) {
        G.lo[a] = lo[a];
        G.g[a] = g[a];
    }
    G.h = h;
    G.inv_h = 1.0 / h;
    if (knn > kLaneMaxK) {  // a k-list spread over a wave per query (pmx_knn_wide.hip; no reuse)
        if (ev_start) (void)hipEventRecord(ev_start, s);
        launch_knn_wide<T>(gpts, gidx, start, &G, 0, rd, N, Tm, knn, maxR2, radii, dists, ids, visited, ctl, gd, spec,
                           s);
        if (ev_end) (void)hipEventRecord(ev_end, s);
    } else {
#define PMX_KT(KT) \
    launch_kt<T, KT>(mode, gpts, gidx, start, G, rd, N, waves, n_waves, Tm, knn, maxR2, max_pts, dists, ids, visited, \
                     ru, ctl, gd, spec, radii, cold, tile_disp, ev_start, ev_end, s)
        // with reuse the list keeps room for the (k+1)-th point (the safe radius;
        // the cold tile writes radius 0 and keeps k entries)
        const int kl = ru.mode && mode >= 1 && knn < 16 && !cold ? knn + 1 : knn;
        if (kl == 1)
            PMX_KT(1);
        else if (kl <= 2)
            PMX_KT(2);
        else if (kl <= 4)
            PMX_KT(4);
        else if (kl <= 5)
            PMX_KT(5);  // (k = 4 with the (k+1)-th entry: 5 fit the 128-VGPR budget, 8 spilled)
        else if (kl <= 8)
            PMX_KT(8);
        else
            PMX_KT(16);
#undef PMX_KT
    }
    if (visited && vout)
        hipLaunchKernelGGL(counter_sum_kernel<T>, dim3(1), dim3(kVSlots), 0, s, visited, vout, iter_err, ctl, spec,
                           spec_st, xseg);
}

template void launch_grid_match<float>(int, const P4<float>*, const int32_t*, const uint32_t*, const double*, double,
                                       const int*, const P4<float>*, int64_t, const uint32_t*, int64_t,
                                       const Mat4<float>&, int, float, uint32_t, float*, int32_t*,
                                       unsigned long long*, unsigned long long*, int*, const GridReuse<float>&,
                                       const LoopCtl*, const GridDesc<float>*, SpecSel*, SelectState*,
                                       unsigned long long*, const float*, bool, bool, hipEvent_t, hipEvent_t,
                                       hipStream_t);
template void launch_grid_match<double>(int, const P4<double>*, const int32_t*, const uint32_t*, const double*, double,
                                        const int*, const P4<double>*, int64_t, const uint32_t*, int64_t,
                                        const Mat4<double>&, int, double, uint32_t, double*, int32_t*,
                                        unsigned long long*, unsigned long long*, int*, const GridReuse<double>&,
                                        const LoopCtl*, const GridDesc<double>*, SpecSel*, SelectState*,
                                        unsigned long long*, const double*, bool, bool, hipEvent_t, hipEvent_t,
                                        hipStream_t);

// map match ids (grid positions, -1 = none) back to reference indices
__global__ void pos_to_index_kernel(const int32_t* __restrict__ pos, const int32_t* __restrict__ gidx,
                                    int32_t* __restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int32_t p = pos[i];
        out[i] = p < 0 ? -1 : gidx[p];
    }
}
void launch_pos_to_index(const int32_t* pos, const int32_t* gidx, int32_t* out, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(pos_to_index_kernel, dim3((unsigned)g), dim3(256), 0, s, pos, gidx, out, n);
}


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_grid() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&grid_lane_kernel<float, 1, 1>));
}

}  // namespace pmx
