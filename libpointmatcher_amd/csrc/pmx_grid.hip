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
// Tile kernel (PMX_GRID_MODE=tile, pmx_grid_tile.inc).  One wave = up to 64
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
#include "pmx_p2plane.h"
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
#ifndef PMX_SCAN_U
#define PMX_SCAN_U 4
#endif
constexpr int kScanU = PMX_SCAN_U;
// phase-1 row grouping of the per-lane search (rows per group, points per row)
#ifndef PMX_P1_G
#define PMX_P1_G 3
#endif
#ifndef PMX_P1_U
#define PMX_P1_U 4
#endif
constexpr int kP1G = PMX_P1_G;
constexpr int kP1U = PMX_P1_U;
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

// Octant search: the 2x2x2 cells nearest to the query (its cell and, per
// axis, the neighbour on the query's side of the cell centre: 4 rows of 2
// cells).  Every point outside the block is at least LB = the distance to
// the block's interior faces (>= h/2) away, so the result is final when it
// passes the same certification as the shell search; true then.
template <typename T, int KT>
__device__ __forceinline__ bool octant_search(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                              const uint32_t* __restrict__ start, const GridGeom& G, T qx, T qy,
                                              T qz, const double q[3], const int c[3], T maxR2, int k, T (&kd)[KT],
                                              int32_t (&ki)[KT], uint32_t& visits) {
    int b0[3], b1[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double mid = G.lo[a] + ((double)c[a] + 0.5) * G.h;
        const int o = q[a] >= mid ? c[a] + 1 : c[a] - 1;
        b0[a] = o < c[a] ? max(o, 0) : c[a];
        b1[a] = o > c[a] ? min(o, G.g[a] - 1) : c[a];
    }
    uint32_t ra[4], rb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int y = (r & 1) ? b1[1] : b0[1], z = (r & 2) ? b1[2] : b0[2];
        const bool ok = !((r & 1) && b1[1] == b0[1]) && !((r & 2) && b1[2] == b0[2]);  // no duplicate rows
        const uint32_t row = ((uint32_t)z * (uint32_t)G.g[1] + (uint32_t)y) * (uint32_t)G.g[0];
        const uint32_t va = gld32(start, row + b0[0]);
        const uint32_t vb = gld32(start, row + b1[0] + 1);
        ra[r] = ok ? va : 0u;
        rb[r] = ok ? vb : 0u;
    }
    constexpr int U = kP1U;
    P4<T> p[4][U];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = ra[r] + u;
            p[r][u] = gld32(gpts, j < rb[r] ? j : 0u);  // masked: any in-range address
        }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = ra[r] + u;
            if (j < rb[r]) consider<T, KT>(gidx, (int32_t)j, gsqd(qx, qy, qz, p[r][u]), kd, ki);
        }
        visits += rb[r] - ra[r];
        if (ra[r] + U < rb[r]) {
            uint32_t v0 = 0;
            scan_range<T, KT>(gpts, gidx, ra[r] + U, rb[r], qx, qy, qz, kd, ki, v0);
        }
    }
    double lb = 1e300;
    bool any = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        if (b0[a] > 0) {
            lb = fmin(lb, q[a] - (G.lo[a] + (double)b0[a] * G.h));
            any = true;
        }
        if (b1[a] < G.g[a] - 1) {
            lb = fmin(lb, (G.lo[a] + (double)(b1[a] + 1) * G.h) - q[a]);
            any = true;
        }
    }
    if (!any) return true;  // the block is the whole grid
    if (lb > 0.0) {
        const double lb2 = lb * lb * (1.0 - 1e-5);
        T dk;
        int32_t ik;
        kth(kd, ki, k, dk, ik);
        if (((double)dk < lb2 && ik != kNoPos) || lb2 > (double)maxR2) return true;
    }
    return false;
}

// Shell walk with batched row scans (R >= 2).  The rows (and single cells)
// of a shell that pass the gap test are queued kShellB at a time; a full
// queue loads all its cell bounds together, then the first kShellU points of
// every queued range together, so a batch costs two dependent round trips
// instead of two per row.  The gap test reads the list as it stands when the
// row is queued; the list only shrinks the limit afterwards, so a queued row
// may be one the row-at-a-time walk would have skipped — never the reverse:
// the set of points that can enter the list, and the result, are the same.
// Off by default (kShellB = 0): measured at C3 the cold match went 0.83 ->
// 1.7 ms (B = 4) and 1.9 ms (B = 6) — lanes fill their queues at different
// rows, so the wave runs the flush once per lane group, and the stale limit
// queues rows the row-at-a-time walk skips.
#ifndef PMX_SHELL_B
#define PMX_SHELL_B 0
#endif
#ifndef PMX_SHELL_U
#define PMX_SHELL_U 0
#endif
constexpr int kShellB = PMX_SHELL_B;
constexpr int kShellU = PMX_SHELL_U;

template <typename T, int KT>
__device__ __forceinline__ void shell_flush(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                            const uint32_t* __restrict__ start, const uint32_t (&ia)[kShellB > 0 ? kShellB : 1],
                                            const uint32_t (&ib)[kShellB > 0 ? kShellB : 1], int np, T qx, T qy, T qz,
                                            T (&kd)[KT], int32_t (&ki)[KT], uint32_t& visits) {
    constexpr int B = kShellB > 0 ? kShellB : 1, U = kShellU;
    uint32_t ra[B], rb[B];
#pragma unroll
    for (int s = 0; s < B; ++s) {
        const bool ok = s < np;
        const uint32_t va = gld32(start, ok ? ia[s] : 0u);
        const uint32_t vb = gld32(start, ok ? ib[s] : 0u);
        ra[s] = ok ? va : 0u;
        rb[s] = ok ? vb : 0u;
    }
    // (U = 0: only the bounds are batched; most shell cells of a surface
    // cloud are empty, and an empty range costs nothing past its bounds)
    P4<T> p[B][U > 0 ? U : 1];
#pragma unroll
    for (int s = 0; s < B; ++s)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = ra[s] + u;
            p[s][u] = gld32(gpts, j < rb[s] ? j : 0u);  // masked: any in-range address
        }
#pragma unroll
    for (int s = 0; s < B; ++s) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = ra[s] + u;
            if (j < rb[s]) consider<T, KT>(gidx, (int32_t)j, gsqd(qx, qy, qz, p[s][u]), kd, ki);
        }
        visits += rb[s] - ra[s];
        if (ra[s] + U < rb[s]) {
            uint32_t v0 = 0;
            scan_range<T, KT>(gpts, gidx, ra[s] + U, rb[s], qx, qy, qz, kd, ki, v0);
        }
    }
}

template <typename T, int KT>
__device__ __forceinline__ void shell_walk_batched(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                                   const uint32_t* __restrict__ start, const GridGeom& G, T qx, T qy,
                                                   T qz, const double q[3], const int c[3], int R, int k,
                                                   T (&kd)[KT], int32_t (&ki)[KT], uint32_t& visits) {
    constexpr int B = kShellB > 0 ? kShellB : 1;
    const double margin = 1.0 - 1e-5;
    const int y0 = max(c[1] - R, 0), y1 = min(c[1] + R, G.g[1] - 1);
    const int z0 = max(c[2] - R, 0), z1 = min(c[2] + R, G.g[2] - 1);
    const int x0 = max(c[0] - R, 0), x1 = min(c[0] + R, G.g[0] - 1);
    uint32_t ia[B], ib[B];
    int np = 0;
    auto push = [&](uint32_t a, uint32_t b) {
#pragma unroll
        for (int s = 0; s < B; ++s)
            if (s == np) {  // (static indexing keeps the queue in registers)
                ia[s] = a;
                ib[s] = b;
            }
        if (++np == B) {
            shell_flush<T, KT>(gpts, gidx, start, ia, ib, np, qx, qy, qz, kd, ki, visits);
            np = 0;
        }
    };
    for (int z = z0; z <= z1; ++z) {
        const double gz = axis_gap(G, 2, z, q[2]), gz2 = gz * gz;
        const bool zface = (z == c[2] - R) || (z == c[2] + R);
        for (int y = y0; y <= y1; ++y) {
            // the limit of the list as it stands (entry k + 1 when the list
            // has room for it: the safe radius bound, see lane_search)
            T dkT;
            int32_t ikT;
            kth(kd, ki, k < KT ? k + 1 : k, dkT, ikT);
            const double lim = ikT == kNoPos ? 1e300 : (double)dkT / margin;
            if (gz2 > lim) break;  // (the whole z slab: gz does not depend on y)
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
                if (xa <= xb) push(row + (uint32_t)xa, row + (uint32_t)xb + 1u);
            } else {
                const int xl = c[0] - R, xr = c[0] + R;
                if (xl >= 0) {
                    const double gx = axis_gap(G, 0, xl, q[0]);
                    if (g2 + gx * gx <= lim) push(row + (uint32_t)xl, row + (uint32_t)xl + 1u);
                }
                if (xr <= G.g[0] - 1) {
                    const double gx = axis_gap(G, 0, xr, q[0]);
                    if (g2 + gx * gx <= lim) push(row + (uint32_t)xr, row + (uint32_t)xr + 1u);
                }
            }
        }
    }
    if (np > 0) shell_flush<T, KT>(gpts, gidx, start, ia, ib, np, qx, qy, qz, kd, ki, visits);
}

// Exact shell search for one query (from scratch); kd/ki must be
// initialised.  Certified on the k-th entry of the list (entries past k, when
// KT > k, are the next-nearest points visited).  lb_exit: the distance from
// the query to the unvisited region at exit (1e300: the whole grid).
template <typename T, int KT>
__device__ __forceinline__ void lane_search(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                            const uint32_t* __restrict__ start, const GridGeom& G, T qx, T qy, T qz,
                            const double q[3], const int c[3], T maxR2, int k, T (&kd)[KT], int32_t (&ki)[KT],
                            uint32_t& visits, double& lb_exit) {
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
        if (R >= 2 && kShellB > 0) {
            shell_walk_batched<T, KT>(gpts, gidx, start, G, qx, qy, qz, q, c, R, k, kd, ki, visits);
        } else if (R >= 2) {
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
                kth(kd, ki, k < KT ? k + 1 : k, dkT, ikT);
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
            out_d[j * k + s] = d;
            out_i[j * k + s] = id;
            if (sa.on) spec_acc<T>(sa, d);
        }
    }
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

// The counter phase folded into the match kernel (PMX_FOLD_COUNTER=1): the
// last workgroup to finish runs it, one launch fewer per iteration.  Off by
// default: measured at C3 (driver command) the match grew 22.4 -> 31.6 us
// against 22.4 + 5.9 us for the two launches — every workgroup must drain its
// stores before it takes its ticket, and that drain costs more than the
// boundary it saves.  Every
// value it reads was published by atomics or write-through (sc1) stores and
// is read with coherent loads, so each workgroup only drains its memory
// operations before it takes its ticket (cdna_hip_programming.md §6 G16,
// the sc1 form of the in-launch reduction).
// Tickets: one counter per group of workgroups (blockIdx % kTicketGroups, each
// on its own 128-byte line), then one for the groups — a single counter
// taken by all 4K workgroups serialises (measured: +27 us at C3).
constexpr size_t kTicketOff = (size_t)4 * kVSlots * kVStride;  // (unsigned long longs into vpart)
constexpr int kTicketGroups = 64;
template <typename T>
__device__ __forceinline__ void counter_fold(unsigned long long* __restrict__ vpart,
                                             unsigned long long* __restrict__ out, int* __restrict__ iter_err,
                                             SpecSel* __restrict__ spec, SelectState* __restrict__ st,
                                             unsigned long long* __restrict__ xseg) {
    __shared__ unsigned s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned* tk = (unsigned*)(vpart + kTicketOff);  // [group g at g * 32] ..., top at kTicketGroups * 32
    if (threadIdx.x == 0) {
        const unsigned G = gridDim.x, b = blockIdx.x;
        const unsigned g = b % kTicketGroups;
        const unsigned ng = G < (unsigned)kTicketGroups ? G : (unsigned)kTicketGroups;
        const unsigned gsize = (G - g + kTicketGroups - 1) / kTicketGroups;  // blocks with this residue
        unsigned last = 0;
        const unsigned o = __hip_atomic_fetch_add(tk + g * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o == gsize - 1) {
            const unsigned t = __hip_atomic_fetch_add(tk + kTicketGroups * 32, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            last = t == ng - 1 ? 1u : 0u;
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    counter_phase<T>(vpart, out, iter_err, spec, st, xseg);
    for (int g = threadIdx.x; g <= kTicketGroups; g += blockDim.x)  // (every group's and the top counter)
        __hip_atomic_store(tk + g * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a deferred counter phase that no select_all consumed
template <typename T>
void launch_counter_sum(unsigned long long* vpart, unsigned long long* vout, int* iter_err, const LoopCtl* ctl,
                        SpecSel* spec, SelectState* st, hipStream_t s) {
    hipLaunchKernelGGL(counter_sum_kernel<T>, dim3(1), dim3(kVSlots), 0, s, vpart, vout, iter_err, ctl, spec, st,
                       nullptr);
}
template void launch_counter_sum<float>(unsigned long long*, unsigned long long*, int*, const LoopCtl*, SpecSel*,
                                        SelectState*, hipStream_t);
template void launch_counter_sum<double>(unsigned long long*, unsigned long long*, int*, const LoopCtl*, SpecSel*,
                                         SelectState*, hipStream_t);

// Several ranks: resolve the quantile from the all-gathered window segments
// (pmx_spec.h).  Every rank runs it on the same segments and writes the same
// limit; a miss leaves the radix passes (with their histogram all-reduce) to
// resolve it.
template <typename T>
__global__ __launch_bounds__(kVSlots) void spec_pick_kernel(const unsigned long long* __restrict__ segs, int nseg,
                                                            SpecSel* __restrict__ spec,
                                                            SelectState* __restrict__ st,
                                                            const LoopCtl* __restrict__ ctl) {
    __shared__ uint32_t lh[2048];
    __shared__ unsigned long long part[kVSlots];
    __shared__ unsigned long long bc[2];
    if (ctl && ctl->done) return;
    unsigned long long fin = 0, below = 0, nk = 0;
    bool overflow = false;
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
    spec_pick<T, kVSlots>(spec, st, fin, below, nk, overflow, src, lh, part, bc);
}

template <typename T>
void launch_spec_pick(const unsigned long long* segs, int nseg, SpecSel* spec, SelectState* st, const LoopCtl* ctl,
                      hipStream_t s) {
    hipLaunchKernelGGL(spec_pick_kernel<T>, dim3(1), dim3(kVSlots), 0, s, segs, nseg, spec, st, ctl);
}
template void launch_spec_pick<float>(const unsigned long long*, int, SpecSel*, SelectState*, const LoopCtl*,
                                      hipStream_t);
template void launch_spec_pick<double>(const unsigned long long*, int, SpecSel*, SelectState*, const LoopCtl*,
                                       hipStream_t);

// counters: 0 pairs, 1 full-search fallbacks, 2 finite distances, 3 below the quantile window
// (+ the fold tickets: kTicketGroups + 1 counters, 128 bytes apart)
size_t grid_counter_bytes() { return sizeof(unsigned long long) * (4 * kVSlots * kVStride + 16 * (kTicketGroups + 1)); }

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

// one query from scratch: octant block (oct) or the shell search
template <typename T, int KT>
__device__ __forceinline__ void full_query(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                           const uint32_t* __restrict__ start, const GridGeom& G,
                                           const P4<T>* __restrict__ rd, int64_t j, const Mat4<T>& Tm, int k,
                                           T maxR2, int oct, T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                           T* __restrict__ safe, uint32_t& visits, SpecAcc<T>& sa) {
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
    if (!qnan) {
        bool done = false;
        if (oct) done = octant_search<T, KT>(gpts, gidx, start, G, qx, qy, qz, q, c, maxR2, k, kd, ki, visits);
        if (!done) {
#pragma unroll
            for (int s = 0; s < KT; ++s) {  // (a k-list must not see the octant's points twice)
                kd[s] = (T)__builtin_huge_val();
                ki[s] = kNoPos;
            }
            lane_search<T, KT>(gpts, gidx, start, G, qx, qy, qz, q, c, maxR2, k, kd, ki, visits, lb_exit);
        }
    }
    write_out<T, KT>(j, k, maxR2, kd, ki, out_d, out_i, sa);
    if (safe) safe[j] = oct ? (T)0 : safe_radius<T, KT>(kd, ki, k, lb_exit);
}

// the certificate for query j; true when the k-list was rewritten from the
// previous one
template <typename T, int KT>
__device__ __forceinline__ bool reuse_query(const P4<T>* __restrict__ gpts, const int32_t* __restrict__ gidx,
                                            const P4<T>& p, T qx, T qy, T qz, const Mat4<T>& Tprev, int64_t j,
                                            int k, T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                            T* __restrict__ safe, uint32_t& visits, SpecAcc<T>& sa) {
    const T rs = safe[j];
    const T dkp = out_d[j * k + k - 1];
    int32_t id[KT];
    bool ok = rs > (T)0 && dkp < (T)__builtin_huge_val();
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        id[s] = s < k ? out_i[j * k + s] : 0;
        ok = ok && id[s] >= 0;
    }
    if (!ok) return false;
    T ox, oy, oz;
    gxform(Tprev, p, ox, oy, oz);
    const double ex = (double)qx - (double)ox, ey = (double)qy - (double)oy, ez = (double)qz - (double)oz;
    const double delta = sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + kReuseMargin);
    const double a = sqrt((double)dkp) * (1.0 + kReuseMargin) + delta;
    const double b = (double)rs * (1.0 - kReuseMargin) - delta;
    if (!(a < b)) return false;
    // the same k points: new distances, sorted as a full search sorts them
    T kd[KT];
    int32_t ki[KT];
#pragma unroll
    for (int s = 0; s < KT; ++s) {
        kd[s] = (T)__builtin_huge_val();
        ki[s] = kNoPos;
    }
#pragma unroll
    for (int s = 0; s < KT; ++s)
        if (s < k) ginsert<T, KT>(gidx, kd, ki, gsqd(qx, qy, qz, gld32(gpts, (uint32_t)id[s])), id[s]);
    visits += (uint32_t)k;
    write_out<T, KT>(j, k, maxR2, kd, ki, out_d, out_i, sa);
    safe[j] = (T)(b * (1.0 - 1e-6));
    return true;
}

// ------------------------------------------------- LDS box full searches --
#include "pmx_grid_box.inc"

// ------------------------------------------------- fused point-to-plane --
// The point-to-plane sums of one slot's pairs, after the match has written
// them (pmx_post.hip has the rest of the scheme): the pairs the block can
// decide are added to the lane's fp64 accumulators (the same T products as
// p2plane_body, PointToPlane.cpp:194-243), the quantile window's are
// recorded for the pick.  With TrimmedDist at chain position 0 a pair whose
// key is below the window is kept once the window resolves the limit (every
// kept pair: d <= limit with limit inside the window) and a pair above it is
// not; without a quantile every pair is decided here.  Counters: kept,
// non-zero weights (no quantile: inf distances may pass the predicates),
// finite distances, points with a kept pair.
// (all lanes of the wave call it; act = the lane holds a slot).  The lane's
// pairs go into its accumulators (this pass only: no array stays live across
// the searches), then one transposed wave sum adds them to the wave's LDS row.
template <typename T, int DIM>
__device__ __forceinline__ void fuse_chunk(const FuseAcc<T>& fa, SpecAcc<T>& sa, unsigned long long* __restrict__ recs,
                                           const P4<T>* __restrict__ gpn, const P4<T>* __restrict__ rd,
                                           const Mat4<T>& Tm, const T* __restrict__ out_d,
                                           const int32_t* __restrict__ out_i, int64_t j, bool act, int k,
                                           double* __restrict__ wrow) {
    using KO = KeyOf<T>;
    constexpr int NSF = DIM == 3 ? 27 : 9;
    double acc[kFuseNV];
#pragma unroll
    for (int v = 0; v < kFuseNV; ++v) acc[v] = 0.0;
    if (act) {
        const T inf = (T)__builtin_huge_val();
        T px, py, pz;
        gxform(Tm, gld(rd, j), px, py, pz);
        bool point_kept = false, appended = false;
        for (int s = 0; s < k; ++s) {
            const T d = out_d[j * k + s];
            const int32_t id = out_i[j * k + s];
            const bool finite = d != inf;
            const bool fx = (!fa.fx_finite || finite) && d >= fa.fx_lo && d <= fa.fx_hi;
            if (finite) acc[NSF + 2] += 1.0;
            bool keep;
            if (fa.quantile) {
                keep = false;
                if (finite) {
                    const bool below = KO::key(d) < (typename KO::K)sa.lo;
                    const unsigned pos = spec_acc<T>(sa, d);
                    if (pos < kSpecCap) {  // inside the window: decided by the pick
                        const bool head = fx && !point_kept && !appended;
                        recs[pos] = (unsigned long long)j << 32 | (fx ? kRecFx : 0ull) | (head ? kRecHead : 0ull) |
                                    ((unsigned long long)id & kRecPos);
                        appended = appended || fx;
                    } else {
                        keep = below && fx;
                    }
                }
            } else {
                if (fx) acc[NSF + 1] += 1.0;  // (w != 0).count(): may include an infinite distance
                keep = fx && finite;
            }
            if (keep) {
                acc[NSF] += 1.0;
                point_kept = true;
                p2plane_add<T, DIM, kFuseNV>(acc, px, py, pz, gld(gpn, 2 * (int64_t)id),
                                             gld(gpn, 2 * (int64_t)id + 1));
            }
        }
        if (point_kept) acc[NSF + 3] += 1.0;
    }
    int idx;
    const double w = wave_transpose_sum<kFuseNV>(acc, idx);
    if (transpose_writer<kFuseNV>()) wrow[idx] += w;
}

// ------------------------------------------------------- per-lane kernel --
// occupancy hint of the per-lane kernel (waves per SIMD; 0 = the compiler's
// choice).  The search is bound by dependent gather latency, so more resident
// waves hide more of it, as long as the register cap does not spill.
// XCD-aware block order of the per-lane kernel (PMX_LANE_XCD, default on)
#ifndef PMX_LANE_XCD
#define PMX_LANE_XCD 1
#endif
#ifndef PMX_LANE_WPE
#define PMX_LANE_WPE 0
#endif
#if PMX_LANE_WPE > 0
#define PMX_LANE_ATTR __attribute__((amdgpu_waves_per_eu(PMX_LANE_WPE)))
#else
#define PMX_LANE_ATTR
#endif
// BOX: the instance with the LDS box path (launched with dynamic LDS while
// many queries need a full search); the plain instance keeps the reuse
// path's registers and occupancy
// FUSE: the fused point-to-plane instance (pmx_post.hip): every block
// writes one record of sums
template <typename T, int KT, bool BOX, bool FUSE>
__global__ __launch_bounds__(256, 4) PMX_LANE_ATTR void grid_lane_kernel(const P4<T>* __restrict__ gpts,
                                                        const int32_t* __restrict__ gidx,
                                                        const uint32_t* __restrict__ start, GridGeom G,
                                                        const P4<T>* __restrict__ rd, int64_t N, Mat4<T> Tm, int k,
                                                        T maxR2, T* __restrict__ out_d, int32_t* __restrict__ out_i,
                                                        unsigned long long* __restrict__ visited, int oct,
                                                        int reuse, T* __restrict__ safe, Mat4<T> Tprev,
                                                        const LoopCtl* __restrict__ ctl,
                                                        const GridDesc<T>* __restrict__ gd,
                                                        SpecSel* __restrict__ spec, unsigned long long* __restrict__ vout,
                                                        int* __restrict__ iter_err, SelectState* __restrict__ spec_st,
                                                        unsigned long long* __restrict__ xseg,
                                                        const T* __restrict__ radii, uint32_t box_bytes,
                                                        int box_grow, FuseAcc<T> fa) {
    extern __shared__ __attribute__((aligned(16))) char box_lds[];  // (box_bytes: the launch's dynamic LDS)
    const P4<T>* gpn = nullptr;  // (fused: the level's point / normal records)
    if (ctl) {  // device loop: transform, level and reuse state from the device
        if (ctl->done) return;
        const GridDesc<T>& D = gd[ctl->level];
        gpts = D.gpts;
        gidx = D.gidx;
        start = D.start;
        G = D.G;
        gpn = D.gpn;
        ctl_transform(ctl, Tm);
        if (reuse) {
            reuse = ctl->prev_level == ctl->level ? 2 : 1;
#pragma unroll
            for (int i = 0; i < 16; ++i) Tprev.m[i] = (T)ctl->Tprev[i];
        }
    }
    if (!reuse) safe = nullptr;
    uint32_t visits = 0;
#if PMX_LANE_XCD
    const int64_t blk = xcd_block();  // (pmx_internal.h: adjacent slot ranges gather through one L2)
#else
    const int64_t blk = blockIdx.x;
#endif
    // quantile window (pmx_spec.h): every written distance is classified
    // (fused: by the fused pass, which also records the window's pairs)
    SpecAcc<T> sa;
    spec_acc_init<T>(sa, spec);
    SpecAcc<T> sw = sa;  // (the writers' view: off when the fused pass classifies)
    if (FUSE) sw.on = false;
    // fused: the window's pairs are recorded only while the window is valid
    // (no window: the post launch reduces every pair itself)
    const bool fuse_on = FUSE && (!fa.quantile || sa.on);
    __shared__ double wacc[4 * kFuseNV];
    if (FUSE)
        for (int v = threadIdx.x; v < 4 * kFuseNV; v += blockDim.x) wacc[v] = 0.0;
    // Phase 1: every lane tries the certificate (reuse 2; otherwise every
    // query misses).  Phase 2: the block's misses, compacted in slot order,
    // run the full search on consecutive lanes — from an LDS box of the grid
    // when the launch has one and enough lanes missed (pmx_grid_box.inc),
    // else the per-lane shell walk (a miss does not make its whole wave pay
    // for both paths).
    __shared__ int miss[256];
    __shared__ int wave_cnt[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long full_total = 0;
    {
        const int64_t base = blk * 256;
        const int64_t j = base + threadIdx.x;
        bool missed = j < N;
        if (reuse == 2 && j < N) {
            const P4<T> p = gld(rd, j);
            T qx, qy, qz;
            gxform(Tm, p, qx, qy, qz);
            missed = !reuse_query<T, KT>(gpts, gidx, p, qx, qy, qz, Tprev, j, k, qr2(radii, j, maxR2), out_d, out_i,
                                         safe, visits, sw);
        }
        const unsigned long long m = __ballot(missed);
        if (lane == 0) wave_cnt[wave] = __popcll(m);
        __syncthreads();
        int off = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int cw = wave_cnt[w];
            off += w < wave ? cw : 0;
            total += cw;
        }
        if (missed) miss[off + __popcll(m & ((1ull << lane) - 1))] = threadIdx.x;
        __syncthreads();
        if (BOX && total >= kBoxMinMiss && !oct) {
            box_phase<T, KT>(gpts, gidx, start, G, rd, base, miss, total, Tm, k, maxR2, radii, out_d, out_i, safe,
                             visits, sw, box_lds, box_bytes, reuse == 2 ? -1 : box_grow, reuse, Tprev);
        } else if ((int)threadIdx.x < total) {
            const int64_t j2 = base + miss[threadIdx.x];
            full_query<T, KT>(gpts, gidx, start, G, rd, j2, Tm, k, qr2(radii, j2, maxR2), oct, out_d, out_i, safe,
                              visits, sw);
        }
        full_total += (unsigned long long)total;
        if (FUSE) {
            __syncthreads();  // (the misses' outputs were written by other lanes of the block)
            if (fuse_on) {
                unsigned long long* recs = spec ? spec->recs : nullptr;
                double* wrow = wacc + wave * kFuseNV;
                if (fa.dim == 3)
                    fuse_chunk<T, 3>(fa, sa, recs, gpn, rd, Tm, out_d, out_i, j, j < N, k, wrow);
                else
                    fuse_chunk<T, 2>(fa, sa, recs, gpn, rd, Tm, out_d, out_i, j, j < N, k, wrow);
            }
        }
    }
    add_visits(visits, visited);
    // queries that took the full search (the "fallback" counter the level choice reads)
    if (threadIdx.x == 0 && visited && full_total && reuse) atomicAdd(vslot(visited, 1), full_total);
    if (sa.on) spec_acc_flush<T>(FUSE ? sa : sw, vslot(visited, 2), vslot(visited, 3));
    if (FUSE) {
        __syncthreads();  // (every wave's rows)
        // the block's record, block-major (the post launch sums the records in block order)
        if (threadIdx.x < kFuseNV)
            fa.partials[(int64_t)blockIdx.x * kFuseNV + threadIdx.x] =
                ((wacc[threadIdx.x] + wacc[kFuseNV + threadIdx.x]) + wacc[2 * kFuseNV + threadIdx.x]) +
                wacc[3 * kFuseNV + threadIdx.x];
    }
    if (vout) counter_fold<T>(visited, vout, iter_err, spec, spec_st, xseg);
}

// ------------------------------------------------------------ tile kernel --
#include "pmx_grid_tile.inc"

template <typename T, int KT>
static void launch_kt(int mode, const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const GridGeom& G,
                      const P4<T>* rd, int64_t N, const uint32_t* waves, int64_t n_waves, const Mat4<T>& Tm, int knn,
                      T maxR2, uint32_t max_pts, T* dists, int32_t* ids, unsigned long long* visited,
                      const GridReuse<T>& ru, const LoopCtl* ctl, const GridDesc<T>* gd, SpecSel* spec,
                      unsigned long long* vout, int* iter_err, SelectState* spec_st, unsigned long long* xseg,
                      const T* radii, uint32_t box_bytes, int box_grow, bool cold, const FuseAcc<T>& fa,
                      hipStream_t s) {
    if (cold) {  // a new reading's first match without an LDS box: the tile kernel's cold form (pmx_grid_tile.inc)
        hipLaunchKernelGGL((grid_tile_kernel<T, KT>), dim3((unsigned)((N + 63) / 64)), dim3(64), 0, s, gpts, gidx, start,
                           G, rd, N, (const uint32_t*)nullptr, Tm, knn, maxR2, max_pts, dists, ids, visited, radii, 1,
                           ctl, gd, spec, ru.safe);
    } else if (mode >= 1) {  // 1: shell search, 2: octant block first
        const int64_t grid = (N + 255) / 256;
#define PMX_LANE(B, F)                                                                                                 \
    hipLaunchKernelGGL((grid_lane_kernel<T, KT, B, F>), dim3((unsigned)grid), dim3(256), box_bytes, s, gpts, gidx, start, \
                       G, rd, N, Tm, knn, maxR2, dists, ids, visited, mode == 2 ? 1 : 0, ru.mode, ru.safe, ru.Tprev, ctl, \
                       gd, spec, vout, iter_err, spec_st, xseg, radii, box_bytes, box_grow, fa)
        if (box_bytes > 0) {
            if (fa.on)
                PMX_LANE(true, true);
            else
                PMX_LANE(true, false);
        } else {
            if (fa.on)
                PMX_LANE(false, true);
            else
                PMX_LANE(false, false);
        }
#undef PMX_LANE
    } else {
        const int64_t W = waves ? n_waves : (N + 63) / 64;
        hipLaunchKernelGGL((grid_tile_kernel<T, KT>), dim3((unsigned)W), dim3(64), 0, s, gpts, gidx, start, G, rd, N,
                           waves, Tm, knn, maxR2, max_pts, dists, ids, visited, radii, 0, (const LoopCtl*)nullptr,
                           (const GridDesc<T>*)nullptr, (SpecSel*)nullptr, (T*)nullptr);
    }
}

template <typename T>
void launch_grid_match(int mode, const P4<T>* gpts, const int32_t* gidx, const uint32_t* start, const double* lo,
                       double h, const int* g, const P4<T>* rd, int64_t N, const uint32_t* waves, int64_t n_waves,
                       const Mat4<T>& Tm, int knn, T maxR2, uint32_t max_pts, T* dists, int32_t* ids,
                       unsigned long long* visited, unsigned long long* vout, int* iter_err,
                       const GridReuse<T>& ru, const LoopCtl* ctl, const GridDesc<T>* gd, SpecSel* spec,
                       SelectState* spec_st, unsigned long long* xseg, bool fold, bool defer, const T* radii,
                       uint32_t box_bytes, int box_grow, bool cold, const FuseAcc<T>& fa, hipEvent_t ev_end,
                       hipStream_t s) {
    if (N <= 0) return;
    if (mode < 1) box_bytes = 0;
    cold = cold && mode >= 1 && box_bytes == 0;
    fold = fold && mode >= 1 && visited && vout && !cold;  // (a cold launch runs the counter kernel after it)
    if (mode < 1 || !visited || !vout) spec = nullptr;  // (the window needs the per-lane kernel and the counters)
    GridGeom G;
    for (int a = 0; a < 3; ++a) {
        G.lo[a] = lo[a];
        G.g[a] = g[a];
    }
    G.h = h;
    G.inv_h = 1.0 / h;
    if (knn > kLaneMaxK) {  // a k-list spread over a wave per query (pmx_knn_wide.hip; no reuse, no fused sums)
        launch_knn_wide<T>(gpts, gidx, start, &G, 0, rd, N, Tm, knn, maxR2, radii, dists, ids, visited, ctl, gd, spec,
                           s);
        if (ev_end) (void)hipEventRecord(ev_end, s);
        if (visited && vout && !defer)
            hipLaunchKernelGGL(counter_sum_kernel<T>, dim3(1), dim3(kVSlots), 0, s, visited, vout, iter_err, ctl, spec,
                               spec_st, xseg);
        return;
    }
#define PMX_KT(KT) \
    launch_kt<T, KT>(mode, gpts, gidx, start, G, rd, N, waves, n_waves, Tm, knn, maxR2, max_pts, dists, ids, visited, \
                     ru, ctl, gd, spec, fold ? vout : nullptr, iter_err, spec_st, xseg, radii, box_bytes, box_grow, cold, \
                     fa, s)
    // with reuse the list keeps room for the (k+1)-th point (the safe radius;
    // the cold tile writes radius 0 and keeps k entries)
    const int kl = ru.mode && mode >= 1 && knn < 16 && !cold ? knn + 1 : knn;
    if (kl == 1)
        PMX_KT(1);
    else if (kl <= 2)
        PMX_KT(2);
    else if (kl <= 4)
        PMX_KT(4);
    else if (kl <= 8)
        PMX_KT(8);
    else
        PMX_KT(16);
#undef PMX_KT
    if (ev_end) (void)hipEventRecord(ev_end, s);  // (timing: the match kernel, with the folded counter phase)
    // (folded: the per-lane kernel's last workgroup ran it; deferred: the
    // select_all launch that follows runs it, pmx_select.hip)
    if (visited && vout && !fold && !defer && !fa.on)
        hipLaunchKernelGGL(counter_sum_kernel<T>, dim3(1), dim3(kVSlots), 0, s, visited, vout, iter_err, ctl, spec,
                           spec_st, xseg);
}

template void launch_grid_match<float>(int, const P4<float>*, const int32_t*, const uint32_t*, const double*, double,
                                       const int*, const P4<float>*, int64_t, const uint32_t*, int64_t,
                                       const Mat4<float>&, int, float, uint32_t, float*, int32_t*,
                                       unsigned long long*, unsigned long long*, int*, const GridReuse<float>&,
                                       const LoopCtl*, const GridDesc<float>*, SpecSel*, SelectState*,
                                       unsigned long long*, bool, bool, const float*, uint32_t, int, bool,
                                       const FuseAcc<float>&, hipEvent_t, hipStream_t);
template void launch_grid_match<double>(int, const P4<double>*, const int32_t*, const uint32_t*, const double*, double,
                                        const int*, const P4<double>*, int64_t, const uint32_t*, int64_t,
                                        const Mat4<double>&, int, double, uint32_t, double*, int32_t*,
                                        unsigned long long*, unsigned long long*, int*, const GridReuse<double>&,
                                        const LoopCtl*, const GridDesc<double>*, SpecSel*, SelectState*,
                                        unsigned long long*, bool, bool, const double*, uint32_t, int, bool,
                                        const FuseAcc<double>&, hipEvent_t, hipStream_t);

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
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&grid_lane_kernel<float, 1, false, false>));
}

}  // namespace pmx
