// pmx_post.hip — the post-match work of a device-loop iteration in one
// launch (point-to-plane, single rank).
//
// The steady-state iteration was six dependent launches: match, counter sum
// + window pick, radix select (a no-op on a window hit), point-to-plane
// reduction (a second pass over the matches, ~56 B per pair re-gathered),
// finalize, step — each boundary ~1.5-2 us on MI355X plus the short kernels'
// latency chains (~43 us of the 70 us iteration at C3, kernel trace).  Now
// it is three: the match, which adds the point-to-plane sums of the pairs it
// can decide itself (pmx_grid.hip fuse_chunk: every pair without a quantile
// filter; with TrimmedDist at chain position 0 the pairs below the quantile
// window, recording the window's own pairs); this launch; the step
// (pmx_loop.hip).  Here:
//
//   block 0: folds the match's counters, picks the quantile inside the
//            window (pmx_spec.h) and publishes the verdict;
//   hit:     every block adds its slice of the match blocks' records and of
//            the window's pairs at or below the limit;
//   miss:    every block runs the radix passes (pmx_selectall.h), then its
//            share of the full point-to-plane reduction with that limit
//            (p2plane_body);
//   then the last block to arrive sums the blocks' partials in block order
//   into the iteration block (the ErrorElements counts included).
//
// A window hit is exact: the limit lies inside [lo, hi], so a pair below lo is
// at or below it and a pair above hi is not (OutlierFiltersImpl.cpp:139-147,
// ties inclusive).  The sums are the same T products in fp64 as p2plane_body
// (PointToPlane.cpp:194-243); only their fp64 summation order differs (the
// window pairs' order follows the match's appends).  Every cross-block
// hand-off is an agent-scope atomic (stores, loads, tickets): no fence.
// The grid is at most the resident block count (every block may wait on
// another's publication; the waits are bounded and raise kSelTimeout).
#include "pmx_internal.h"
#include "pmx_p2plane.h"
#include "pmx_selectall.h"
#include "pmx_loop.h"
#include "pmx_spec.h"

namespace pmx {

template <typename T>
struct PostArgs {
    const T* d;            // match distances (N * k, slot-major)
    const int32_t* ids;    // match grid positions
    const P4<T>* rd;       // reading (slot order)
    int64_t N;
    int k;
    LoopCtl* ctl;
    const GridDesc<T>* gd;
    int quantile;          // chain position 0 is TrimmedDist
    double ratio;
    SelX* sx;
    SelectState* st;
    SpecSel* spec;
    int* iter_err;
    unsigned long long* vpart;  // the match's spread counters
    unsigned long long* vout;   // [pairs, full searches] of the iteration block
    const double* fuse_part;    // the match blocks' records [fuse_blocks][kFuseNV]
    int fuse_blocks;
    double* part2;              // miss path: [NV][gridDim.x]
    WChain<T> chain;            // the chain (miss path), position 0 = the quantile
    double* res_out;            // the iteration block's result area (host mirror)
    LoopState<T>* S;
    LoopCfg cfg;
    T* trace;
};

// the window pairs of this block's slice and its slice of the match records,
// in the fused layout; hit path
template <typename T, int DIM>
__device__ __forceinline__ void post_hit_slice(const PostArgs<T>& a, double L, double (&acc)[kFuseNV]) {
    constexpr int NSF = DIM == 3 ? 27 : 9;
    const int t = threadIdx.x;
    const int G = gridDim.x;
    // the match records: block b adds records [b R, (b + 1) R) in order, thread t of them every 256th
    const int R = (a.fuse_blocks + G - 1) / G;
    const int r0 = blockIdx.x * R, r1 = min(a.fuse_blocks, r0 + R);
    for (int r = r0 + t; r < r1; r += 256) {
        const double2* p = reinterpret_cast<const double2*>(a.fuse_part + (int64_t)r * kFuseNV);
        double2 x[kFuseNV / 2];
#pragma unroll
        for (int q = 0; q < kFuseNV / 2; ++q) x[q] = p[q];
#pragma unroll
        for (int q = 0; q < kFuseNV / 2; ++q) {
            acc[2 * q] += x[q].x;
            acc[2 * q + 1] += x[q].y;
        }
    }
    if (!a.quantile) return;
    // the window's pairs at or below the limit (every load of a round issued first)
    using KO = KeyOf<T>;
    using K = typename KO::K;
    const K kl = KO::key((T)L);
    Mat4<T> Tm;
    ctl_transform(a.ctl, Tm);
    const P4<T>* gpn = a.gd[a.ctl->level].gpn;
    // (published with the verdict by block 0 in this launch: a coherent load)
    const unsigned nu = (unsigned)ald(&a.sx->nused);
    const K* keys = (const K*)a.spec->keys;
    constexpr int U = 4;
    const unsigned stride = (unsigned)G * 256u;
    for (unsigned i0 = blockIdx.x * 256u + (unsigned)t; i0 < nu; i0 += U * stride) {
        bool kp[U];
        unsigned long long rc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned i = i0 + (unsigned)u * stride;
            rc[u] = i < nu ? a.spec->recs[i] : 0ull;
            const K key = i < nu ? keys[i] : (K)0;
            kp[u] = i < nu && (rc[u] & kRecFx) && key <= kl;
        }
        P4<T> pr[U], q[U], n[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = kp[u] ? (int64_t)(rc[u] >> 32) : 0, pos = kp[u] ? (int64_t)(rc[u] & kRecPos) : 0;
            pr[u] = gld(a.rd, j);
            q[u] = gld(gpn, 2 * pos);
            n[u] = gld(gpn, 2 * pos + 1);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!kp[u]) continue;
            T px, py, pz;
            xform3(Tm, pr[u], px, py, pz);
            p2plane_add<T, DIM, kFuseNV>(acc, px, py, pz, q[u], n[u]);
            acc[NSF] += 1.0;
            if (rc[u] & kRecHead) acc[NSF + 3] += 1.0;
        }
    }
}

// every block's ticket after its stores drained; true on the last block
__device__ __forceinline__ bool post_ticket(SelX* sx) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(&sx->post_arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (old + 1u) % gridDim.x == 0u;
    }
    __syncthreads();
    return s_last != 0;
}

// the last block: every block's partials in block order (coherent loads);
// hit: the fused layout's counts become the point-to-plane layout's (kept,
// non-zero weights, rejected matches, rejected points, sum of the weights)
template <typename T, int DIM>
__device__ void post_final(const PostArgs<T>& a, bool hit) {
    constexpr int NSF = DIM == 3 ? 27 : 9;
    constexpr int NV = NSF + 5;
    __shared__ double red[4][kFuseNV];
    __shared__ double tot[kFuseNV];
    const int t = threadIdx.x, wave = t >> 6;
    const int G = gridDim.x;
    double x[kFuseNV];
#pragma unroll
    for (int v = 0; v < kFuseNV; ++v)
        x[v] = t < G ? __hip_atomic_load(&a.part2[(int64_t)v * G + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0.0;
    int idx;
    const double w = wave_transpose_sum<kFuseNV>(x, idx);
    if (transpose_writer<kFuseNV>()) red[wave][idx] = w;
    __syncthreads();
    if (t < kFuseNV) tot[t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    __syncthreads();
    if (t < NSF) a.res_out[t] = tot[t];
    if (t == 0) {
        if (hit) {
            const double kept = tot[NSF], nz = a.quantile ? kept : tot[NSF + 1], fin = tot[NSF + 2];
            a.res_out[NSF] = kept;
            a.res_out[NSF + 1] = nz;
            a.res_out[NSF + 2] = fin - kept;
            a.res_out[NSF + 3] = (double)a.N - tot[NSF + 3];
            a.res_out[NSF + 4] = kept;
        } else {
            for (int v = NSF; v < NV; ++v) a.res_out[v] = tot[v];
        }
    }
}

template <typename T, int DIM>
__global__ __launch_bounds__(256) void post_kernel(PostArgs<T> a) {
    if (a.ctl->done) return;  // (uniform)
    double L = 0.0;
    bool hit = true, ok = true;
    if (a.quantile) {
        ok = select_all_body<T>(a.d, a.N * a.k, a.sx, a.st, a.ratio, nullptr, a.iter_err, 0, a.spec, a.vpart, a.vout,
                                true, &L, &hit);
    } else if (blockIdx.x == 0) {
        counter_phase<T>(a.vpart, a.vout, a.iter_err, nullptr, nullptr, nullptr);
    }
    if (ok && hit) {
        double acc[kFuseNV];
#pragma unroll
        for (int v = 0; v < kFuseNV; ++v) acc[v] = 0.0;
        post_hit_slice<T, DIM>(a, L, acc);
        block_store<kFuseNV, true>(acc, a.part2);
    } else if (ok) {  // miss: the full reduction with the resolved limit
        __shared__ SelectState s_lim;
        if (threadIdx.x == 0) s_lim.limit = L;
        __syncthreads();
        WChain<T> ch = a.chain;
        ch.st[0] = &s_lim;
        Mat4<T> Tm;
        ctl_transform(a.ctl, Tm);
        const P4<T>* ref = a.gd[a.ctl->level].gpn;
        p2plane_body<T, DIM, true>(a.rd, Tm, ref, ref + 1, 2, a.d, a.ids, ch, a.k, a.N, a.part2);
    }
    // (an error or a timed-out wait: the step kernel raises it; the sums are unused)
    if (!post_ticket(a.sx) || !ok) return;
    post_final<T, DIM>(a, hit);
}

// the post launch's grid: at most the resident blocks (every block may wait
// on another's publication), a power of two (the tickets' generations)
template <typename T>
static int post_grid(int rows, int cu_count) {
    static int cached[2] = {0, 0};
    int& g = cached[rows == 4 ? 1 : 0];
    if (g == 0) {
        int per = 0;
        const void* f = rows == 4 ? reinterpret_cast<const void*>(&post_kernel<T, 3>)
                                  : reinterpret_cast<const void*>(&post_kernel<T, 2>);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, 256, 0) != hipSuccess || per < 1) per = 1;
        const int64_t lim = std::min<int64_t>((int64_t)per * cu_count, 256);
        int p2 = 1;
        while (p2 * 2 <= lim) p2 *= 2;
        g = p2;
    }
    return g;
}

template <typename T>
void launch_post(const PostLaunch<T>& p, hipStream_t s) {
    PostArgs<T> a;
    a.d = p.d;
    a.ids = p.ids;
    a.rd = p.rd;
    a.N = p.N;
    a.k = p.k;
    a.ctl = p.ctl;
    a.gd = p.gd;
    a.quantile = p.quantile;
    a.ratio = p.ratio;
    a.sx = (SelX*)p.selx;
    a.st = p.st;
    a.spec = p.spec;
    a.iter_err = p.iter_err;
    a.vpart = p.vpart;
    a.vout = p.vout;
    a.fuse_part = p.fuse_part;
    a.fuse_blocks = p.fuse_blocks;
    a.part2 = p.part2;
    a.chain = p.chain;
    a.res_out = p.res_out;
    a.S = p.S;
    a.cfg = p.cfg;
    a.trace = p.trace;
    const int G = post_grid<T>(p.cfg.rows, p.cu_count);
    if (p.cfg.rows == 4)
        hipLaunchKernelGGL((post_kernel<T, 3>), dim3(G), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((post_kernel<T, 2>), dim3(G), dim3(256), 0, s, a);
}

template void launch_post<float>(const PostLaunch<float>&, hipStream_t);
template void launch_post<double>(const PostLaunch<double>&, hipStream_t);

void preload_post() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&post_kernel<float, 3>));
}

}  // namespace pmx
