// pmx_spec.h — windowed quantile select fused into the grid match.
//
// TrimmedDist / MedianDist need one order statistic of the k*N match
// distances per iteration (Matches::getDistsQuantile, Matches.cpp:60-87).
// The radix select of pmx_select.hip finds it exactly in three dependent
// passes over the distances (f32).  Across ICP iterations the quantile moves
// little, so the match kernel itself classifies every distance it writes
// against a key window [lo, hi] around the previous iteration's limit:
//
//   fin    = number of finite distances          (Matches.cpp:71)
//   below  = number of finite keys  <  lo
//   keys[] = the keys inside [lo, hi]             (appended, capacity cap)
//
// The target rank r = (size_t)((T)fin * ratio) (clamped; ratio == 1 -> the
// maximum) is in the window iff below <= r < below + n_keys, and then the
// limit is exactly the (r - below)-th smallest appended key: the select runs
// over a few thousand keys inside counter_sum_kernel (pmx_grid.hip), which
// follows the match anyway.  Nothing is approximated: when the window misses
// (rank outside, overflow, first iteration, any error condition) `hit` stays
// 0 and the regular radix passes run and produce the limit, exactly as
// without the window.  Either way the next window is centred on the resolved
// limit, its half-width from the last movement of the limit and capped by the
// observed key density so the expected append count stays below cap/2.
//
// Used by the device-resident loop, chain position 0.  With several ranks the
// counters and window keys are exchanged first (SpecKeys segments below).
#pragma once

#include "pmx_internal.h"

namespace pmx {

template <typename T>
struct KeyOf;
template <>
struct KeyOf<float> {
    using K = uint32_t;
    static constexpr int bits = 32;
    static __device__ __forceinline__ K key(float v) { return __float_as_uint(v); }
    static __device__ __forceinline__ float val(K k) { return __uint_as_float(k); }
    static constexpr K inf_key = 0x7F800000u;
};
template <>
struct KeyOf<double> {
    using K = unsigned long long;
    static constexpr int bits = 64;
    static __device__ __forceinline__ K key(double v) { return (K)__double_as_longlong(v); }
    static __device__ __forceinline__ double val(K k) { return __longlong_as_double((long long)k); }
    static constexpr K inf_key = 0x7FF0000000000000ull;
};

constexpr unsigned kSpecCap = 16384;  // appended keys per iteration

// radix-select digit layout (pmx_select.hip): 11-bit digits from the top,
// the last one(s) 10-bit
// f32: [31:21] [20:10] [9:0]          f64: [63:53] [52:42] [41:31] [30:20] [19:10] [9:0]
__host__ __device__ inline void digit_of(int key_bits, int pass, int& shift, int& bits) {
    if (key_bits == 32) {
        const int sh[3] = {21, 10, 0};
        const int bt[3] = {11, 11, 10};
        shift = sh[pass];
        bits = bt[pass];
    } else {
        const int sh[6] = {53, 42, 31, 20, 10, 0};
        const int bt[6] = {11, 11, 11, 11, 10, 10};
        shift = sh[pass];
        bits = bt[pass];
    }
}

struct SpecSel {
    unsigned long long lo, hi;  // key window (inclusive); valid != 0
    unsigned long long prev;    // last resolved limit key
    double ratio;               // quantile ratio (T value)
    void* keys;                 // K[kSpecCap]
    unsigned int n_keys;        // appended by the match (may exceed the capacity)
    int valid;                  // lo / hi describe a window
    int have_prev;              // prev holds a limit
    int hit;                    // this iteration's limit came from the window
    unsigned long long n_hit, n_miss;  // statistics (host-readable)
    double dens;                // key density estimate of the last radix select (keys per key unit)
    int wide;                   // several ranks: a miss costs a stall and a replay, so a wider window
};

// ---- match side: classify every distance the match writes ----
template <typename T>
struct SpecAcc {
    using K = typename KeyOf<T>::K;
    K lo, hi;
    K* keys;
    unsigned int* n_keys;
    uint32_t fin, below;
    bool on;
};
// off when there is no window (no spec, or the radix passes resolve this
// iteration): the match then classifies nothing
template <typename T>
__device__ __forceinline__ void spec_acc_init(SpecAcc<T>& a, SpecSel* sp) {
    using K = typename KeyOf<T>::K;
    a.on = sp && sp->valid;  // (uniform)
    a.fin = 0;
    a.below = 0;
    a.lo = 0;
    a.hi = 0;
    a.keys = nullptr;
    a.n_keys = nullptr;
    if (!a.on) return;
    a.lo = (K)sp->lo;
    a.hi = (K)sp->hi;
    a.keys = (K*)sp->keys;
    a.n_keys = &sp->n_keys;
}
// classify one written distance; returns its append position inside the
// window's buffers (kSpecCap or more: not appended)
template <typename T>
__device__ __forceinline__ unsigned spec_acc(SpecAcc<T>& a, T d) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    const K k = KO::key(d);
    unsigned pos = kSpecCap;
    if (k < KO::inf_key) {  // (+inf and NaN excluded; distances are >= +0)
        a.fin += 1;
        if (k < a.lo) {
            a.below += 1;
        } else if (k <= a.hi) {  // rare: a few thousand of k*N
            pos = atomicAdd(a.n_keys, 1u);
            // (write-through: the match kernel's last block reads the keys in the same launch)
            if (pos < kSpecCap) __hip_atomic_store(&a.keys[pos], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    return pos;
}
// wave sums into the spread counters (all lanes of the wave call it)
template <typename T>
__device__ __forceinline__ void spec_acc_flush(const SpecAcc<T>& a, unsigned long long* c_fin,
                                               unsigned long long* c_below) {
    uint32_t f = a.fin, b = a.below;
    for (int off = 32; off > 0; off >>= 1) {
        f += __shfl_xor(f, off);
        b += __shfl_xor(b, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (f) atomicAdd(c_fin, (unsigned long long)f);
        if (b) atomicAdd(c_below, (unsigned long long)b);
    }
}

// ---- next window, centred on the resolved limit key kl ----
// density: keys per key unit around the limit (observed)
template <typename T>
__device__ __forceinline__ void spec_update(SpecSel* sp, typename KeyOf<T>::K kl, double density) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    const double move = sp->have_prev ? (double)(kl > (K)sp->prev ? kl - (K)sp->prev : (K)sp->prev - kl) : 0.0;
    // (several ranks: a miss stalls the blind batch and replays it, so the
    // window is wider — C3 sharded: no stall in 20 iterations instead of 1-2,
    // profiles/r06/scale/wide_window.txt; one rank resolves a miss inside the
    // select launch, and a wider window costs it appends)
    double hw = sp->wide ? 6.0 * move + 256.0 : 3.0 * move + 64.0;
    const double dens = density > 1e-30 ? density : 1e-30;
    // expected appends <= cap / 8: every append is an atomic on one counter
    // inside the match kernel, so the window is kept small
    const double cap_hw = (double)(kSpecCap / 16) / dens;
    if (hw > cap_hw) hw = cap_hw;
    if (hw > 1.0e15) hw = 1.0e15;
    if (hw < 1.0) hw = 1.0;
    const K h = (K)hw;
    const K lo = kl > h ? kl - h : (K)0;
    const K hi = (KO::inf_key - 1 - kl) > h ? kl + h : KO::inf_key - 1;
    sp->lo = lo;
    sp->hi = hi;
    sp->prev = kl;
    sp->have_prev = 1;
    sp->valid = 1;
}

// ---- several ranks: the window's keys are exchanged ----
// Every rank packs its counters and window keys into one segment
//   [fin, below, n_keys, key_0 .. key_{n-1}]   (unsigned long long each)
// after its match; the segments are all-gathered (pmx_capi.hip) and every
// rank resolves the same limit from the union (spec_pick over nseg
// segments).  A rank that appended more than kSpecXCap keys makes the window
// miss on every rank (its segment carries the true count).
constexpr unsigned kSpecXCap = 4096;
constexpr unsigned kSpecXHdr = 3;
constexpr unsigned kSpecXStride = kSpecXHdr + kSpecXCap;  // unsigned long longs per segment

// the keys a pick runs over: one local append buffer, or nseg exchanged segments
template <typename T>
struct SpecKeys {
    using K = typename KeyOf<T>::K;
    const K* local = nullptr;                    // single rank: K[n_local]
    unsigned n_local = 0;
    const unsigned long long* segs = nullptr;    // several ranks: nseg * kSpecXStride
    int nseg = 0;
    const K* lds = nullptr;                      // single rank: the keys copied to LDS (every pass reads them)
    __device__ __forceinline__ int count() const { return segs ? nseg : 1; }
    __device__ __forceinline__ unsigned n(int s) const {
        if (!segs) return n_local;
        const unsigned long long c = segs[(size_t)s * kSpecXStride + 2];
        return c < kSpecXCap ? (unsigned)c : kSpecXCap;
    }
    __device__ __forceinline__ K key(int s, unsigned i) const {
        // (local keys: appended in the same launch when the match's last block picks: coherent loads)
        if (lds) return lds[i];
        return segs ? (K)segs[(size_t)s * kSpecXStride + kSpecXHdr + i] : local[i];
    }
};

// inclusive scan over a block of kThreads (a multiple of 64, <= 1024):
// wave scans with shuffles, then the waves' totals (two barriers, against
// 2 log2(kThreads) for a Hillis-Steele scan through LDS).  wsum: LDS of
// kThreads / 64 entries.
template <int kThreads>
__device__ __forceinline__ unsigned long long block_incl_scan(unsigned long long v, unsigned long long* wsum) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    if (lane == 63) wsum[wave] = v;
    __syncthreads();
    unsigned long long before = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) before += w < wave ? wsum[w] : 0ull;
    __syncthreads();  // (wsum reusable)
    return before + v;
}

// ---- counter side: resolve the limit from the window (one block) ----
// fin / below: the match's counters (global), nk_raw: keys appended inside
// the window (global; more than the buffers hold means a miss), keys: where
// they are.  Writes st (as the radix select's last pass would) and sp->hit;
// resets the append counter (commit = false: reads only, the verdict and the
// limit key in *kl_out, for spec_commit).  Block of kThreads.
template <typename T>
__device__ __forceinline__ void spec_commit(SpecSel* __restrict__ sp, SelectState* __restrict__ st, bool hit,
                                            typename KeyOf<T>::K lo, typename KeyOf<T>::K hi,
                                            typename KeyOf<T>::K kl, unsigned long long fin, unsigned long long nk) {
    using KO = KeyOf<T>;
    if (!hit) {
        sp->hit = 0;
        sp->n_miss += 1;
        sp->n_keys = 0;
        return;
    }
    st->err = 0;
    st->count = fin;
    st->prefix = (unsigned long long)kl;
    st->rank = 0;
    st->ratio = (double)(T)sp->ratio;
    st->limit = (double)KO::val(kl);
    sp->hit = 1;
    sp->n_hit += 1;
    sp->n_keys = 0;
    const double width = (double)(hi - lo) + 1.0;
    spec_update<T>(sp, kl, (double)nk / width);
}

template <typename T, int kThreads>
__device__ __forceinline__ bool spec_pick(SpecSel* __restrict__ sp, SelectState* __restrict__ st,
                                          unsigned long long fin, unsigned long long below,
                                          unsigned long long nk_raw, bool overflow, const SpecKeys<T>& src,
                                          uint32_t* lh, unsigned long long* part, unsigned long long* bc,
                                          bool commit = true, unsigned long long* kl_out = nullptr) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    const int t = threadIdx.x;
    const unsigned long long nk = nk_raw;
    const K lo = (K)sp->lo, hi = (K)sp->hi;
    // target rank (Matches.cpp:83-86 via pick_phase's rule)
    bool ok = sp->valid && !overflow && fin > 0;
    const T q = (T)sp->ratio;
    unsigned long long rank = 0;
    if (ok) {
        if (!(q >= (T)0 && q <= (T)1)) {
            ok = false;
        } else if (q == (T)1) {
            rank = fin - 1;
        } else {
            rank = (unsigned long long)((T)fin * q);
            if (rank >= fin) rank = fin - 1;
        }
    }
    ok = ok && rank >= below && rank < below + nk;
    __syncthreads();
    if (!ok) {
        if (t == 0 && commit) spec_commit<T>(sp, st, false, lo, hi, (K)0, fin, nk);
        return false;
    }
    unsigned long long r = rank - below;
    // radix select over offsets (key - lo) < 2^nb, 11-bit digits from the top
    const unsigned long long w = (unsigned long long)(hi - lo);
    const int nb = w == 0 ? 1 : 64 - __builtin_clzll(w);
    unsigned long long prefix = 0;  // resolved high bits of the offset
    int done_bits = 0;
    while (done_bits < nb) {  // uniform
        const int bits = (nb - done_bits) < 11 ? (nb - done_bits) : 11;
        const int shift = nb - done_bits - bits;
        const int nbins = 1 << bits;
        for (int i = t; i < 2048; i += kThreads) lh[i] = 0;
        __syncthreads();
        for (int s = 0; s < src.count(); ++s) {
            const unsigned ns = src.n(s);
            for (unsigned i = t; i < ns; i += kThreads) {
                const unsigned long long off = (unsigned long long)(src.key(s, i) - lo);
                if (done_bits == 0 || (off >> (shift + bits)) == prefix)
                    atomicAdd(&lh[(off >> shift) & (unsigned long long)(nbins - 1)], 1u);
            }
        }
        __syncthreads();
        // each thread owns 2048 / kThreads consecutive bins
        constexpr int per = 2048 / kThreads;
        unsigned long long mine = 0;
        for (int j = 0; j < per; ++j) mine += lh[t * per + j];
        const unsigned long long incl = block_incl_scan<kThreads>(mine, part);
        const unsigned long long excl = incl - mine;
        if (r >= excl && r < incl) {
            unsigned long long cum = excl;
            for (int j = 0; j < per; ++j) {
                const unsigned long long c = lh[t * per + j];
                if (r < cum + c) {
                    bc[0] = (unsigned long long)(t * per + j);
                    bc[1] = r - cum;
                    break;
                }
                cum += c;
            }
        }
        __syncthreads();
        prefix = (prefix << bits) | bc[0];
        r = bc[1];
        done_bits += bits;
        __syncthreads();
    }
    const K kl = lo + (K)prefix;
    if (kl_out) *kl_out = (unsigned long long)kl;
    if (t == 0 && commit) spec_commit<T>(sp, st, true, lo, hi, kl, fin, nk);
    return true;
}

// ---- the counter phase after a match (one block of kVSlots threads) ----
// Pair / fallback / window counters: every wave of the match adds into one of
// kVSlots spread counters (each on its own 128-byte line); this folds them.
constexpr int kVSlots = 256;
constexpr int kVStride = 16;  // unsigned long longs: 128 bytes
// (also clears the iteration's error word: it runs first after the match,
// before any filter can raise one).  With a quantile window (pmx_spec.h) it
// also resolves the iteration's quantile from the window when it can — or,
// with several ranks (xseg != null), packs this rank's window segment for the
// exchange and leaves the pick to spec_pick_kernel.
template <typename T>
__device__ __forceinline__ void counter_phase(unsigned long long* __restrict__ vpart,
                                              unsigned long long* __restrict__ out, int* __restrict__ iter_err,
                                              SpecSel* __restrict__ spec, SelectState* __restrict__ st,
                                              unsigned long long* __restrict__ xseg) {
    __shared__ unsigned long long red[4][kVSlots / 64];
    __shared__ uint32_t lh[2048];
    __shared__ unsigned long long part[kVSlots];
    __shared__ unsigned long long bc[2];
    const int t = threadIdx.x;
    unsigned long long v[4];
    // the window's append count, read with the counters (one round trip)
    const unsigned nk_raw = spec ? __hip_atomic_load(&spec->n_keys, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    // (coherent loads / stores: the counters of another launch's workgroups,
    // possibly on other XCDs)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        unsigned long long* p = vpart + (size_t)(c * kVSlots + t) * kVStride;
        v[c] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next match
    }
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] += __shfl_xor(v[c], off);
    }
    if ((t & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) red[c][t >> 6] = v[c];
    }
    __syncthreads();
    unsigned long long sum[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < kVSlots / 64; ++w) sum[c] += red[c][w];
    if (t == 0) {
        // (coherent: the fused post launch may read them from another block)
        __hip_atomic_store(&out[0], sum[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&out[1], sum[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (iter_err) __hip_atomic_store(iter_err, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (coherent: a select may write it in the same launch)
    }
    if (!spec) return;
    if (xseg) {  // several ranks: this rank's segment [fin, below, n, keys...]
        using K = typename KeyOf<T>::K;
        const unsigned nk = nk_raw;
        const unsigned nc = nk < kSpecXCap ? nk : kSpecXCap;
        const K* keys = (const K*)spec->keys;
        if (t == 0) {
            xseg[0] = sum[2];
            xseg[1] = sum[3];
            xseg[2] = spec->valid ? nk : 0ull;
        }
        for (unsigned i = t; i < nc; i += kVSlots)
            xseg[kSpecXHdr + i] = (unsigned long long)__hip_atomic_load(&keys[i], __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // (every lane read n_keys before it is reset)
        if (t == 0) spec->n_keys = 0;
        return;
    }
    using K = typename KeyOf<T>::K;
    SpecKeys<T> src;
    src.local = (const K*)spec->keys;
    src.n_local = nk_raw < kSpecCap ? nk_raw : kSpecCap;
    // the keys into LDS once (every radix pass of the pick reads them all)
    constexpr unsigned kSpecLds = 4096;
    __shared__ K lkeys[kSpecLds];
    if (src.n_local <= kSpecLds && spec->valid) {
        for (unsigned i = t; i < src.n_local; i += kVSlots) lkeys[i] = src.local[i];
        __syncthreads();
        src.lds = lkeys;
    }
    (void)spec_pick<T, kVSlots>(spec, st, sum[2], sum[3], src.n_local, nk_raw > kSpecCap, src, lh, part, bc);
}

}  // namespace pmx
