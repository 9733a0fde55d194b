// pmx_select.hip — outlier weighting on the device.
//
// Replaces OutlierFiltersImpl.cpp:51-223 and Matches::getDistsQuantile
// (Matches.cpp:60-87).  The reference copies the finite distances into a
// std::vector and runs nth_element; here the exact order statistic is found
// by a most-significant-digit radix select on the IEEE bit patterns (squared
// distances are >= +0, so the unsigned bit order is the numeric order; +inf
// and NaN keys are excluded exactly as `dists != inf` excludes them).  Each
// pass is one streaming histogram kernel (k*N*sizeof(T) bytes, HBM-bound) and
// one single-block "pick" kernel; with several ranks the 2048-bin histogram is
// all-reduced between the two (pmx_capi.hip), which makes the select exact
// over the global, sharded match set.
//
// Index rule (Matches.cpp:83-86): target = (size_t)((T)count * ratio) over the
// finite distances, ratio == 1 -> maximum; the weight is (dist <= value).
//
// VarTrimmedDist (OutlierFiltersImpl.cpp:166-220): compaction of the finite
// positive distances, a device LSD radix sort, the sequential std::partial_sum
// in T (one wave, bit-identical to the CPU), the FRMS curve and a first-index
// argmin, then the same radix select with the optimised ratio.
#include "pmx_internal.h"
#include "pmx_radix.h"
#include "pmx_sort.h"
#include "pmx_spec.h"
#include "pmx_selectall.h"


#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace pmx {

// digit layout: digit_of (pmx_spec.h)
int select_bins(int pass, int key_bits) {
    int sh, bt;
    digit_of(key_bits, pass, sh, bt);
    return 1 << bt;
}
template <>
int select_passes<float>() {
    return 3;
}
template <>
int select_passes<double>() {
    return 6;
}

// Block-local histogram of digit `pass` over the keys that match the
// resolved prefix, flushed into the global histogram with one atomic per
// non-empty bin.  Pass 0 starts a fresh select (the state is not read).
template <typename T>
__device__ __forceinline__ void hist_phase(const T* __restrict__ d, int64_t n, uint32_t* __restrict__ hist,
                                           const SelectState* __restrict__ st, int pass, uint32_t* lh) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    int shift, bits;
    digit_of(KO::bits, pass, shift, bits);
    const int nb = 1 << bits;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) lh[i] = 0;
    __syncthreads();
    const bool skip = pass > 0 && st->err != 0;
    const K prefix = pass > 0 ? (K)st->prefix : (K)0;
    const int hs = shift + bits;
    if (!skip) {
        // Each thread loads kSelPer consecutive keys at once (vector loads,
        // all in flight: the pass is latency-bound otherwise).  Plain LDS
        // atomics: aggregating equal bins per wave first measured slower
        // (pass 0 at C3: 11.4 us plain vs 39.7 us aggregated — a wave of noisy
        // neighbouring distances sees ~20-30 distinct bins).
        const int64_t tile = (int64_t)blockDim.x * kSelPer;
        for (int64_t base = (int64_t)blockIdx.x * tile; base < n; base += (int64_t)gridDim.x * tile) {  // uniform
            const int64_t i0 = base + (int64_t)threadIdx.x * kSelPer;
            T v[kSelPer];
            load_keys<T>(d, i0, n, v);
#pragma unroll
            for (int j = 0; j < kSelPer; ++j) {
                const K k = KO::key(v[j]);
                // +inf (and NaN, and the padding past n) excluded, Matches.cpp:71;
                // later passes keep the resolved prefix
                if (k < KO::inf_key && (pass == 0 || (k >> hs) == prefix))
                    atomicAdd(&lh[(uint32_t)(k >> shift) & (uint32_t)(nb - 1)], 1u);
            }
        }
    }
    __syncthreads();
    // flush with returning atomics and wait for the returns: once they are
    // back the adds are performed at the device coherence point, which is
    // what select_all_kernel's arrival counters rely on (no release fence,
    // which would write back the whole L2)
    uint32_t ret = 0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) {
        const uint32_t c = lh[i];
        if (c) ret |= atomicAdd(&hist[i], c);
    }
    asm volatile("" ::"v"(ret));
}

template <typename T>
__global__ __launch_bounds__(256) void select_hist_kernel(const T* __restrict__ d, int64_t n,
                                                          uint32_t* __restrict__ hist,
                                                          const SelectState* __restrict__ st, int pass,
                                                          const LoopCtl* __restrict__ ctl,
                                                          const SpecSel* __restrict__ spec) {
    __shared__ uint32_t lh[2048];
    if (ctl && ctl->done) return;
    if (spec && spec->hit) return;  // the quantile window resolved it (pmx_spec.h)
    hist_phase<T>(d, n, hist, st, pass, lh);
}

// Few blocks: every block flushes its non-empty bins with global atomics, and
// the first digits of squared distances fall into a handful of bins, so more
// blocks mostly add same-address atomic traffic.
static int64_t select_blocks(int64_t n) {
    // (64: the select_all launch is a no-op whenever the quantile window
    // resolved the limit, and its cost is then the dispatch of its blocks;
    // same-box A/B at C3, driver command: 256 -> 81.6, 128 -> 80.4,
    // 64 -> 80.2, 32 -> 81.0 us per iteration)
    constexpr int64_t cap = 64;
    int64_t g = (n + 256 * kSelPer - 1) / (256 * kSelPer);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    // a power of two: select_all_kernel's uint32 arrival counters then wrap
    // at a multiple of the grid, and the generation stamps stay aligned
    int64_t p2 = 1;
    while (p2 * 2 <= g) p2 *= 2;
    return p2;
}

template <typename T>
void launch_select_hist(const T* d, int64_t n, uint32_t* hist, const SelectState* st, int pass, const LoopCtl* ctl,
                        const SpecSel* spec, hipStream_t s) {
    hipLaunchKernelGGL(select_hist_kernel<T>, dim3((unsigned)select_blocks(n)), dim3(256), 0, s, d, n, hist, st,
                       pass, ctl, spec);
}

// one block of 256 threads; each thread owns 8 consecutive bins.  Pass 0
// starts a fresh select state (count, rank from the ratio, error).
template <typename T, bool kCoherent>
__device__ __forceinline__ void pick_phase(uint32_t* __restrict__ hist, SelectState* __restrict__ st, int pass,
                                           double ratio_host, const double* __restrict__ ratio_dev,
                                           int* __restrict__ iter_err, int last, unsigned long long* part,
                                           unsigned long long& s_rank, int& s_err, SpecSel* __restrict__ spec) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    int shift, bits;
    digit_of(KO::bits, pass, shift, bits);
    const int nb = 1 << bits;
    const int per = nb / 256;  // 8 or 4
    const int t = threadIdx.x;
    // this thread's bins, read once (independent reads, all in flight)
    uint32_t hv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) hv[j] = j < per ? hbin<kCoherent>(&hist[t * per + j]) : 0u;
    unsigned long long mine = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) mine += hv[j];
    {  // inclusive scan over the 256 partials (pmx_spec.h block_incl_scan)
        __shared__ unsigned long long wsum[4];
        part[t] = block_incl_scan<256>(mine, wsum);
        __syncthreads();
    }
    if (t == 0) {
        s_err = pass == 0 ? 0 : st->err;
        if (pass == 0) {
            const unsigned long long count = part[255];
            st->err = 0;
            st->count = count;
            st->prefix = 0;
            const T q = ratio_dev ? (T)(*ratio_dev) : (T)ratio_host;
            st->ratio = (double)q;
            if (count == 0) {
                s_err = -2;  // PMX_E_EMPTY_QUANTILE: ConvergenceError("no outlier to filter")
            } else if (!ratio_dev && ratio_host == kRatioMedianIndex) {
                st->rank = count / 2;  // nth_element at size / 2 (Matches.cpp:110-120)
            } else if (q < (T)0 || q > (T)1) {
                s_err = -3;  // ConvergenceError("quantile must be between 0 and 1")
            } else if (q == (T)1) {
                st->rank = count - 1;  // max_element
            } else {
                unsigned long long r = (unsigned long long)((T)count * q);
                if (r >= count) r = count - 1;  // reference reads out of range (UB); clamp
                st->rank = r;
            }
            if (s_err) {
                st->err = s_err;
                *iter_err = s_err;
                st->limit = __builtin_nan("");
            }
        }
        s_rank = st->rank;
        // key density around the quantile for the next window (pmx_spec.h):
        // the finest bucket of this select still holding >= 64 keys (the
        // last pass's 2^10-key bucket holds ~1 key for f64)
        if (spec) {
            const unsigned long long cnt = part[255];
            if (pass == 0) spec->dens = -1.0;
            if (cnt >= 64) spec->dens = (double)cnt / ldexp(1.0, shift + bits);
        }
    }
    __syncthreads();
    if (s_err == 0) {
        const unsigned long long rank = s_rank;
        const unsigned long long excl = t > 0 ? part[t - 1] : 0ull;
        if (rank >= excl && rank < part[t]) {
            unsigned long long cum = excl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j >= per) break;
                const unsigned long long c = hv[j];
                if (rank < cum + c) {
                    const K digit = (K)(t * per + j);
                    const K prefix = ((K)st->prefix << bits) | digit;
                    st->prefix = (unsigned long long)prefix;
                    st->rank = rank - cum;
                    if (last) {
                        st->limit = (double)KO::val(prefix);
                        // next iteration's quantile window, centred here
                        if (spec)
                            spec_update<T>(spec, prefix,
                                           spec->dens > 0.0 ? spec->dens : (double)(part[255] + 1) / (double)nb);
                    }
                    break;
                }
                cum += c;
            }
        }
    }
    __syncthreads();
    for (int j = 0; j < per; ++j) hzero<kCoherent>(&hist[t * per + j]);  // ready for the next pass
}

template <typename T>
__global__ __launch_bounds__(256) void select_pick_kernel(uint32_t* __restrict__ hist, SelectState* __restrict__ st,
                                                          int pass, double ratio_host,
                                                          const double* __restrict__ ratio_dev,
                                                          int* __restrict__ iter_err, int last,
                                                          const LoopCtl* __restrict__ ctl,
                                                          SpecSel* __restrict__ spec) {
    __shared__ unsigned long long part[256];
    __shared__ unsigned long long s_rank;
    __shared__ int s_err;
    if (ctl && ctl->done) return;
    if (spec && spec->hit) return;  // the quantile window resolved it (pmx_spec.h)
    pick_phase<T, false>(hist, st, pass, ratio_host, ratio_dev, iter_err, last, part, s_rank, s_err, spec);
}

size_t selx_bytes() { return sizeof(SelX) + (size_t)kSelMaxPasses * 2048 * sizeof(uint32_t); }
int64_t select_all_blocks(int64_t n) { return select_blocks(n); }

template <typename T>
__global__ __launch_bounds__(256) void select_all_kernel(const T* __restrict__ d, int64_t n, SelX* __restrict__ sx,
                                                         SelectState* __restrict__ st, double ratio_host,
                                                         const double* __restrict__ ratio_dev,
                                                         int* __restrict__ iter_err, const LoopCtl* __restrict__ ctl,
                                                         SpecSel* __restrict__ spec,
                                                         const unsigned long long* __restrict__ vpart,
                                                         unsigned long long* __restrict__ vout) {
    if (ctl && ctl->done) return;  // (uniform: no block arrives anywhere)
    select_all_body<T>(d, n, sx, st, ratio_host, ratio_dev, iter_err, spec, vpart, vout);
}

template <typename T>
void launch_select_all(const T* d, int64_t n, void* selx, SelectState* st, double ratio, const double* ratio_dev,
                       int* iter_err, const LoopCtl* ctl, SpecSel* spec, const unsigned long long* vpart,
                       unsigned long long* vout, hipStream_t s) {
    hipLaunchKernelGGL(select_all_kernel<T>, dim3((unsigned)select_blocks(n)), dim3(256), 0, s, d, n, (SelX*)selx, st,
                       ratio, ratio_dev, iter_err, ctl, spec, vpart, vout);
}

template <typename T>
void launch_select_pick(uint32_t* hist, SelectState* st, int pass, double ratio, const double* ratio_dev,
                        int* iter_err, const LoopCtl* ctl, SpecSel* spec, hipStream_t s) {
    const int last = pass == select_passes<T>() - 1;
    hipLaunchKernelGGL(select_pick_kernel<T>, dim3(1), dim3(256), 0, s, hist, st, pass, ratio, ratio_dev,
                       iter_err, last, ctl, spec);
}

static unsigned grid_for(int64_t n) {
    int64_t g = (n + 1023) / 1024;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (unsigned)g;
}

// ============================================================ VarTrimmed ==
// scratch layout (bytes, 256-aligned pieces; launch_vartrim):
//   [hdr: 256 B]         int count, int err, ..., the head's running sum
//   RsHead               the radix sort's histograms and tile counters
//                        (zeroed once at allocation: vartrim_scratch_head)
//   keysA[n], keysB[n]   the keys, then sorted (K)
//   cum[n]               sequential partial sums (T)
//   argmin partials      (kFrmsBlocks values + indices)
//   the radix sort's look-back state, the chunk table, Q_even / Q_odd / P1
//   (8 B per key) and W1 (4 B per key), the walk's trace
// deno: host-computed table pow(id / points_nbr, lambda) in T (the same libm
// call as the reference's Eigen pow, OutlierFiltersImpl.cpp:209)
static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }



// The finite positive distances (OutlierFiltersImpl.cpp:186-188) as sort
// keys in place, every other distance as the all-ones key (sorted after every
// finite positive float's bits); the count of the kept ones.  The LSD radix
// sort of pmx_radix.h then orders all n keys — the kept ones first.
// (with the radix sort's histogram pass folded in, pmx_radix.h rs_hist_block:
// the sort then starts with its first scatter pass)
template <typename T>
__global__ __launch_bounds__(256) void vt_keys_kernel(const T* __restrict__ d, int64_t n,
                                                      typename KeyOf<T>::K* __restrict__ keys, int* __restrict__ count,
                                                      const LoopCtl* __restrict__ ctl, RsHead* __restrict__ rsh,
                                                      unsigned long long* __restrict__ rs_state0,
                                                      int64_t rs_words) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    constexpr int npass = KO::bits / kRsBits;
    static_assert(KO::bits % kRsBits == 0 && npass <= kRsMaxPasses, "whole digits");
    __shared__ int wtot[4], wz[4];
    __shared__ unsigned int h[npass][kRsDigits];
    if (ctl && ctl->done) return;
    for (int p = 0; p < npass; ++p) h[p][threadIdx.x] = 0;
    __syncthreads();
    int c = 0, z = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const T v = d[i];
        const bool keep = v != (T)__builtin_huge_val() && v > (T)0;
        const K key = keep ? KO::key(v) : ~(K)0;
        keys[i] = key;
#pragma unroll
        for (int p = 0; p < npass; ++p) atomicAdd(&h[p][rs_digit<K>(key, p * kRsBits, kRsBits)], 1u);
        c += keep ? 1 : 0;
        z += v == (T)0 ? 1 : 0;  // (finite, not kept: the quantile's population has them)
    }
    for (int off = 32; off > 0; off >>= 1) {
        c += __shfl_xor(c, off);
        z += __shfl_xor(z, off);
    }
    if ((threadIdx.x & 63) == 0) {
        wtot[threadIdx.x >> 6] = c;
        wz[threadIdx.x >> 6] = z;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = (wtot[0] + wtot[1]) + (wtot[2] + wtot[3]);
        const int zt = (wz[0] + wz[1]) + (wz[2] + wz[3]);
        if (tot) atomicAdd(count, tot);
        if (zt) atomicAdd(count + 2, zt);
    }
    rs_hist_block<K>(h, npass, rsh, rs_state0, rs_words);  // (after the barrier above: every bin counted)
}

template <typename K>
static size_t vt_sort_temp_bytes(int64_t n) {
    size_t t = 0;
    (void)pmx_sort_keys(nullptr, t, (const K*)nullptr, (K*)nullptr, (int)std::max<int64_t>(n, 1),
                                            0, (int)(8 * sizeof(K)));
    return t;
}

// std::partial_sum in T with the sequential rounding, computed in parallel.
// The running sum s only grows (sorted positive keys), so it stays in one
// binade [2^e, 2^(e+1)) for long stretches, where every sum is a multiple of
// u = ulp(2^e) and one IEEE step is exactly
//     fl(s + x) = s + u * rnd(x / u)      (rnd: nearest; a tie, x / u = m + 1/2,
//                                          goes to the even result: parity of s/u + m)
// as long as the result stays below 2^(e+1).  So inside a binade the sums are
// S_j = S_0 + P_j + C_j in units of u: P_j an integer prefix sum of rnd(x/u)
// (ties counted as m), C_j the ties that rounded up, resolved in order by one
// thread from the parity of the sum before each (ties are rare).  The first
// step whose result reaches 2^(e+1) is done as a plain T addition, and the
// next stretch starts in the new binade.  Bit-identical to the sequential
// loop for any input; a chunk with more ties than the LDS list holds is
// summed sequentially.  One block of kCumThreads, chunks of kCumThreads *
// kCumPer keys.
constexpr int kCumThreads = 1024;
// (4 keys per thread: 4 K-key chunks — a chunk then rarely holds two binade
// crossings, and the preparation runs on 4x as many blocks; 16 K chunks put
// the first ~5 crossings after the head into one chunk, walked with one
// block-wide pass per crossing)
constexpr int kCumPer = 4;
constexpr int kCumMaxTies = 1024;
template <typename T>
struct CumBits;
template <>
struct CumBits<float> {
    static constexpr int P = 24;  // significand bits
    static __device__ __forceinline__ float min_normal() { return 1.17549435e-38f; }
    static __device__ __forceinline__ int binade(float s) { return (int)((__float_as_uint(s) >> 23) & 0xffu) - 127; }
    // s / ulp(2^binade): the significand with its hidden bit (s normal)
    static __device__ __forceinline__ long long units(float s) {
        return (long long)((__float_as_uint(s) & 0x7fffffu) | 0x800000u);
    }
};
template <>
struct CumBits<double> {
    static constexpr int P = 53;
    static __device__ __forceinline__ double min_normal() { return 2.2250738585072014e-308; }
    static __device__ __forceinline__ int binade(double s) {
        return (int)(((unsigned long long)__double_as_longlong(s) >> 52) & 0x7ffull) - 1023;
    }
    static __device__ __forceinline__ long long units(double s) {
        return (long long)(((unsigned long long)__double_as_longlong(s) & 0xfffffffffffffull) | (1ull << 52));
    }
};
__device__ __forceinline__ long long sat_add(long long a, long long b, long long lim) {
    const long long v = a + b;
    return v < lim ? v : lim;
}
// exclusive saturating scan over the block (values and result <= lim; a
// saturating add is associative, so every unsaturated prefix is exact).  The
// exclusive value is the previous lane's inclusive one, not incl - v: a
// thread whose own total saturates (its keys reach the crossing) still needs
// the exact prefix before it for its keys ahead of the crossing.
__device__ __forceinline__ long long cum_block_scan(long long v, long long lim, long long* wsum, long long& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long u = __shfl_up(incl, off);
        if (lane >= off) incl = sat_add(incl, u, lim);
    }
    long long ex = __shfl_up(incl, 1);
    if (lane == 0) ex = 0;
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    long long before = 0;
    total = 0;
    for (int w = 0; w < kCumThreads / 64; ++w) {
        before = w < wave ? sat_add(before, wsum[w], lim) : before;
        total = sat_add(total, wsum[w], lim);
    }
    __syncthreads();
    return sat_add(before, ex, lim);
}

// The head (the first kCumHead keys, where the running sum leaves its binade
// every few keys) is summed sequentially; the rest is cut into chunks of
// kCumChunk keys.  vt_chunk_prep_kernel prepares every chunk in parallel
// under the binade e GUESSED from a double prefix of the chunk sums, and under
// e + 1: per key the integer prefix of rnd(x / u), with binade e's ties
// already resolved for an even and for an odd start (Q_even, Q_odd) and binade
// e + 1's ties counted as m (P1) beside a word locating the e + 1 ties (W1).
// The ties resolve in parallel: tie k rounds up iff the units before it plus
// m_k are odd, and with d_k = parity(pb_k + m_k) (pb_k: the prefix before the
// tie, ties counted as m) the first tie after a start of parity B rounds up
// iff B ^ d_k, every later one iff d_k ^ d_(k-1) — independent of the start,
// so a prefix count D_k of those changes gives every tie's rounding for either
// start parity.  vt_cumsum_kernel then walks the chunks in order with the
// exact running sum S, wave 0 alone:
//   fast   S in binade e, S / u + Q[end] < 2^P: the chunk's end sum in O(1)
//          from the chunk table (preloaded in LDS), 64 chunks per step;
//   cross  the sum leaves binade e inside the chunk: the crossing step (the
//          first j with S / u + Q[j] >= 2^P, a two-level search of the stored
//          Q, 64 keys per level) is a plain T addition, and when it lands in
//          binade e + 1 and the rest of the chunk stays there, the rest's sums
//          are the e + 1 prefix from there (its ties by the D_k rule);
//   slow   anything else (a wrong guess, many ties, two crossings, a
//          subnormal sum): the block's passes below, which write the chunk.
// vt_chunk_write_kernel writes the fast and crossing chunks' sums in
// parallel.  Every path computes the sequential loop's bits.
constexpr int kCumChunk = kCumThreads * kCumPer;
// (the head is summed by the preparation launch's extra block while the
// other blocks prepare their chunks; 8 K measured slower: the serial sum of
// the head, ~10 ns per key, outlasts the passes it saves)
constexpr int kCumHead = 4096;
constexpr int kFastTies = 256;
constexpr int kChunkLds = 512;  // chunk-table entries the walk preloads into LDS

// the prefixes saturate here (a chunk far above its guessed binade would
// overflow 64 bits; any value this large only says "past 2^P")
constexpr long long kCumCap = 1ll << 61;

struct VtChunk {
    double sum;       // double sum of the chunk's keys (the guess)
    long long P[2];   // integer totals under binades e and e + 1 (ties as m; saturated at kCumCap)
    long long C[2];   // binade e: ties rounded up over the chunk, for an even / odd start
    double S0;        // exact start sum (T value): fast and crossing chunks
    double S1;        // crossing: the sum after the crossing step
    int e;            // guessed binade
    int nt[2];        // ties under e, e + 1 (kFastTies + 1: too many)
    int D1;           // binade e + 1: D_k of the chunk's last tie
    int ok;           // 0: the passes wrote it; 1 fast; 2 crossing
    int par;          // parity of S0 / u
    int jc;           // crossing: chunk-local index of the crossing step
    int k0, r0, Dk0;  // crossing: the first e + 1 tie after jc, its rounding, D_k0
};

// the per-key arrays of the prepared chunks, index j - kCumHead
// (launch_vartrim lays them out)
struct VtPrep {
    long long* Q[2];  // binade e: units added by keys up to j, ties resolved, even / odd start
    long long* P1;    // binade e + 1: inclusive prefix, ties counted as m
    int* W1;          // binade e + 1 ties up to j: count | d_next << 9 | d_last << 10 | D_last << 11
};

constexpr int kVtTraceMax = 2048;  // (development trace of the walk: marks, then the count)

static int64_t vt_chunks(int64_t n) { return n > kCumHead ? (n - kCumHead + kCumChunk - 1) / kCumChunk : 0; }

// the part of the VarTrimmed scratch that must be zero when it is allocated
// (the radix sort's persistent counters); bytes from the scratch's start
size_t vartrim_scratch_head() { return 256 + al256(sizeof(RsHead)); }

template <typename T>
size_t vartrim_scratch_bytes(int64_t n) {
    using K = typename KeyOf<T>::K;
    const int64_t nch = vt_chunks(n);
    return 256 + al256(sizeof(RsHead)) + 2 * al256(sizeof(K) * n) + al256(sizeof(T) * n) + 2 * al256(8 * 256) +
           al256(rs_state_bytes(n)) + al256(sizeof(VtChunk) * (nch + 1)) + 3 * al256(8 * (size_t)n) +
           al256(4 * (size_t)n) + al256(8 * (2 * (size_t)kVtTraceMax + 1));
}

// this thread's kCumPer keys from j0 (16-byte loads when in range)
template <typename T>
__device__ __forceinline__ void vt_load(const typename KeyOf<T>::K* __restrict__ keys, int64_t c, int64_t j0,
                                        typename KeyOf<T>::K (&kv)[kCumPer]) {
    using K = typename KeyOf<T>::K;
    if (j0 + kCumPer <= c) {
        using V = typename std::conditional<sizeof(K) == 4, uint4, ulonglong2>::type;
        constexpr int E = 16 / sizeof(K);
        const V* vp = reinterpret_cast<const V*>(keys + j0);
#pragma unroll
        for (int w = 0; w < kCumPer / E; ++w) {
            const V x = vp[w];
            const K* xe = reinterpret_cast<const K*>(&x);
#pragma unroll
            for (int e = 0; e < E; ++e) kv[w * E + e] = xe[e];
        }
    } else {
#pragma unroll
        for (int i = 0; i < kCumPer; ++i) kv[i] = j0 + i < c ? keys[j0 + i] : (K)0;
    }
}

// 1 / u = 2^sh as two finite factors: in double's lowest binades sh reaches
// 1075 (u = 2^-1074), beyond the largest double power of two; x * a * b is
// still exact (power-of-two scalings of a value that stays in range)
struct UScale {
    double a, b;
};
__device__ __forceinline__ UScale uscale(int sh) {
    const int h = sh > 1000 ? 1000 : sh;
    return {ldexp(1.0, h), ldexp(1.0, sh - h)};
}

// x / u rounded to nearest (a tie counted as m and flagged) for the active
// keys [p, q1); returns the thread's saturated total
template <typename T>
__device__ __forceinline__ long long vt_round(const typename KeyOf<T>::K (&kv)[kCumPer], int64_t j0, int64_t p,
                                              int64_t q1, UScale inv_u, long long (&r)[kCumPer],
                                              bool (&tie)[kCumPer], int& ntie) {
    using KO = KeyOf<T>;
    constexpr long long LIM = 1ll << CumBits<T>::P;
    long long loc = 0;
    ntie = 0;
#pragma unroll
    for (int i = 0; i < kCumPer; ++i) {
        const int64_t j = j0 + i;
        r[i] = 0;
        tie[i] = false;
        if (j >= p && j < q1) {
            const double q = ((double)KO::val(kv[i]) * inv_u.a) * inv_u.b;  // exact (power-of-two scales)
            if (!(q < (double)LIM)) {
                r[i] = LIM;  // (this step alone leaves the binade)
            } else {
                const double m = floor(q), f = q - m;
                tie[i] = f == 0.5;
                r[i] = (long long)m + (f > 0.5 ? 1 : 0);
            }
        }
        loc = sat_add(loc, r[i], LIM);
        ntie += tie[i] ? 1 : 0;
    }
    return loc;
}

// chunk sums in double (block 0: the head; block b + 1: chunk b)
template <typename T>
__global__ __launch_bounds__(kCumThreads) void vt_chunk_sum_kernel(const typename KeyOf<T>::K* __restrict__ keys,
                                                                   const int* __restrict__ count,
                                                                   VtChunk* __restrict__ ch,
                                                                   const LoopCtl* __restrict__ ctl) {
    using KO = KeyOf<T>;
    __shared__ double ws[kCumThreads / 64];
    if (ctl && ctl->done) return;
    const int64_t c = *count;
    const int64_t lo = blockIdx.x == 0 ? 0 : kCumHead + (int64_t)(blockIdx.x - 1) * kCumChunk;
    const int64_t hi = blockIdx.x == 0 ? (c < kCumHead ? c : kCumHead) : (lo + kCumChunk < c ? lo + kCumChunk : c);
    if (lo >= hi) return;
    double v = 0.0;
    for (int64_t j = lo + threadIdx.x; j < hi; j += kCumThreads) v += (double)KO::val(keys[j]);
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < kCumThreads / 64; ++w) t += ws[w];
        ch[blockIdx.x].sum = t;
    }
}

// exclusive scan of int64 values over the block (no saturation: the chunk
// totals stay below 2^38); wsum: kCumThreads / 64 entries
__device__ __forceinline__ long long block_excl_scan_ll(long long v, long long* wsum, long long& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long u = __shfl_up(incl, off);
        if (lane >= off) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    long long before = 0;
    total = 0;
    for (int w = 0; w < kCumThreads / 64; ++w) {
        before += w < wave ? wsum[w] : 0ll;
        total += wsum[w];
    }
    __syncthreads();
    return before + (incl - v);
}

// per chunk: the guessed binade e; under e and e + 1 the inclusive prefixes,
// the totals and the ties; binade e's ties resolved for both start parities
// The head's sums (std::partial_sum's first kCumHead steps, sequentially in
// T): keys staged in LDS by the block, one thread sums into LDS (no global
// store in the serial loop), the block writes them out coalesced.  head_out
// = the running sum after the head, for the walk.
template <typename T>
__device__ __forceinline__ void vt_cum_head(const typename KeyOf<T>::K* __restrict__ keys, int64_t c,
                                            T* __restrict__ cum, T* __restrict__ head_out) {
    using KO = KeyOf<T>;
    __shared__ __attribute__((aligned(16))) T s_h[kCumHead];
    const int ph = c < kCumHead ? (int)c : kCumHead;
    for (int j = threadIdx.x; j < ph; j += kCumThreads) s_h[j] = KO::val(keys[j]);
    __syncthreads();
    if (threadIdx.x == 0) {
        // Batches of 16 keys in 16-byte LDS vectors, software-pipelined: the
        // next batch's loads are issued before this batch's dependent adds
        // and its stores (LDS operations complete in order, so a store queued
        // ahead of a load would make the load's wait cover it too); the adds
        // then hide the load latency.  acc starts at -0: -0 + x0 = x0 exactly,
        // partial_sum's first output.
        using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
        constexpr int E = 16 / sizeof(T), NV = 16 / E;
        V* hv = reinterpret_cast<V*>(s_h);
        T acc = (T)-0.0;
        const int nb = ph / 16;
        V cur[NV], nxt[NV];
        if (nb > 0) {
#pragma unroll
            for (int w = 0; w < NV; ++w) cur[w] = hv[w];
        }
        for (int bt = 0; bt < nb; ++bt) {
            if (bt + 1 < nb) {
#pragma unroll
                for (int w = 0; w < NV; ++w) nxt[w] = hv[(bt + 1) * NV + w];
            }
#pragma unroll
            for (int w = 0; w < NV; ++w) {
                T* x = reinterpret_cast<T*>(&cur[w]);
#pragma unroll
                for (int q = 0; q < E; ++q) {
                    acc = acc + x[q];
                    x[q] = acc;
                }
            }
#pragma unroll
            for (int w = 0; w < NV; ++w) hv[bt * NV + w] = cur[w];
#pragma unroll
            for (int w = 0; w < NV; ++w) cur[w] = nxt[w];
        }
        for (int j = nb * 16; j < ph; ++j) {
            acc = acc + s_h[j];
            s_h[j] = acc;
        }
        *head_out = acc;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < ph; j += kCumThreads) cum[j] = s_h[j];
}

template <typename T>
__global__ __launch_bounds__(kCumThreads) void vt_chunk_prep_kernel(const typename KeyOf<T>::K* __restrict__ keys,
                                                                    const int* __restrict__ count,
                                                                    VtChunk* __restrict__ ch, VtPrep pr,
                                                                    const LoopCtl* __restrict__ ctl,
                                                                    T* __restrict__ cum, T* __restrict__ head_out) {
    using K = typename KeyOf<T>::K;
    constexpr int P = CumBits<T>::P;
    __shared__ long long wsum[kCumThreads / 64];
    __shared__ double s_approx;
    __shared__ double wsd[kCumThreads / 64];
    __shared__ int l_d[kFastTies], l_D[kFastTies];
    static_assert(kFastTies <= kCumThreads, "one tie per thread");
    if (ctl && ctl->done) return;
    const int64_t c = *count;
    const int b = blockIdx.x, t = threadIdx.x;
    if (b == (int)gridDim.x - 1 && cum) {  // (the extra block: the head, vt_cum_head)
        vt_cum_head<T>(keys, c, cum, head_out);
        return;
    }
    const int64_t lo = kCumHead + (int64_t)b * kCumChunk;
    if (lo >= c) return;
    const int64_t hi = lo + kCumChunk < c ? lo + kCumChunk : c;
    {
        // the head and every earlier chunk: an estimate of the running sum
        // (its binade is only a guess the walk verifies: any order will do;
        // a fixed one keeps it deterministic), the block's threads in parallel
        double a = 0.0;
        for (int i = t; i <= b; i += kCumThreads) a += ch[i].sum;
        for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
        if ((t & 63) == 0) wsd[t >> 6] = a;
        __syncthreads();
        if (t == 0) {
            double s2 = 0.0;
            for (int w = 0; w < kCumThreads / 64; ++w) s2 += wsd[w];
            s_approx = s2;
        }
    }
    __syncthreads();
    const int e = CumBits<T>::binade((T)s_approx);
    const int64_t j0 = lo + (int64_t)t * kCumPer;
    K kv[kCumPer];
    vt_load<T>(keys, c, j0, kv);
    for (int v = 0; v < 2; ++v) {  // (uniform) binade e, then e + 1
        const UScale inv_u = uscale(P - 1 - (e + v));
        long long r[kCumPer];
        bool tie[kCumPer];
        int ntie;
        (void)vt_round<T>(kv, j0, lo, hi, inv_u, r, tie, ntie);
        long long loc = 0;
#pragma unroll
        for (int i = 0; i < kCumPer; ++i) loc = sat_add(loc, r[i], kCumCap);
        long long tot, tt;
        long long run = cum_block_scan(loc, kCumCap, wsum, tot);
        const long long tbase = block_excl_scan_ll((long long)ntie, wsum, tt);
        const int nt = tt <= kFastTies ? (int)tt : kFastTies + 1;
        if (nt <= kFastTies) {  // each tie's d = parity of (the prefix before it + m)
            int k = (int)tbase;
            long long pb = run;
#pragma unroll
            for (int i = 0; i < kCumPer; ++i) {
                if (tie[i]) l_d[k++] = (int)((pb + r[i]) & 1ll);
                pb = sat_add(pb, r[i], kCumCap);
            }
        }
        __syncthreads();
        {  // D_k: the changes of d over ties 1..k, one tie per thread
            const long long x = t > 0 && t < nt && nt <= kFastTies ? (long long)(l_d[t] ^ l_d[t - 1]) : 0ll;
            long long xt;
            const long long ex = block_excl_scan_ll(x, wsum, xt);
            if (t < nt && nt <= kFastTies) l_D[t] = (int)(ex + x);
        }
        __syncthreads();
        if (nt <= kFastTies) {
            const int d0 = nt > 0 ? l_d[0] : 0;
            int kt = (int)tbase;  // ties at or before the key
#pragma unroll
            for (int i = 0; i < kCumPer; ++i) {
                run = sat_add(run, r[i], kCumCap);
                kt += tie[i] ? 1 : 0;
                const int64_t j = j0 + i;
                if (j >= hi) continue;
                if (v == 0) {  // the rounded-up ties so far, for an even / odd start
                    const long long D = kt > 0 ? (long long)l_D[kt - 1] : 0ll;
                    pr.Q[0][j - kCumHead] = run + (kt > 0 ? (long long)d0 + D : 0ll);
                    pr.Q[1][j - kCumHead] = run + (kt > 0 ? (long long)(1 ^ d0) + D : 0ll);
                } else {
                    pr.P1[j - kCumHead] = run;
                    const int dn = kt < nt ? l_d[kt] : 0, dl = kt > 0 ? l_d[kt - 1] : 0;
                    const int Dl = kt > 0 ? l_D[kt - 1] : 0;
                    pr.W1[j - kCumHead] = kt | (dn << 9) | (dl << 10) | (Dl << 11);
                }
            }
        }
        if (t == 0) {
            ch[b + 1].P[v] = tot;
            ch[b + 1].nt[v] = nt;
            const int Dt = nt > 0 && nt <= kFastTies ? l_D[nt - 1] : 0;
            if (v == 0) {
                const int d0 = nt > 0 && nt <= kFastTies ? l_d[0] : 0;
                ch[b + 1].C[0] = nt > 0 ? d0 + Dt : 0;
                ch[b + 1].C[1] = nt > 0 ? (1 ^ d0) + Dt : 0;
            } else {
                ch[b + 1].D1 = Dt;
            }
        }
        __syncthreads();  // (the LDS tie list is rewritten for e + 1)
    }
    if (t == 0) {
        ch[b + 1].e = e;
        ch[b + 1].ok = 0;
    }
}

// the fast and crossing chunks' sums: S0 + Q_par[j] in units of binade e,
// then after a crossing S1 + (P1[j] - P1[jc]) + the rest's rounded-up ties in
// units of binade e + 1
template <typename T>
__global__ __launch_bounds__(kCumThreads) void vt_chunk_write_kernel(const typename KeyOf<T>::K* __restrict__ keys,
                                                                     const int* __restrict__ count,
                                                                     const VtChunk* __restrict__ ch, VtPrep pr,
                                                                     T* __restrict__ cum,
                                                                     const LoopCtl* __restrict__ ctl) {
    constexpr int P = CumBits<T>::P;
    (void)keys;
    if (ctl && ctl->done) return;
    const int64_t c = *count;
    const int b = blockIdx.x, t = threadIdx.x;
    const int64_t lo = kCumHead + (int64_t)b * kCumChunk;
    if (lo >= c) return;
    const VtChunk q = ch[b + 1];
    if (!q.ok) return;  // (uniform: the passes wrote this chunk)
    const int64_t hi = lo + kCumChunk < c ? lo + kCumChunk : c;
    const int jc = q.ok == 2 ? q.jc : 0x7fffffff;
    const double u0 = ldexp(1.0, q.e - (P - 1)), u1 = ldexp(1.0, q.e + 1 - (P - 1));
    const long long U0 = CumBits<T>::units((T)q.S0);
    const long long U1 = q.ok == 2 ? CumBits<T>::units((T)q.S1) : 0;
    const long long P1jc = q.ok == 2 ? pr.P1[lo + jc - kCumHead] : 0;
    const long long* __restrict__ Q = pr.Q[q.par];
#pragma unroll
    for (int i = 0; i < kCumPer; ++i) {
        const int li = t * kCumPer + i;
        const int64_t j = lo + li;
        if (j >= hi) continue;
        T v;
        if (li < jc) {
            v = (T)((double)(U0 + Q[j - kCumHead]) * u0);
        } else if (li == jc) {
            v = (T)q.S1;
        } else {
            const int w = pr.W1[j - kCumHead];
            const int kt = w & 0x1ff;
            const long long ups = kt > q.k0 ? (long long)(q.r0 + (w >> 11) - q.Dk0) : 0ll;
            v = (T)((double)(U1 + (pr.P1[j - kCumHead] - P1jc) + ups) * u1);
        }
        cum[j] = v;
    }
}

int g_vt_trace = 0;
template <typename T>
__global__ __launch_bounds__(kCumThreads) void vt_cumsum_kernel(const typename KeyOf<T>::K* __restrict__ keys,
                                                                const int* __restrict__ count, T* __restrict__ cum,
                                                                VtChunk* __restrict__ ch, VtPrep pr, int nch,
                                                                const LoopCtl* __restrict__ ctl,
                                                                unsigned long long* __restrict__ trace,
                                                                const T* __restrict__ head_in) {
    using KO = KeyOf<T>;
    // (development trace, PMX_VT_TRACE: thread 0 stamps each step of the walk
    // with the 100 MHz real-time counter; pmx_vartrim_partial_sums prints it)
    int nmark = 0;
#define VT_MARK(type, bb, detail)                                                                               \
    if (trace && threadIdx.x == 0 && nmark < kVtTraceMax) {                                                     \
        trace[2 * nmark] = __builtin_amdgcn_s_memrealtime();                                                    \
        trace[2 * nmark + 1] = ((unsigned long long)(type) << 56) | ((unsigned long long)(unsigned)(bb) << 24) | \
                               ((unsigned long long)(detail) & 0xffffffull);                                    \
        ++nmark;                                                                                                \
    }
    constexpr int P = CumBits<T>::P;
    constexpr long long LIM = 1ll << P;
    __shared__ long long wsum[kCumThreads / 64];
    __shared__ int s_nt;
    __shared__ int tie_idx[kCumMaxTies];        // chunk-local index, in order
    __shared__ long long tie_pb[kCumMaxTies];   // P before the tie (ties counted as m)
    __shared__ long long tie_m[kCumMaxTies];
    __shared__ int tie_c[kCumMaxTies];          // rounded-up ties up to and including this one
    __shared__ int s_cross;
    __shared__ long long s_lo;                  // the walk's position (chunk start, chunk)
    __shared__ int s_b;
    __shared__ T s_run;                         // the running sum after the chunk
    // the chunk table of the fast test (the walk's per-chunk decision then
    // reads no global memory)
    __shared__ long long c_P0[kChunkLds], c_C[2][kChunkLds], c_P1[kChunkLds];
    __shared__ int c_e[kChunkLds], c_nt0[kChunkLds], c_nt1[kChunkLds], c_D1[kChunkLds];
    if (ctl && ctl->done) return;
    const int t = threadIdx.x;
    const int64_t c = *count;
    if (c <= 0) return;
    const int nchl = nch < kChunkLds ? nch : kChunkLds;
    for (int i = t; i < nchl; i += kCumThreads) {
        const VtChunk& q = ch[i + 1];
        c_P0[i] = q.P[0];
        c_C[0][i] = q.C[0];
        c_C[1][i] = q.C[1];
        c_e[i] = q.e;
        c_nt0[i] = q.nt[0];
        c_P1[i] = q.P[1];
        c_nt1[i] = q.nt[1];
        c_D1[i] = q.D1;
    }
    // the head: summed (and written) by the preparation launch's extra block
    // when there are chunks (head_in), else here, the same way
    const int ph = c < kCumHead ? (int)c : kCumHead;
    if (head_in) {
        if (t == 0) s_run = *head_in;
    } else {
        vt_cum_head<T>(keys, c, cum, &s_run);
    }
    VT_MARK(1, 0, ph);
    __syncthreads();
    T s = s_run;
    __syncthreads();
    // The walk.  Wave 0 settles runs of fast chunks and the crossings
    // between them (no block barrier: one per chunk made the ~250 fast
    // chunks of a 1M sum most of the walk); the block then takes the first
    // chunk that is neither, through the passes.
    int64_t lo = ph;
    int b = 0;
    while (lo < c) {  // (uniform)
        if (t < 64) {
            // Fast chunks, 64 per step: the guessed binade is the running
            // sum's, few ties, and the chunk's last sum stays below the next
            // binade.  The run stays in S's binade es, so chunk i's start
            // units are U + the increments of the chunks before it, an
            // integer prefix sum, and each increment Q_par[end] = P0 +
            // C[parity] depends on the parity of its start only: the
            // parities are a prefix composition of 1-bit maps (p -> p ^
            // parity(P0 + C_p)).  Bit-identical to the chunk-by-chunk walk.
            const int lane = t;
            T sr = s;
            if (sr >= CumBits<T>::min_normal()) {
                int es = CumBits<T>::binade(sr);
                double u = ldexp(1.0, es - (P - 1));
                long long U = CumBits<T>::units(sr);
                for (;;) {  // (wave-uniform)
                    const int bi = b + lane;
                    const int64_t loi = lo + (int64_t)lane * kCumChunk;
                    int e = 0, nt0 = kFastTies + 1;
                    long long P0 = 0, C0 = 0, C1 = 0;
                    if (loi < c) {
                        if (bi < kChunkLds) {
                            e = c_e[bi];
                            nt0 = c_nt0[bi];
                            P0 = c_P0[bi];
                            C0 = c_C[0][bi];
                            C1 = c_C[1][bi];
                        } else {
                            const VtChunk& g = ch[bi + 1];
                            e = g.e;
                            nt0 = g.nt[0];
                            P0 = g.P[0];
                            C0 = g.C[0];
                            C1 = g.C[1];
                        }
                    }
                    const bool valid = loi < c && nt0 <= kFastTies && e == es;
                    // this chunk's parity map as (image of 0, image of 1)
                    int f0 = (int)((P0 + C0) & 1ll), f1 = 1 ^ (int)((P0 + C1) & 1ll);
                    // exclusive prefix composition (lane i: the map from the
                    // window's start parity to chunk i's start parity)
                    int g0 = 0, g1 = 1;  // identity
                    {
                        int a0 = f0, a1 = f1;  // inclusive composition, scanned
#pragma unroll
                        for (int off = 1; off < 64; off <<= 1) {
                            const int b0 = __shfl_up(a0, off), b1 = __shfl_up(a1, off);
                            if (lane >= off) {  // a = a o b (b first)
                                const int n0 = b0 ? a1 : a0, n1 = b1 ? a1 : a0;
                                a0 = n0;
                                a1 = n1;
                            }
                        }
                        const int p0 = __shfl_up(a0, 1), p1 = __shfl_up(a1, 1);
                        if (lane > 0) {
                            g0 = p0;
                            g1 = p1;
                        }
                    }
                    const int par0 = (int)(U & 1ll);
                    const int par = par0 ? g1 : g0;
                    // (clamped: an increment of 2^P ends the run anyway; 64 of
                    // them stay far from overflow)
                    long long inc = P0 + (par ? C1 : C0);
                    inc = inc < LIM ? inc : LIM;
                    long long incl = inc;
#pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const long long v2 = __shfl_up(incl, off);
                        if (lane >= off) incl += v2;
                    }
                    const long long Ui = U + (incl - inc), fin = U + incl;
                    const bool stop = !valid || fin >= LIM;
                    const unsigned long long sm = __ballot(stop);
                    const int first = sm ? __builtin_ctzll(sm) : 64;
                    if (lane < first) {
                        VtChunk& q = ch[bi + 1];
                        q.S0 = (double)Ui * u;  // (the T value of the start sum, exactly)
                        q.par = par;
                        q.ok = 1;
                    }
                    if (first == 64) {
                        U = __shfl(fin, 63);
                        lo += (int64_t)64 * kCumChunk;
                        b += 64;
                        if (lo >= c) break;
                        continue;
                    }
                    const long long Uf = __shfl(Ui, first);
                    const int parf = __shfl(par, first);
                    const int vf = __shfl(valid ? 1 : 0, first);
                    U = Uf;
                    lo += (int64_t)first * kCumChunk;
                    b += first;
                    if (!vf) break;  // (the passes)
                    // A valid chunk whose end leaves the binade: the crossing.
                    int nt1, D1;
                    long long P1t;
                    if (b < kChunkLds) {
                        nt1 = c_nt1[b];
                        D1 = c_D1[b];
                        P1t = c_P1[b];
                    } else {
                        const VtChunk& g = ch[b + 1];
                        nt1 = g.nt[1];
                        D1 = g.D1;
                        P1t = g.P[1];
                    }
                    if (nt1 > kFastTies || P1t >= kCumCap) break;
                    const int64_t cend = lo + kCumChunk < c ? lo + kCumChunk : c;
                    const int nl = (int)(cend - lo);
                    const long long* __restrict__ Q = pr.Q[parf] + (lo - kCumHead);
                    const long long need = LIM - Uf;  // the crossing: the first key with Q >= need
                    // the 64-key segment holding it (Q is non-decreasing; the
                    // chunk's last Q reaches need), then the key in it
                    long long v1 = 0;
                    if (64 * lane < nl) v1 = Q[64 * lane + 63 < nl ? 64 * lane + 63 : nl - 1];
                    const unsigned long long m1 = __ballot(64 * lane < nl && v1 >= need);
                    const int sg = m1 ? __builtin_ctzll(m1) : 0;
                    const int pos = 64 * sg + lane;
                    long long q2 = 0, p1 = 0;
                    int w1 = 0;
                    typename KO::K kx = 0;
                    if (pos < nl) {
                        q2 = Q[pos];
                        p1 = pr.P1[lo - kCumHead + pos];
                        w1 = pr.W1[lo - kCumHead + pos];
                        kx = keys[lo + pos];
                    }
                    const unsigned long long m2 = __ballot(pos < nl && q2 >= need);
                    if (!m1 || !m2) break;  // (not reached: Q's last value reaches need)
                    const int li = __builtin_ctzll(m2);
                    const int jc = 64 * sg + li;
                    const long long qin = __shfl(q2, li > 0 ? li - 1 : 0);
                    const long long qseg = __shfl(v1, sg > 0 ? sg - 1 : 0);
                    const long long qb = li > 0 ? qin : qseg;  // Q before the crossing (jc > 0)
                    const T before = (T)((double)(Uf + (jc > 0 ? qb : 0ll)) * u);
                    const T S1 = before + KO::val(__shfl(kx, li));  // the crossing step, in T
                    if (!(S1 >= CumBits<T>::min_normal()) || CumBits<T>::binade(S1) != es + 1) break;
                    // the rest of the chunk in binade e + 1: its ties from k0,
                    // the first after jc (r0 its rounding, then the D_k rule)
                    const long long U1 = CumBits<T>::units(S1);
                    const long long P1jc = __shfl(p1, li);
                    const int w = __shfl(w1, li);
                    const int k0 = w & 0x1ff, dn = (w >> 9) & 1, dl = (w >> 10) & 1, Dl = w >> 11;
                    const int Dk0 = k0 > 0 ? Dl + (dn ^ dl) : 0;
                    const int r0 = (int)((U1 - P1jc) & 1ll) ^ dn;
                    const long long ups = k0 < nt1 ? (long long)(r0 + D1 - Dk0) : 0ll;
                    const long long fin1 = U1 + (P1t - P1jc) + ups;
                    if (fin1 >= LIM) break;  // (a second crossing: the passes)
                    if (lane == 0) {
                        VtChunk& q = ch[b + 1];
                        q.S0 = (double)Uf * u;
                        q.par = parf;
                        q.jc = jc;
                        q.S1 = (double)S1;
                        q.k0 = k0;
                        q.r0 = r0;
                        q.Dk0 = Dk0;
                        q.ok = 2;
                    }
                    VT_MARK(3, b, jc);
                    es += 1;
                    u = ldexp(1.0, es - (P - 1));
                    U = fin1;
                    lo += kCumChunk;
                    b += 1;
                    if (lo >= c) break;
                }
                sr = (T)((double)U * u);
            }
            if (lane == 0) {
                s_run = sr;
                s_lo = lo;
                s_b = b;
                s_cross = 0x7fffffff;
            }
            VT_MARK(2, b, 0);
        }
        __syncthreads();
        s = s_run;
        lo = s_lo;
        b = s_b;
        __syncthreads();  // (read before thread 0 rewrites them)
        if (lo >= c) break;
        const int64_t cend = lo + kCumChunk < c ? lo + kCumChunk : c;
        int64_t p = lo;
        while (p < cend) {  // (uniform) passes over [p, cend)
            VT_MARK(4, b, p - lo);
            const int eb = CumBits<T>::binade(s);
            const UScale inv_u = uscale(P - 1 - eb);  // 1 / ulp(2^eb)
            const double u = ldexp(1.0, eb - (P - 1));
            const long long S0 = CumBits<T>::units(s);  // in [2^(P-1), 2^P)
            // the pass starts at p rounded down to a multiple of kCumPer (each
            // thread's keys then come in 16-byte vector loads); keys below p
            // are inactive (contribute 0, written earlier)
            const int64_t jb = p & ~(int64_t)(kCumPer - 1);
            const int64_t q1 = jb + (int64_t)kCumChunk < cend ? jb + (int64_t)kCumChunk : cend;
            if (!(s >= CumBits<T>::min_normal())) {
                // a subnormal running sum (every key so far below the
                // smallest normal): units() would add a hidden bit s does not
                // have — this pass sequentially, exactly as partial_sum
                if (t == 0) {
                    T acc = s;
                    for (int64_t j = p; j < q1; ++j) {
                        acc = acc + KO::val(keys[j]);
                        cum[j] = acc;
                    }
                    s_run = acc;
                }
                __syncthreads();
                s = s_run;
                p = q1;
                __syncthreads();
                continue;
            }
            const int64_t j0 = jb + (int64_t)t * kCumPer;
            typename KO::K kv[kCumPer];
            vt_load<T>(keys, c, j0, kv);
            long long r[kCumPer];
            bool tie[kCumPer];
            int ntie;
            const long long loc = vt_round<T>(kv, j0, p, q1, inv_u, r, tie, ntie);
            long long tot;
            const long long base = cum_block_scan(loc, LIM, wsum, tot);
            // the ties, in element order, with the P before each
            long long tt;
            const long long tbase = cum_block_scan((long long)ntie, LIM, wsum, tt);
            if (t == 0) s_nt = (int)tt;
            if (tt <= kCumMaxTies) {
                long long run = base;
                int k = (int)tbase;
#pragma unroll
                for (int i = 0; i < kCumPer; ++i) {
                    if (tie[i]) {
                        tie_idx[k] = t * kCumPer + i;
                        tie_pb[k] = run;
                        tie_m[k] = r[i];
                        ++k;
                    }
                    run = sat_add(run, r[i], LIM);
                }
            }
            __syncthreads();
            const int nt = s_nt;
            if (nt > kCumMaxTies) {
                // (many ties: this pass sequentially, exactly as partial_sum)
                if (t == 0) {
                    T acc = s;
                    for (int64_t j = p; j < q1; ++j) {
                        acc = acc + KO::val(keys[j]);
                        cum[j] = acc;
                    }
                    s_run = acc;
                }
                __syncthreads();
                s = s_run;
                p = q1;
                __syncthreads();
                continue;
            }
            // the ties' rounding, in parallel: tie k rounds up iff the units
            // before it plus m_k are odd, i.e. c_k ^ parity(up_(k-1)) with
            // c_k = (S0 + pb_k + m_k) & 1 — and then parity(up_k) = c_k.  So
            // tie k rounds up iff c_k != c_(k-1) (c_(-1) = 0), and up_k is a
            // prefix sum of those (a serial loop over the ties before; past a
            // crossing the saturated values are as meaningless either way)
            {
                static_assert(kCumMaxTies <= kCumThreads, "one tie per thread");
                const int ck = t < nt ? (int)((S0 + tie_pb[t] + tie_m[t]) & 1ll) : 0;
                const int cp = t > 0 && t - 1 < nt ? (int)((S0 + tie_pb[t - 1] + tie_m[t - 1]) & 1ll) : 0;
                const long long inc = t < nt ? (long long)(ck ^ cp) : 0ll;
                long long ttot;
                const long long upx = block_excl_scan_ll(inc, wsum, ttot);
                if (t < nt) tie_c[t] = (int)(upx + inc);
                if (t == 0) s_cross = 0x7fffffff;
            }
            __syncthreads();
            // every element's sum in units of u; the first that leaves the binade
            long long run = base;
            int first = 0x7fffffff;
            int kt = 0;  // ties at chunk-local index <= the element: binary search over tie_idx
            {
                int lo2 = 0, hi2 = nt;  // first tie with index >= t * kCumPer
                while (lo2 < hi2) {
                    const int mid = (lo2 + hi2) >> 1;
                    if (tie_idx[mid] < t * kCumPer) lo2 = mid + 1; else hi2 = mid;
                }
                kt = lo2;
            }
            long long Sv[kCumPer];
#pragma unroll
            for (int i = 0; i < kCumPer; ++i) {
                run = sat_add(run, r[i], LIM);
                const int li = t * kCumPer + i;
                if (kt < nt && tie_idx[kt] == li) ++kt;
                const long long C = kt > 0 ? (long long)tie_c[kt - 1] : 0ll;
                Sv[i] = S0 + run + C;
                if (j0 + i >= p && j0 + i < q1 && Sv[i] >= LIM && first == 0x7fffffff) first = li;
            }
            if (first != 0x7fffffff) atomicMin(&s_cross, first);
            __syncthreads();
            const int cross = s_cross;
#pragma unroll
            for (int i = 0; i < kCumPer; ++i) {
                const int li = t * kCumPer + i;
                const int64_t j = j0 + i;
                if (j >= p && j < q1 && li < cross) cum[j] = (T)((double)Sv[i] * u);
                // the running sum: before the crossing, or after the whole pass
                if (j >= p && ((cross != 0x7fffffff && li == cross - 1) || (cross == 0x7fffffff && j == q1 - 1)))
                    s_run = (T)((double)Sv[i] * u);
            }
            __syncthreads();
            if (cross == 0x7fffffff) {
                s = s_run;
                p = q1;
            } else {
                // the crossing step as a plain T addition, then the next binade
                if (t == 0) {
                    const T prev = jb + cross == p ? s : s_run;  // (the crossing is the pass's first active key)
                    const T nv = prev + KO::val(keys[jb + cross]);
                    cum[jb + cross] = nv;
                    s_run = nv;
                }
                __syncthreads();
                s = s_run;
                p = jb + cross + 1;
            }
            __syncthreads();
        }
        lo += kCumChunk;
        ++b;
    }
    VT_MARK(7, b, 0);
    if (trace && threadIdx.x == 0) trace[2 * kVtTraceMax] = (unsigned long long)nmark;
#undef VT_MARK
}

// FRMS_j = (cum[minEl+j] * (1/id)) * ((1/deno)^2), first argmin; writes the
// optimised ratio (OutlierFiltersImpl.cpp:202-217)
// (value, index) argmin with the first index on equal values: associative,
// so block partials combine to the sequential minCoeff's answer (a NaN FRMS
// value is never taken, as in the sequential scan)
template <typename T>
__device__ __forceinline__ void argmin_merge(T& bv, int& bi, T ov, int oi) {
    if (ov < bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
    }
}
template <typename T>
__device__ __forceinline__ void block_argmin256(T& bv, int& bi, T* sv, int* si) {
    const int t = threadIdx.x;
    sv[t] = bv;
    si[t] = bi;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
            T v = sv[t];
            int i = si[t];
            argmin_merge(v, i, sv[t + off], si[t + off]);
            sv[t] = v;
            si[t] = i;
        }
        __syncthreads();
    }
    bv = sv[0];
    bi = si[0];
}

// FRMS_j = (cum[minEl+j] * (1/id)) * ((1/deno)^2) (OutlierFiltersImpl.cpp:202-213),
// each block's first argmin over a grid-stride slice
constexpr int kFrmsBlocks = 256;
template <typename T>
__global__ __launch_bounds__(256) void vt_frms_part_kernel(const T* __restrict__ cum, const int* __restrict__ count,
                                                           const T* __restrict__ deno, int minEl, int maxEl,
                                                           T* __restrict__ part_v, int* __restrict__ part_i,
                                                           const LoopCtl* __restrict__ ctl) {
    __shared__ T sv[256];
    __shared__ int si[256];
    if (ctl && ctl->done) return;
    const int c = *count;
    const int hi = maxEl < c ? maxEl : c;  // reference reads past the filtered count (UB); build clamps
    const int n = hi - minEl;
    T bv = (T)__builtin_huge_val();
    int bi = 0x7fffffff;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
        const T id = (T)(minEl + 1 + j);
        const T inv_id = (T)1 / id;
        const T invd = (T)1 / deno[j];
        argmin_merge(bv, bi, (cum[minEl + j] * inv_id) * (invd * invd), j);
    }
    block_argmin256(bv, bi, sv, si);
    if (threadIdx.x == 0) {
        part_v[blockIdx.x] = bv;
        part_i[blockIdx.x] = bi;
    }
}

// the blocks' argmins combined; writes the optimised ratio (:214-217)
// VarTrimmed's quantile at the optimised ratio (OutlierFiltersImpl.cpp:
// 221-223, Matches::getDistsQuantile) straight from the sort: the radix
// select over the same distances finds the same order statistic, and its
// population — the finite distances — is the zeros (not sort keys: the
// partial sum takes the positive ones only) followed by the sorted positive
// keys.  The rank rule and the final select state are select_all_kernel's
// (pick_phase, pass 0); one thread, one load instead of the radix passes —
// run by the FRMS argmin's final block once it has the ratio (one launch).
// header words: [0] kept keys (atomic), [1] error, [2] zero distances
// (atomic), [8, 10) the head's running sum; the last call's counters are
// copied from kVtHdrCopy on (the counters themselves are zeroed after use)
constexpr int kVtHdrCopy = 16;
int vartrim_hdr_copy() { return kVtHdrCopy; }

template <typename T>
__device__ __forceinline__ void vt_quantile_body(const typename KeyOf<T>::K* __restrict__ sorted,
                                                 int* __restrict__ hdr, const double* __restrict__ ratio_dev,
                                                 SelectState* __restrict__ st, int* __restrict__ iter_err) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    // the last reader of this call's counters: they are kept for
    // pmx_vartrim_partial_sums at kVtHdrCopy and zeroed for the next call
    // (no reset launch; an iteration queued after the loop stopped returns
    // before this, leaving the last call's copy)
    const int h0 = hdr[0], h2 = hdr[2];
    hdr[kVtHdrCopy] = h0;
    hdr[kVtHdrCopy + 2] = h2;
    hdr[0] = 0;
    hdr[2] = 0;
    const unsigned long long zeros = (unsigned)h2;
    const unsigned long long total = (unsigned long long)(unsigned)h0 + zeros;
    const T q = (T)(*ratio_dev);
    unsigned long long rank = 0;
    int err = 0;
    if (total == 0) {
        err = -2;  // PMX_E_EMPTY_QUANTILE: ConvergenceError("no outlier to filter")
    } else if (q < (T)0 || q > (T)1) {
        err = -3;  // ConvergenceError("quantile must be between 0 and 1")
    } else if (q == (T)1) {
        rank = total - 1;  // max_element
    } else {
        rank = (unsigned long long)((T)total * q);
        if (rank >= total) rank = total - 1;
    }
    st->err = err;
    st->count = total;
    st->ratio = (double)q;
    st->rank = 0;
    if (err) {
        st->prefix = 0;
        st->limit = __builtin_nan("");
        __hip_atomic_store(iter_err, err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const K key = rank < zeros ? KO::key((T)0) : sorted[rank - zeros];
    st->prefix = (unsigned long long)key;
    st->limit = (double)KO::val(key);
}

template <typename T>
__global__ __launch_bounds__(256) void vt_frms_final_kernel(const T* __restrict__ part_v,
                                                            const int* __restrict__ part_i,
                                                            int* __restrict__ count, int minEl, int maxEl,
                                                            int points_nbr, double* __restrict__ ratio_dev,
                                                            int* __restrict__ err, int* __restrict__ iter_err,
                                                            const LoopCtl* __restrict__ ctl,
                                                            const typename KeyOf<T>::K* __restrict__ sorted,
                                                            SelectState* __restrict__ st) {
    __shared__ T sv[256];
    __shared__ int si[256];
    if (ctl && ctl->done) return;
    const int t = threadIdx.x;
    const int c = *count;
    const int hi = maxEl < c ? maxEl : c;
    if (c == 0 || hi - minEl <= 0) {
        if (t == 0) {
            const int e = c == 0 ? -2 : -3;
            *err = e;
            *iter_err = e;
            *ratio_dev = __builtin_nan("");
            vt_quantile_body<T>(sorted, count, ratio_dev, st, iter_err);
        }
        return;
    }
    T bv = (T)__builtin_huge_val();
    int bi = 0x7fffffff;
    for (int b = t; b < kFrmsBlocks; b += 256) argmin_merge(bv, bi, part_v[b], part_i[b]);
    block_argmin256(bv, bi, sv, si);  // (its barriers: every thread has read the count)
    if (t == 0) {
        const int minIndex = bi == 0x7fffffff ? 0 : bi;
        *ratio_dev = (double)(T)((float)(minIndex + minEl) / (float)points_nbr);
        vt_quantile_body<T>(sorted, count, ratio_dev, st, iter_err);
    }
}

template <typename T>
void launch_vartrim(const T* d, int64_t n, int points_nbr, T minRatio, T maxRatio, const T* deno, void* scratch,
                    size_t scratch_bytes, double* ratio_dev, int* err_dev, SelectState* st, const LoopCtl* ctl,
                    hipStream_t s) {
    (void)scratch_bytes;
    using K = typename KeyOf<T>::K;
    char* p = static_cast<char*>(scratch);
    int* hdr = reinterpret_cast<int*>(p);
    p += 256;
    RsHead* rsh = reinterpret_cast<RsHead*>(p);  // (zeroed when the scratch is allocated: vartrim_scratch_head)
    p += al256(sizeof(RsHead));
    K* keysA = reinterpret_cast<K*>(p);
    p += al256(sizeof(K) * n);
    K* keysB = reinterpret_cast<K*>(p);
    p += al256(sizeof(K) * n);
    T* cum = reinterpret_cast<T*>(p);
    p += al256(sizeof(T) * n);
    T* part_v = reinterpret_cast<T*>(p);  // (the FRMS argmin's block partials)
    p += al256(8 * 256);
    int* part_i = reinterpret_cast<int*>(p);
    p += al256(8 * 256);
    void* rs_state = p;  // the radix sort's look-back state (pmx_radix.h)
    p += al256(rs_state_bytes(n));
    const int64_t nch = vt_chunks(n);
    VtChunk* ch = reinterpret_cast<VtChunk*>(p);
    p += al256(sizeof(VtChunk) * (nch + 1));
    VtPrep pr;
    for (int v = 0; v < 2; ++v) {
        pr.Q[v] = reinterpret_cast<long long*>(p);
        p += al256(8 * (size_t)n);
    }
    pr.P1 = reinterpret_cast<long long*>(p);
    p += al256(8 * (size_t)n);
    pr.W1 = reinterpret_cast<int*>(p);
    p += al256(4 * (size_t)n);

    K* src = keysB;  // (the sorted keys: the kept ones first)
    if (n > 0) {
        hipLaunchKernelGGL(vt_keys_kernel<T>, dim3(rs_hist_blocks(n)), dim3(256), 0, s, d, n, keysA, hdr, ctl, rsh,
                           (unsigned long long*)rs_state, rs_tiles(n) * kRsDigits);
        src = launch_radix_sort_keys<K>(keysA, keysB, n, 0, KeyOf<T>::bits, rsh, rs_state, ctl, s, true);
    }
    // the head's running sum (written by the preparation launch's extra block)
    T* head = reinterpret_cast<T*>(hdr + 8);
    if (nch > 0) {
        hipLaunchKernelGGL(vt_chunk_sum_kernel<T>, dim3((unsigned)(nch + 1)), dim3(kCumThreads), 0, s, src, hdr, ch, ctl);
        hipLaunchKernelGGL(vt_chunk_prep_kernel<T>, dim3((unsigned)(nch + 1)), dim3(kCumThreads), 0, s, src, hdr, ch, pr,
                           ctl, cum, head);
    }
    unsigned long long* trace = g_vt_trace ? reinterpret_cast<unsigned long long*>(p) : nullptr;
    hipLaunchKernelGGL(vt_cumsum_kernel<T>, dim3(1), dim3(kCumThreads), 0, s, src, hdr, cum, ch, pr, (int)nch, ctl,
                       trace, nch > 0 ? (const T*)head : (const T*)nullptr);
    if (nch > 0)
        hipLaunchKernelGGL(vt_chunk_write_kernel<T>, dim3((unsigned)nch), dim3(kCumThreads), 0, s, src, hdr, ch, pr,
                           cum, ctl);
    const int minEl = (int)std::floor(minRatio * (T)points_nbr);
    const int maxEl = (int)std::floor(maxRatio * (T)points_nbr);
    hipLaunchKernelGGL(vt_frms_part_kernel<T>, dim3(kFrmsBlocks), dim3(256), 0, s, cum, hdr, deno, minEl, maxEl, part_v,
                       part_i, ctl);
    // (with the quantile at the optimised ratio: vt_quantile_body)
    hipLaunchKernelGGL(vt_frms_final_kernel<T>, dim3(1), dim3(256), 0, s, part_v, part_i, hdr, minEl, maxEl,
                       points_nbr, ratio_dev, hdr + 1, err_dev, ctl, (const K*)src, st);
}

// explicit instantiations
template void launch_select_hist<float>(const float*, int64_t, uint32_t*, const SelectState*, int, const LoopCtl*,
                                        const SpecSel*, hipStream_t);
template void launch_select_hist<double>(const double*, int64_t, uint32_t*, const SelectState*, int, const LoopCtl*,
                                         const SpecSel*, hipStream_t);
template void launch_select_pick<float>(uint32_t*, SelectState*, int, double, const double*, int*, const LoopCtl*,
                                        SpecSel*, hipStream_t);
template void launch_select_pick<double>(uint32_t*, SelectState*, int, double, const double*, int*, const LoopCtl*,
                                         SpecSel*, hipStream_t);
template void launch_select_all<float>(const float*, int64_t, void*, SelectState*, double, const double*, int*,
                                       const LoopCtl*, SpecSel*, const unsigned long long*, unsigned long long*,
                                       hipStream_t);
template void launch_select_all<double>(const double*, int64_t, void*, SelectState*, double, const double*, int*,
                                        const LoopCtl*, SpecSel*, const unsigned long long*, unsigned long long*,
                                        hipStream_t);
template void launch_vartrim<float>(const float*, int64_t, int, float, float, const float*, void*, size_t, double*,
                                    int*, SelectState*, const LoopCtl*, hipStream_t);
template void launch_vartrim<double>(const double*, int64_t, int, double, double, const double*, void*, size_t,
                                     double*, int*, SelectState*, const LoopCtl*, hipStream_t);
template <typename T>
size_t vartrim_trace_offset(int64_t n) {
    return vartrim_scratch_bytes<T>(n) - al256(8 * (2 * (size_t)kVtTraceMax + 1));
}
int vartrim_trace_max() { return kVtTraceMax; }
template size_t vartrim_trace_offset<float>(int64_t);
template size_t vartrim_trace_offset<double>(int64_t);
template size_t vartrim_scratch_bytes<float>(int64_t);
template size_t vartrim_scratch_bytes<double>(int64_t);


// Load this translation unit's code object now (pmx_ctx_create): HIP loads a
// module at the first launch of any of its kernels, and that host-side stall
// (milliseconds for the large grid module) would otherwise land inside the
// first ICP iteration.
void preload_select() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&select_all_kernel<float>));
}

}  // namespace pmx
