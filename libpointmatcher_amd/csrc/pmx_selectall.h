// pmx_selectall.h — the radix select with every pass in one launch (the
// select_all_kernel of pmx_select.hip), and the histogram helpers it shares
// with the per-pass kernels of the sharded select.
#pragma once

#include "pmx_internal.h"
#include "pmx_spec.h"

#include <type_traits>

namespace pmx {

// ------------------------------------------------------------- histogram --
constexpr int kSelPer = 16;  // keys per thread per tile

// kSelPer consecutive values from i0 (16-byte vector loads when the whole run
// is in range; +inf pads past n and is excluded like any infinite distance)
template <typename T>
__device__ __forceinline__ void load_keys(const T* __restrict__ d, int64_t i0, int64_t n, T (&v)[kSelPer]) {
    if (i0 + kSelPer <= n) {
        using V = typename std::conditional<sizeof(T) == 4, float4, double2>::type;
        constexpr int E = 16 / sizeof(T);
        const V* p = reinterpret_cast<const V*>(d + i0);  // i0 * sizeof(T) is a multiple of 64
#pragma unroll
        for (int q = 0; q < kSelPer / E; ++q) {
            const V x = p[q];
            const T* xe = reinterpret_cast<const T*>(&x);
#pragma unroll
            for (int e = 0; e < E; ++e) v[q * E + e] = xe[e];
        }
    } else {
#pragma unroll
        for (int j = 0; j < kSelPer; ++j) v[j] = i0 + j < n ? d[i0 + j] : (T)__builtin_huge_val();
    }
}
// ------------------------------------------------------------------ pick --
// histogram bin reads/resets; kCoherent: device-scope atomics (the fused pass
// kernel reads bins other blocks - on other XCDs - have just added to)
template <bool kCoherent>
__device__ __forceinline__ uint32_t hbin(uint32_t* h) {
    // (a fetch-add of 0 is performed where the other blocks' adds were)
    if constexpr (kCoherent) return __hip_atomic_fetch_add(h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return *h;
}
template <bool kCoherent>
__device__ __forceinline__ void hzero(uint32_t* h) {
    if constexpr (kCoherent) {
        __hip_atomic_store(h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *h = 0;
    }
}

// ------------------------------------------------- all passes, one launch --
// Every kernel boundary costs ~4.5 us on MI355X (measured: an empty select
// pass takes 4.6 us in the kernel trace — the dispatch's release / acquire
// over the 8 XCD L2s), and the three (f64: six) passes of the radix select
// are three boundaries per iteration even when the quantile window already
// resolved the limit.  select_all_kernel runs every pass in ONE launch: the
// blocks histogram a digit, the last block to arrive (arrival counter) picks
// it and publishes it, the others wait for the publication and go on with
// the next digit.  A window hit makes the whole launch a no-op.
//
// Cross-block traffic uses device-scope atomics only (flushes with returning
// atomics, as the ticket pass does; reads of what another block wrote with
// fetch-add 0 / atomic loads): no fence, no L2 write-back.  Nothing is reset:
// the arrival counters only grow (one launch adds exactly `grid` arrivals per
// pass it reaches), so arrival a belongs to generation a / grid + 1, and the
// picker of that generation stamps its publication with it.  The waits are
// bounded (an exit condition every wave reaches): a timeout raises
// kSelTimeout in the iteration's error word instead of hanging.  The grid
// is clamped to the blocks the device holds at once (select_all_blocks: at
// most 64 blocks of 256 threads, far below one block per CU), so every block
// is resident unless other processes fill the GPU; then the bounded waits
// turn a starved block into an error, not a hang.
constexpr int kSelMaxPasses = 6;
struct SelX {
    unsigned int arrive[8];                  // per pass (monotonic)
    unsigned long long go[kSelMaxPasses];    // gen << 56 | err << 55 | resolved prefix (<= 54 bits)
    unsigned long long rank[kSelMaxPasses];  // rank left inside the prefix after pass p
    unsigned long long tot[kSelMaxPasses];   // keys histogrammed in pass p
    unsigned long long count;                // finite keys (pass 0)
    unsigned int cread;                      // merged counter phase: blocks done reading (monotonic)
    unsigned int pad_;
};

__device__ __forceinline__ unsigned long long ald(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (returning: the caller makes later publications depend on the return)
__device__ __forceinline__ unsigned long long ast(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The match's counter phase merged into the select launch (device loop,
// single rank, window on): EVERY block folds the spread counters and picks
// from the window keys itself (reads only: the same inputs give every block
// the same verdict, so no block waits for another's); block 0 then waits
// until every block has read (an arrival count: the readers never wait, so
// this needs no co-residency) and writes the results — the iteration
// block's counters, the error word, the select state and the next window.
// The spread counters are zeroed by the point-to-plane launch that follows.
// Returns the verdict (block-uniform).
template <typename T>
__device__ __forceinline__ bool counter_merged(const unsigned long long* __restrict__ vpart,
                                               unsigned long long* __restrict__ out, int* __restrict__ iter_err,
                                               SpecSel* __restrict__ spec, SelectState* __restrict__ st,
                                               SelX* __restrict__ sx) {
    using K = typename KeyOf<T>::K;
    constexpr unsigned kLds = 4096;
    __shared__ unsigned long long red[4][kVSlots / 64];
    __shared__ uint32_t lh[2048];
    __shared__ unsigned long long part[kVSlots];
    __shared__ unsigned long long bc[2];
    __shared__ K lkeys[kLds];
    const int t = threadIdx.x;
    const unsigned nk_raw = spec->n_keys;
    const K lo = (K)spec->lo, hi = (K)spec->hi;
    const bool valid = spec->valid != 0;
    unsigned long long v[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] = vpart[(size_t)(c * kVSlots + t) * kVStride];
    for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] += __shfl_xor(v[c], off);
    }
    if ((t & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) red[c][t >> 6] = v[c];
    }
    SpecKeys<T> src;
    src.local = (const K*)spec->keys;
    src.n_local = nk_raw < kSpecCap ? nk_raw : kSpecCap;
    if (src.n_local <= kLds && valid) {
        for (unsigned i = t; i < src.n_local; i += kVSlots) lkeys[i] = src.local[i];
        src.lds = lkeys;
    }
    __syncthreads();
    unsigned long long sum[4] = {0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 4; ++c)
        for (int w = 0; w < kVSlots / 64; ++w) sum[c] += red[c][w];
    unsigned long long kl = 0;
    const bool hit = spec_pick<T, kVSlots>(spec, st, sum[2], sum[3], src.n_local, nk_raw > kSpecCap, src, lh, part,
                                           bc, false, &kl);
    __syncthreads();  // (every thread of the block has read)
    if (t == 0) {
        const unsigned old = atomicAdd(&sx->cread, 1u);
        if (blockIdx.x == 0) {
            // every block of this launch has read once the count reaches the
            // generation's end (a power-of-two grid: the count wraps cleanly)
            const unsigned G = gridDim.x, base = old - old % G;
            bool all = false;
            for (int it = 0; it < (1 << 22); ++it) {
                if (__hip_atomic_load(&sx->cread, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base >= G) {
                    all = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            __hip_atomic_store(&out[0], sum[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&out[1], sum[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(iter_err, all ? 0 : kSelTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            spec_commit<T>(spec, st, hit, lo, hi, (K)kl, sum[2], nk_raw);
        }
    }
    return hit;
}

// The select itself (every block of select_all_kernel): the resolved
// limit and select state in *st, the next window re-centred (spec).
template <typename T>
__device__ __forceinline__ void select_all_body(const T* __restrict__ d, int64_t n, SelX* __restrict__ sx,
                                                SelectState* __restrict__ st, double ratio_host,
                                                const double* __restrict__ ratio_dev, int* __restrict__ iter_err,
                                                SpecSel* __restrict__ spec,
                                                const unsigned long long* __restrict__ vpart = nullptr,
                                                unsigned long long* __restrict__ vout = nullptr) {
    using KO = KeyOf<T>;
    using K = typename KO::K;
    __shared__ uint32_t lh[2048];
    __shared__ unsigned long long part[256];
    __shared__ unsigned long long s_w[2];  // (published word, its generation)
    __shared__ int s_last;
    __shared__ unsigned int s_old;
    if (vpart) {
        if (counter_merged<T>(vpart, vout, iter_err, spec, st, sx)) return;  // (the window resolved it)
    } else if (spec && spec->hit) {
        return;  // (the window resolved it in the counter kernel before this launch)
    }
    constexpr int passes = KO::bits == 32 ? 3 : 6;
    uint32_t* hist0 = reinterpret_cast<uint32_t*>(sx + 1);
    const int t = threadIdx.x;
    const unsigned G = gridDim.x;
    K prefix = 0;
    const T q = ratio_dev ? (T)(*ratio_dev) : (T)ratio_host;
    for (int pass = 0; pass < passes; ++pass) {
        int shift, bits;
        digit_of(KO::bits, pass, shift, bits);
        const int nb = 1 << bits;
        uint32_t* hist = hist0 + pass * 2048;
        // ---- histogram of this digit over the keys inside the prefix ----
        for (int i = t; i < nb; i += 256) lh[i] = 0;
        __syncthreads();
        {
            const int hs = shift + bits;
            const int64_t tile = (int64_t)256 * kSelPer;
            for (int64_t base = (int64_t)blockIdx.x * tile; base < n; base += (int64_t)G * tile) {
                T v[kSelPer];
                load_keys<T>(d, base + (int64_t)t * kSelPer, n, v);
#pragma unroll
                for (int j = 0; j < kSelPer; ++j) {
                    const K k = KO::key(v[j]);
                    if (k < KO::inf_key && (pass == 0 || (k >> hs) == prefix))
                        atomicAdd(&lh[(uint32_t)(k >> shift) & (uint32_t)(nb - 1)], 1u);
                }
            }
        }
        __syncthreads();
        uint32_t ret = 0;  // returning flushes: done at the coherence point once back
        for (int i = t; i < nb; i += 256) {
            const uint32_t c = lh[i];
            if (c) ret |= atomicAdd(&hist[i], c);
        }
        asm volatile("" ::"v"(ret));
        __syncthreads();
        if (t == 0) {
            const unsigned old = atomicAdd(&sx->arrive[pass], 1u);
            s_old = old;
            s_last = (old + 1) % G == 0;
        }
        __syncthreads();
        const unsigned long long gen = ((unsigned long long)(s_old / G) + 1ull) & 0xffull;
        if (s_last) {
            // ---- the picker: pick_phase's rule over the flushed bins ----
            const int per = nb / 256;
            uint32_t hv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) hv[j] = j < per ? hbin<true>(&hist[t * per + j]) : 0u;
            unsigned long long mine = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) mine += hv[j];
            {  // inclusive scan over the 256 partials (pmx_spec.h block_incl_scan)
                __shared__ unsigned long long wsum[4];
                part[t] = block_incl_scan<256>(mine, wsum);
                __syncthreads();
            }
            const unsigned long long total = part[255];
            unsigned long long rank = 0;
            int err = 0;
            if (pass == 0) {
                if (total == 0) {
                    err = -2;  // PMX_E_EMPTY_QUANTILE: ConvergenceError("no outlier to filter")
                } else if (!ratio_dev && ratio_host == kRatioMedianIndex) {
                    rank = total / 2;  // nth_element at size / 2 (Matches.cpp:110-120)
                } else if (q < (T)0 || q > (T)1) {
                    err = -3;  // ConvergenceError("quantile must be between 0 and 1")
                } else if (q == (T)1) {
                    rank = total - 1;  // max_element
                } else {
                    rank = (unsigned long long)((T)total * q);
                    if (rank >= total) rank = total - 1;  // reference reads out of range (UB); clamp
                }
            } else {
                rank = __hip_atomic_fetch_add(&sx->rank[pass - 1], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (err == 0) {
                const unsigned long long excl = t > 0 ? part[t - 1] : 0ull;
                if (rank >= excl && rank < part[t]) {
                    unsigned long long cum = excl;
                    for (int j = 0; j < per; ++j) {
                        const unsigned long long c = hv[j];
                        if (rank < cum + c) {
                            s_w[0] = (unsigned long long)(t * per + j);
                            s_w[1] = rank - cum;
                            break;
                        }
                        cum += c;
                    }
                }
            }
            __syncthreads();
            for (int j = 0; j < per; ++j) hzero<true>(&hist[t * per + j]);  // ready for the next launch
            const K np = err ? (K)0 : (K)((prefix << bits) | (K)s_w[0]);
            const unsigned long long nrank = err ? 0ull : s_w[1];
            if (t == 0) {
                unsigned long long r0 = 0;
                if (pass == 0) r0 |= ast(&sx->count, total);
                r0 |= ast(&sx->tot[pass], total);
                if (err || pass == passes - 1) {
                    // the final state, as the pass kernels leave it
                    const unsigned long long count = pass == 0 ? total : ald(&sx->count);
                    st->err = err;
                    st->count = count;
                    st->prefix = (unsigned long long)np;
                    st->rank = nrank;
                    st->ratio = (double)q;
                    if (err) {
                        st->limit = __builtin_nan("");
                        __hip_atomic_store(iter_err, err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        st->limit = (double)KO::val(np);
                        if (spec) {
                            // density for the next window: the finest bucket with >= 64 keys
                            double dens = -1.0;
                            for (int p = 0; p < passes; ++p) {
                                int sh, bt;
                                digit_of(KO::bits, p, sh, bt);
                                const unsigned long long c = p == pass ? total : ald(&sx->tot[p]);
                                if (c >= 64) dens = (double)c / ldexp(1.0, sh + bt);
                            }
                            spec_update<T>(spec, np, dens > 0.0 ? dens : (double)(total + 1) / (double)nb);
                        }
                    }
                } else {
                    r0 |= ast(&sx->rank[pass], nrank);
                }
                // publish once the data above has returned (performed where every block reads it)
                asm volatile("" ::"v"(r0));
                (void)ast(&sx->go[pass],
                          gen << 56 | (err ? 1ull << 55 : 0ull) | ((unsigned long long)np & ((1ull << 55) - 1)));
            }
            if (err) return;
            prefix = np;
            __syncthreads();
            if (pass == passes - 1) return;
        } else {
            if (pass == passes - 1) return;  // (the picker finishes alone)
            // ---- wait for this generation's publication (bounded) ----
            if (t == 0) {
                unsigned long long w = 0;
                bool ok = false;
                for (int it = 0; it < (1 << 22); ++it) {
                    w = ald(&sx->go[pass]);
                    if ((w >> 56) == gen) {
                        ok = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                s_w[0] = w;
                s_w[1] = ok ? 1ull : 0ull;
                if (!ok) __hip_atomic_store(iter_err, kSelTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            const unsigned long long w = s_w[0];
            if (!s_w[1] || (w >> 55) & 1ull) return;  // timeout, or the quantile failed
            prefix = (K)(w & ((1ull << 55) - 1));
        }
    }
}

}  // namespace pmx
