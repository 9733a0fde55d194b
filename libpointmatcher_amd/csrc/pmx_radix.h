// pmx_radix.h — LSD radix sort of unsigned keys (32 or 64 bit) for the
// device loop's per-iteration sorts (VarTrimmedDist's distances).
//
// rocPRIM's onesweep sort (pmx_sort.h) runs one launch per 8-bit digit, but
// fills its look-back state with hipMemsetAsync before every pass: at the 1M
// keys of a C3 VarTrimmed iteration that was 9 fills of ~4.9 us beside 6
// kernels, 114 us of the iteration (profiles/r05/exp).  This sort has the
// same structure — one histogram launch for every digit, then one launch per
// digit whose blocks rank a 4096-key tile, publish per-digit counts with a
// decoupled look-back and scatter — and no fill: each launch zeroes what the
// next one needs (the histogram launch the first pass's look-back state and
// tile counter, pass p those of pass p + 1, the last block of the last pass
// the histogram), so the scratch is in its initial state between calls.
//
// Ranking is stable (LSD radix sort needs it): in a tile, wave w owns keys
// [w * 64 * kRsItems, (w + 1) * 64 * kRsItems) in striped order (item i, lane
// l = key i * 64 + l), so processing items in order ranks keys in index order;
// waves and tiles are prefixed in order.  Lane ranks come from a bit-sliced
// match of the digit over the wave (8 ballots).
#pragma once

#include "pmx_internal.h"

namespace pmx {

constexpr int kRsBits = 8;
constexpr int kRsDigits = 1 << kRsBits;  // = threads per block: thread d owns digit d
constexpr int kRsThreads = 256;
constexpr int kRsItems = 16;  // (8 measured slower: 28.7 vs 22.1 us per pass)
constexpr int kRsTile = kRsThreads * kRsItems;
constexpr int kRsMaxPasses = 8;
constexpr int kRsLook = 8;  // look-back words loaded per round
static_assert(kRsDigits == kRsThreads, "one thread per digit");

// persistent part of the scratch (zero at allocation, zero between calls)
struct RsHead {
    unsigned int hist[kRsMaxPasses][kRsDigits];  // digit counts of every pass
    unsigned int tile_ctr[kRsMaxPasses];         // dynamic tile ids, per pass
    unsigned int done;                           // last pass: blocks finished
    unsigned int pad[7];
};

inline int64_t rs_tiles(int64_t n) { return (n + kRsTile - 1) / kRsTile; }
// look-back state: two buffers (pass parity) of tiles x digits words
inline size_t rs_state_bytes(int64_t n) { return 2 * sizeof(unsigned long long) * (size_t)rs_tiles(n) * kRsDigits; }

template <typename K>
__device__ __forceinline__ unsigned rs_digit(K k, int shift, int bits) {
    return (unsigned)((k >> shift) & (K)((1u << bits) - 1u));
}

// every pass's digit histogram; zeroes pass 0's look-back state and tile counter
template <typename K>
__global__ __launch_bounds__(kRsThreads) void rs_hist_kernel(const K* __restrict__ keys, int64_t n, int begin_bit,
                                                             int end_bit, int npass, RsHead* __restrict__ head,
                                                             unsigned long long* __restrict__ state0,
                                                             int64_t state_words, const LoopCtl* __restrict__ ctl) {
    __shared__ unsigned int h[kRsMaxPasses][kRsDigits];
    if (ctl && ctl->done) return;
    const int t = threadIdx.x;
    for (int p = 0; p < npass; ++p) h[p][t] = 0;
    __syncthreads();
    const int64_t stride = (int64_t)gridDim.x * kRsThreads;
    for (int64_t i = (int64_t)blockIdx.x * kRsThreads + t; i < n; i += stride) {
        const K k = keys[i];
        for (int p = 0; p < npass; ++p) {
            // (the last pass's digit is narrower when the key range is not a
            // whole number of digits: the same width rs_pass_kernel scatters by)
            const int sh = begin_bit + p * kRsBits;
            atomicAdd(&h[p][rs_digit<K>(k, sh, min(kRsBits, end_bit - sh))], 1u);
        }
    }
    __syncthreads();
    for (int p = 0; p < npass; ++p)
        if (h[p][t]) atomicAdd(&head->hist[p][t], h[p][t]);
    for (int64_t i = (int64_t)blockIdx.x * kRsThreads + t; i < state_words; i += stride) state0[i] = 0ull;
    if (blockIdx.x == 0 && t == 0) head->tile_ctr[0] = 0u;
}

// the histogram launch's grid (a grid-stride loop: ~16 keys per thread)
inline int rs_hist_blocks(int64_t n) {
    return (int)std::min<int64_t>(256, std::max<int64_t>(1, (n + kRsThreads - 1) / kRsThreads / 16));
}
// the histogram pass folded into a kernel that produces the keys (one block
// of kRsThreads; h: its LDS bins, zeroed and synchronised by the caller,
// counted by it): the block's bins into head->hist, the first pass's
// look-back words zeroed (grid-stride), the first tile counter reset
template <typename K>
__device__ __forceinline__ void rs_hist_block(unsigned int (*h)[kRsDigits], int npass, RsHead* __restrict__ head,
                                              unsigned long long* __restrict__ state0, int64_t state_words) {
    const int t = threadIdx.x;
    for (int p = 0; p < npass; ++p)
        if (h[p][t]) atomicAdd(&head->hist[p][t], h[p][t]);
    const int64_t stride = (int64_t)gridDim.x * kRsThreads;
    for (int64_t i = (int64_t)blockIdx.x * kRsThreads + t; i < state_words; i += stride) state0[i] = 0ull;
    if (blockIdx.x == 0 && t == 0) head->tile_ctr[0] = 0u;
}

// look-back words: value in the low 32 bits, flag in the high ones
constexpr unsigned long long kRsAgg = 1ull << 32, kRsInc = 2ull << 32;

template <typename K>
__global__ __launch_bounds__(kRsThreads) void rs_pass_kernel(const K* __restrict__ in, K* __restrict__ out, int64_t n,
                                                             int pass, int npass, int shift, int bits,
                                                             RsHead* __restrict__ head,
                                                             unsigned long long* __restrict__ state,
                                                             unsigned long long* __restrict__ state_next,
                                                             const LoopCtl* __restrict__ ctl) {
    __shared__ unsigned int wcnt[kRsThreads / 64][kRsDigits];
    __shared__ unsigned int goff[kRsDigits];
    __shared__ unsigned int s_tile;
    __shared__ unsigned int scan_w[kRsThreads / 64];
    if (ctl && ctl->done) return;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t == 0) s_tile = atomicAdd(&head->tile_ctr[pass], 1u);
    for (int w = 0; w < kRsThreads / 64; ++w) wcnt[w][t] = 0;
    __syncthreads();
    const unsigned tile = s_tile;
    const int64_t ntiles = (n + kRsTile - 1) / kRsTile;
    // (the next pass's look-back state of this tile, and its tile counter)
    if (state_next) state_next[(int64_t)tile * kRsDigits + t] = 0ull;
    if (tile == 0 && t == 0 && pass + 1 < kRsMaxPasses) head->tile_ctr[pass + 1] = 0u;
    // ---- rank the tile's keys inside each wave (striped, items in order) ----
    const int64_t wbase = (int64_t)tile * kRsTile + (int64_t)wave * 64 * kRsItems;
    K kv[kRsItems];
    unsigned loc[kRsItems];
#pragma unroll
    for (int i = 0; i < kRsItems; ++i) {
        const int64_t idx = wbase + (int64_t)i * 64 + lane;
        kv[i] = idx < n ? in[idx] : (K)0;
    }
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < kRsItems; ++i) {
        const int64_t idx = wbase + (int64_t)i * 64 + lane;
        const bool act = idx < n;
        const unsigned d = rs_digit<K>(kv[i], shift, bits);
        unsigned long long peers = __ballot(act);
#pragma unroll
        for (int b = 0; b < kRsBits; ++b) {
            const bool bit = (d >> b) & 1u;
            const unsigned long long bal = __ballot(act && bit);
            peers &= bit ? bal : ~bal;
        }
        unsigned base = 0;
        if (act) base = wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        if (act) {
            const unsigned rank = (unsigned)__popcll(peers & lt);
            loc[i] = base + rank;
            if (rank == 0) wcnt[wave][d] = base + (unsigned)__popcll(peers);  // (the lowest peer: the digit's leader)
        }
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // ---- thread d: the tile's count of digit d, the waves' prefixes ----
    unsigned wpre[kRsThreads / 64];
    unsigned tot = 0;
#pragma unroll
    for (int w = 0; w < kRsThreads / 64; ++w) {
        wpre[w] = tot;
        tot += wcnt[w][t];
    }
    // publish the aggregate, then the look-back over the earlier tiles
    unsigned long long* my = state + (int64_t)tile * kRsDigits + t;
    if (tile == 0) {
        __hip_atomic_store(my, kRsInc | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(my, kRsAgg | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the digit's start in the output: the counts of the smaller digits
    const unsigned hd = head->hist[pass][t];
    unsigned dexcl;
    {
        unsigned v = hd;  // block exclusive scan over the 256 digits
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned u = __shfl_up(v, off);
            if (lane >= off) v += u;
        }
        if (lane == 63) scan_w[wave] = v;
        __syncthreads();
        unsigned before = 0;
        for (int w = 0; w < wave; ++w) before += scan_w[w];
        dexcl = before + v - hd;
    }
    unsigned excl = 0;
    if (tile > 0) {
        // the words of up to kRsLook earlier tiles per round, loaded together
        // (one dependent round trip per round instead of per tile); the
        // round's usable prefix: from the nearest tile down to the first
        // inclusive word, stopping at the first one not published yet
        int64_t j = (int64_t)tile - 1;
        for (;;) {
            unsigned long long w[kRsLook];
#pragma unroll
            for (int q = 0; q < kRsLook; ++q)
                w[q] = j - q >= 0 ? __hip_atomic_load(state + (j - q) * kRsDigits + t, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : kRsInc;  // (before tile 0: an inclusive zero)
            int used = 0;
            bool done = false;
#pragma unroll
            for (int q = 0; q < kRsLook; ++q) {
                if (done || used < q) continue;  // (stopped earlier in this round)
                const unsigned long long flag = w[q] >> 32;
                if (flag == 0) continue;  // (not published: resume from here next round)
                excl += (unsigned)w[q];
                used = q + 1;
                if (flag == 2) done = true;
            }
            if (done) break;
            j -= used;
            if (used == 0) __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(my, kRsInc | (excl + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    (void)ntiles;
#pragma unroll
    for (int w = 0; w < kRsThreads / 64; ++w) wcnt[w][t] = wpre[w];  // (now the waves' prefixes)
    goff[t] = dexcl + excl;
    __syncthreads();
    // ---- scatter ----
#pragma unroll
    for (int i = 0; i < kRsItems; ++i) {
        const int64_t idx = wbase + (int64_t)i * 64 + lane;
        if (idx < n) {
            const unsigned d = rs_digit<K>(kv[i], shift, bits);
            out[goff[d] + wcnt[wave][d] + loc[i]] = kv[i];
        }
    }
    // the last pass's last finishing block leaves the histogram zero
    if (pass == npass - 1) {
        __syncthreads();
        __shared__ int s_last;
        if (t == 0) {
            __atomic_thread_fence(__ATOMIC_RELEASE);
            const unsigned old = __hip_atomic_fetch_add(&head->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == (unsigned)(ntiles - 1) ? 1 : 0;
        }
        __syncthreads();
        if (s_last) {
            for (int p = 0; p < npass; ++p)
                __hip_atomic_store(&head->hist[p][t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t == 0) __hip_atomic_store(&head->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Sort the n keys of `a` on bits [begin_bit, end_bit), the passes
// alternating between a and b; returns the buffer holding the result (b after
// an odd number of passes, else a).  head: an RsHead, zero when allocated;
// state: rs_state_bytes(n).
// hist_ready: the keys' producer already added every pass's histogram into
// head->hist, zeroed the first pass's look-back words and tile counter
// (rs_hist_block below) — no histogram launch here.
template <typename K>
K* launch_radix_sort_keys(K* a, K* b, int64_t n, int begin_bit, int end_bit, RsHead* head, void* state,
                          const LoopCtl* ctl, hipStream_t s, bool hist_ready = false) {
    if (n <= 0) return a;
    const int npass = (end_bit - begin_bit + kRsBits - 1) / kRsBits;
    const int64_t ntiles = rs_tiles(n);
    const int64_t words = ntiles * kRsDigits;
    unsigned long long* st[2] = {(unsigned long long*)state, (unsigned long long*)state + words};
    const int hb = rs_hist_blocks(n);
    if (!hist_ready)
        hipLaunchKernelGGL(rs_hist_kernel<K>, dim3(hb), dim3(kRsThreads), 0, s, a, n, begin_bit, end_bit, npass, head, st[0],
                           words, ctl);
    K* src = a;
    K* dst = b;
    for (int p = 0; p < npass; ++p) {
        const int sh = begin_bit + p * kRsBits;
        const int bits = std::min(kRsBits, end_bit - sh);
        hipLaunchKernelGGL(rs_pass_kernel<K>, dim3((unsigned)ntiles), dim3(kRsThreads), 0, s, src, dst, n, p, npass, sh,
                           bits, head, st[p % 2], p + 1 < npass ? st[(p + 1) % 2] : (unsigned long long*)nullptr, ctl);
        K* t = src;
        src = dst;
        dst = t;
    }
    return src;
}

}  // namespace pmx
