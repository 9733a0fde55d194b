// pmx_setup.hip — the once-per-compute setup on the device.
//
// Matcher::init (MatchersImpl.cpp:77-83: libnabo builds its kd-tree over the
// filtered reference) becomes, here, the multi-level uniform grid of
// pmx_grid.hip; the reading copy of ICP.cpp:337-347 becomes the reading in
// slot (Morton) order.  Both used to be built on the host (a counting sort
// per grid level and a std::sort of the Morton keys: ~0.4 s at 1M points);
// they are built here from the uploaded clouds:
//
//   pack        rows x n point-major T -> P4<T> (2-D clouds as (x, y, 0, h)),
//               normals D x n -> P4<T>, the reference padded with +inf points
//   bbox        lo / hi of the finite points in double (min / max: exact,
//               order-free) and their count
//   occupancy   distinct cells at a trial cell size (the local-dimension
//               estimate that sizes the levels)
//   cell keys   cell of every finite point (+ a histogram of the cells);
//               the keys sorted stably with their indices (hipcub radix
//               sort: the index order inside a cell is kept, as the host
//               counting sort kept it); cell starts = exclusive scan of the
//               histogram; points / normals / indices gathered in key order
//   morton      the reading's Morton keys of its initially transformed cell,
//               sorted with their indices: the slot order
//
// Every cell computation is the host's double arithmetic,
// floor((q - lo) / h) clamped to the grid, so the device build is the host
// build bit for bit (the grid / loop / config tests check the matches it
// serves against the oracle).
#include <algorithm>

#include <hipcub/hipcub.hpp>

#include "pmx_internal.h"
#include "pmx_sort.h"

namespace pmx {

// ------------------------------------------------------------------ pack --
// off (may be null): subtracted per axis in T — the centring of ICP.cpp:299
// (features.topRows(dim - 1) -= mean), the same one rounding per coordinate
template <typename T>
__global__ void pack_p4_kernel(const T* __restrict__ raw, int rows, int64_t n, int64_t n_pad, P4<T>* __restrict__ out,
                               Off3<T> off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    if (i >= n) {
        const T inf = (T)__builtin_huge_val();
        out[i] = P4<T>{inf, inf, inf, (T)1};
        return;
    }
    const T* p = raw + i * rows;
    P4<T> q = rows == 4 ? P4<T>{p[0], p[1], p[2], p[3]} : P4<T>{p[0], p[1], (T)0, p[2]};
    if (off.on) {
        q.x = q.x - off.v[0];
        q.y = q.y - off.v[1];
        if (rows == 4) q.z = q.z - off.v[2];
    }
    out[i] = q;
}

template <typename T>
__global__ void pack_nrm_kernel(const T* __restrict__ raw, int D, int64_t n, P4<T>* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const T* p = raw + i * D;
    out[i] = D == 3 ? P4<T>{p[0], p[1], p[2], (T)0} : P4<T>{p[0], p[1], (T)0, (T)0};
}

static unsigned blocks_for(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per > 0 ? (n + per - 1) / per : 1); }

template <typename T>
void launch_pack_p4(const T* raw, int rows, int64_t n, int64_t n_pad, P4<T>* out, hipStream_t s, const T* offset) {
    if (n_pad <= 0) return;
    Off3<T> off{};
    if (offset) {
        off.on = 1;
        for (int a = 0; a < rows - 1; ++a) off.v[a] = offset[a];
    }
    hipLaunchKernelGGL(pack_p4_kernel<T>, dim3(blocks_for(n_pad)), dim3(256), 0, s, raw, rows, n, n_pad, out, off);
}
template <typename T>
void launch_pack_nrm(const T* raw, int D, int64_t n, P4<T>* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(pack_nrm_kernel<T>, dim3(blocks_for(n)), dim3(256), 0, s, raw, D, n, out);
}

// ------------------------------------------------------------------ bbox --
template <typename T>
__device__ __forceinline__ bool dfinite(const P4<T>& p) {
    return isfinite((double)p.x) && isfinite((double)p.y) && isfinite((double)p.z);
}

constexpr int kBBoxBlocks = 256;

// per-block partials: lo[3], hi[3], valid
template <typename T>
__global__ __launch_bounds__(256) void bbox_kernel(const P4<T>* __restrict__ p, int64_t n, double* __restrict__ part) {
    __shared__ double red[7][256];
    double v[7] = {1e300, 1e300, 1e300, -1e300, -1e300, -1e300, 0.0};
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const P4<T> q = p[i];
        if (!dfinite(q)) continue;
        const double c[3] = {(double)q.x, (double)q.y, (double)q.z};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            v[a] = fmin(v[a], c[a]);
            v[3 + a] = fmax(v[3 + a], c[a]);
        }
        v[6] += 1.0;
    }
    const int t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < 7; ++k) red[k][t] = v[k];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                red[a][t] = fmin(red[a][t], red[a][t + off]);
                red[3 + a][t] = fmax(red[3 + a][t], red[3 + a][t + off]);
            }
            red[6][t] += red[6][t + off];
        }
        __syncthreads();
    }
    if (t < 7) part[blockIdx.x * 8 + t] = red[t][0];
}

// (min / max are order-free and the count is an exact integer in double:
// the block tree gives the same result as a sequential walk)
__global__ __launch_bounds__(256) void bbox_final_kernel(const double* __restrict__ part, int nb,
                                                         double* __restrict__ out) {
    __shared__ double red[7][256];
    const int t = threadIdx.x;
    double v[7] = {1e300, 1e300, 1e300, -1e300, -1e300, -1e300, 0.0};
    for (int b = t; b < nb; b += 256) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            v[a] = fmin(v[a], part[b * 8 + a]);
            v[3 + a] = fmax(v[3 + a], part[b * 8 + 3 + a]);
        }
        v[6] += part[b * 8 + 6];
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) red[k][t] = v[k];
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                red[a][t] = fmin(red[a][t], red[a][t + off]);
                red[3 + a][t] = fmax(red[3 + a][t], red[3 + a][t + off]);
            }
            red[6][t] += red[6][t + off];
        }
        __syncthreads();
    }
    if (t < 7) out[t] = red[t][0];
}

// out[7]: lo xyz, hi xyz, finite count; scratch: kBBoxBlocks * 8 doubles
template <typename T>
void launch_bbox(const P4<T>* p, int64_t n, double* scratch, double* out, hipStream_t s) {
    int64_t nb = (n + 255) / 256;
    if (nb > kBBoxBlocks) nb = kBBoxBlocks;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(bbox_kernel<T>, dim3((unsigned)nb), dim3(256), 0, s, p, n, scratch);
    hipLaunchKernelGGL(bbox_final_kernel, dim3(1), dim3(256), 0, s, scratch, (int)nb, out);
}
size_t bbox_scratch_bytes() { return sizeof(double) * kBBoxBlocks * 8; }

// --------------------------------------------------------------- cells ---
// the host build's cell (pmx_capi.hip cell_of): floor((q - lo) / h) in
// double, clamped to the grid; x fastest
__device__ __forceinline__ int64_t dcell_of(const SetupShape& s, double x, double y, double z, int64_t ci[3]) {
    const double q[3] = {x, y, z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double f = floor((q[a] - s.lo[a]) / s.h);
        if (f < 0) f = 0;
        if (f > s.g[a] - 1) f = s.g[a] - 1;
        ci[a] = (int64_t)f;
    }
    return (ci[2] * s.g[1] + ci[1]) * s.g[0] + ci[0];
}

// distinct occupied cells of a trial grid, with no global atomics: block
// (slice, part) sets, in an LDS bitmap, the bits of the cells of its slice of
// the points that fall in its part of the bitmap (kOccWords words), and
// writes that part to its own slice of `slices`; occupancy_count_kernel ORs
// the slices word by word and counts the bits.  (Global atomicOr on a shared
// bitmap serialised on contended words: 300 us non-returning, 600 us with the
// returned bits counted, at 1M points.)
constexpr int kOccWords = 32768;  // 128 KB of LDS
constexpr int kOccSlices = 32;
// gfx950 gives a workgroup up to 160 KB of LDS; the bitmap must fit it (a
// 64 KB-LDS target would need kOccWords <= 16384)
static_assert(kOccWords * sizeof(uint32_t) <= 160 * 1024, "occupancy bitmap exceeds the gfx950 LDS budget");

size_t occupancy_bytes(int64_t cells) { return 256 + sizeof(uint32_t) * (size_t)kOccSlices * (size_t)((cells + 31) / 32); }

template <typename T>
__global__ __launch_bounds__(1024) void occupancy_kernel(const P4<T>* __restrict__ p, int64_t n, SetupShape s,
                                                         int64_t words, uint32_t* __restrict__ slices) {
    __shared__ uint32_t bm[kOccWords];
    const int64_t w0 = (int64_t)blockIdx.y * kOccWords;
    const int nw = (int)(words - w0 < kOccWords ? words - w0 : kOccWords);
    for (int i = threadIdx.x; i < nw; i += 1024) bm[i] = 0;
    __syncthreads();
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t a = (int64_t)blockIdx.x * per, b = a + per < n ? a + per : n;
    for (int64_t i = a + threadIdx.x; i < b; i += 1024) {
        const P4<T> q = p[i];
        if (dfinite(q)) {
            int64_t ci[3];
            const int64_t c = dcell_of(s, (double)q.x, (double)q.y, (double)q.z, ci);
            const int64_t w = (c >> 5) - w0;
            if (w >= 0 && w < nw) atomicOr(&bm[w], 1u << (uint32_t)(c & 31));
        }
    }
    __syncthreads();
    uint32_t* out = slices + (int64_t)blockIdx.x * words + w0;
    for (int i = threadIdx.x; i < nw; i += 1024) out[i] = bm[i];
}

__global__ __launch_bounds__(256) void occupancy_count_kernel(const uint32_t* __restrict__ slices, int64_t words,
                                                              unsigned long long* __restrict__ count) {
    __shared__ unsigned long long part[4];
    unsigned long long v = 0;
    for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < words; w += (int64_t)gridDim.x * blockDim.x) {
        uint32_t o = 0;
#pragma unroll 8
        for (int sl = 0; sl < kOccSlices; ++sl) o |= slices[(int64_t)sl * words + w];
        v += (unsigned)__popc(o);
    }
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(count, t);
    }
}

// scratch: occupancy_bytes(s.cells) at `scratch`; the count (zeroed by the
// caller) in its first 8 bytes
template <typename T>
void launch_occupancy(const P4<T>* p, int64_t n, const SetupShape& s, void* scratch, hipStream_t st) {
    // (the caller sized `scratch` with occupancy_bytes(s.cells) and checked
    // s.cells <= kOccMaxCells)
    const int64_t words = (s.cells + 31) / 32;
    unsigned long long* count = (unsigned long long*)scratch;
    uint32_t* slices = (uint32_t*)((char*)scratch + 256);
    const unsigned parts = (unsigned)((words + kOccWords - 1) / kOccWords);
    hipLaunchKernelGGL(occupancy_kernel<T>, dim3(kOccSlices, parts), dim3(1024), 0, st, p, n, s, words, slices);
    const int64_t cb = std::min<int64_t>(1024, std::max<int64_t>(1, (words + 255) / 256));
    hipLaunchKernelGGL(occupancy_count_kernel, dim3((unsigned)cb), dim3(256), 0, st, slices, words, count);
}

// cell key of every point (non-finite: the sentinel C, sorted last) and the
// histogram of the finite ones
template <typename T>
__global__ void cell_keys_kernel(const P4<T>* __restrict__ p, int64_t n, SetupShape s, uint32_t* __restrict__ keys,
                                 int32_t* __restrict__ idx, uint32_t* __restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const P4<T> q = p[i];
    uint32_t k = (uint32_t)s.cells;
    if (dfinite(q)) {
        int64_t ci[3];
        k = (uint32_t)dcell_of(s, (double)q.x, (double)q.y, (double)q.z, ci);
        atomicAdd(&counts[k], 1u);
    }
    keys[i] = k;
    idx[i] = (int32_t)i;
}

// gpn: the point-to-plane reduction's gather records, point and normal side
// by side (one 32 / 64-byte record per position instead of two gathers from
// two arrays)
template <typename T>
__global__ void grid_gather_kernel(const P4<T>* __restrict__ p, const P4<T>* __restrict__ nrm,
                                   const int32_t* __restrict__ sidx, int64_t valid, P4<T>* __restrict__ gp,
                                   P4<T>* __restrict__ gpn, int32_t* __restrict__ gi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= valid) return;
    const int32_t j = sidx[i];
    const P4<T> q = p[j];
    gp[i] = q;
    gi[i] = j;
    if (gpn) {
        gpn[2 * i] = q;
        gpn[2 * i + 1] = nrm[j];
    }
}

static int bits_for(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

// hipcub scratch of the setup sorts / scans
template <typename K>
static size_t sort_temp_bytes(int64_t n) {
    size_t t = 0;
    (void)pmx_sort_pairs(nullptr, t, (const K*)nullptr, (K*)nullptr, (const int32_t*)nullptr,
                                             (int32_t*)nullptr, (int)n, 0, (int)(8 * sizeof(K)));
    return t;
}
static size_t scan_temp_bytes(int64_t n) {
    size_t t = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, t, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
    return t;
}

// one grid level (sizes from the host): the layout of pmx_grid.hip
template <typename T>
int build_level_device(const P4<T>* pts, int64_t M, const P4<T>* nrm, const SetupShape& s, int64_t valid,
                       const SetupScratch& sc, P4<T>* gp, P4<T>* gpn, int32_t* gi, uint32_t* gstart, hipStream_t st) {
    const int64_t C = s.cells;
    hipError_t e = hipMemsetAsync(sc.counts, 0, sizeof(uint32_t) * (size_t)(C + 1), st);
    if (e != hipSuccess) return -1;
    if (M > 0) {
        hipLaunchKernelGGL(cell_keys_kernel<T>, dim3(blocks_for(M)), dim3(256), 0, st, pts, M, s, sc.keys32,
                           sc.idx, sc.counts);
        size_t tb = sc.temp_bytes;
        e = pmx_sort_pairs(sc.temp, tb, sc.keys32, sc.keys32_out, sc.idx, sc.idx_out, (int)M, 0,
                                               bits_for((uint64_t)C), st);
        if (e != hipSuccess) return -2;
    }
    size_t tb = sc.temp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(sc.temp, tb, sc.counts, gstart, (int)(C + 1), st);
    if (e != hipSuccess) return -3;
    if (valid > 0)
        hipLaunchKernelGGL(grid_gather_kernel<T>, dim3(blocks_for(valid)), dim3(256), 0, st, pts, nrm, sc.idx_out,
                           valid, gp, gpn, gi);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

size_t setup_temp_bytes(int64_t n, int64_t max_cells) {
    size_t a = sort_temp_bytes<uint32_t>(n), b = sort_temp_bytes<unsigned long long>(n),
           c = scan_temp_bytes(max_cells + 1);
    return std::max(a, std::max(b, c));
}

// ------------------------------------------------------------------ tree --
// The cold match's bounding-box tree over one grid level (MatchersImpl.cpp:
// 77-83: libnabo builds a kd-tree once per Matcher::init; here a 4-ary box
// tree whose leaves are the level's occupied cells, so a leaf is a contiguous
// position range and the search returns that level's positions).  Built from
// the level's sorted cell keys in five steps, no host synchronisation:
//   keys     the first position of every occupied cell gets the cell's
//            Morton code, every other position a sentinel (sorted last); the
//            occupied cells are counted into hdr[0]
//   sort     (Morton code, cell) pairs, stable (pmx_sort_pairs): the leaves
//            in Morton order come first
//   leaves   a leaf's position range from the cell starts and its box from its
//            points (float, rounded outward) into the level-1 records
//   levels   level l's record c-th box = the union of record (l-1, 4r + c)'s
//            four boxes, one launch per level up to the layout's top
// The record count of a level and the top level follow from hdr[0] on the
// device (the host sizes the layout from the point count, an upper bound).
constexpr uint32_t kTreeSentinel = 0xffffffffu;

__device__ __forceinline__ uint32_t spread3_10(uint32_t v) {
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(256) void tree_keys_kernel(const uint32_t* __restrict__ ckey, int64_t valid, int g0,
                                                        int g1, int shift, uint32_t* __restrict__ okey,
                                                        int32_t* __restrict__ oval, uint32_t* __restrict__ hdr) {
    __shared__ uint32_t cnt[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool first = false;
    if (i < valid) {
        const uint32_t c = ckey[i];
        first = i == 0 || ckey[i - 1] != c;
        uint32_t k = kTreeSentinel;
        if (first) {
            const uint32_t x = c % (uint32_t)g0, y = (c / (uint32_t)g0) % (uint32_t)g1,
                           z = c / ((uint32_t)g0 * (uint32_t)g1);
            k = spread3_10(x >> shift) | (spread3_10(y >> shift) << 1) | (spread3_10(z >> shift) << 2);
        }
        okey[i] = k;
        oval[i] = (int32_t)c;
    }
    const unsigned long long b = __ballot(first);
    if ((threadIdx.x & 63) == 0) cnt[threadIdx.x >> 6] = (uint32_t)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t n = cnt[0] + cnt[1] + cnt[2] + cnt[3];
        if (n) atomicAdd(hdr, n);
    }
}

// records at level l of a tree with n leaves (l = 0: the leaves)
__device__ __forceinline__ uint32_t tree_records(uint32_t n, int l) {
    for (int i = 0; i < l; ++i) n = (n + 3u) >> 2;
    return n;
}

template <typename T>
__device__ __forceinline__ float f_down(T v);
template <>
__device__ __forceinline__ float f_down<float>(float v) { return v; }
template <>
__device__ __forceinline__ float f_down<double>(double v) { return __double2float_rd(v); }
template <typename T>
__device__ __forceinline__ float f_up(T v);
template <>
__device__ __forceinline__ float f_up<float>(float v) { return v; }
template <>
__device__ __forceinline__ float f_up<double>(double v) { return __double2float_ru(v); }

// one record slot: box (mn, mx) of child c of record r
__device__ __forceinline__ void tree_put(float4* __restrict__ rec, uint32_t r, int c, const float (&mn)[3],
                                         const float (&mx)[3]) {
    float* R = reinterpret_cast<float*>(rec + (size_t)r * kTreeRecF4);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        R[4 * a + c] = mn[a];
        R[12 + 4 * a + c] = mx[a];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void tree_leaf_kernel(const int32_t* __restrict__ cells,
                                                        const uint32_t* __restrict__ gstart,
                                                        const P4<T>* __restrict__ gp, int64_t slots,
                                                        uint32_t* __restrict__ hdr, float4* __restrict__ rec) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= slots) return;
    const uint32_t n = hdr[0];
    float mn[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float mx[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    uint32_t a = 0, b = 0;
    if (i < (int64_t)n) {
        const uint32_t cell = (uint32_t)cells[i];
        a = gstart[cell];
        b = gstart[cell + 1];
        for (uint32_t p = a; p < b; ++p) {
            const P4<T> q = gp[p];
            mn[0] = fminf(mn[0], f_down<T>(q.x));
            mn[1] = fminf(mn[1], f_down<T>(q.y));
            mn[2] = fminf(mn[2], f_down<T>(q.z));
            mx[0] = fmaxf(mx[0], f_up<T>(q.x));
            mx[1] = fmaxf(mx[1], f_up<T>(q.y));
            mx[2] = fmaxf(mx[2], f_up<T>(q.z));
        }
    }
    const uint32_t r = (uint32_t)(i >> 2);
    const int c = (int)(i & 3);
    tree_put(rec, r, c, mn, mx);
    uint32_t* U = reinterpret_cast<uint32_t*>(rec + (size_t)r * kTreeRecF4) + 24;
    U[2 * c] = a;
    U[2 * c + 1] = b;
    if (i == 0) {
        uint32_t R = (n + 3u) >> 2;
        int l = 1;
        while (R > 1u) {
            R = (R + 3u) >> 2;
            ++l;
        }
        hdr[1] = (uint32_t)l;
    }
}

__global__ __launch_bounds__(256) void tree_level_kernel(float4* __restrict__ rec, uint32_t off_child,
                                                         uint32_t off_cur, int lvl, int64_t slots,
                                                         const uint32_t* __restrict__ hdr) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= slots) return;
    const uint32_t n = hdr[0];
    const uint32_t child = (uint32_t)i;  // (record 4r + c of level lvl - 1)
    float mn[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float mx[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    if (child < tree_records(n, lvl - 1)) {
        const float4* C = rec + (size_t)(off_child + child) * kTreeRecF4;
        const float4 v[6] = {C[0], C[1], C[2], C[3], C[4], C[5]};
        mn[0] = fminf(fminf(v[0].x, v[0].y), fminf(v[0].z, v[0].w));
        mn[1] = fminf(fminf(v[1].x, v[1].y), fminf(v[1].z, v[1].w));
        mn[2] = fminf(fminf(v[2].x, v[2].y), fminf(v[2].z, v[2].w));
        mx[0] = fmaxf(fmaxf(v[3].x, v[3].y), fmaxf(v[3].z, v[3].w));
        mx[1] = fmaxf(fmaxf(v[4].x, v[4].y), fmaxf(v[4].z, v[4].w));
        mx[2] = fmaxf(fmaxf(v[5].x, v[5].y), fmaxf(v[5].z, v[5].w));
    }
    tree_put(rec, off_cur + (uint32_t)(i >> 2), (int)(i & 3), mn, mx);
}

int tree_layout(int64_t valid, uint32_t off[kTreeMaxLevels], int64_t* records) {
    for (int l = 0; l < kTreeMaxLevels; ++l) off[l] = 0;
    int64_t R = (std::max<int64_t>(valid, 1) + 3) / 4, total = R;
    int l = 1;
    off[1] = 0;
    while (R > 1) {
        R = (R + 3) / 4;
        ++l;
        if (l >= kTreeMaxLevels) return -1;
        off[l] = (uint32_t)total;
        total += R;
    }
    if (records) *records = total;
    return l;  // the layout's top level
}

template <typename T>
int build_tree_device(const P4<T>* gp, const uint32_t* gstart, const SetupShape& s, int64_t valid,
                      const SetupScratch& sc, float4* rec, uint32_t* hdr, const uint32_t off[kTreeMaxLevels],
                      hipStream_t st) {
    (void)off;  // (the caller's copy of the same layout)
    uint32_t lay[kTreeMaxLevels];
    int64_t nrec = 0;
    const int top = tree_layout(valid, lay, &nrec);
    if (top < 1) return -5;
    hipError_t e = hipMemsetAsync(hdr, 0, 2 * sizeof(uint32_t), st);
    if (e != hipSuccess) return -1;
    if (valid > 0) {
        int gm = std::max(s.g[0], std::max(s.g[1], s.g[2])), shift = 0;
        while (((gm - 1) >> shift) >= 1024) ++shift;
        hipLaunchKernelGGL(tree_keys_kernel, dim3(blocks_for(valid)), dim3(256), 0, st, sc.keys32_out, valid,
                           s.g[0], s.g[1], shift, sc.keys32, sc.idx, hdr);
        size_t tb = sc.temp_bytes;
        e = pmx_sort_pairs(sc.temp, tb, sc.keys32, sc.keys32_out, sc.idx, sc.idx_out, (int)valid, 0, 32, st);
        if (e != hipSuccess) return -2;
    }
    int64_t R = (std::max<int64_t>(valid, 1) + 3) / 4;
    hipLaunchKernelGGL(tree_leaf_kernel<T>, dim3(blocks_for(4 * R)), dim3(256), 0, st, sc.idx_out, gstart, gp, 4 * R,
                       hdr, rec);
    for (int l = 2; l <= top; ++l) {
        R = (R + 3) / 4;  // (every record of level l in the layout; the ones past the tree's get empty boxes)
        hipLaunchKernelGGL(tree_level_kernel, dim3(blocks_for(4 * R)), dim3(256), 0, st, rec, lay[l - 1], lay[l], l,
                           4 * R, (const uint32_t*)hdr);
    }
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
template int build_tree_device<float>(const P4<float>*, const uint32_t*, const SetupShape&, int64_t,
                                      const SetupScratch&, float4*, uint32_t*, const uint32_t*, hipStream_t);
template int build_tree_device<double>(const P4<double>*, const uint32_t*, const SetupShape&, int64_t,
                                       const SetupScratch&, float4*, uint32_t*, const uint32_t*, hipStream_t);

// ---------------------------------------------------------------- morton --
__device__ __forceinline__ uint64_t dspread3(uint64_t v) {
    v &= 0x1fffffull;
    v = (v | v << 32) & 0x1f00000000ffffull;
    v = (v | v << 16) & 0x1f0000ff0000ffull;
    v = (v | v << 8) & 0x100f00f00f00f00full;
    v = (v | v << 4) & 0x10c30c30c30c30c3ull;
    v = (v | v << 2) & 0x1249249249249249ull;
    return v;
}

// slot key of a reading point: Morton code of the cell (finest level) of the
// point transformed by M0 in double (the host's build_order arithmetic);
// non-finite points last
template <typename T>
__global__ void morton_keys_kernel(const P4<T>* __restrict__ p, int64_t n, Mat4<T> M0, SetupShape s, int morton,
                                   unsigned long long sentinel, unsigned long long* __restrict__ keys,
                                   int32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const P4<T> r = p[i];
    const double x = ((double)M0.m[0] * r.x + (double)M0.m[1] * r.y) + (double)M0.m[2] * r.z + (double)M0.m[3] * r.w;
    const double y = ((double)M0.m[4] * r.x + (double)M0.m[5] * r.y) + (double)M0.m[6] * r.z + (double)M0.m[7] * r.w;
    const double z = ((double)M0.m[8] * r.x + (double)M0.m[9] * r.y) + (double)M0.m[10] * r.z + (double)M0.m[11] * r.w;
    unsigned long long k = sentinel;
    if (isfinite(x) && isfinite(y) && isfinite(z)) {
        int64_t ci[3];
        const int64_t c = dcell_of(s, x, y, z, ci);
        k = morton ? (dspread3((uint64_t)ci[0]) | (dspread3((uint64_t)ci[1]) << 1) | (dspread3((uint64_t)ci[2]) << 2))
                   : (unsigned long long)c;
    }
    keys[i] = k;
    idx[i] = (int32_t)i;
}

template <typename T>
__global__ void slot_gather_kernel(const P4<T>* __restrict__ raw, const int32_t* __restrict__ order, int64_t n,
                                   P4<T>* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = raw[order[i]];
}

// sc.keys64_out / sc.idx_out receive the sorted keys and the slot -> query order
template <typename T>
int reading_order_device(const P4<T>* raw, int64_t n, const Mat4<T>& M0, const SetupShape& s, bool morton,
                         const SetupScratch& sc, P4<T>* sorted, hipStream_t st) {
    if (n <= 0) return 0;
    // the sort runs over the key bits in use only (one onesweep pass per 8):
    // the Morton code of the largest cell coordinate, or the cell count, and
    // one more bit for the non-finite points' key (past every finite key)
    int gb = 1;
    while (gb < 21 && (((int64_t)1 << gb) < (int64_t)std::max(s.g[0], std::max(s.g[1], s.g[2])))) ++gb;
    const unsigned long long sentinel = morton ? (1ull << (3 * gb)) : (unsigned long long)s.cells;
    const int end_bit = bits_for(sentinel);
    hipLaunchKernelGGL(morton_keys_kernel<T>, dim3(blocks_for(n)), dim3(256), 0, st, raw, n, M0, s, morton ? 1 : 0,
                       sentinel, sc.keys64, sc.idx);
    size_t tb = sc.temp_bytes;
    hipError_t e = pmx_sort_pairs(sc.temp, tb, sc.keys64, sc.keys64_out, sc.idx, sc.idx_out, (int)n, 0, end_bit, st);
    if (e != hipSuccess) return -2;
    hipLaunchKernelGGL(slot_gather_kernel<T>, dim3(blocks_for(n)), dim3(256), 0, st, raw, sc.idx_out, n, sorted);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

// slot-major device array -> query-major (the mirrors' unpermute), 4 / 8-byte elements
template <typename E>
__global__ void unpermute_kernel(const E* __restrict__ src, const int32_t* __restrict__ order, int64_t n, int span,
                                 E* __restrict__ dst) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * span) return;
    const int64_t s = i / span, j = i - s * span;
    dst[(int64_t)order[s] * span + j] = src[i];
}
void launch_unpermute(const void* src, const int32_t* order, int64_t n, int span, size_t esz, void* dst,
                      hipStream_t s) {
    if (n <= 0) return;
    const int64_t tot = n * span;
    if (esz == 8)
        hipLaunchKernelGGL(unpermute_kernel<unsigned long long>, dim3(blocks_for(tot)), dim3(256), 0, s,
                           (const unsigned long long*)src, order, n, span, (unsigned long long*)dst);
    else
        hipLaunchKernelGGL(unpermute_kernel<uint32_t>, dim3(blocks_for(tot)), dim3(256), 0, s, (const uint32_t*)src,
                           order, n, span, (uint32_t*)dst);
}

// ---- KDTreeVarDistMatcher radii ----
template <typename T>
__global__ void gather_scalar_kernel(const T* __restrict__ src, const int32_t* __restrict__ order, int64_t n,
                                     T* __restrict__ dst) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[order ? order[i] : i];
}
template <typename T>
void launch_gather_scalar(const T* src, const int32_t* order, int64_t n, T* dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(gather_scalar_kernel<T>, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)), dim3(256),
                       0, s, src, order, n, dst);
}
template <typename T>
__global__ void apply_radii_kernel(T* __restrict__ d, int32_t* __restrict__ ids, const T* __restrict__ radii,
                                   int64_t N, int k) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N * k; e += stride) {
        const T r = radii[e / k];
        if (!(d[e] <= r * r)) {
            d[e] = (T)__builtin_huge_val();
            ids[e] = -1;
        }
    }
}
template <typename T>
void launch_apply_radii(T* dists, int32_t* ids, const T* radii, int64_t N, int k, hipStream_t s) {
    if (N <= 0) return;
    hipLaunchKernelGGL(apply_radii_kernel<T>, dim3((unsigned)std::min<int64_t>((N * k + 255) / 256, 4096)), dim3(256),
                       0, s, dists, ids, radii, N, k);
}

#define PMX_SETUP_INST(T)                                                                                            \
    template void launch_pack_p4<T>(const T*, int, int64_t, int64_t, P4<T>*, hipStream_t, const T*);                \
    template void launch_pack_nrm<T>(const T*, int, int64_t, P4<T>*, hipStream_t);                                  \
    template void launch_bbox<T>(const P4<T>*, int64_t, double*, double*, hipStream_t);                             \
    template void launch_occupancy<T>(const P4<T>*, int64_t, const SetupShape&, void*,                             \
                                      hipStream_t);                                                                 \
    template int build_level_device<T>(const P4<T>*, int64_t, const P4<T>*, const SetupShape&, int64_t,           \
                                       const SetupScratch&, P4<T>*, P4<T>*, int32_t*, uint32_t*, hipStream_t);      \
    template int reading_order_device<T>(const P4<T>*, int64_t, const Mat4<T>&, const SetupShape&, bool,           \
                                         const SetupScratch&, P4<T>*, hipStream_t);
PMX_SETUP_INST(float)
PMX_SETUP_INST(double)
template void launch_gather_scalar<float>(const float*, const int32_t*, int64_t, float*, hipStream_t);
template void launch_gather_scalar<double>(const double*, const int32_t*, int64_t, double*, hipStream_t);
template void launch_apply_radii<float>(float*, int32_t*, const float*, int64_t, int, hipStream_t);
template void launch_apply_radii<double>(double*, int32_t*, const double*, int64_t, int, hipStream_t);
#undef PMX_SETUP_INST

void preload_setup() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&cell_keys_kernel<float>));
}

}  // namespace pmx
