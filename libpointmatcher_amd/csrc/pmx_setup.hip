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
