// pmx_voxel.hip — VoxelGridDataPointsFilter on the device
// (DataPointsFilters/VoxelGrid.cpp:60-343).
//
// The reference walks the points once, giving every point the linear index of
// its voxel (unsigned 32-bit arithmetic on floor(x / vSize - minBound)) and
// every voxel its first point; then, with useCentroid, it adds each later
// point of a voxel into that first point (in point order, in T) and divides
// by the count; without it, it overwrites feature rows 1..3 of the first
// point with the voxel centre (sic: the rows are shifted by one, so x stays,
// the homogeneous row of a 3-D cloud receives the z centre — reproduced as
// is); descriptors are averaged the same way (averageExistingDescriptors).
// The kept first points come out in index order.
//
// On the device: one pass for the per-axis min / max (exact: min / max of T
// values), the host derives the bounds and division counts in T exactly as
// the reference; one pass for the voxel keys; a stable radix sort of
// (key, point index) — within a voxel the points stay in index order, so the
// segment's first entry is the voxel's first point and a sequential sum over
// the segment is the reference's summation order; one thread per voxel then
// builds the output record; a last radix sort orders the voxels by their
// first point.  Bit-identical to the reference's arithmetic.
#include <algorithm>
#include <cmath>
#include <memory>
#include <string>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "pmx_internal.h"
#include "pmx_sort.h"

#include "../../include/pmx.h"

namespace pmx {

template <typename T>
__global__ __launch_bounds__(256) void vox_minmax_kernel(const T* __restrict__ f, int rows, int64_t n,
                                                         T* __restrict__ part) {
    const int D = rows - 1;
    T mn[3], mx[3];
    for (int a = 0; a < 3; ++a) {
        mn[a] = (T)__builtin_huge_val();
        mx[a] = -(T)__builtin_huge_val();
    }
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        for (int a = 0; a < D; ++a) {
            const T v = f[i * rows + a];
            mn[a] = v < mn[a] ? v : mn[a];  // (a NaN never wins: the reference's minCoeff skips it too)
            mx[a] = v > mx[a] ? v : mx[a];
        }
    __shared__ T smn[3][256], smx[3][256];
    for (int a = 0; a < 3; ++a) {
        smn[a][threadIdx.x] = mn[a];
        smx[a][threadIdx.x] = mx[a];
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int a = 0; a < 3; ++a) {
                const T b = smn[a][threadIdx.x + s], c = smx[a][threadIdx.x + s];
                smn[a][threadIdx.x] = b < smn[a][threadIdx.x] ? b : smn[a][threadIdx.x];
                smx[a][threadIdx.x] = c > smx[a][threadIdx.x] ? c : smx[a][threadIdx.x];
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < 3; ++a) {
            part[blockIdx.x * 6 + a] = smn[a][0];
            part[blockIdx.x * 6 + 3 + a] = smx[a][0];
        }
}

template <typename T>
struct VoxGeom {
    T vs[3];     // voxel sizes
    T minB[3];   // min / vSize
    uint32_t ndx, ndy, ndz;
    int rows;
};

// VoxelGrid.cpp:146-162: the voxel of a point, in the reference's unsigned arithmetic
template <typename T>
__global__ void vox_key_kernel(const T* __restrict__ f, int64_t n, VoxGeom<T> g, uint32_t* __restrict__ key,
                               uint32_t* __restrict__ idx) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += stride) {
        const T* x = f + p * g.rows;
        const uint32_t i = (uint32_t)floor(x[0] / g.vs[0] - g.minB[0]);
        const uint32_t j = (uint32_t)floor(x[1] / g.vs[1] - g.minB[1]);
        uint32_t v;
        if (g.rows == 4) {
            const uint32_t k = (uint32_t)floor(x[2] / g.vs[2] - g.minB[2]);
            v = i + j * g.ndx + k * g.ndx * g.ndy;
        } else {
            v = i + j * g.ndx;
        }
        key[p] = v;
        idx[p] = (uint32_t)p;
    }
}

__global__ void vox_iota_kernel(uint32_t* __restrict__ a, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += stride) a[s] = (uint32_t)s;
}

__global__ void vox_heads_kernel(const uint32_t* __restrict__ key, int64_t n, uint32_t* __restrict__ head) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n; s += stride)
        head[s] = (s == 0 || key[s] != key[s - 1]) ? 1u : 0u;
}

// one thread per voxel: the output record at slot v (VoxelGrid.cpp:165-314)
template <typename T>
__global__ void vox_record_kernel(const T* __restrict__ f, const T* __restrict__ desc, int desc_dim,
                                  const uint32_t* __restrict__ key, const uint32_t* __restrict__ idx,
                                  const uint32_t* __restrict__ seg_start, int64_t nseg, int64_t n, VoxGeom<T> g,
                                  int centroid, int avg, T* __restrict__ rf, T* __restrict__ rdsc,
                                  uint32_t* __restrict__ first_out, uint32_t* __restrict__ seg_id) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int rows = g.rows, D = rows - 1;
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nseg; v += stride) {
        const uint32_t a = seg_start[v];
        const uint32_t b = v + 1 < nseg ? seg_start[v + 1] : (uint32_t)n;
        const uint32_t first = idx[a];
        const uint32_t cnt = b - a;
        const T* x0 = f + (int64_t)first * rows;
        T* out = rf + v * rows;
        for (int r = 0; r < rows; ++r) out[r] = x0[r];
        if (centroid) {
            for (int r = 0; r < D; ++r) {  // (the homogeneous row is not summed)
                T s = x0[r];
                for (uint32_t q = a + 1; q < b; ++q) s += f[(int64_t)idx[q] * rows + r];
                out[r] = s / (T)cnt;
            }
        } else {
            const uint32_t vid = key[a];
            uint32_t k = 0;
            if (rows == 4) {
                k = vid / (g.ndx * g.ndy);
                out[3] = (T)k * g.vs[2] + g.vs[2] / (T)2;  // (the reference's k == numDivZ branch is unreachable)
            }
            const uint32_t j = (vid - k * g.ndx * g.ndy) / g.ndx;
            out[2] = (T)j * g.vs[1] + g.vs[1] / (T)2;
            const uint32_t i = vid - k * g.ndx * g.ndy - j * g.ndx;
            out[1] = (T)i * g.vs[0] + g.vs[0] / (T)2;
        }
        if (desc_dim > 0) {
            const T* d0 = desc + (int64_t)first * desc_dim;
            T* od = rdsc + v * desc_dim;
            for (int r = 0; r < desc_dim; ++r) {
                if (!avg) {
                    od[r] = d0[r];
                    continue;
                }
                T s = d0[r];
                for (uint32_t q = a + 1; q < b; ++q) s += desc[(int64_t)idx[q] * desc_dim + r];
                od[r] = s / (T)cnt;
            }
        }
        first_out[v] = first;
        seg_id[v] = (uint32_t)v;
    }
}

template <typename T>
__global__ void vox_gather_kernel(const T* __restrict__ rf, const T* __restrict__ rdsc, int rows, int desc_dim,
                                  const uint32_t* __restrict__ order, int64_t nseg, T* __restrict__ of,
                                  T* __restrict__ od) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nseg; i += stride) {
        const uint32_t v = order[i];
        for (int r = 0; r < rows; ++r) of[i * rows + r] = rf[(int64_t)v * rows + r];
        for (int r = 0; r < desc_dim; ++r) od[i * desc_dim + r] = rdsc[(int64_t)v * desc_dim + r];
    }
}

static unsigned vox_grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

// d_f: rows x n point-major on the device, d_desc desc_dim x n (or null).
// Outputs (device, capacity n): d_of, d_od; *n_out.  err: the reference's
// InvalidParameter message on a failure.
template <typename T>
int voxel_run(const T* d_f, int rows, int64_t n, const T* d_desc, int desc_dim, const double vsize[3], bool centroid,
              bool avg, T* d_of, T* d_od, int64_t* n_out, hipStream_t st, std::string& err) {
    *n_out = 0;
    if (n <= 0) return PMX_OK;
    if (n > (int64_t)0x7fffffff) {
        err = "VoxelGridDataPointsFilter: more than 2^31 points";
        return PMX_E_BAD_PARAM;
    }
    const int D = rows - 1;
    // bounds (VoxelGrid.cpp:87-120), all in T
    const unsigned nb = std::min<unsigned>(vox_grid(n), 1024);
    T* part = nullptr;
    if (hipMalloc(&part, sizeof(T) * 6 * nb) != hipSuccess) return PMX_E_HIP;
    std::unique_ptr<void, void (*)(void*)> free_part(part, [](void* p) { (void)hipFree(p); });
    hipLaunchKernelGGL(vox_minmax_kernel<T>, dim3(nb), dim3(256), 0, st, d_f, rows, n, part);
    std::vector<T> hp((size_t)6 * nb);
    if (hipMemcpyAsync(hp.data(), part, sizeof(T) * 6 * nb, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return PMX_E_HIP;
    T mn[3], mx[3];
    for (int a = 0; a < 3; ++a) {
        mn[a] = (T)INFINITY;
        mx[a] = -(T)INFINITY;
        for (unsigned b = 0; b < nb; ++b) {
            mn[a] = std::min(mn[a], hp[b * 6 + a]);
            mx[a] = std::max(mx[a], hp[b * 6 + 3 + a]);
        }
    }
    VoxGeom<T> g;
    g.rows = rows;
    T maxB[3];
    for (int a = 0; a < 3; ++a) {
        g.vs[a] = (T)vsize[a];
        g.minB[a] = a < D ? mn[a] / g.vs[a] : (T)0;
        maxB[a] = a < D ? mx[a] / g.vs[a] : (T)0;
    }
    // numDiv = 1 + maxBound - minBound in T, truncated to unsigned; a NaN or
    // an overflowing count is the reference's "couldn't be computed" / "memory allocation" error
    double cnt[3] = {1, 1, 1};
    for (int a = 0; a < D; ++a) {
        const T v = (T)1 + maxB[a] - g.minB[a];
        if (!(v >= (T)1) || !(v < (T)4294967296.0)) {
            err = "VoxelGridDataPointsFilter: The number of voxel couldn't be computed. There might be NaNs in the "
                  "feature matrix. Use the fileter RemoveNaNDataPointsFilter before this one if it's the case.";
            return PMX_E_BAD_PARAM;
        }
        cnt[a] = (double)(uint32_t)v;
    }
    g.ndx = (uint32_t)cnt[0];
    g.ndy = (uint32_t)cnt[1];
    g.ndz = D == 3 ? (uint32_t)cnt[2] : 0u;
    const double nvox = cnt[0] * cnt[1] * (D == 3 ? cnt[2] : 1.0);
    if (nvox > 4294967295.0) {  // (the reference's unsigned product wraps and indexes out of its vector)
        err = "VoxelGridDataPointsFilter: Memory allocation error with " + std::to_string((long long)nvox) +
              " voxels.  Try increasing the voxel dimensions.";
        return PMX_E_BAD_PARAM;
    }
    // keys, stable sort by voxel, segments
    uint32_t *key = nullptr, *key2 = nullptr, *idx = nullptr, *idx2 = nullptr, *head = nullptr, *segs = nullptr;
    int64_t* nsel = nullptr;
    void* temp = nullptr;
    size_t tsort = 0, tsel = 0, tsort2 = 0;
    (void)pmx_sort_pairs(nullptr, tsort, key, key2, idx, idx2, (int)n, 0, 32, st);
    (void)hipcub::DeviceSelect::Flagged(nullptr, tsel, idx, head, segs, nsel, (int)n, st);
    (void)pmx_sort_pairs(nullptr, tsort2, key, key2, idx, idx2, (int)n, 0, 32, st);
    const size_t tb = std::max(std::max(tsort, tsel), tsort2);
    const size_t words = (size_t)n;
    char* buf = nullptr;
    const size_t bytes = 6 * words * sizeof(uint32_t) + 256 + tb + 256 + sizeof(T) * (size_t)n * (rows + desc_dim);
    if (hipMalloc(&buf, bytes) != hipSuccess) {
        err = "VoxelGridDataPointsFilter: device allocation failed";
        return PMX_E_HIP;
    }
    std::unique_ptr<void, void (*)(void*)> free_buf(buf, [](void* p) { (void)hipFree(p); });
    key = (uint32_t*)buf;
    key2 = key + words;
    idx = key2 + words;
    idx2 = idx + words;
    head = idx2 + words;
    segs = head + words;
    nsel = (int64_t*)(segs + words);
    temp = (char*)nsel + 256;
    T* rf = (T*)((char*)temp + ((tb + 255) & ~(size_t)255));
    T* rdsc = rf + (size_t)n * rows;
    const unsigned G = vox_grid(n);
    hipLaunchKernelGGL(vox_key_kernel<T>, dim3(G), dim3(256), 0, st, d_f, n, g, key, idx);
    size_t t = tb;
    if (pmx_sort_pairs(temp, t, key, key2, idx, idx2, (int)n, 0, 32, st) != hipSuccess)
        return PMX_E_HIP;
    hipLaunchKernelGGL(vox_heads_kernel, dim3(G), dim3(256), 0, st, key2, n, head);
    // segment starts: the positions whose head flag is set (the positions are the iota in key)
    hipLaunchKernelGGL(vox_iota_kernel, dim3(G), dim3(256), 0, st, key, n);
    t = tb;
    if (hipcub::DeviceSelect::Flagged(temp, t, key, head, segs, nsel, (int)n, st) != hipSuccess) return PMX_E_HIP;
    int64_t nseg = 0;
    if (hipMemcpyAsync(&nseg, nsel, sizeof(int64_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return PMX_E_HIP;
    // records (first point per voxel in `key`, voxel slot ids in `head`), then index order
    hipLaunchKernelGGL(vox_record_kernel<T>, dim3(vox_grid(nseg)), dim3(256), 0, st, d_f, d_desc, desc_dim, key2, idx2,
                       segs, nseg, n, g, centroid ? 1 : 0, avg ? 1 : 0, rf, rdsc, key, head);
    t = tb;  // (first points -> idx, scratch; voxel slots in that order -> segs)
    if (pmx_sort_pairs(temp, t, key, idx, head, segs, (int)nseg, 0, 32, st) != hipSuccess)
        return PMX_E_HIP;
    hipLaunchKernelGGL(vox_gather_kernel<T>, dim3(vox_grid(nseg)), dim3(256), 0, st, rf, rdsc, rows, desc_dim, segs,
                       nseg, d_of, d_od);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess) return PMX_E_HIP;
    *n_out = nseg;
    return PMX_OK;
}

template int voxel_run<float>(const float*, int, int64_t, const float*, int, const double[3], bool, bool, float*,
                              float*, int64_t*, hipStream_t, std::string&);
template int voxel_run<double>(const double*, int, int64_t, const double*, int, const double[3], bool, bool, double*,
                               double*, int64_t*, hipStream_t, std::string&);

}  // namespace pmx
