// pmx_ssn.hip — SamplingSurfaceNormalDataPointsFilter on the device
// (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342; computeNormal /
// computeDensity / serializeEigVec / argMax, utils/utils.h:86-156).
//
// The reference splits the cloud recursively (buildNew, :171-221): a box
// with more than knn points is cut at the median of its longest side
// (std::nth_element), the halves recurse; a box of <= knn points is a leaf
// whose points get the leaf's normal / density / eigen pairs (fuseRange,
// :223-342) and are sub-sampled (rand() < ratio) or replaced by their mean.
//
// Here the recursion runs breadth-first, one level per round, over every box
// at once:
//   ranks      the (coordinate, index) rank of every point along each axis
//              (one radix sort per axis): comparing ranks is comparing
//              coordinates with the index breaking ties, a total order;
//   level      key = (box, rank along the box's cut axis) for every point,
//              one stable radix sort of all points: every box is sorted
//              along its own axis, its first count - count/2 points are the
//              left half; the cut value and the children's bounds follow
//              (the reference's leftMax / rightMin, :209-214);
//   leaves     a last sort by (leaf, index) puts every leaf's points in index
//              order, one thread per leaf does fuseRange.
// Deterministic where the reference is implementation-defined: ties of the
// median split broken by index (nth_element leaves them anywhere), a leaf's
// points in index order (the reference's order after nth_element is
// unspecified: it decides the mean's summation order, which point
// samplingMethod 1 keeps and the order of the rand() draws), eigen pairs as
// pmx_normals.hip (Jacobi in double, ascending, signed).  The CPU oracle
// (oracle/pmo_impl.inc) makes the same choices.
//
// The device does the sorts, the levels and the per-leaf statistics; the host
// assembles the output cloud (the sampling draws use the process's rand()
// state in the reference's order, and the output is in index order, :145-164).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "pmx_internal.h"
#include "pmx_sort.h"

#include "common/pmx_dense.h"

namespace pmx {

// (pmx_normals.hip)
template <int D>
__device__ void sym_eigen_ssn(double (&a)[D][D], double (&w)[D], double (&V)[D][D]) {
    double fro = 0.0;
    for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) {
            fro += a[r][c] * a[r][c];
            V[r][c] = r == c ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < D; ++p)
            for (int q = p + 1; q < D; ++q) off += a[p][q] * a[p][q];
        if (!(off > 1e-36 * fro)) break;
        for (int p = 0; p < D; ++p)
            for (int q = p + 1; q < D; ++q) {
                if (a[p][q] == 0.0) continue;
                const double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
                for (int r = 0; r < D; ++r) {
                    const double arp = a[r][p], arq = a[r][q];
                    a[r][p] = c * arp - s * arq;
                    a[r][q] = s * arp + c * arq;
                }
                for (int r = 0; r < D; ++r) {
                    const double apr = a[p][r], aqr = a[q][r];
                    a[p][r] = c * apr - s * aqr;
                    a[q][r] = s * apr + c * aqr;
                }
                for (int r = 0; r < D; ++r) {
                    const double vrp = V[r][p], vrq = V[r][q];
                    V[r][p] = c * vrp - s * vrq;
                    V[r][q] = s * vrp + c * vrq;
                }
            }
    }
    for (int i = 0; i < D; ++i) w[i] = a[i][i];
    for (int i = 0; i < D; ++i)
        for (int j = i + 1; j < D; ++j)
            if (w[j] < w[i]) {
                double t = w[i];
                w[i] = w[j];
                w[j] = t;
                for (int r = 0; r < D; ++r) {
                    t = V[r][i];
                    V[r][i] = V[r][j];
                    V[r][j] = t;
                }
            }
    for (int j = 0; j < D; ++j) {
        double big = V[0][j];
        for (int r = 1; r < D; ++r)
            if (fabs(V[r][j]) > fabs(big)) big = V[r][j];
        if (big < 0.0)
            for (int r = 0; r < D; ++r) V[r][j] = -V[r][j];
    }
}

template <typename T>
__device__ __forceinline__ T ssn_coord(const P4<T>& p, int r) {
    return r == 0 ? p.x : (r == 1 ? p.y : p.z);
}

// orderable key of a coordinate (-0 as +0: the reference's `<` ties them)
__device__ __forceinline__ unsigned long long okey(float v) {
    uint32_t b = __float_as_uint(v == 0.0f ? 0.0f : v);
    b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return (unsigned long long)b;
}
__device__ __forceinline__ unsigned long long okey(double v) {
    unsigned long long b = (unsigned long long)__double_as_longlong(v == 0.0 ? 0.0 : v);
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

static unsigned nblk(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

template <typename T>
__global__ void axis_keys_kernel(const P4<T>* __restrict__ p, int64_t n, int axis, unsigned long long* __restrict__ k,
                                 int32_t* __restrict__ idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    k[i] = okey(ssn_coord(p[i], axis));
    idx[i] = (int32_t)i;
}
__global__ void rank_scatter_kernel(const int32_t* __restrict__ sorted_idx, int64_t n, uint32_t* __restrict__ rank) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rank[sorted_idx[i]] = (uint32_t)i;
}

// box table (one level): first, count, bounds; cut axis (-1: leaf), children
template <typename T>
struct Boxes {
    int32_t* first;
    int32_t* cnt;
    T* lo;  // 3 per box
    T* hi;
    int32_t* cut;
    int32_t* nchild;  // 1 (leaf) or 2
};

// argMax (utils.h:141-156) over the box's extent: strict >, from 0 (the
// homogeneous row's zero extent never wins)
template <typename T>
__global__ void box_plan_kernel(Boxes<T> b, int64_t nbox, int D, int knn) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nbox) return;
    int cut = -1;
    if (b.cnt[s] > knn) {
        cut = 0;
        T best = 0;
        for (int r = 0; r < D; ++r) {
            const T e = b.hi[s * 3 + r] - b.lo[s * 3 + r];
            if (e > best) {
                best = e;
                cut = r;
            }
        }
    }
    b.cut[s] = cut;
    b.nchild[s] = cut >= 0 ? 2 : 1;
}

__global__ void level_keys_kernel(const int32_t* __restrict__ boxof, const int32_t* __restrict__ cut,
                                  const uint32_t* __restrict__ rank, const int32_t* __restrict__ perm, int64_t n,
                                  unsigned long long* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = boxof[i];
    const int c = cut[s];
    keys[i] = ((unsigned long long)(uint32_t)s << 32) | (c >= 0 ? (unsigned long long)rank[(int64_t)c * n + perm[i]] : 0ull);
}

// children (buildNew :189-220): left = first count - count/2 points, cut
// value = the left half's end point's coordinate
template <typename T>
__global__ void box_split_kernel(Boxes<T> b, int64_t nbox, const int32_t* __restrict__ base, Boxes<T> nb,
                                 const P4<T>* __restrict__ p, const int32_t* __restrict__ perm) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nbox) return;
    const int32_t o = base[s], f = b.first[s], c = b.cnt[s], cut = b.cut[s];
    T lo[3], hi[3];
    for (int r = 0; r < 3; ++r) {
        lo[r] = b.lo[s * 3 + r];
        hi[r] = b.hi[s * 3 + r];
    }
    if (cut < 0) {
        nb.first[o] = f;
        nb.cnt[o] = c;
        for (int r = 0; r < 3; ++r) {
            nb.lo[o * 3 + r] = lo[r];
            nb.hi[o * 3 + r] = hi[r];
        }
        return;
    }
    const int32_t right = c / 2, left = c - right;
    const T cv = ssn_coord(p[perm[f + left]], cut);
    nb.first[o] = f;
    nb.cnt[o] = left;
    nb.first[o + 1] = f + left;
    nb.cnt[o + 1] = right;
    for (int r = 0; r < 3; ++r) {
        nb.lo[o * 3 + r] = lo[r];
        nb.hi[o * 3 + r] = r == cut ? cv : hi[r];
        nb.lo[(o + 1) * 3 + r] = r == cut ? cv : lo[r];
        nb.hi[(o + 1) * 3 + r] = hi[r];
    }
}

__global__ void boxof_kernel(const int32_t* __restrict__ boxof, const int32_t* __restrict__ first,
                             const int32_t* __restrict__ cnt, const int32_t* __restrict__ cut,
                             const int32_t* __restrict__ base, int64_t n, int32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t s = boxof[i];
    int32_t o = base[s];
    if (cut[s] >= 0 && i >= first[s] + (cnt[s] - cnt[s] / 2)) ++o;
    out[i] = o;
}

__global__ void leaf_index_keys_kernel(const int32_t* __restrict__ boxof, const int32_t* __restrict__ perm, int64_t n,
                                       unsigned long long* __restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[i] = ((unsigned long long)(uint32_t)boxof[i] << 32) | (uint32_t)perm[i];
}

// fuseRange (:223-342) for one leaf per thread, its points in index order.
// rec: mean (D), normal (D), density, eigen values (D), eigen vectors (D*D);
// fit: 1, or 0 when the box is too large / C fails the rank test.
template <typename T, int D>
__global__ void leaf_kernel(const P4<T>* __restrict__ p, const int32_t* __restrict__ perm,
                            const int32_t* __restrict__ first, const int32_t* __restrict__ cnt, int64_t nleaf,
                            T max_box, int want_eig, T* __restrict__ rec, int32_t* __restrict__ fit) {
    const int64_t l = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nleaf) return;
    constexpr int RS = D + D + 1 + D + D * D;
    const int32_t f = first[l], c = cnt[l];
    // box (:233-243)
    T boxDim = 0;
    for (int r = 0; r < D; ++r) {
        T a = ssn_coord(p[perm[f]], r), b = a;
        for (int i = 1; i < c; ++i) {
            const T v = ssn_coord(p[perm[f + i]], r);
            a = v < a ? v : a;
            b = v > b ? v : b;
        }
        if (r == 0 || b - a > boxDim) boxDim = b - a;
    }
    if (boxDim > max_box) {
        fit[l] = 0;
        return;
    }
    T mean[D];
    for (int r = 0; r < D; ++r) {
        T s = ssn_coord(p[perm[f]], r);
        for (int i = 1; i < c; ++i) s = s + ssn_coord(p[perm[f + i]], r);
        mean[r] = s / (T)c;
    }
    T C[D * D];
    for (int e = 0; e < D * D; ++e) C[e] = 0;
    T maxn = 0;
    for (int i = 0; i < c; ++i) {
        const P4<T> q = p[perm[f + i]];
        T nn[D], n2 = 0;
        for (int r = 0; r < D; ++r) {
            nn[r] = ssn_coord(q, r) - mean[r];
            n2 = n2 + nn[r] * nn[r];
        }
        for (int a = 0; a < D; ++a)
            for (int b = 0; b < D; ++b) C[a * D + b] = C[a * D + b] + nn[a] * nn[b];
        const T nr = (T)sqrt((double)n2);
        maxn = nr > maxn ? nr : maxn;
    }
    T ev[D], evec[D][D];
    for (int r = 0; r < D; ++r) {
        ev[r] = r == 0 ? (T)1 : (T)0;  // Vector::Identity(D, 1)
        for (int cc = 0; cc < D; ++cc) evec[r][cc] = r == cc ? (T)1 : (T)0;
    }
    if (want_eig) {
        pmx_dense::FullPivQR<T> qr;
        qr.compute(C, D);
        if (!(qr.rank() + 1 >= D)) {  // (:254-264)
            fit[l] = 0;
            return;
        }
        double a[D][D], w[D], V[D][D];
        for (int r = 0; r < D; ++r)
            for (int cc = 0; cc < D; ++cc) a[r][cc] = (double)C[r * D + cc];
        sym_eigen_ssn<D>(a, w, V);
        for (int r = 0; r < D; ++r) {
            ev[r] = (T)w[r];
            for (int cc = 0; cc < D; ++cc) evec[r][cc] = (T)V[r][cc];
        }
    }
    T* R = rec + l * RS;
    for (int r = 0; r < D; ++r) {
        R[r] = mean[r];
        R[D + r] = evec[r][0];  // computeNormal: the smallest eigenvalue's vector
        R[2 * D + 1 + r] = ev[r];
    }
    R[2 * D] = (T)c / (T)((4.0 / 3.0) * 3.14159265358979323846 * pow((double)maxn, 3.0));  // computeDensity
    for (int r = 0; r < D; ++r)
        for (int cc = 0; cc < D; ++cc) R[3 * D + 1 + r * D + cc] = evec[r][cc];  // serializeEigVec: row-major
    fit[l] = 1;
}

// ------------------------------------------------------------------- host --
struct DevBuf {
    std::vector<void*> ptrs;
    ~DevBuf() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <typename X>
    X* get(size_t count) {
        void* p = nullptr;
        if (hipMalloc(&p, sizeof(X) * std::max<size_t>(count, 1)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return (X*)p;
    }
};

static int bits_of(uint64_t v) {
    int b = 1;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

// error codes as pmx.h (PMX_E_HIP = -10, PMX_E_BAD_PARAM = -3)
template <typename T>
int ssn_run(const P4<T>* d_pts, int D, int64_t n, int knn, T max_box, bool want_eig, hipStream_t st,
            std::vector<int32_t>& perm_h, std::vector<int32_t>& lfirst, std::vector<int32_t>& lcnt,
            std::vector<int32_t>& fit_h, std::vector<T>& rec_h, std::string& err) {
    DevBuf m;
    const int64_t nb_max = n;  // boxes never outnumber points
    unsigned long long* keys = m.get<unsigned long long>(n);
    unsigned long long* keys2 = m.get<unsigned long long>(n);
    int32_t* idx = m.get<int32_t>(n);
    int32_t* idx2 = m.get<int32_t>(n);
    uint32_t* rank = m.get<uint32_t>((size_t)n * D);
    int32_t* boxof = m.get<int32_t>(n);
    int32_t* boxof2 = m.get<int32_t>(n);
    Boxes<T> B[2];
    for (int k = 0; k < 2; ++k) {
        B[k].first = m.get<int32_t>(nb_max);
        B[k].cnt = m.get<int32_t>(nb_max);
        B[k].lo = m.get<T>(nb_max * 3);
        B[k].hi = m.get<T>(nb_max * 3);
        B[k].cut = m.get<int32_t>(nb_max);
        B[k].nchild = m.get<int32_t>(nb_max);
    }
    int32_t* base = m.get<int32_t>(nb_max + 1);
    size_t tsort = 0, tscan = 0;
    (void)pmx_sort_pairs(nullptr, tsort, keys, keys2, idx, idx2, (int)n, 0, 64, st);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tscan, B[0].nchild, base, (int)(nb_max + 1), st);
    const size_t tbytes = std::max(tsort, tscan);
    void* temp = m.get<char>(tbytes);
    for (void* q : m.ptrs)
        if (!q) {
            err = "SamplingSurfaceNormalDataPointsFilter: device allocation failed";
            return -10;
        }
    auto fail_hip = [&](const char* what) {
        err = std::string("SamplingSurfaceNormalDataPointsFilter: ") + what + ": " + hipGetErrorString(hipGetLastError());
        return -10;
    };
    // per-axis (coordinate, index) ranks
    for (int a = 0; a < D; ++a) {
        hipLaunchKernelGGL(axis_keys_kernel<T>, dim3(nblk(n)), dim3(256), 0, st, d_pts, n, a, keys, idx);
        size_t tb = tbytes;
        if (pmx_sort_pairs(temp, tb, keys, keys2, idx, idx2, (int)n, 0,
                                               sizeof(T) == 4 ? 32 : 64, st) != hipSuccess)
            return fail_hip("axis sort");
        hipLaunchKernelGGL(rank_scatter_kernel, dim3(nblk(n)), dim3(256), 0, st, idx2, n, rank + (size_t)a * n);
    }
    // the root box: the whole cloud, bounds = its coordinate extent
    // (rowwise min / max, :139-140: the first / last of each axis order)
    {
        std::vector<T> lo(3, 0), hi(3, 0);
        std::vector<P4<T>> ends(2);
        for (int a = 0; a < D; ++a) {
            hipLaunchKernelGGL(axis_keys_kernel<T>, dim3(nblk(n)), dim3(256), 0, st, d_pts, n, a, keys, idx);
            size_t tb = tbytes;
            if (pmx_sort_pairs(temp, tb, keys, keys2, idx, idx2, (int)n, 0,
                                                   sizeof(T) == 4 ? 32 : 64, st) != hipSuccess)
                return fail_hip("bounds sort");
            int32_t e[2];
            if (hipMemcpyAsync(&e[0], idx2, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipMemcpyAsync(&e[1], idx2 + n - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return fail_hip("bounds copy");
            for (int k = 0; k < 2; ++k)
                if (hipMemcpy(&ends[k], d_pts + e[k], sizeof(P4<T>), hipMemcpyDeviceToHost) != hipSuccess)
                    return fail_hip("bounds copy");
            lo[a] = a == 0 ? ends[0].x : a == 1 ? ends[0].y : ends[0].z;
            hi[a] = a == 0 ? ends[1].x : a == 1 ? ends[1].y : ends[1].z;
        }
        const int32_t f0 = 0, c0 = (int32_t)n;
        if (hipMemcpyAsync(B[0].first, &f0, sizeof(f0), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(B[0].cnt, &c0, sizeof(c0), hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(B[0].lo, lo.data(), sizeof(T) * 3, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(B[0].hi, hi.data(), sizeof(T) * 3, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemsetAsync(boxof, 0, sizeof(int32_t) * n, st) != hipSuccess)
            return fail_hip("root box");
    }
    // perm = identity (index order)
    {
        std::vector<int32_t> id((size_t)n);
        for (int64_t i = 0; i < n; ++i) id[(size_t)i] = (int32_t)i;
        if (hipMemcpyAsync(idx, id.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail_hip("identity");
    }
    int32_t* perm = idx;
    int32_t* perm2 = idx2;
    int cur = 0;
    int64_t nbox = 1;
    for (int level = 0; level < 64; ++level) {
        Boxes<T>& b = B[cur];
        hipLaunchKernelGGL(box_plan_kernel<T>, dim3(nblk(nbox)), dim3(256), 0, st, b, nbox, D, knn);
        size_t tb = tbytes;
        if (hipcub::DeviceScan::ExclusiveSum(temp, tb, b.nchild, base, (int)nbox, st) != hipSuccess)
            return fail_hip("box scan");
        int32_t nnew = 0;  // the new box count: base[nbox - 1] + nchild[nbox - 1]
        int32_t last_base = 0, last_child = 0;
        if (hipMemcpyAsync(&last_base, base + nbox - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(&last_child, b.nchild + nbox - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail_hip("box count");
        nnew = last_base + last_child;
        if (nnew == nbox) break;  // every box is a leaf
        // every box sorted along its own cut axis
        hipLaunchKernelGGL(level_keys_kernel, dim3(nblk(n)), dim3(256), 0, st, boxof, b.cut, rank, perm, n, keys);
        tb = tbytes;
        if (pmx_sort_pairs(temp, tb, keys, keys2, perm, perm2, (int)n, 0,
                                               32 + bits_of((uint64_t)nbox), st) != hipSuccess)
            return fail_hip("level sort");
        std::swap(perm, perm2);
        Boxes<T>& nb = B[cur ^ 1];
        hipLaunchKernelGGL(box_split_kernel<T>, dim3(nblk(nbox)), dim3(256), 0, st, b, nbox, base, nb, d_pts, perm);
        hipLaunchKernelGGL(boxof_kernel, dim3(nblk(n)), dim3(256), 0, st, boxof, b.first, b.cnt, b.cut, base, n,
                           boxof2);
        std::swap(boxof, boxof2);
        cur ^= 1;
        nbox = nnew;
    }
    // leaves in index order
    hipLaunchKernelGGL(leaf_index_keys_kernel, dim3(nblk(n)), dim3(256), 0, st, boxof, perm, n, keys);
    size_t tb = tbytes;
    if (pmx_sort_pairs(temp, tb, keys, keys2, perm, perm2, (int)n, 0, 32 + bits_of((uint64_t)nbox),
                                           st) != hipSuccess)
        return fail_hip("leaf sort");
    std::swap(perm, perm2);
    const int RS = D + D + 1 + D + D * D;
    T* rec = m.get<T>((size_t)nbox * RS);
    int32_t* fit = m.get<int32_t>(nbox);
    if (!rec || !fit) {
        err = "SamplingSurfaceNormalDataPointsFilter: device allocation failed";
        return -10;
    }
    const Boxes<T>& L = B[cur];
    if (D == 3)
        hipLaunchKernelGGL((leaf_kernel<T, 3>), dim3(nblk(nbox)), dim3(256), 0, st, d_pts, perm, L.first, L.cnt, nbox,
                           max_box, want_eig ? 1 : 0, rec, fit);
    else
        hipLaunchKernelGGL((leaf_kernel<T, 2>), dim3(nblk(nbox)), dim3(256), 0, st, d_pts, perm, L.first, L.cnt, nbox,
                           max_box, want_eig ? 1 : 0, rec, fit);
    if (hipGetLastError() != hipSuccess) return fail_hip("leaf kernel");
    perm_h.resize((size_t)n);
    lfirst.resize((size_t)nbox);
    lcnt.resize((size_t)nbox);
    fit_h.resize((size_t)nbox);
    rec_h.resize((size_t)nbox * RS);
    if (hipMemcpyAsync(perm_h.data(), perm, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(lfirst.data(), L.first, sizeof(int32_t) * nbox, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(lcnt.data(), L.cnt, sizeof(int32_t) * nbox, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(fit_h.data(), fit, sizeof(int32_t) * nbox, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(rec_h.data(), rec, sizeof(T) * nbox * RS, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail_hip("results copy");
    return 0;
}

template int ssn_run<float>(const P4<float>*, int, int64_t, int, float, bool, hipStream_t, std::vector<int32_t>&,
                            std::vector<int32_t>&, std::vector<int32_t>&, std::vector<int32_t>&,
                            std::vector<float>&, std::string&);
template int ssn_run<double>(const P4<double>*, int, int64_t, int, double, bool, hipStream_t, std::vector<int32_t>&,
                             std::vector<int32_t>&, std::vector<int32_t>&, std::vector<int32_t>&,
                             std::vector<double>&, std::string&);

void preload_ssn() {
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&leaf_kernel<float, 3>));
}

}  // namespace pmx
