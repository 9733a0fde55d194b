// pmx_filters_capi.hip — the stand-alone data filters of include/pmx.h:
// SurfaceNormal, SamplingSurfaceNormal and VoxelGrid on the device, each on a
// temporary context (the self-match of the normals uses the grid match).
#include "pmx_ctx.h"

namespace pmxc {

// SurfaceNormalDataPointsFilter (DataPointsFilters/SurfaceNormal.cpp:80-290):
// self-match on a temporary context, the statistics kernel, and the
// smoothNormals pass on the host (the reference smooths in place, point by
// point: later points see the already smoothed normals of earlier ones,
// :256-283 — a sequential dependency kept as is).
template <typename T>
int surface_normals_impl(int device, const T* feat, int rows, int64_t n, int knn, double maxDist, unsigned flags,
                         T* o_nrm, T* o_dens, T* o_eval, T* o_evec, T* o_ids, T* o_mdist, int64_t* degenerate) {
    if (rows != 3 && rows != 4) {
        g_err = "SurfaceNormalDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    if (knn < 1) {  // (SurfaceNormal.h:68: min 1; k > 16 on the wave-per-query search)
        g_err = "SurfaceNormalDataPointsFilter: knn must be >= 1";
        return PMX_E_BAD_PARAM;
    }
    if (degenerate) *degenerate = 0;
    if (n <= 0) return PMX_OK;
    pmx_ctx* c = nullptr;
    int rc = pmx_ctx_create(device, sizeof(T) == 8 ? PMX_F64 : PMX_F32, &c);
    if (rc) {
        g_err = "SurfaceNormalDataPointsFilter: no HIP device";
        return rc;
    }
    struct Guard {
        pmx_ctx* c;
        ~Guard() { pmx_ctx_destroy(c); }
    } guard{c};
    auto err = [&](int r) {
        g_err = c->err;
        return r;
    };
    c->reuse_on = false;
    c->search_type = 1;
    if (c->grid_mode == 0) c->grid_mode = 1;
    const int D = rows - 1;
    std::vector<T> I((size_t)rows * rows, (T)0);
    for (int i = 0; i < rows; ++i) I[(size_t)i * rows + i] = 1;
    if ((rc = set_reference_impl<T>(c, feat, rows, n, nullptr))) return err(rc);
    if ((rc = set_reading_impl<T>(c, feat, rows, n, I.data()))) return err(rc);
    if ((rc = match_impl<T>(c, I.data(), knn, maxDist, nullptr))) return err(rc);
    const int64_t per = D + 1 + D + D * D + 1;  // normals, density, eigen values, eigen vectors, mean distance
    T* d_out = nullptr;
    unsigned long long* d_deg = nullptr;
    HIPCHK(c, hipMalloc((void**)&d_out, sizeof(T) * (size_t)(n * per)));
    std::unique_ptr<void, void (*)(void*)> free_out(d_out, [](void* p) { (void)hipFree(p); });
    HIPCHK(c, hipMalloc((void**)&d_deg, sizeof(unsigned long long)));
    std::unique_ptr<void, void (*)(void*)> free_deg(d_deg, [](void* p) { (void)hipFree(p); });
    HIPCHK(c, hipMemsetAsync(d_deg, 0, sizeof(unsigned long long), c->stream));
    T* d_nrm = d_out;
    T* d_dens = d_nrm + n * D;
    T* d_eval = d_dens + n;
    T* d_evec = d_eval + n * D;
    T* d_md = d_evec + n * D * D;
    const GridLevel& L = c->lv(c->ids_level);
    launch_surface_normals<T>((const P4<T>*)c->d_rd, (const P4<T>*)L.gpts, c->d_ids, (const T*)c->d_dists, n, knn, D,
                              d_nrm, d_dens, d_eval, d_evec, d_md, d_deg, c->stream);
    HIPCHK(c, hipGetLastError());
    std::vector<T> h((size_t)(n * per));
    unsigned long long deg = 0;
    HIPCHK(c, hipMemcpyAsync(h.data(), d_out, sizeof(T) * h.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&deg, d_deg, sizeof(deg), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // slot order -> point order
    auto take = [&](int64_t off, int span, T* dst) {
        if (!dst) return;
        std::vector<T> src(h.begin() + off, h.begin() + off + n * span);
        (void)unpermute<T>(c, src, dst, span);  // (host_order below has run)
    };
    const bool smooth = (flags & PMX_SN_SMOOTH) && o_nrm;
    if ((rc = host_order(c))) return err(rc);
    take(0, D, o_nrm);
    take(n * D, 1, o_dens);
    take(n * (D + 1), D, o_eval);
    take(n * (2 * D + 1), D * D, o_evec);
    take(n * (2 * D + 1 + D * D), 1, o_mdist);
    if (o_ids || smooth) {
        std::vector<T> dd((size_t)(n * knn));
        std::vector<int32_t> ii((size_t)(n * knn));
        if ((rc = get_matches_impl<T>(c, dd.data(), ii.data()))) return err(rc);
        if (o_ids)  // matches.ids.cast<T>() (SurfaceNormal.cpp:250-253)
            for (size_t e = 0; e < ii.size(); ++e) o_ids[e] = (T)ii[e];
        if (smooth) {  // SurfaceNormal.cpp:256-283, in place, point order
            const T inf = std::numeric_limits<T>::infinity();
            for (int64_t i = 0; i < n; ++i) {
                T cur[3] = {0, 0, 0}, mean[3] = {0, 0, 0};
                for (int r = 0; r < D; ++r) cur[r] = o_nrm[i * D + r];
                int cnt = 0;
                for (int j = 0; j < knn; ++j) {
                    if (dd[(size_t)(i * knn + j)] == inf) continue;
                    const int64_t ref = ii[(size_t)(i * knn + j)];
                    const T* nb = o_nrm + ref * D;
                    T dot = 0;
                    for (int r = 0; r < D; ++r) dot = dot + cur[r] * nb[r];
                    for (int r = 0; r < D; ++r) mean[r] = dot > (T)0 ? mean[r] + nb[r] : mean[r] - nb[r];
                    ++cnt;
                }
                for (int r = 0; r < D; ++r) o_nrm[i * D + r] = mean[r] / (T)cnt;
            }
        }
    }
    if (degenerate) *degenerate = (int64_t)deg;
    return PMX_OK;
}

// SamplingSurfaceNormalDataPointsFilter::inPlaceFilter
// (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342): the split and the leaf
// statistics on the device (pmx_ssn.hip), the sampling and the output cloud
// here — fuseRange's draws in leaf order (:285-309), the output in index
// order (:145-164).
template <typename T>
int voxel_impl(int device, const T* feat, int rows, int64_t n, const T* desc, int desc_dim, const double* vsize,
               bool centroid, bool avg, T* feat_out, T* desc_out, int64_t* n_out) {
    if (rows != 3 && rows != 4) {
        g_err = "VoxelGridDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    *n_out = 0;
    if (n <= 0) return PMX_OK;
    if (hipSetDevice(device) != hipSuccess) {
        g_err = "VoxelGridDataPointsFilter: no HIP device";
        return PMX_E_HIP;
    }
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return PMX_E_HIP;
    std::unique_ptr<std::remove_pointer<hipStream_t>::type, void (*)(hipStream_t)> free_st(
        st, [](hipStream_t s) { (void)hipStreamDestroy(s); });
    const size_t fb = sizeof(T) * (size_t)rows * n, db = sizeof(T) * (size_t)desc_dim * n;
    char* buf = nullptr;
    if (hipMalloc(&buf, 2 * (fb + db) + 512) != hipSuccess) {
        g_err = "VoxelGridDataPointsFilter: device allocation failed";
        return PMX_E_HIP;
    }
    std::unique_ptr<void, void (*)(void*)> free_buf(buf, [](void* p) { (void)hipFree(p); });
    T* d_f = (T*)buf;
    T* d_d = (T*)(buf + ((fb + 255) & ~(size_t)255));
    T* d_of = (T*)((char*)d_d + ((db + 255) & ~(size_t)255));
    T* d_od = d_of + (size_t)rows * n;
    if (hipMemcpyAsync(d_f, feat, fb, hipMemcpyHostToDevice, st) != hipSuccess) return PMX_E_HIP;
    if (db && hipMemcpyAsync(d_d, desc, db, hipMemcpyHostToDevice, st) != hipSuccess) return PMX_E_HIP;
    std::string err;
    int64_t m = 0;
    const int rc = voxel_run<T>(d_f, rows, n, db ? d_d : nullptr, desc_dim, vsize, centroid, avg, d_of, d_od, &m, st,
                                err);
    if (rc) {
        g_err = err.empty() ? std::string("VoxelGridDataPointsFilter: HIP failure") : err;
        return rc;
    }
    if (hipMemcpyAsync(feat_out, d_of, sizeof(T) * (size_t)rows * m, hipMemcpyDeviceToHost, st) != hipSuccess)
        return PMX_E_HIP;
    if (db && desc_out &&
        hipMemcpyAsync(desc_out, d_od, sizeof(T) * (size_t)desc_dim * m, hipMemcpyDeviceToHost, st) != hipSuccess)
        return PMX_E_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return PMX_E_HIP;
    *n_out = m;
    return PMX_OK;
}

template <typename T>
int ssn_impl(int device, const T* feat, int rows, int64_t n, const T* desc, int desc_dim, int knn, int method,
             double ratio_d, double max_box_d, unsigned flags, T* feat_out, T* desc_out, T* o_nrm, T* o_dens,
             T* o_eval, T* o_evec, int64_t* n_out, int64_t* unfit_out) {
    if (rows != 3 && rows != 4) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: clouds must be 2-D or 3-D (3 or 4 homogeneous rows)";
        return PMX_E_BAD_PARAM;
    }
    if (knn < 3) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: knn must be >= 3";
        return PMX_E_BAD_PARAM;
    }
    if (method != 0 && method != 1) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: samplingMethod must be 0 or 1";
        return PMX_E_BAD_PARAM;
    }
    if (n > (int64_t)0x7fffffff) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: more than 2^31 points";
        return PMX_E_BAD_PARAM;
    }
    if (n_out) *n_out = 0;
    if (unfit_out) *unfit_out = 0;
    if (n <= 0) return PMX_OK;
    pmx_ctx* c = nullptr;
    int rc = pmx_ctx_create(device, sizeof(T) == 8 ? PMX_F64 : PMX_F32, &c);
    if (rc) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: no HIP device";
        return rc;
    }
    struct Guard {
        pmx_ctx* c;
        ~Guard() { pmx_ctx_destroy(c); }
    } guard{c};
    const int D = rows - 1;
    void* d_pts = nullptr;
    if (hipMalloc(&d_pts, sizeof(P4<T>) * n) != hipSuccess) {
        g_err = "SamplingSurfaceNormalDataPointsFilter: device allocation failed";
        return PMX_E_HIP;
    }
    std::unique_ptr<void, void (*)(void*)> free_pts(d_pts, [](void* p) { (void)hipFree(p); });
    if ((rc = upload_raw(c, feat, sizeof(T) * (size_t)rows * n))) {
        g_err = c->err;
        return rc;
    }
    launch_pack_p4<T>((const T*)c->d_raw, rows, n, n, (P4<T>*)d_pts, c->stream);
    const T ratio = (T)ratio_d, max_box = (T)max_box_d;
    const bool want_eig = (flags & (PMX_SSN_NORMALS | PMX_SSN_EIGVALUES | PMX_SSN_EIGVECTORS)) != 0;
    std::vector<int32_t> perm, lf, lc, fit;
    std::vector<T> rec;
    std::string err;
    if ((rc = ssn_run<T>((const P4<T>*)d_pts, D, n, knn, max_box, want_eig, c->stream, perm, lf, lc, fit, rec, err))) {
        g_err = err;
        return rc;
    }
    const int RS = D + D + 1 + D + D * D;
    // fuseRange's sampling, leaf by leaf in the recursion's order
    std::vector<int32_t> keep_leaf((size_t)n, -1);  // by point index: the leaf whose record it takes
    int64_t unfit = 0, kept = 0;
    for (size_t l = 0; l < lf.size(); ++l) {
        const int32_t f = lf[l], cnt = lc[l];
        if (!fit[l]) {
            unfit += cnt;
            continue;
        }
        if (method == 0) {
            for (int32_t i = 0; i < cnt; ++i) {
                const float r = (float)std::rand() / (float)RAND_MAX;
                if (r < ratio) {
                    keep_leaf[(size_t)perm[(size_t)(f + i)]] = (int32_t)l;
                    ++kept;
                }
            }
        } else {  // the smallest index of the leaf carries its mean
            keep_leaf[(size_t)perm[(size_t)f]] = (int32_t)l;
            ++kept;
        }
    }
    int64_t o = 0;
    for (int64_t k = 0; k < n; ++k) {
        const int32_t l = keep_leaf[(size_t)k];
        if (l < 0) continue;
        const T* R = rec.data() + (size_t)l * RS;
        if (feat_out) {
            if (method == 0) {
                for (int r = 0; r < rows; ++r) feat_out[o * rows + r] = feat[k * rows + r];
            } else {
                for (int r = 0; r < D; ++r) feat_out[o * rows + r] = R[r];
                feat_out[o * rows + D] = 1;
            }
        }
        if (desc_out && desc && desc_dim > 0) {
            if (method == 1 && (flags & PMX_SSN_AVERAGE)) {  // mergedDesc (:320-328)
                const int32_t f = lf[(size_t)l], cnt = lc[(size_t)l];
                for (int cc = 0; cc < desc_dim; ++cc) {
                    T s = 0;
                    for (int32_t i = 0; i < cnt; ++i) s = s + desc[(int64_t)perm[(size_t)(f + i)] * desc_dim + cc];
                    desc_out[o * desc_dim + cc] = s / (T)cnt;
                }
            } else {
                for (int cc = 0; cc < desc_dim; ++cc) desc_out[o * desc_dim + cc] = desc[k * desc_dim + cc];
            }
        }
        if (o_nrm)
            for (int r = 0; r < D; ++r) o_nrm[o * D + r] = R[D + r];
        if (o_dens) o_dens[o] = R[2 * D];
        if (o_eval)
            for (int r = 0; r < D; ++r) o_eval[o * D + r] = R[2 * D + 1 + r];
        if (o_evec)
            for (int e = 0; e < D * D; ++e) o_evec[o * D * D + e] = R[3 * D + 1 + e];
        ++o;
    }
    (void)kept;
    if (n_out) *n_out = o;
    if (unfit_out) *unfit_out = unfit;
    return PMX_OK;
}

}  // namespace pmxc

using namespace pmxc;

extern "C" {

int pmx_sampling_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc,
                                 int desc_dim, int knn, int sampling_method, double ratio, double max_box_dim,
                                 unsigned flags, void* feat_out, void* desc_out, void* normals, void* densities,
                                 void* eig_values, void* eig_vectors, int64_t* n_out, int64_t* unfit) {
    if ((!feat && n > 0) || (desc_dim > 0 && !desc && n > 0)) {
        g_err = "null cloud";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return ssn_impl<float>(device, (const float*)feat, rows, n, (const float*)desc, desc_dim, knn, sampling_method,
                               ratio, max_box_dim, flags, (float*)feat_out, (float*)desc_out, (float*)normals,
                               (float*)densities, (float*)eig_values, (float*)eig_vectors, n_out, unfit);
    if (dtype == PMX_F64)
        return ssn_impl<double>(device, (const double*)feat, rows, n, (const double*)desc, desc_dim, knn,
                                sampling_method, ratio, max_box_dim, flags, (double*)feat_out, (double*)desc_out,
                                (double*)normals, (double*)densities, (double*)eig_values, (double*)eig_vectors,
                                n_out, unfit);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

int pmx_voxel_grid(int device, int dtype, const void* feat, int rows, int64_t n, const void* desc, int desc_dim,
                   const double* vsize, int use_centroid, int average_desc, void* feat_out, void* desc_out,
                   int64_t* n_out) {
    if ((!feat && n > 0) || (desc_dim > 0 && !desc && n > 0) || !vsize || !n_out || (!feat_out && n > 0) ||
        desc_dim < 0) {
        g_err = "null argument";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return voxel_impl<float>(device, (const float*)feat, rows, n, (const float*)desc, desc_dim, vsize,
                                 use_centroid != 0, average_desc != 0, (float*)feat_out, (float*)desc_out, n_out);
    if (dtype == PMX_F64)
        return voxel_impl<double>(device, (const double*)feat, rows, n, (const double*)desc, desc_dim, vsize,
                                  use_centroid != 0, average_desc != 0, (double*)feat_out, (double*)desc_out, n_out);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

int pmx_surface_normals(int device, int dtype, const void* feat, int rows, int64_t n, int knn, double maxDist,
                        unsigned flags, void* normals, void* densities, void* eig_values, void* eig_vectors,
                        void* matched_ids, void* mean_dists, int64_t* degenerate) {
    if (!feat && n > 0) {
        g_err = "null cloud";
        return PMX_E_BAD_PARAM;
    }
    if (dtype == PMX_F32)
        return surface_normals_impl<float>(device, (const float*)feat, rows, n, knn, maxDist, flags, (float*)normals,
                                           (float*)densities, (float*)eig_values, (float*)eig_vectors,
                                           (float*)matched_ids, (float*)mean_dists, degenerate);
    if (dtype == PMX_F64)
        return surface_normals_impl<double>(device, (const double*)feat, rows, n, knn, maxDist, flags,
                                            (double*)normals, (double*)densities, (double*)eig_values,
                                            (double*)eig_vectors, (double*)matched_ids, (double*)mean_dists,
                                            degenerate);
    g_err = "dtype must be PMX_F32 or PMX_F64";
    return PMX_E_BAD_PARAM;
}

}  // extern "C"
