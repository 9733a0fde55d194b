// pm_capi.cpp — extern "C" front-end of the host ICP chain (include/pmx_icp.h).
#include <cstring>
#include <memory>

#include "pm_icp.h"
#include "pmx_icp.h"

using namespace pm;

struct pmx_icp {
    int dtype = 0;
    // descriptors staged for the next compute / prepare: (cloud 0 reading /
    // 1 reference, name, span, point-major values as doubles)
    struct Desc {
        int cloud;
        std::string name;
        int span;
        std::vector<double> v;
    };
    std::vector<Desc> staged;
    std::unique_ptr<PointMatcher<float>::ICP> f;
    std::unique_ptr<PointMatcher<double>::ICP> d;
    std::string err;
};

namespace {

template <typename F>
int guarded(pmx_icp* icp, F&& fn) {
    try {
        fn();
        return PMX_ICP_OK;
    } catch (const ConvergenceError& e) {
        icp->err = e.what();
        return PMX_ICP_CONVERGENCE_ERROR;
    } catch (const InvalidParameter& e) {
        icp->err = e.what();
        return PMX_ICP_INVALID_PARAMETER;
    } catch (const TransformationError& e) {
        icp->err = e.what();
        return PMX_ICP_TRANSFORMATION_ERROR;
    } catch (const InvalidElement& e) {
        icp->err = e.what();
        return PMX_ICP_INVALID_ELEMENT;
    } catch (const InvalidModuleType& e) {
        icp->err = e.what();
        return PMX_ICP_INVALID_MODULE_TYPE;
    } catch (const ConfigurationError& e) {
        icp->err = e.what();
        return PMX_ICP_CONFIGURATION_ERROR;
    } catch (const std::exception& e) {
        icp->err = e.what();
        return PMX_ICP_RUNTIME_ERROR;
    }
}

template <typename T>
DataPoints<T> make_cloud(const void* feat, int rows, int64_t n, const void* normals) {
    DataPoints<T> c;
    c.rows = rows;
    c.n = n;
    // (borrowed: the caller's arrays stay valid for the call; DataPoints copies own their data)
    c.ext = static_cast<const T*>(feat);
    const char* xyz[] = {"x", "y", "z"};
    for (int r = 0; r < rows - 1; ++r) c.featureLabels.push_back({xyz[r], 1});
    c.featureLabels.push_back({"pad", 1});
    if (normals) {
        c.descriptorLabels.push_back({"normals", rows - 1});
        c.descDim = rows - 1;
        c.extDesc = static_cast<const T*>(normals);
    }
    return c;
}

template <typename T>
typename PointMatcher<T>::ICP& get(pmx_icp* icp);
template <>
PointMatcher<float>::ICP& get<float>(pmx_icp* icp) {
    return *icp->f;
}
template <>
PointMatcher<double>::ICP& get<double>(pmx_icp* icp) {
    return *icp->d;
}

// descriptors staged for `cloud` (0 reading, 1 reference) into c
template <typename T>
void take_staged(pmx_icp* icp, int cloud, DataPoints<T>& c) {
    std::vector<pmx_icp::Desc> rest;
    for (auto& d : icp->staged) {
        if (d.cloud != cloud) {
            rest.push_back(std::move(d));
            continue;
        }
        if ((int64_t)d.v.size() != c.n * d.span)
            throw InvalidParameter("descriptor " + d.name + ": " + std::to_string(d.v.size() / std::max(d.span, 1)) +
                                   " points staged for a cloud of " + std::to_string(c.n));
        std::vector<T> t(d.v.begin(), d.v.end());
        c.addDescriptor(d.name, d.span, t.data());
    }
    icp->staged = std::move(rest);
}

template <typename T>
std::vector<T> init_of(const void* T_init, int rows) {
    std::vector<T> Ti((size_t)rows * rows, (T)0);
    if (T_init) {
        const T* p = static_cast<const T*>(T_init);
        Ti.assign(p, p + (size_t)rows * rows);
    } else {
        for (int i = 0; i < rows; ++i) Ti[i * rows + i] = 1;
    }
    return Ti;
}

template <typename T>
void prepare_impl(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* reference, int64_t M,
                  const void* nrm, const void* T_init) {
    auto rd = make_cloud<T>(reading, rows, N, nullptr);
    auto ref = make_cloud<T>(reference, rows, M, nrm);
    take_staged<T>(icp, 0, rd);
    take_staged<T>(icp, 1, ref);
    get<T>(icp).prepare(rd, ref, init_of<T>(T_init, rows));
}

template <typename T>
void set_map_impl(pmx_icp* icp, const void* map, int rows, int64_t M, const void* nrm, int* accepted) {
    auto c = make_cloud<T>(map, rows, M, nrm);
    take_staged<T>(icp, 1, c);
    const bool ok = get<T>(icp).setMap(c);
    if (accepted) *accepted = ok ? 1 : 0;
}

template <typename T>
void get_map_impl(pmx_icp* icp, void* feat, int64_t capacity, int64_t* n, int* rows) {
    const auto g = get<T>(icp).getPrefilteredMap();
    if (n) *n = g.n;
    if (rows) *rows = g.rows;
    if (!feat) return;
    if (capacity < 0 || (uint64_t)capacity < (uint64_t)g.features.size())
        throw InvalidParameter("pmx_icp_get_map: capacity below n * rows");
    std::memcpy(feat, g.features.data(), sizeof(T) * g.features.size());
}

// 1: prepared (iterate / finish follow), 0: no map (T_out = identity)
template <typename T>
int seq_prepare_impl(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* T_init) {
    auto rd = make_cloud<T>(reading, rows, N, nullptr);
    take_staged<T>(icp, 0, rd);
    return get<T>(icp).prepareSequence(rd, init_of<T>(T_init, rows)) ? 1 : 0;
}

template <typename T>
void finish_impl(pmx_icp* icp, void* T_out) {
    auto out = get<T>(icp).finish();
    std::memcpy(T_out, out.data(), sizeof(T) * out.size());
}

template <typename T>
void stats_impl(const pmx_icp* icp, pmx_icp_stats* s) {
    auto& I = get<T>(const_cast<pmx_icp*>(icp));
    std::memset(s, 0, sizeof(*s));
    s->iterations = I.iterationCount;
    s->point_count_touched = I.matcher ? (int64_t)I.matcher->getVisitCount() : 0;
    if (I.errorMinimizer) {
        s->overlap_ratio = (double)I.errorMinimizer->getWeightedPointUsedRatio();
        s->point_used_ratio = (double)I.errorMinimizer->getPointUsedRatio();
        s->kept = I.errorMinimizer->keptPoints;
        s->rejected_matches = I.errorMinimizer->nbRejectedMatches;
        s->rejected_points = I.errorMinimizer->nbRejectedPoints;
    }
    s->convergence_duration = I.convergenceDuration;
    s->reference_preprocessing_duration = I.referencePreprocessingDuration;
    s->reading_preprocessing_duration = I.readingPreprocessingDuration;
    s->max_iterations_reached = I.maxNumIterationsReached ? 1 : 0;
}

}  // namespace

#define BOTH(icp, expr_f, expr_d) ((icp)->dtype == 1 ? (expr_d) : (expr_f))

extern "C" {

int pmx_icp_create(int dtype, int device, pmx_icp** out) {
    if (!out || (dtype != 0 && dtype != 1)) return PMX_ICP_INVALID_PARAMETER;
    pmx_icp* icp = new pmx_icp();
    icp->dtype = dtype;
    if (dtype == 1)
        icp->d.reset(new PointMatcher<double>::ICP(device));
    else
        icp->f.reset(new PointMatcher<float>::ICP(device));
    *out = icp;
    return PMX_ICP_OK;
}

void pmx_icp_destroy(pmx_icp* icp) { delete icp; }

const char* pmx_icp_last_error(const pmx_icp* icp) { return icp ? icp->err.c_str() : "null"; }

int pmx_icp_set_default(pmx_icp* icp) {
    return guarded(icp, [&] { BOTH(icp, icp->f->setDefault(), icp->d->setDefault()); });
}

int pmx_icp_load_yaml(pmx_icp* icp, const char* text) {
    return guarded(icp, [&] {
        const std::string s(text ? text : "");
        BOTH(icp, icp->f->loadFromYaml(s), icp->d->loadFromYaml(s));
    });
}

int pmx_icp_comm_init(pmx_icp* icp, const void* uid, int nranks, int rank) {
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        if (dev.ctx) throw std::runtime_error("pmx_icp_comm_init must precede the first compute");
        dev.nranks = nranks;
        dev.rank = rank;
        const unsigned char* p = static_cast<const unsigned char*>(uid);
        dev.uid.assign(p, p + 128);
    });
}

int pmx_icp_comm_init_host(pmx_icp* icp, int nranks, int rank, pmx_allreduce_fn allreduce, pmx_allgather_fn allgather,
                           void* user) {
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        if (dev.ctx) throw std::runtime_error("pmx_icp_comm_init_host must precede the first compute");
        if (!allreduce || !allgather || nranks < 1 || rank < 0 || rank >= nranks)
            throw InvalidParameter("pmx_icp_comm_init_host: bad arguments");
        dev.nranks = nranks;
        dev.rank = rank;
        dev.host_ar = allreduce;
        dev.host_ag = allgather;
        dev.host_user = user;
    });
}

int pmx_icp_keep_trace(pmx_icp* icp, int on) {
    return guarded(icp, [&] { BOTH(icp, icp->f->keepTrace = on != 0, icp->d->keepTrace = on != 0); });
}

int pmx_icp_prepare(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* reference, int64_t M,
                    const void* nrm, const void* T_init) {
    return guarded(icp, [&] {
        BOTH(icp, prepare_impl<float>(icp, reading, rows, N, reference, M, nrm, T_init),
             prepare_impl<double>(icp, reading, rows, N, reference, M, nrm, T_init));
    });
}

int pmx_icp_iterate(pmx_icp* icp, int n, int* done) {
    return guarded(icp, [&] {
        const bool more = BOTH(icp, icp->f->iterate(n), icp->d->iterate(n));
        if (done) *done = more ? 0 : 1;
    });
}

int pmx_icp_finish(pmx_icp* icp, void* T_out) {
    return guarded(icp, [&] { BOTH(icp, finish_impl<float>(icp, T_out), finish_impl<double>(icp, T_out)); });
}

int pmx_icp_add_descriptor(pmx_icp* icp, int cloud, const char* name, int span, const void* values, int64_t n) {
    if (!icp) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        if (!name || span < 1 || n < 0 || (!values && n > 0) || (cloud != 0 && cloud != 1))
            throw InvalidParameter("pmx_icp_add_descriptor: bad arguments");
        if (n > 0 && (uint64_t)n > ((uint64_t)1 << 40) / (uint64_t)span)
            throw InvalidParameter("pmx_icp_add_descriptor: descriptor too large");
        pmx_icp::Desc d{cloud, name, span, {}};
        d.v.resize((size_t)(n * span));
        for (int64_t i = 0; i < n * span; ++i)
            d.v[(size_t)i] = icp->dtype == 1 ? ((const double*)values)[i] : (double)((const float*)values)[i];
        icp->staged.push_back(std::move(d));
    });
}

int pmx_icp_compute(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* reference, int64_t M,
                    const void* nrm, const void* T_init, void* T_out) {
    int rc = pmx_icp_prepare(icp, reading, rows, N, reference, M, nrm, T_init);
    if (rc) return rc;
    int done = 0;
    while (!done) {
        rc = pmx_icp_iterate(icp, 1 << 20, &done);
        if (rc) return rc;
    }
    return pmx_icp_finish(icp, T_out);
}

int pmx_icp_set_map(pmx_icp* icp, const void* map, int rows, int64_t M, const void* nrm, int* accepted) {
    if (!icp) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        if ((!map && M > 0) || M < 0 || (rows != 3 && rows != 4)) throw InvalidParameter("pmx_icp_set_map: bad arguments");
        BOTH(icp, set_map_impl<float>(icp, map, rows, M, nrm, accepted),
             set_map_impl<double>(icp, map, rows, M, nrm, accepted));
    });
}

int pmx_icp_clear_map(pmx_icp* icp) {
    if (!icp) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] { BOTH(icp, icp->f->clearMap(), icp->d->clearMap()); });
}

int pmx_icp_has_map(const pmx_icp* icp, int* has) {
    if (!icp || !has) return PMX_ICP_INVALID_PARAMETER;
    *has = (icp->dtype == 1 ? icp->d->hasMap() : icp->f->hasMap()) ? 1 : 0;
    return PMX_ICP_OK;
}

int pmx_icp_get_map(pmx_icp* icp, void* features, int64_t capacity, int64_t* n, int* rows) {
    if (!icp) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        BOTH(icp, get_map_impl<float>(icp, features, capacity, n, rows),
             get_map_impl<double>(icp, features, capacity, n, rows));
    });
}

int pmx_icp_sequence_prepare(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* T_init, int* prepared) {
    if (!icp) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        // (the pmx_icp_set_map checks: make_cloud reads rows - 1 coordinates per point)
        if ((!reading && N > 0) || N < 0 || (rows != 3 && rows != 4))
            throw InvalidParameter("pmx_icp_sequence_prepare: bad arguments");
        const int p = BOTH(icp, seq_prepare_impl<float>(icp, reading, rows, N, T_init),
                           seq_prepare_impl<double>(icp, reading, rows, N, T_init));
        if (prepared) *prepared = p;
    });
}

int pmx_icp_sequence_compute(pmx_icp* icp, const void* reading, int rows, int64_t N, const void* T_init,
                             void* T_out) {
    if (!icp || !T_out) return PMX_ICP_INVALID_PARAMETER;
    if ((!reading && N > 0) || N < 0 || (rows != 3 && rows != 4)) {  // (before the identity is written)
        icp->err = "pmx_icp_sequence_compute: bad arguments";
        return PMX_ICP_INVALID_PARAMETER;
    }
    int prepared = 0;
    int rc = pmx_icp_sequence_prepare(icp, reading, rows, N, T_init, &prepared);
    if (rc) return rc;
    if (!prepared) {  // ICP.cpp:599-604: no map, identity
        for (int i = 0; i < rows * rows; ++i) {
            const double v = i % (rows + 1) == 0 ? 1.0 : 0.0;
            if (icp->dtype == 1)
                ((double*)T_out)[i] = v;
            else
                ((float*)T_out)[i] = (float)v;
        }
        return PMX_ICP_OK;
    }
    int done = 0;
    while (!done) {
        rc = pmx_icp_iterate(icp, 1 << 20, &done);
        if (rc) return rc;
    }
    return pmx_icp_finish(icp, T_out);
}

int pmx_icp_stats_get(const pmx_icp* icp, pmx_icp_stats* out) {
    if (!icp || !out) return PMX_ICP_INVALID_PARAMETER;
    if (icp->dtype == 1)
        stats_impl<double>(icp, out);
    else
        stats_impl<float>(icp, out);
    return PMX_ICP_OK;
}

int pmx_icp_trace_get(const pmx_icp* icp, void* out, int max_iters) {
    if (!icp || !out) return 0;
    int n = 0;
    if (icp->dtype == 1) {
        for (auto& t : icp->d->trace) {
            if (n >= max_iters) break;
            std::memcpy((double*)out + (size_t)n * t.size(), t.data(), sizeof(double) * t.size());
            ++n;
        }
    } else {
        for (auto& t : icp->f->trace) {
            if (n >= max_iters) break;
            std::memcpy((float*)out + (size_t)n * t.size(), t.data(), sizeof(float) * t.size());
            ++n;
        }
    }
    return n;
}

int pmx_icp_timing(pmx_icp* icp, int on) {
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        dev.ensure();
        dev.check(pmx_timing_enable(dev.ctx, on));
    });
}

int pmx_icp_timing_read(pmx_icp* icp, double* ms, int64_t* launches) {
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        dev.ensure();
        double other = 0;
        dev.check(pmx_timing_read(dev.ctx, ms, launches, &other));
    });
}

int pmx_icp_select_stats(pmx_icp* icp, uint64_t* hits, uint64_t* misses) {
    if (!icp || !hits || !misses) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        dev.ensure();
        dev.check(pmx_loop_select_stats(dev.ctx, hits, misses));
    });
}

int pmx_icp_loop_diag(pmx_icp* icp, int first, int count, int64_t* out) {
    if (!icp || (!out && count > 0)) return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        dev.ensure();
        dev.check(pmx_loop_diag(dev.ctx, first, count, out));
    });
}

int pmx_icp_comm_stats(pmx_icp* icp, uint64_t* allreduces, uint64_t* allgathers, uint64_t* verdict_syncs,
                       uint64_t* async_iterations, uint64_t* stalls) {
    if (!icp || !allreduces || !allgathers || !verdict_syncs || !async_iterations || !stalls)
        return PMX_ICP_INVALID_PARAMETER;
    return guarded(icp, [&] {
        Device& dev = icp->dtype == 1 ? icp->d->dev : icp->f->dev;
        dev.ensure();
        dev.check(pmx_comm_stats(dev.ctx, allreduces, allgathers));
        dev.check(pmx_comm_loop_stats(dev.ctx, verdict_syncs, async_iterations, stalls));
    });
}

}  // extern "C"

// ---------------------------------------------------------------- clouds --
struct pmx_cloud {
    int dtype = 0;
    pm::DataPoints<float> f;
    pm::DataPoints<double> d;
};

namespace {
thread_local std::string g_cloud_err;
template <typename T>
const pm::DataPoints<T>& cloud_of(const pmx_cloud* c);
template <>
const pm::DataPoints<float>& cloud_of<float>(const pmx_cloud* c) { return c->f; }
template <>
const pm::DataPoints<double>& cloud_of<double>(const pmx_cloud* c) { return c->d; }
template <typename T>
void cloud_copy(const pmx_cloud* c, void* feat, void* desc) {
    const auto& dp = cloud_of<T>(c);
    if (feat) std::memcpy(feat, dp.features.data(), sizeof(T) * dp.features.size());
    if (desc) std::memcpy(desc, dp.descriptors.data(), sizeof(T) * dp.descriptors.size());
}
}  // namespace

extern "C" {

int pmx_cloud_load(const char* path, int dtype, pmx_cloud** out) {
    if (!path || !out || (dtype != 0 && dtype != 1)) {
        g_cloud_err = "null argument or bad dtype";
        return PMX_ICP_INVALID_PARAMETER;
    }
    *out = nullptr;
    try {
        auto* c = new pmx_cloud;
        c->dtype = dtype;
        if (dtype == 1)
            c->d = pm::load_cloud<double>(path);
        else
            c->f = pm::load_cloud<float>(path);
        *out = c;
        return PMX_ICP_OK;
    } catch (const std::exception& e) {
        g_cloud_err = e.what();
        return PMX_ICP_RUNTIME_ERROR;
    }
}

void pmx_cloud_destroy(pmx_cloud* c) { delete c; }

const char* pmx_cloud_last_error(void) { return g_cloud_err.c_str(); }

int pmx_cloud_info(const pmx_cloud* c, int64_t* n, int* rows, int* desc_dim, int* nfl, int* ndl) {
    if (!c) return PMX_ICP_INVALID_PARAMETER;
    auto fill = [&](const auto& dp) {
        if (n) *n = dp.n;
        if (rows) *rows = dp.rows;
        if (desc_dim) *desc_dim = dp.descDim;
        if (nfl) *nfl = (int)dp.featureLabels.size();
        if (ndl) *ndl = (int)dp.descriptorLabels.size();
    };
    if (c->dtype == 1)
        fill(c->d);
    else
        fill(c->f);
    return PMX_ICP_OK;
}

int pmx_cloud_label(const pmx_cloud* c, int which, int i, char* name, int cap, int* span) {
    if (!c || !name || cap < 1) return PMX_ICP_INVALID_PARAMETER;
    auto get = [&](const auto& dp) -> int {
        const auto& ls = which == 0 ? dp.featureLabels : dp.descriptorLabels;
        if (i < 0 || i >= (int)ls.size()) return PMX_ICP_INVALID_PARAMETER;
        std::snprintf(name, (size_t)cap, "%s", ls[(size_t)i].text.c_str());
        if (span) *span = ls[(size_t)i].span;
        return PMX_ICP_OK;
    };
    return c->dtype == 1 ? get(c->d) : get(c->f);
}

int pmx_cloud_data(const pmx_cloud* c, void* feat, void* desc) {
    if (!c) return PMX_ICP_INVALID_PARAMETER;
    if (c->dtype == 1)
        cloud_copy<double>(c, feat, desc);
    else
        cloud_copy<float>(c, feat, desc);
    return PMX_ICP_OK;
}

}  // extern "C"

