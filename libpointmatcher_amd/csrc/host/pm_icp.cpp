// pm_icp.cpp — modules, registry and the ICP loop of the GPU path.
//
// Module names, parameter names, defaults and bounds are those of the
// reference so that libpointmatcher YAML chain files load unchanged:
//   KDTreeMatcher, KDTreeVarDistMatcher  MatchersImpl.h:74-134
//   Null/MaxDist/MinDist/MedianDist/TrimmedDist/VarTrimmedDist/Robust OutlierFilter
//                                 OutlierFiltersImpl.h:51-260
//   PointToPlane / PointToPoint ErrorMinimizer
//                                 ErrorMinimizers/PointToPlane.h:61-90, PointToPoint.h
//   Counter / Differential / Bound TransformationChecker
//                                 TransformationCheckersImpl.h:60-130
//   Identity / SurfaceNormal / MaxDist / MinDist / RandomSampling / FixStepSampling /
//   BoundingBox DataPointsFilter  DataPointsFilters/{SurfaceNormal,MaxDist,MinDist,RandomSampling,FixStepSampling,BoundingBox}.h
//   NullInspector, NullLogger (+ no-op stand-ins for
//   the VTK/Performance inspectors and FileLogger, accepted for config
//   compatibility)
#include "pm_icp.h"

#include <cstdlib>
#include <cstring>
#include <iostream>

namespace pm {

// ------------------------------------------------------------------ Device --
Device::~Device() {
    if (ctx) pmx_ctx_destroy(ctx);
}

void Device::ensure() {
    if (ctx) return;
    const int rc = pmx_ctx_create(device, dtype, &ctx);
    if (rc != PMX_OK) {
        ctx = nullptr;
        throw std::runtime_error("pmx_ctx_create failed (" + std::to_string(rc) + "): no usable HIP device " +
                                 std::to_string(device) + " (" + std::to_string(pmx_device_count()) + " visible)");
    }
    if (host_ar) {
        check(pmx_comm_init_host(ctx, nranks, rank, host_ar, host_ag, host_user));
    } else if (!uid.empty()) {  // (a communicator issues its collectives at any nranks, also 1)
        if (uid.size() != 128) throw std::runtime_error("multi-rank ICP needs a 128-byte RCCL unique id");
        check(pmx_comm_init(ctx, uid.data(), nranks, rank));
    }
}

void Device::check(int rc) const {
    if (rc == PMX_OK) return;
    const std::string msg = ctx ? pmx_last_error(ctx) : "no device context";
    switch (rc) {
    case PMX_E_NO_POINTS:
    case PMX_E_EMPTY_QUANTILE:
        throw ConvergenceError(msg);
    case PMX_E_CONVERGENCE:
        throw ConvergenceError(msg);
    case PMX_E_BAD_PARAM:
        throw InvalidParameter(msg);
    case PMX_E_TRANSFORMATION:
        throw TransformationError(msg);
    default:
        throw std::runtime_error("pmx error " + std::to_string(rc) + ": " + msg);
    }
}

template <typename T>
static int dtype_of() {
    return sizeof(T) == 8 ? PMX_F64 : PMX_F32;
}

// ----------------------------------------------------------------- Matches --
template <typename T>
void PointMatcher<T>::Matches::mirror() const {
    if (mirrored) return;
    dists.resize((size_t)n * knn);
    ids.resize((size_t)n * knn);
    dev->check(pmx_get_matches(dev->ctx, dists.data(), ids.data()));
    mirrored = true;
}

template <typename T>
T PointMatcher<T>::Matches::getDistsQuantile(T quantile) const {
    mirror();
    std::vector<T> v;
    v.reserve(dists.size());
    for (T d : dists)
        if (d != std::numeric_limits<T>::infinity()) v.push_back(d);
    if (v.empty()) throw ConvergenceError("no outlier to filter");
    if (quantile < (T)0 || quantile > (T)1) throw ConvergenceError("quantile must be between 0 and 1");
    if (quantile == (T)1) return *std::max_element(v.begin(), v.end());
    size_t idx = (size_t)((T)v.size() * quantile);
    if (idx >= v.size()) idx = v.size() - 1;
    std::nth_element(v.begin(), v.begin() + idx, v.end());
    return v[idx];
}

// ================================================================= modules ==
namespace {

template <typename T>
using PM = PointMatcher<T>;

// ---- KDTreeMatcher on the GPU (exact search; see pmx_match.hip) ----------
// Matcher::init of both kd-tree matchers: the reference (and its normals,
// for the point-to-plane minimiser) to HBM, the search structure built there
template <typename T>
void matcher_init(Device& dev, const DataPoints<T>& ref, int searchType, const T* centre, T* mean_out) {
    dev.ensure();
    std::vector<T> nrm;
    const T* np = nullptr;
    if (ref.descriptorLabels.size() == 1 && ref.descriptorLabels[0].text == "normals" &&
        ref.descriptorLabels[0].span == ref.rows - 1) {
        np = ref.desc();  // (the only descriptor: already the dense D x n block, no copy)
    } else if (ref.descriptorExists("normals")) {
        int span = 0;
        nrm = ref.descriptor("normals", &span);
        if (span < ref.rows - 1) throw InvalidElement("normals descriptor has fewer rows than the dimension");
        if (span != ref.rows - 1) {
            std::vector<T> t((size_t)(ref.rows - 1) * ref.n);
            for (int64_t i = 0; i < ref.n; ++i)
                for (int r = 0; r < ref.rows - 1; ++r) t[i * (ref.rows - 1) + r] = nrm[i * span + r];
            nrm.swap(t);
        }
        np = nrm.data();
    }
    dev.check(pmx_set_search(dev.ctx, searchType));  // 0: brute force, 1/2: exact grid search
    if (mean_out)
        dev.check(pmx_set_reference_mean_centred(dev.ctx, ref.feat(), ref.rows, ref.n, np, mean_out));
    else if (centre)
        dev.check(pmx_set_reference_centred(dev.ctx, ref.feat(), ref.rows, ref.n, np, centre));
    else
        dev.check(pmx_set_reference(dev.ctx, ref.feat(), ref.rows, ref.n, np));
}
template <typename T>
typename PM<T>::Matches device_matches(Device& dev, int knn) {
    typename PM<T>::Matches m;
    m.dev = &dev;
    m.knn = knn;
    int64_t n = 0;
    pmx_get_shape(dev.ctx, &n, nullptr);
    m.n = n;
    return m;
}

template <typename T>
struct KDTreeMatcherGPU : PM<T>::Matcher {
    typedef typename PM<T>::Matches Matches;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("knn", "number of nearest neighbors to consider it the reference", "1", "1", "2147483647",
                     &Parametrizable::Comp<unsigned>),
                PDoc("epsilon", "approximation to use for the nearest-neighbor search", "0", "0", "inf",
                     &Parametrizable::Comp<T>),
                PDoc("searchType", "Nabo search type (the GPU search is exact for every type)", "1", "0", "2",
                     &Parametrizable::Comp<unsigned>),
                PDoc("maxDist", "maximum distance to consider for neighbors", "inf", "0", "inf",
                     &Parametrizable::Comp<T>)};
    }
    int knn;
    T epsilon;
    int searchType;
    T maxDist;
    explicit KDTreeMatcherGPU(const Parametrizable::Parameters& p)
        : PM<T>::Matcher("KDTreeMatcher", doc(), p),
          knn(this->template get<int>("knn")),
          epsilon(this->template get<T>("epsilon")),
          searchType(this->template get<int>("searchType")),
          maxDist(this->template get<T>("maxDist")) {}

    void init(Device& dev, const DataPoints<T>& ref, const T* centre, T* mean_out) override {
        matcher_init<T>(dev, ref, searchType, centre, mean_out);
    }
    Matches findClosests(Device& dev, const std::vector<T>& T_iter) override {
        // PointCountTouched is added from the minimiser's pmx_stats.visited
        // once the (asynchronous) match has completed, see ICP::step
        dev.check(pmx_match(dev.ctx, T_iter.data(), knn, (double)maxDist, (double)epsilon, nullptr));
        return device_matches<T>(dev, knn);
    }
    bool loopConfig(pmx_loop_cfg& cfg) const override {
        cfg.knn = knn;
        cfg.max_dist = (double)maxDist;
        return true;
    }
};

// ---- KDTreeVarDistMatcher (MatchersImpl.h:105-134, MatchersImpl.cpp:106-150):
// the radius of each reading point is its maxDistField descriptor; the GPU
// search takes the radii per query (pmx_set_reading_radii)
template <typename T>
struct KDTreeVarDistMatcherGPU : PM<T>::Matcher {
    typedef typename PM<T>::Matches Matches;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("knn", "number of nearest neighbors to consider it the reference", "1", "1", "2147483647",
                     &Parametrizable::Comp<unsigned>),
                PDoc("epsilon", "approximation to use for the nearest-neighbor search", "0", "0", "inf",
                     &Parametrizable::Comp<T>),
                PDoc("searchType", "Nabo search type (the GPU search is exact for every type)", "1", "0", "2",
                     &Parametrizable::Comp<unsigned>),
                PDoc("maxDistField", "descriptor field name used to set a maximum distance to consider for neighbors "
                                     "per point", "maxSearchDist")};
    }
    int knn;
    T epsilon;
    int searchType;
    std::string maxDistField;
    explicit KDTreeVarDistMatcherGPU(const Parametrizable::Parameters& p)
        : PM<T>::Matcher("KDTreeVarDistMatcher", doc(), p),
          knn(this->template get<int>("knn")),
          epsilon(this->template get<T>("epsilon")),
          searchType(this->template get<int>("searchType")),
          maxDistField(this->template get<std::string>("maxDistField")) {}
    void init(Device& dev, const DataPoints<T>& ref, const T* centre, T* mean_out) override {
        matcher_init<T>(dev, ref, searchType, centre, mean_out);
    }
    void initReading(Device& dev, const DataPoints<T>& reading) override {
        // getDescriptorViewByName(maxDistField).transpose(): one radius per point
        int span = 0;
        const std::vector<T> r = reading.descriptor(maxDistField, &span);
        if (span != 1)
            throw InvalidElement("KDTreeVarDistMatcher: descriptor " + maxDistField + " must have one row, not " +
                                 std::to_string(span));
        dev.check(pmx_set_reading_radii(dev.ctx, r.data()));
    }
    Matches findClosests(Device& dev, const std::vector<T>& T_iter) override {
        dev.check(pmx_match(dev.ctx, T_iter.data(), knn, INFINITY, (double)epsilon, nullptr));
        return device_matches<T>(dev, knn);
    }
    bool loopConfig(pmx_loop_cfg& cfg) const override {
        cfg.knn = knn;
        cfg.max_dist = INFINITY;  // (the per-point radii stay set on the context)
        return true;
    }
};

// ---- outlier filters ------------------------------------------------------
template <typename T>
struct NullOF : PM<T>::OutlierFilter {
    explicit NullOF(const Parametrizable::Parameters&) {}
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_null(d.ctx, pos));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_NULL;
        return true;
    }
};
template <typename T>
struct MaxDistOF : PM<T>::OutlierFilter {
    T maxDist;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("maxDist", "threshold distance (Euclidean norm)", "1", "0.0000001", "inf", &Parametrizable::Comp<T>)};
    }
    explicit MaxDistOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("MaxDistOutlierFilter", doc(), p), maxDist(this->template get<T>("maxDist")) {}
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_maxdist(d.ctx, pos, (double)maxDist));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_MAXDIST;
        cfg.filter_p[pos][0] = (double)maxDist;
        return true;
    }
};
template <typename T>
struct MinDistOF : PM<T>::OutlierFilter {
    T minDist;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("minDist", "threshold distance (Euclidean norm)", "1", "0.0000001", "inf", &Parametrizable::Comp<T>)};
    }
    explicit MinDistOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("MinDistOutlierFilter", doc(), p), minDist(this->template get<T>("minDist")) {}
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_mindist(d.ctx, pos, (double)minDist));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_MINDIST;
        cfg.filter_p[pos][0] = (double)minDist;
        return true;
    }
};
template <typename T>
struct MedianDistOF : PM<T>::OutlierFilter {
    T factor;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("factor", "points farther away factor * median will be considered outliers.", "3", "0.0000001",
                     "inf", &Parametrizable::Comp<T>)};
    }
    explicit MedianDistOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("MedianDistOutlierFilter", doc(), p), factor(this->template get<T>("factor")) {}
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_mediandist(d.ctx, pos, (double)factor));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_MEDIANDIST;
        cfg.filter_p[pos][0] = (double)factor;
        return true;
    }
};
template <typename T>
struct TrimmedDistOF : PM<T>::OutlierFilter {
    T ratio;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("ratio", "percentage to keep", "0.85", "0.0000001", "1.0", &Parametrizable::Comp<T>)};
    }
    explicit TrimmedDistOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("TrimmedDistOutlierFilter", doc(), p), ratio(this->template get<T>("ratio")) {}
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_trimmed(d.ctx, pos, (double)ratio));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_TRIMMED;
        cfg.filter_p[pos][0] = (double)ratio;
        return true;
    }
};
template <typename T>
struct VarTrimmedDistOF : PM<T>::OutlierFilter {
    T minRatio, maxRatio, lambda;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("minRatio", "min ratio", "0.05", "0.0000001", "1", &Parametrizable::Comp<T>),
                PDoc("maxRatio", "max ratio", "0.99", "0.0000001", "1", &Parametrizable::Comp<T>),
                PDoc("lambda", "lambda (part of the term that balance the rmsd: 1/ratio^lambda", "2.35")};
    }
    explicit VarTrimmedDistOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("VarTrimmedDistOutlierFilter", doc(), p),
          minRatio(this->template get<T>("minRatio")),
          maxRatio(this->template get<T>("maxRatio")),
          lambda(this->template get<T>("lambda")) {
        if (minRatio >= maxRatio)  // OutlierFiltersImpl.cpp:160-163
            throw InvalidParameter("VarTrimmedDistOutlierFilter: minRatio (" + std::to_string(minRatio) +
                                   ") should be smaller than maxRatio (" + std::to_string(maxRatio) + ")");
    }
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        d.check(pmx_outlier_vartrimmed(d.ctx, pos, (double)minRatio, (double)maxRatio, (double)lambda));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_VARTRIMMED;
        cfg.filter_p[pos][0] = (double)minRatio;
        cfg.filter_p[pos][1] = (double)maxRatio;
        cfg.filter_p[pos][2] = (double)lambda;
        return true;
    }
};

// RobustOutlierFilter (OutlierFiltersImpl.h:220-260, OutlierFiltersImpl.cpp:380-598):
// the parameters and the filter's state (iteration, berg target, tuning
// substitution) stay here as in the reference object; the scale and the
// weights are computed on the device (pmx_outlier_robust).  In the device
// loop the same schedule runs from the loop's iteration index (loopConfig
// hands over the call counter; loopAdvance counts the iterations that ran).
template <typename T>
struct RobustOF : PM<T>::OutlierFilter {
    std::string robustFctName, scaleEstimator, distanceType;
    T tuning, squaredApproximation, approximation;
    int nbIterationForScale;
    int robustFctId = -1;
    int iteration = 1;
    T berg_target_scale = 0;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("robustFct", "Type of robust function used. Available fct: 'cauchy', 'welsch', 'sc', 'gm', "
                                  "'tukey', 'huber', 'L1' and 'student'.", "cauchy"),
                PDoc("tuning", "Tuning parameter used to limit the influence of outliers (the target scale with "
                               "'berg').", "1.0", "0.0000001", "inf", &Parametrizable::Comp<T>),
                PDoc("scaleEstimator", "'none', 'mad', 'berg' or 'std'", "mad"),
                PDoc("nbIterationForScale", "iterations the scale is recomputed for (0: every iteration)", "0", "0",
                     "100", &Parametrizable::Comp<int>),
                PDoc("distanceType", "'point2point' or 'point2plane'", "point2point"),
                PDoc("approximation", "weights of errors above this threshold are forced to zero (inf: none)", "inf",
                     "0.0", "inf", &Parametrizable::Comp<T>)};
    }
    explicit RobustOF(const Parametrizable::Parameters& p)
        : PM<T>::OutlierFilter("RobustOutlierFilter", doc(), p),
          robustFctName(this->template get<std::string>("robustFct")),
          scaleEstimator(this->template get<std::string>("scaleEstimator")),
          distanceType(this->template get<std::string>("distanceType")),
          tuning(this->template get<T>("tuning")),
          approximation(this->template get<T>("approximation")),
          nbIterationForScale(this->template get<int>("nbIterationForScale")) {
        squaredApproximation = (T)std::pow(approximation, 2);
        if (scaleEstimator != "none" && scaleEstimator != "mad" && scaleEstimator != "berg" && scaleEstimator != "std")
            throw InvalidParameter("Invalid scale estimator name.");
        if (distanceType != "point2point" && distanceType != "point2plane")
            throw InvalidParameter("Invalid distance type name.");
        static const char* names[] = {"cauchy", "welsch", "sc", "gm", "tukey", "huber", "L1", "student"};
        for (int i = 0; i < 8; ++i)
            if (robustFctName == names[i]) robustFctId = i;  // (PMX_RF_* order)
        if (robustFctId < 0) throw InvalidParameter("Invalid robust function name.");
        if (scaleEstimator == "berg") {  // Bergstrom 2014 tunings (:419-433)
            berg_target_scale = tuning;
            if (robustFctId == PMX_RF_CAUCHY) tuning = (T)4.3040;
            else if (robustFctId == PMX_RF_TUKEY) tuning = (T)7.0589;
            else if (robustFctId == PMX_RF_HUBER) tuning = (T)2.0138;
        }
    }
    void compute(Device& d, const typename PM<T>::Matches&, int pos) override {
        // robustFiltering's scale schedule (:500-531); iteration counts the
        // filter's calls over its lifetime, as the reference member does
        const bool recompute = iteration <= nbIterationForScale || nbIterationForScale == 0;
        int mode = PMX_RS_NONE;
        if (scaleEstimator == "mad") mode = recompute ? PMX_RS_MAD : PMX_RS_KEEP;
        else if (scaleEstimator == "std") mode = recompute ? PMX_RS_STD : PMX_RS_KEEP;
        else if (scaleEstimator == "berg")
            mode = !recompute ? PMX_RS_KEEP : (iteration == 1 ? PMX_RS_BERG_FIRST : PMX_RS_BERG_NEXT);
        ++iteration;
        d.check(pmx_outlier_robust(d.ctx, pos, robustFctId, (double)tuning, (double)approximation, mode,
                                   (double)berg_target_scale, distanceType == "point2plane" ? 1 : 0));
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.filter_kind[pos] = PMX_FILTER_ROBUST;
        cfg.robust_fct = robustFctId;
        cfg.robust_estimator = scaleEstimator == "mad"   ? PMX_RSE_MAD
                               : scaleEstimator == "std" ? PMX_RSE_STD
                               : scaleEstimator == "berg" ? PMX_RSE_BERG
                                                          : PMX_RSE_NONE;
        cfg.robust_p2pl = distanceType == "point2plane" ? 1 : 0;
        cfg.robust_nb_iter_for_scale = nbIterationForScale;
        cfg.robust_first_call = iteration;
        cfg.robust_tuning = (double)tuning;
        cfg.robust_approx = (double)approximation;
        cfg.robust_berg_target = (double)berg_target_scale;
        return true;
    }
    void loopAdvance(int64_t iterations) override { iteration += (int)iterations; }
};

// ---- error minimisers -----------------------------------------------------
template <typename T>
void build_p2plane_transform(int rows, const T* x, std::vector<T>& out) {
    // PointToPlane.cpp:245-312 (shared with the device loop: pmx_dense.h)
    out.assign((size_t)rows * rows, (T)0);
    dense::p2plane_transform(rows, x, out.data());
}

template <typename T>
struct PointToPlaneEM : PM<T>::ErrorMinimizer {
    bool force2D, force4DOF;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("force2D",
                     "If set to true(1), the minimization will be forced to give a solution in 2D (i.e., on the "
                     "XY-plane) even with 3D inputs.",
                     "0", "0", "1", &Parametrizable::Comp<bool>),
                PDoc("force4DOF",
                     "If set to true(1), the minimization will optimize only yaw and translation, pitch and roll "
                     "will follow the prior.",
                     "0", "0", "1", &Parametrizable::Comp<bool>)};
    }
    explicit PointToPlaneEM(const Parametrizable::Parameters& p)
        : PM<T>::ErrorMinimizer("PointToPlaneErrorMinimizer", doc(), p),
          force2D(this->template get<T>("force2D") != (T)0),
          force4DOF(this->template get<T>("force4DOF") != (T)0) {
        if (force2D && force4DOF)
            throw ConfigurationError("Force 2D cannot be used together with force4DOF.");
    }
    std::vector<T> compute(Device& d, int rows) override {
        if (force2D || force4DOF)
            throw ConfigurationError("PointToPlaneErrorMinimizer: force2D / force4DOF are outside the GPU path");
        const int n = rows == 4 ? 6 : 3;
        double A[36], b[6];
        pmx_stats st;
        d.check(pmx_p2plane_system(d.ctx, A, b, &st));
        this->setStats(st);
        T At[36], bt[6], x[6];
        for (int i = 0; i < n * n; ++i) At[i] = (T)A[i];
        for (int i = 0; i < n; ++i) bt[i] = (T)b[i];
        dense::solve_underdetermined(At, bt, n, x);
        std::vector<T> out;
        build_p2plane_transform(rows, x, out);
        return out;
    }
    bool loopConfig(pmx_loop_cfg& cfg) const override {
        cfg.minimizer = 0;
        return !force2D && !force4DOF;
    }
};

template <typename T>
struct PointToPointEM : PM<T>::ErrorMinimizer {
    explicit PointToPointEM(const Parametrizable::Parameters&) { this->className = "PointToPointErrorMinimizer"; }
    std::vector<T> compute(Device& d, int rows) override {
        // PointToPoint.cpp:61-101
        const int D = rows - 1;
        double mp[3], mq[3], md[9];
        pmx_stats st;
        d.check(pmx_p2point_system(d.ctx, mp, mq, md, &st));
        this->setStats(st);
        T m[9], mpT[3], mqT[3];
        for (int i = 0; i < D * D; ++i) m[i] = (T)md[i];
        for (int i = 0; i < D; ++i) {
            mpT[i] = (T)mp[i];
            mqT[i] = (T)mq[i];
        }
        std::vector<T> out((size_t)rows * rows, (T)0);
        dense::p2point_transform(rows, m, mpT, mqT, out.data());  // (shared with the device loop)
        return out;
    }
    bool loopConfig(pmx_loop_cfg& cfg) const override {
        cfg.minimizer = 1;
        return true;
    }
};

// ---- transformation checkers ------------------------------------------------
template <typename T>
void rot3(const std::vector<T>& M, int rows, T* m3) {
    // topLeftCorner(3,3) — in 2-D this is the whole 3x3 homogeneous matrix,
    // exactly as the reference's check() uses it
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) m3[r * 3 + c] = M[r * rows + c];
}

template <typename T>
struct CounterTC : PM<T>::TransformationChecker {
    unsigned maxIterationCount;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("maxIterationCount", "maximum number of iterations ", "40", "0", "2147483647",
                     &Parametrizable::Comp<unsigned>)};
    }
    explicit CounterTC(const Parametrizable::Parameters& p)
        : PM<T>::TransformationChecker("CounterTransformationChecker", doc(), p),
          maxIterationCount(this->template get<unsigned>("maxIterationCount")) {
        this->limits = {(T)maxIterationCount};
        this->conditionVariableNames = {"Iteration"};
        this->limitNames = {"Max iteration"};
    }
    void init(const std::vector<T>&, int, bool&) override { this->conditionVariables = {(T)0}; }
    void check(const std::vector<T>&, int, bool& iterate) override {
        this->conditionVariables[0] = this->conditionVariables[0] + (T)1;
        if (this->conditionVariables[0] >= this->limits[0]) {  // TransformationCheckersImpl.cpp:71-75
            iterate = false;
            throw typename PM<T>::MaxNumIterationsReached();
        }
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.checker_kind[pos] = PMX_CHECK_COUNTER;
        cfg.checker_p[pos][0] = (double)this->limits[0];
        return true;
    }
};

template <typename T>
struct DifferentialTC : PM<T>::TransformationChecker {
    T minDiffRotErr, minDiffTransErr;
    unsigned smoothLength;
    std::vector<std::array<T, 4>> rotations;
    std::vector<std::array<T, 3>> translations;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("minDiffRotErr", "threshold for rotation error (radian)", "0.001", "0.", "6.2831854",
                     &Parametrizable::Comp<T>),
                PDoc("minDiffTransErr", "threshold for translation error", "0.001", "0.", "inf", &Parametrizable::Comp<T>),
                PDoc("smoothLength", "number of iterations over which to average the differencial error", "3", "0",
                     "2147483647", &Parametrizable::Comp<unsigned>)};
    }
    explicit DifferentialTC(const Parametrizable::Parameters& p)
        : PM<T>::TransformationChecker("DifferentialTransformationChecker", doc(), p),
          minDiffRotErr(this->template get<T>("minDiffRotErr")),
          minDiffTransErr(this->template get<T>("minDiffTransErr")),
          smoothLength(this->template get<unsigned>("smoothLength")) {
        this->limits = {minDiffRotErr, minDiffTransErr};
    }
    void push(const std::vector<T>& M, int rows, bool init2d) {
        T m3[9], q[4];
        if (init2d) {
            // TransformationCheckersImpl.cpp:107-110: 2-D init uses [R 0; 0 1]
            for (int i = 0; i < 9; ++i) m3[i] = (i % 4 == 0) ? (T)1 : (T)0;
            m3[0] = M[0];
            m3[1] = M[1];
            m3[3] = M[3];
            m3[4] = M[4];
        } else {
            rot3(M, rows, m3);
        }
        dense::quat_from_matrix(m3, q);
        rotations.push_back({q[0], q[1], q[2], q[3]});
        std::array<T, 3> t{0, 0, 0};
        for (int r = 0; r < rows - 1; ++r) t[r] = M[r * rows + rows - 1];
        translations.push_back(t);
    }
    void init(const std::vector<T>& M, int rows, bool&) override {
        this->conditionVariables = {(T)0, (T)0};
        rotations.clear();
        translations.clear();
        push(M, rows, rows != 4);
    }
    void check(const std::vector<T>& M, int rows, bool& iterate) override {
        push(M, rows, false);
        T cv0 = 0, cv1 = 0;
        if (rotations.size() > smoothLength) {
            for (size_t i = rotations.size() - 1; i >= rotations.size() - smoothLength; i--) {
                cv0 = cv0 + std::fabs(dense::angular_distance(rotations[i].data(), rotations[i - 1].data()));
                T nn = 0;
                for (int r = 0; r < rows - 1; ++r) {
                    const T d = translations[i][r] - translations[i - 1][r];
                    nn = nn + d * d;
                }
                cv1 = cv1 + std::fabs(std::sqrt(nn));
            }
            cv0 = cv0 / (T)smoothLength;
            cv1 = cv1 / (T)smoothLength;
            if (cv0 < this->limits[0] && cv1 < this->limits[1]) iterate = false;
        }
        this->conditionVariables = {cv0, cv1};
        if (cv0 != cv0) throw ConvergenceError("abs rotation norm not a number");
        if (cv1 != cv1) throw ConvergenceError("abs translation norm not a number");
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.checker_kind[pos] = PMX_CHECK_DIFFERENTIAL;
        cfg.checker_p[pos][0] = (double)minDiffRotErr;
        cfg.checker_p[pos][1] = (double)minDiffTransErr;
        cfg.checker_p[pos][2] = (double)smoothLength;
        return smoothLength < 64;  // the device history ring
    }
};

template <typename T>
struct BoundTC : PM<T>::TransformationChecker {
    T maxRotationNorm, maxTranslationNorm;
    std::array<T, 4> q0{};
    T rot2d0 = 0;
    std::array<T, 3> t0{};
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("maxRotationNorm", "rotation bound", "1", "0", "inf", &Parametrizable::Comp<T>),
                PDoc("maxTranslationNorm", "translation bound", "1", "0", "inf", &Parametrizable::Comp<T>)};
    }
    explicit BoundTC(const Parametrizable::Parameters& p)
        : PM<T>::TransformationChecker("BoundTransformationChecker", doc(), p),
          maxRotationNorm(this->template get<T>("maxRotationNorm")),
          maxTranslationNorm(this->template get<T>("maxTranslationNorm")) {
        this->limits = {maxRotationNorm, maxTranslationNorm};
    }
    void init(const std::vector<T>& M, int rows, bool&) override {
        this->conditionVariables = {(T)0, (T)0};
        if (rows == 4) {
            T m3[9];
            rot3(M, rows, m3);
            dense::quat_from_matrix(m3, q0.data());
        } else {
            rot2d0 = std::acos(M[0]);
        }
        for (int r = 0; r < rows - 1; ++r) t0[r] = M[r * rows + rows - 1];
    }
    void check(const std::vector<T>& M, int rows, bool&) override {
        T cv0;
        if (rows == 4) {
            T m3[9], q[4];
            rot3(M, rows, m3);
            dense::quat_from_matrix(m3, q);
            cv0 = dense::angular_distance(q, q0.data());
        } else {
            T v = std::acos(M[0]) - rot2d0;
            while (v > (T)3.14159265358979323846) v -= (T)(2 * 3.14159265358979323846);
            while (v < (T)-M_PI) v += (T)(2 * 3.14159265358979323846);
            cv0 = v;
        }
        T nn = 0;
        for (int r = 0; r < rows - 1; ++r) {
            const T d = M[r * rows + rows - 1] - t0[r];
            nn = nn + d * d;
        }
        const T cv1 = std::sqrt(nn);
        this->conditionVariables = {cv0, cv1};
        if (cv0 > this->limits[0] || cv1 > this->limits[1]) {
            std::ostringstream oss;
            oss << "limit out of bounds: rot: " << cv0 << "/" << this->limits[0] << " tr: " << cv1 << "/"
                << this->limits[1];
            throw ConvergenceError(oss.str());
        }
    }
    bool loopConfig(pmx_loop_cfg& cfg, int pos) const override {
        cfg.checker_kind[pos] = PMX_CHECK_BOUND;
        cfg.checker_p[pos][0] = (double)maxRotationNorm;
        cfg.checker_p[pos][1] = (double)maxTranslationNorm;
        return true;
    }
};

// ---- data filters / inspectors / loggers -----------------------------------
template <typename T>
struct IdentityDPF : PM<T>::DataPointsFilter {
    explicit IdentityDPF(const Parametrizable::Parameters&) { this->className = "IdentityDataPointsFilter"; }
    void inPlaceFilter(DataPoints<T>&) override {}
};

// SurfaceNormalDataPointsFilter (DataPointsFilters/SurfaceNormal.cpp:50-290,
// parameters SurfaceNormal.h:64-80): the self k-NN and the per-point
// statistics on the GPU (pmx_surface_normals, pmx_normals.hip); descriptors
// in the reference's label order.  epsilon > 0 is accepted: the search is
// exact, which any approximation bound admits.
template <typename T>
struct SurfaceNormalDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("knn", "number of nearest neighbors to consider, including the point itself", "5", "3",
                     "2147483647", &P::Comp<unsigned>),
                PDoc("maxDist", "maximum distance to consider for neighbors", "inf", "0", "inf", &P::Comp<T>),
                PDoc("epsilon", "approximation to use for the nearest-neighbor search", "0", "0", "inf", &P::Comp<T>),
                PDoc("keepNormals", "whether the normals should be added as descriptors to the resulting cloud", "1"),
                PDoc("keepDensities", "whether the point densities should be added as descriptors to the resulting cloud",
                     "0"),
                PDoc("keepEigenValues", "whether the eigen values should be added as descriptors to the resulting cloud",
                     "0"),
                PDoc("keepEigenVectors",
                     "whether the eigen vectors should be added as descriptors to the resulting cloud", "0"),
                PDoc("keepMatchedIds",
                     "whether the identifiers of matches points should be added as descriptors to the resulting cloud",
                     "0"),
                PDoc("keepMeanDist", "whether the distance to the nearest neighbor mean should be added as descriptors "
                                     "to the resulting cloud",
                     "0"),
                PDoc("sortEigen", "whether the eigenvalues and eigenvectors should be sorted (ascending) based on the "
                                  "eigenvalues",
                     "0"),
                PDoc("smoothNormals", "whether the normal vector should be average with the nearest neighbors", "0")};
    }
    unsigned knn;
    T maxDist, epsilon;
    bool keepNormals, keepDensities, keepEigenValues, keepEigenVectors, keepMatchedIds, keepMeanDist, sortEigen,
        smoothNormals;
    explicit SurfaceNormalDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("SurfaceNormalDataPointsFilter", doc(), p),
          knn(this->template get<unsigned>("knn")),
          maxDist(this->template get<T>("maxDist")),
          epsilon(this->template get<T>("epsilon")),
          keepNormals(this->template get<bool>("keepNormals")),
          keepDensities(this->template get<bool>("keepDensities")),
          keepEigenValues(this->template get<bool>("keepEigenValues")),
          keepEigenVectors(this->template get<bool>("keepEigenVectors")),
          keepMatchedIds(this->template get<bool>("keepMatchedIds")),
          keepMeanDist(this->template get<bool>("keepMeanDist")),
          sortEigen(this->template get<bool>("sortEigen")),
          smoothNormals(this->template get<bool>("smoothNormals")) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const int D = cloud.rows - 1;
        const int64_t n = cloud.n;
        // (eigenpairs are always returned in ascending order: sortEigen's
        // order, and the order computeNormal's choice does not depend on)
        std::vector<T> nrm, dens, eva, eve, ids, md;
        if (keepNormals || smoothNormals) nrm.resize((size_t)(n * D));
        if (keepDensities) dens.resize((size_t)n);
        if (keepEigenValues) eva.resize((size_t)(n * D));
        if (keepEigenVectors) eve.resize((size_t)(n * D * D));
        if (keepMatchedIds) ids.resize((size_t)(n * knn));
        if (keepMeanDist) md.resize((size_t)n);
        auto ptr = [](std::vector<T>& v) { return v.empty() ? nullptr : (void*)v.data(); };
        int64_t degenerate = 0;
        const int rc = pmx_surface_normals(this->device, dtype_of<T>(), cloud.features.data(), cloud.rows, n,
                                           (int)std::min<unsigned>(knn, 1u << 30), (double)maxDist,
                                           smoothNormals ? PMX_SN_SMOOTH : 0u, ptr(nrm), ptr(dens), ptr(eva), ptr(eve),
                                           ptr(ids), ptr(md), &degenerate);
        if (rc == PMX_E_BAD_PARAM) throw InvalidParameter(pmx_last_error(nullptr));
        if (rc) throw std::runtime_error(std::string("SurfaceNormalDataPointsFilter: ") + pmx_last_error(nullptr));
        if (keepNormals) cloud.setDescriptor("normals", D, nrm.data());
        if (keepDensities) cloud.setDescriptor("densities", 1, dens.data());
        if (keepEigenValues) cloud.setDescriptor("eigValues", D, eva.data());
        if (keepEigenVectors) cloud.setDescriptor("eigVectors", D * D, eve.data());
        if (keepMatchedIds) cloud.setDescriptor("matchedIds", (int)knn, ids.data());
        if (keepMeanDist) cloud.setDescriptor("meanDists", 1, md.data());
    }
};

// Stable in-place compaction of a cloud's points (features and descriptors),
// keep(f) called once per point in index order — DataPoints::setColFrom +
// conservativeResize of the reference's subsampling filters.
template <typename T, typename Keep>
void compact_points(DataPoints<T>& cloud, Keep keep) {
    int64_t j = 0;
    for (int64_t i = 0; i < cloud.n; ++i) {
        const T* f = &cloud.features[(size_t)i * cloud.rows];
        if (!keep(f)) continue;
        if (j != i) {
            std::copy(f, f + cloud.rows, &cloud.features[(size_t)j * cloud.rows]);
            const T* d = &cloud.descriptors[(size_t)i * cloud.descDim];
            std::copy(d, d + cloud.descDim, &cloud.descriptors[(size_t)j * cloud.descDim]);
        }
        ++j;
    }
    cloud.n = j;
    cloud.features.resize((size_t)j * cloud.rows);
    cloud.descriptors.resize((size_t)j * cloud.descDim);
}

// MaxDist / MinDist data filters (DataPointsFilters/MaxDist.cpp:55-96,
// MinDist.cpp:55-96, parameters MaxDist.h:57-61, MinDist.h:57-61): keep the
// points whose coordinate `dim` (or Euclidean norm when dim == -1, against
// |limit|) is strictly below (Max) / strictly above (Min) the limit,
// stable compaction of features and descriptors; dim >= D throws.  Host code,
// once per compute and outside the ICP loop, as in the reference.
template <typename T, bool kMax>
struct DistDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static const char* pname() { return kMax ? "maxDist" : "minDist"; }
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("dim", "dimension on which the filter will be applied. x=0, y=1, z=2, radius=-1", "-1", "-1", "2",
                     &P::Comp<int>),
                PDoc(pname(), kMax ? "maximum distance authorized" : "minimum value authorized", "1", "-inf", "inf",
                     &P::Comp<T>)};
    }
    const int dim;
    const T limit;
    explicit DistDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter(kMax ? "MaxDistDataPointsFilter" : "MinDistDataPointsFilter", doc(), p),
          dim(this->template get<int>("dim")),
          limit(this->template get<T>(pname())) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const int D = cloud.rows - 1;
        if (dim >= D)
            throw InvalidParameter(this->className + ": Error, filtering on dimension number " + std::to_string(dim) +
                                   ", larger than authorized axis id " + std::to_string(D - 1));
        const T absLimit = std::abs(limit);
        compact_points(cloud, [&](const T* f) {
            if (dim == -1) {
                T s = 0;
                for (int r = 0; r < D; ++r) s += f[r] * f[r];
                const T norm = std::sqrt(s);
                return kMax ? (norm < absLimit) : (norm > absLimit);
            }
            return kMax ? (f[dim] < limit) : (f[dim] > limit);
        });
    }
};

// DistanceLimitDataPointsFilter (DataPointsFilters/DistanceLimit.cpp:57-128,
// DistanceLimit.h:57-63): MaxDist (removeInside 0: keep < dist) and MinDist
// (removeInside 1: keep > dist) in one filter, on coordinate dim or the
// Euclidean norm against |dist| (dim -1); dim >= D throws.
template <typename T>
struct DistanceLimitDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("dim", "dimension on which the filter will be applied. x=0, y=1, z=2, radius=-1", "-1", "-1", "2",
                     &P::Comp<int>),
                PDoc("dist",
                     "distance limit of the filter. If dim is set to -1 (radius), the absolute value of dist will be used",
                     "1", "-inf", "inf", &P::Comp<T>),
                PDoc("removeInside",
                     "If set to true (1), remove points before the distance limit; else (0), remove points beyond the "
                     "distance limit",
                     "1", "0", "1", &P::Comp<bool>)};
    }
    const int dim;
    const T dist;
    const bool removeInside;
    explicit DistanceLimitDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("DistanceLimitDataPointsFilter", doc(), p),
          dim(this->template get<int>("dim")),
          dist(this->template get<T>("dist")),
          removeInside(this->template get<bool>("removeInside")) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const int D = cloud.rows - 1;
        if (dim >= D)
            throw InvalidParameter("DistanceLimitDataPointsFilter: Error, filtering on dimension number " +
                                   std::to_string(dim) + ", larger than authorized axis id " + std::to_string(D - 1));
        const T absMaxDist = std::abs(dist);
        compact_points(cloud, [&](const T* f) {
            if (dim == -1) {
                T s = 0;
                for (int r = 0; r < D; ++r) s += f[r] * f[r];
                const T norm = std::sqrt(s);
                return removeInside ? (norm > absMaxDist) : (norm < absMaxDist);
            }
            return removeInside ? (f[dim] > dist) : (f[dim] < dist);
        });
    }
};

// RandomSamplingDataPointsFilter (DataPointsFilters/RandomSampling.cpp:55-74,
// RandomSampling.h:59-62): keep point i when (float)std::rand() /
// (float)RAND_MAX < prob, one draw per point in order — the same C library
// generator and state as the reference, so the kept set is identical for the
// same srand seed.
template <typename T>
struct RandomSamplingDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("prob", "probability to keep a point, one over decimation factor ", "0.75", "0", "1",
                     &P::Comp<T>)};
    }
    const double prob;
    explicit RandomSamplingDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("RandomSamplingDataPointsFilter", doc(), p), prob(this->template get<double>("prob")) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        compact_points(cloud, [&](const T*) {
            const float r = (float)std::rand() / (float)RAND_MAX;
            return r < prob;
        });
    }
    bool usesRandState() const override { return true; }
};

// BoundingBoxDataPointsFilter (DataPointsFilters/BoundingBox.cpp:76-108,
// BoundingBox.h:57-67): open box (strict < / >) on x, y and z (z ignored for
// 2-D clouds); removeInside keeps the points outside the box, else inside.
template <typename T>
struct BoundingBoxDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("xMin", "minimum value on x-axis defining one side of the bounding box", "-1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("xMax", "maximum value on x-axis defining one side of the bounding box", "1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("yMin", "minimum value on y-axis defining one side of the bounding box", "-1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("yMax", "maximum value on y-axis defining one side of the bounding box", "1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("zMin", "minimum value on z-axis defining one side of the bounding box", "-1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("zMax", "maximum value on z-axis defining one side of the bounding box", "1", "-inf", "inf",
                     &P::Comp<T>),
                PDoc("removeInside",
                     "If set to true (1), remove points inside the bounding box; else (0), remove points outside the "
                     "bounding box",
                     "1", "0", "1", &P::Comp<bool>)};
    }
    const T xMin, xMax, yMin, yMax, zMin, zMax;
    const bool removeInside;
    explicit BoundingBoxDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("BoundingBoxDataPointsFilter", doc(), p),
          xMin(this->template get<T>("xMin")),
          xMax(this->template get<T>("xMax")),
          yMin(this->template get<T>("yMin")),
          yMax(this->template get<T>("yMax")),
          zMin(this->template get<T>("zMin")),
          zMax(this->template get<T>("zMax")),
          removeInside(this->template get<bool>("removeInside")) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const bool flat = cloud.rows == 3;
        compact_points(cloud, [&](const T* f) {
            const bool in = f[0] > xMin && f[0] < xMax && f[1] > yMin && f[1] < yMax &&
                            ((f[2] > zMin && f[2] < zMax) || flat);
            return removeInside ? !in : in;
        });
    }
};

// FixStepSamplingDataPointsFilter (DataPointsFilters/FixStepSampling.cpp:37-93,
// FixStepSampling.h:57-72): keep every step-th point from a random phase
// rand() % step; step starts at startStep (reset by init) and is multiplied by
// stepMult after each application, clamped at endStep.
template <typename T>
struct FixStepSamplingDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("startStep", "initial number of point to skip (initial decimation factor)", "10", "1",
                     "2147483647", &P::Comp<unsigned>),
                PDoc("endStep", "maximal or minimal number of points to skip (final decimation factor)", "10", "1",
                     "2147483647", &P::Comp<unsigned>),
                PDoc("stepMult", "multiplication factor to compute the new decimation factor for each iteration", "1",
                     "0.0000001", "inf", &P::Comp<double>)};
    }
    const unsigned startStep, endStep;
    const double stepMult;
    double step;
    explicit FixStepSamplingDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("FixStepSamplingDataPointsFilter", doc(), p),
          startStep(this->template get<unsigned>("startStep")),
          endStep(this->template get<unsigned>("endStep")),
          stepMult(this->template get<double>("stepMult")),
          step(startStep) {}
    void init() override { step = startStep; }
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const int iStep((int)step);
        const int64_t phase = std::rand() % iStep;
        int64_t i = -1;
        compact_points(cloud, [&](const T*) {
            ++i;
            return i >= phase && (i - phase) % iStep == 0;
        });
        const double deltaStep(startStep * stepMult - startStep);
        step *= stepMult;
        if (deltaStep < 0 && step < endStep) step = endStep;
        if (deltaStep > 0 && step > endStep) step = endStep;
    }
    bool usesRandState() const override { return true; }
};

// SamplingSurfaceNormalDataPointsFilter (DataPointsFilters/SamplingSurfaceNormal.cpp:80-342,
// parameters SamplingSurfaceNormal.h:64-79): the recursive median split and
// the leaf statistics on the GPU, the sampling on the process's rand() state
// (pmx_sampling_surface_normals, pmx_ssn.hip); existing descriptors averaged
// per leaf (samplingMethod 1) or kept, the new ones in the reference's label
// order.
// VoxelGridDataPointsFilter (DataPointsFilters/VoxelGrid.h:40-98,
// VoxelGrid.cpp:60-343) on the device (pmx_voxel_grid)
template <typename T>
struct VoxelGridDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("vSizeX", "Dimension of each voxel cell in x direction", "1.0", "0.001", "+inf", &P::Comp<T>),
                PDoc("vSizeY", "Dimension of each voxel cell in y direction", "1.0", "0.001", "+inf", &P::Comp<T>),
                PDoc("vSizeZ", "Dimension of each voxel cell in z direction", "1.0", "0.001", "+inf", &P::Comp<T>),
                PDoc("useCentroid", "If 1 (true), down-sample by using centroid of voxel cell.  If false (0), use "
                                    "center of voxel cell.", "1", "0", "1", &P::Comp<bool>),
                PDoc("averageExistingDescriptors", "whether the filter keep the existing point descriptors and average "
                                                   "them or should it drop them", "1", "0", "1", &P::Comp<bool>)};
    }
    T vSizeX, vSizeY, vSizeZ;
    bool useCentroid, averageExistingDescriptors;
    explicit VoxelGridDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("VoxelGridDataPointsFilter", doc(), p),
          vSizeX(this->template get<T>("vSizeX")),
          vSizeY(this->template get<T>("vSizeY")),
          vSizeZ(this->template get<T>("vSizeZ")),
          useCentroid(this->template get<bool>("useCentroid")),
          averageExistingDescriptors(this->template get<bool>("averageExistingDescriptors")) {}
    void inPlaceFilter(DataPoints<T>& cloud) override {
        if (averageExistingDescriptors) {  // (VoxelGrid.cpp:83-90)
            int sum = 0;
            for (auto& l : cloud.descriptorLabels) sum += l.span;
            if (sum != cloud.descDim)
                throw InvalidElement("VoxelGridDataPointsFilter: Error, descriptor labels do not match descriptor data");
        }
        const int64_t n = cloud.n;
        std::vector<T> feat((size_t)(n * cloud.rows)), desc((size_t)(n * cloud.descDim));
        const double vs[3] = {(double)vSizeX, (double)vSizeY, (double)vSizeZ};
        int64_t nout = 0;
        const int rc = pmx_voxel_grid(this->device, dtype_of<T>(), cloud.features.data(), cloud.rows, n,
                                      cloud.descDim ? cloud.descriptors.data() : nullptr, cloud.descDim, vs,
                                      useCentroid ? 1 : 0, averageExistingDescriptors ? 1 : 0, feat.data(),
                                      cloud.descDim ? desc.data() : nullptr, &nout);
        if (rc == PMX_E_BAD_PARAM) throw InvalidParameter(pmx_last_error(nullptr));
        if (rc) throw std::runtime_error(std::string("VoxelGridDataPointsFilter: ") + pmx_last_error(nullptr));
        cloud.n = nout;
        feat.resize((size_t)(nout * cloud.rows));
        cloud.features.swap(feat);
        desc.resize((size_t)(nout * cloud.descDim));
        cloud.descriptors.swap(desc);
    }
};

template <typename T>
struct SamplingSurfaceNormalDPF : PM<T>::DataPointsFilter {
    typedef Parametrizable P;
    static Parametrizable::ParametersDoc doc() {
        return {PDoc("ratio", "ratio of points to keep with random subsampling. Matrix (normal, density, etc.) will be "
                              "associated to all points in the same bin.",
                     "0.5", "0.0000001", "1.0", &P::Comp<T>),
                PDoc("knn", "determined how many points are used to compute the normals. Direct link with the "
                            "rapidity of the computation (large = fast). Technically, limit over which a box is "
                            "splitted in two",
                     "7", "3", "2147483647", &P::Comp<unsigned>),
                PDoc("samplingMethod", "if set to 0, random subsampling using the parameter ratio. If set to 1, bin "
                                       "subsampling with the resulting number of points being 1/knn.",
                     "0", "0", "1", &P::Comp<unsigned>),
                PDoc("maxBoxDim", "maximum length of a box above which the box is discarded", "inf"),
                PDoc("averageExistingDescriptors",
                     "whether the filter keep the existing point descriptors and average them or should it drop them",
                     "1"),
                PDoc("keepNormals", "whether the normals should be added as descriptors to the resulting cloud", "1"),
                PDoc("keepDensities", "whether the point densities should be added as descriptors to the resulting cloud",
                     "0"),
                PDoc("keepEigenValues", "whether the eigen values should be added as descriptors to the resulting cloud",
                     "0"),
                PDoc("keepEigenVectors",
                     "whether the eigen vectors should be added as descriptors to the resulting cloud", "0")};
    }
    T ratio;
    unsigned knn, samplingMethod;
    T maxBoxDim;
    bool averageExistingDescriptors, keepNormals, keepDensities, keepEigenValues, keepEigenVectors;
    explicit SamplingSurfaceNormalDPF(const Parametrizable::Parameters& p)
        : PM<T>::DataPointsFilter("SamplingSurfaceNormalDataPointsFilter", doc(), p),
          ratio(this->template get<T>("ratio")),
          knn(this->template get<unsigned>("knn")),
          samplingMethod(this->template get<unsigned>("samplingMethod")),
          maxBoxDim(this->template get<T>("maxBoxDim")),
          averageExistingDescriptors(this->template get<bool>("averageExistingDescriptors")),
          keepNormals(this->template get<bool>("keepNormals")),
          keepDensities(this->template get<bool>("keepDensities")),
          keepEigenValues(this->template get<bool>("keepEigenValues")),
          keepEigenVectors(this->template get<bool>("keepEigenVectors")) {}
    bool usesRandState() const override { return samplingMethod == 0; }
    void inPlaceFilter(DataPoints<T>& cloud) override {
        const int D = cloud.rows - 1;
        const int64_t n = cloud.n;
        if (averageExistingDescriptors) {  // (:93-101)
            int sum = 0;
            for (auto& l : cloud.descriptorLabels) sum += l.span;
            if (sum != cloud.descDim)
                throw InvalidParameter("SamplingSurfaceNormalDataPointsFilter: Error, descriptor labels do not match "
                                       "descriptor data");
        }
        std::vector<T> feat((size_t)(n * cloud.rows)), desc((size_t)(n * cloud.descDim)), nrm, dens, eva, eve;
        if (keepNormals) nrm.resize((size_t)(n * D));
        if (keepDensities) dens.resize((size_t)n);
        if (keepEigenValues) eva.resize((size_t)(n * D));
        if (keepEigenVectors) eve.resize((size_t)(n * D * D));
        auto ptr = [](std::vector<T>& v) { return v.empty() ? nullptr : (void*)v.data(); };
        unsigned flags = (keepNormals ? PMX_SSN_NORMALS : 0u) | (keepDensities ? PMX_SSN_DENSITIES : 0u) |
                         (keepEigenValues ? PMX_SSN_EIGVALUES : 0u) | (keepEigenVectors ? PMX_SSN_EIGVECTORS : 0u) |
                         (averageExistingDescriptors ? PMX_SSN_AVERAGE : 0u);
        int64_t nout = 0, unfit = 0;
        const int rc = pmx_sampling_surface_normals(
            this->device, dtype_of<T>(), cloud.features.data(), cloud.rows, n,
            cloud.descDim ? cloud.descriptors.data() : nullptr, cloud.descDim,
            (int)std::min<unsigned>(knn, 0x7fffffffu), (int)samplingMethod, (double)ratio, (double)maxBoxDim, flags,
            feat.data(), ptr(desc), ptr(nrm), ptr(dens), ptr(eva), ptr(eve), &nout, &unfit);
        if (rc == PMX_E_BAD_PARAM) throw InvalidParameter(pmx_last_error(nullptr));
        if (rc) throw std::runtime_error(std::string("SamplingSurfaceNormalDataPointsFilter: ") + pmx_last_error(nullptr));
        cloud.n = nout;
        feat.resize((size_t)(nout * cloud.rows));
        cloud.features.swap(feat);
        desc.resize((size_t)(nout * cloud.descDim));
        cloud.descriptors.swap(desc);
        if (keepNormals) cloud.setDescriptor("normals", D, nrm.data());
        if (keepDensities) cloud.setDescriptor("densities", 1, dens.data());
        if (keepEigenValues) cloud.setDescriptor("eigValues", D, eva.data());
        if (keepEigenVectors) cloud.setDescriptor("eigVectors", D * D, eve.data());
    }
};

// no-op stand-in accepting a reference module's parameters (reads them all so
// the "set but not used" check passes)
template <typename Base>
struct NoOp : Base {
    NoOp(const std::string& name, const Parametrizable::ParametersDoc& d, const Parametrizable::Parameters& p)
        : Base(name, d, p) {
        for (auto& pd : d) this->getParamValueString(pd.name);
    }
};

template <typename T>
Parametrizable::ParametersDoc perf_doc() {
    return {PDoc("baseFileName", "base file name for the statistics files (if empty, disabled)", ""),
            PDoc("dumpPerfOnExit", "dump performance statistics to stderr on exit", "0"),
            PDoc("dumpStats", "dump the statistics on first and last step", "0")};
}
template <typename T>
Parametrizable::ParametersDoc vtk_doc() {
    return {PDoc("baseFileName", "base file name for the VTK files ", "point-matcher-output"),
            PDoc("dumpPerfOnExit", "dump performance statistics to stderr on exit", "0"),
            PDoc("dumpStats", "dump the statistics on first and last step", "0"),
            PDoc("dumpIterationInfo", "dump iteration info", "0"),
            PDoc("dumpDataLinks", "dump data links at each iteration", "0"),
            PDoc("dumpReading", "dump the reading cloud at each iteration", "0"),
            PDoc("dumpReference", "dump the reference cloud at each iteration", "0"),
            PDoc("writeBinary", "write binary VTK files", "0")};
}
inline Parametrizable::ParametersDoc filelogger_doc() {
    return {PDoc("infoFileName", "name of the file to output infos to", ""),
            PDoc("warningFileName", "name of the file to output warnings to", ""),
            PDoc("displayLocation", "display the location of message in source code", "0")};
}

}  // namespace

// --------------------------------------------------------------- registry --
template <typename T>
PointMatcher<T>::PointMatcher() {
    typedef Parametrizable::Parameters Ps;
    MatcherRegistrar.reg("KDTreeMatcher", [](const Ps& p) { return std::make_shared<KDTreeMatcherGPU<T>>(p); }, true,
                         "This matcher matches a point from the reading to its closest neighbors in the reference.");
    MatcherRegistrar.reg("KDTreeVarDistMatcher",
                         [](const Ps& p) { return std::make_shared<KDTreeVarDistMatcherGPU<T>>(p); }, true,
                         "This matcher matches a point from the reading to its closest neighbors in the reference. A "
                         "maximum search radius per point can be defined.");
    OutlierFilterRegistrar.reg("NullOutlierFilter", [](const Ps& p) { return std::make_shared<NullOF<T>>(p); }, false);
    OutlierFilterRegistrar.reg("MaxDistOutlierFilter", [](const Ps& p) { return std::make_shared<MaxDistOF<T>>(p); }, true);
    OutlierFilterRegistrar.reg("MinDistOutlierFilter", [](const Ps& p) { return std::make_shared<MinDistOF<T>>(p); }, true);
    OutlierFilterRegistrar.reg("MedianDistOutlierFilter", [](const Ps& p) { return std::make_shared<MedianDistOF<T>>(p); },
                               true);
    OutlierFilterRegistrar.reg("TrimmedDistOutlierFilter", [](const Ps& p) { return std::make_shared<TrimmedDistOF<T>>(p); },
                               true);
    OutlierFilterRegistrar.reg("VarTrimmedDistOutlierFilter",
                               [](const Ps& p) { return std::make_shared<VarTrimmedDistOF<T>>(p); }, true);
    OutlierFilterRegistrar.reg("RobustOutlierFilter", [](const Ps& p) { return std::make_shared<RobustOF<T>>(p); },
                               true);
    ErrorMinimizerRegistrar.reg("PointToPlaneErrorMinimizer",
                                [](const Ps& p) { return std::make_shared<PointToPlaneEM<T>>(p); }, true);
    ErrorMinimizerRegistrar.reg("PointToPointErrorMinimizer",
                                [](const Ps& p) { return std::make_shared<PointToPointEM<T>>(p); }, false);
    TransformationCheckerRegistrar.reg("CounterTransformationChecker",
                                       [](const Ps& p) { return std::make_shared<CounterTC<T>>(p); }, true);
    TransformationCheckerRegistrar.reg("DifferentialTransformationChecker",
                                       [](const Ps& p) { return std::make_shared<DifferentialTC<T>>(p); }, true);
    TransformationCheckerRegistrar.reg("BoundTransformationChecker",
                                       [](const Ps& p) { return std::make_shared<BoundTC<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("IdentityDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<IdentityDPF<T>>(p); }, false);
    DataPointsFilterRegistrar.reg("SurfaceNormalDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<SurfaceNormalDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("RandomSamplingDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<RandomSamplingDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("BoundingBoxDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<BoundingBoxDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("FixStepSamplingDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<FixStepSamplingDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("MaxDistDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<DistDPF<T, true>>(p); }, true);
    DataPointsFilterRegistrar.reg("MinDistDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<DistDPF<T, false>>(p); }, true);
    DataPointsFilterRegistrar.reg("DistanceLimitDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<DistanceLimitDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("VoxelGridDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<VoxelGridDPF<T>>(p); }, true);
    DataPointsFilterRegistrar.reg("SamplingSurfaceNormalDataPointsFilter",
                                  [](const Ps& p) { return std::make_shared<SamplingSurfaceNormalDPF<T>>(p); }, true);
    InspectorRegistrar.reg("NullInspector", [](const Ps& p) {
        return std::make_shared<NoOp<Inspector>>("NullInspector", Parametrizable::ParametersDoc(), p);
    }, false);
    InspectorRegistrar.reg("PerformanceInspector", [](const Ps& p) {
        return std::make_shared<NoOp<Inspector>>("PerformanceInspector", perf_doc<T>(), p);
    }, true);
    InspectorRegistrar.reg("VTKFileInspector", [](const Ps& p) {
        return std::make_shared<NoOp<Inspector>>("VTKFileInspector", vtk_doc<T>(), p);
    }, true);
    LoggerRegistrar.reg("NullLogger", [](const Ps& p) {
        return std::make_shared<NoOp<Logger>>("NullLogger", Parametrizable::ParametersDoc(), p);
    }, false);
    LoggerRegistrar.reg("FileLogger", [](const Ps& p) {
        return std::make_shared<NoOp<Logger>>("FileLogger", filelogger_doc(), p);
    }, true);
}

template <typename T>
const PointMatcher<T>& PointMatcher<T>::get() {
    static const PointMatcher<T> instance;
    return instance;
}

template <typename T>
void PointMatcher<T>::ErrorMinimizer::setStats(const pmx_stats& st) {
    const double kn = (double)st.n_total;
    keptPoints = st.kept;
    pointUsedRatio = (T)((double)st.kept / kn);
    weightedPointUsedRatio = (T)(st.sum_w / kn);
    nbRejectedMatches = st.rejected_matches;
    nbRejectedPoints = st.rejected_points;
    lastVisited = st.visited;
}

template <typename T>
void PointMatcher<T>::OutlierFilters::compute(Device& dev, const Matches& m) {
    if (this->empty()) {
        dev.check(pmx_outlier_default(dev.ctx));
        return;
    }
    int pos = 0;
    for (auto& f : *this) f->compute(dev, m, pos++);
}

template <typename T>
void PointMatcher<T>::TransformationCheckers::init(const TransformationParameters& T_, int rows, bool& iterate) {
    for (auto& c : *this) c->init(T_, rows, iterate);
}
template <typename T>
void PointMatcher<T>::TransformationCheckers::check(const TransformationParameters& T_, int rows, bool& iterate) {
    for (auto& c : *this) c->check(T_, rows, iterate);
}

// ==================================================================== ICP ==
template <typename T>
PointMatcher<T>::ICP::ICP(int device) {
    dev.device = device;
    dev.dtype = dtype_of<T>();
    if (const char* e = std::getenv("PMX_DEVICE_LOOP")) deviceLoop = std::strcmp(e, "0") != 0;
}

template <typename T>
void PointMatcher<T>::ICP::cleanup() {
    readingDataPointsFilters.clear();
    readingStepDataPointsFilters.clear();
    referenceDataPointsFilters.clear();
    matcher.reset();
    outlierFilters.clear();
    errorMinimizer.reset();
    transformationCheckers.clear();
    inspector.reset();
}

template <typename T>
void PointMatcher<T>::ICP::setDefault() {
    // ICP.cpp:99-113: RandomSampling (prob 0.75) on the reading,
    // SamplingSurfaceNormal on the reference, TrimmedDist, KDTreeMatcher,
    // PointToPlane, Counter + Differential, NullInspector.
    cleanup();
    const PointMatcher& pm = PointMatcher::get();
    readingDataPointsFilters.push_back(pm.DataPointsFilterRegistrar.create("RandomSamplingDataPointsFilter"));
    referenceDataPointsFilters.push_back(pm.DataPointsFilterRegistrar.create("SamplingSurfaceNormalDataPointsFilter"));
    outlierFilters.push_back(pm.OutlierFilterRegistrar.create("TrimmedDistOutlierFilter"));
    matcher = pm.MatcherRegistrar.create("KDTreeMatcher");
    errorMinimizer = pm.ErrorMinimizerRegistrar.create("PointToPlaneErrorMinimizer");
    transformationCheckers.push_back(pm.TransformationCheckerRegistrar.create("CounterTransformationChecker"));
    transformationCheckers.push_back(pm.TransformationCheckerRegistrar.create("DifferentialTransformationChecker"));
    inspector = pm.InspectorRegistrar.create("NullInspector");
    reinitMap();  // ICPSequence::setDefault, ICP.cpp:520-528
}

template <typename T>
void PointMatcher<T>::ICP::loadFromYaml(const std::string& text) {
    cleanup();
    const YNode doc = parse_yaml(text);
    if (doc.kind != YNode::Map && doc.kind != YNode::Null) throw ConfigurationError("YAML chain must be a map");
    const PointMatcher& pm = PointMatcher::get();
    std::set<std::string> used;
    auto many = [&](const std::string& key, auto& reg, auto& vec) {
        used.insert(key);
        const YNode* n = doc.find(key);
        if (!n) return;
        for (const YNode& item : n->seq) vec.push_back(reg.createFromYAML(item));
    };
    auto one = [&](const std::string& key, auto& reg, auto& ptr) {
        used.insert(key);
        const YNode* n = doc.find(key);
        if (n)
            ptr = reg.createFromYAML(*n);
        else
            ptr.reset();
    };
    one("logger", pm.LoggerRegistrar, logger);  // ICP.cpp:131-135 (logger first)
    many("readingDataPointsFilters", pm.DataPointsFilterRegistrar, readingDataPointsFilters);
    many("readingStepDataPointsFilters", pm.DataPointsFilterRegistrar, readingStepDataPointsFilters);
    many("referenceDataPointsFilters", pm.DataPointsFilterRegistrar, referenceDataPointsFilters);
    one("matcher", pm.MatcherRegistrar, matcher);
    many("outlierFilters", pm.OutlierFilterRegistrar, outlierFilters);
    one("errorMinimizer", pm.ErrorMinimizerRegistrar, errorMinimizer);
    many("transformationCheckers", pm.TransformationCheckerRegistrar, transformationCheckers);
    one("inspector", pm.InspectorRegistrar, inspector);
    for (const auto& kv : doc.map)  // ICP.cpp:158-166
        if (!used.count(kv.first)) throw InvalidModuleType("Module type " + kv.first + " does not exist");
    reinitMap();  // ICPSequence::loadFromYaml, ICP.cpp:530-539
}

template <typename T>
typename PointMatcher<T>::TransformationParameters PointMatcher<T>::ICP::operator()(const DataPoints& reading,
                                                                                     const DataPoints& reference) {
    const int dim = reading.rows;
    TransformationParameters I((size_t)dim * dim, (T)0);
    for (int i = 0; i < dim; ++i) I[i * dim + i] = 1;
    return compute(reading, reference, I);
}

template <typename T>
typename PointMatcher<T>::TransformationParameters PointMatcher<T>::ICP::compute(
    const DataPoints& reading, const DataPoints& reference, const TransformationParameters& T_init) {
    prepare(reading, reference, T_init);
    while (iterate(1 << 30)) {
    }
    return finish();
}

template <typename T>
static double since(const std::chrono::steady_clock::time_point& t) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
}

template <typename T>
void PointMatcher<T>::ICP::prepare(const DataPoints& readingIn, const DataPoints& referenceIn,
                                   const TransformationParameters& T_init) {
    // ICP::compute, ICP.cpp:265-313
    if (!matcher) throw std::runtime_error("You must setup a matcher before running ICP");
    if (!errorMinimizer) throw std::runtime_error("You must setup an error minimizer before running ICP");
    if (!inspector) throw std::runtime_error("You must setup an inspector before running ICP");
    auto t = std::chrono::steady_clock::now();
    const int dim = referenceIn.rows;
    if (dim != 3 && dim != 4) throw std::runtime_error("clouds must be 2-D or 3-D (3 or 4 homogeneous rows)");
    if (dev.sharded())  // (every rank filters its own reading shard)
        for (const DataPointsFilters* chain :
             {&readingDataPointsFilters, &readingStepDataPointsFilters, &referenceDataPointsFilters})
            for (const auto& f : *chain)
                if (f->usesRandState())
                    throw ConfigurationError(f->className + " draws from the process's rand() state: it cannot run on "
                                             "the reading shards of a multi-rank ICP");
    for (auto& f : referenceDataPointsFilters) f->device = dev.device;
    for (auto& f : readingDataPointsFilters) f->device = dev.device;
    // (no reference filters: the caller's cloud is uploaded as it is and
    // centred on the device — no host copy of the reference)
    const bool filtered = !referenceDataPointsFilters.empty();
    DataPoints refCopy;
    if (filtered) {
        refCopy = referenceIn;
        referenceDataPointsFilters.init();
        referenceDataPointsFilters.apply(refCopy);
    }
    const DataPoints& reference = filtered ? refCopy : referenceIn;
    const int64_t M = reference.n;
    if (M <= 0) throw ConvergenceError("empty reference");
    // mean of the reference columns in T, ICP.cpp:291-292 (each coordinate's
    // sum sequential in point order), computed by the matcher's init on a
    // host thread while the cloud uploads (pmx_set_reference_mean_centred)
    T_refIn_refMean_.assign((size_t)dim * dim, (T)0);
    for (int i = 0; i < dim; ++i) T_refIn_refMean_[i * dim + i] = 1;
    T mean[3] = {0, 0, 0};
    dev.ensure();
    mapIndexed_ = false;  // (an ICPSequence map is no longer the device's reference, even if init throws)
    matcher->init(dev, reference, nullptr, mean);  // ICP.cpp:302 (features - mean, ICP.cpp:299, on the device)
    for (int r = 0; r < dim - 1; ++r) T_refIn_refMean_[r * dim + dim - 1] = mean[r];
    referencePreprocessingDuration = since<T>(t);
    prefilteredReferencePtsCount = M;
    prepareReading(readingIn, T_init);
}

// computeWithTransformedReference up to the loop, ICP.cpp:317-370
// (T_refIn_refMean_ and the matcher describe the reference)
template <typename T>
void PointMatcher<T>::ICP::prepareReading(const DataPoints& readingIn, const TransformationParameters& T_init) {
    const int dim = (int)std::lround(std::sqrt((double)T_refIn_refMean_.size()));
    if ((int64_t)T_init.size() != (int64_t)dim * dim)
        throw std::runtime_error("The shape of initial transformation matrix must be NxN. Where N is the number of "
                                 "rows in the read/reference scans.");
    if (readingIn.rows != dim) throw std::runtime_error("reading and reference dimensions differ");
    const auto t = std::chrono::steady_clock::now();
    // (no reading filters: the caller's cloud directly, no host copy)
    DataPoints readCopy;
    if (!readingDataPointsFilters.empty()) {
        readCopy = readingIn;
        readingDataPointsFilters.init();
        readingDataPointsFilters.apply(readCopy);
    }
    const DataPoints& reading = readingDataPointsFilters.empty() ? readingIn : readCopy;
    // T_refMean_dataIn = T_refIn_refMean^-1 * T_init (the inverse of a pure
    // translation is exact), ICP.cpp:345-346
    TransformationParameters inv((size_t)dim * dim, (T)0);
    for (int i = 0; i < dim; ++i) inv[i * dim + i] = 1;
    for (int r = 0; r < dim - 1; ++r) inv[r * dim + dim - 1] = -T_refIn_refMean_[r * dim + dim - 1];
    T_refMean_dataIn_.assign((size_t)dim * dim, (T)0);
    dense::matmul(inv.data(), T_init.data(), dim, T_refMean_dataIn_.data());
    if (std::fabs((T)1 - dense::det_rot(T_refMean_dataIn_.data(), dim)) > (T)0.001)
        throw TransformationError("RigidTransformation: Error, rotation matrix is not orthogonal.");
    // transformations.apply(reading, T_refMean_dataIn): done on the device
    dev.check(pmx_set_reading(dev.ctx, reading.feat(), dim, reading.n, T_refMean_dataIn_.data()));
    matcher->initReading(dev, reading);  // (per-reading matcher inputs: KDTreeVarDistMatcher's radii)
    // readingStepDataPointsFilters (ICP.cpp:349-350, 373-377): the step
    // filters see the reading in <refMean> every iteration; keep that copy on
    // the host (the device's transform, restated: the same separately rounded
    // terms in the same order) — each iteration filters it and uploads the result
    stepBase_ = DataPoints();
    if (!readingStepDataPointsFilters.empty()) {
        stepBase_ = reading;
        const int D = dim - 1;
        for (int64_t j = 0; j < reading.n; ++j) {
            const T* f = reading.feat() + (size_t)j * dim;
            T* o = &stepBase_.features[(size_t)j * dim];
            for (int r = 0; r < D; ++r) {
                const T* m = &T_refMean_dataIn_[(size_t)r * dim];
                T v = m[0] * f[0];
                v = v + m[1] * f[1];
                v = v + (D == 3 ? m[2] * f[2] : (T)0 * (T)0);
                v = v + m[D] * f[D];
                o[r] = v;
            }
        }
        for (auto& f : readingStepDataPointsFilters) f->device = dev.device;
        readingStepDataPointsFilters.init();
    }
    rows_ = dim;
    T_iter_.assign((size_t)dim * dim, (T)0);
    for (int i = 0; i < dim; ++i) T_iter_[i * dim + i] = 1;
    iterate_ = true;
    maxNumIterationsReached = false;
    transformationCheckers.init(T_iter_, dim, iterate_);
    iterationCount = 0;
    trace.clear();
    loopMode_ = 0;
    loopIters_ = 0;
    loopTouched_ = 0;
    readingPreprocessingDuration = since<T>(t);
    prefilteredReadingPtsCount = reading.n;
    t0_ = std::chrono::steady_clock::now();
}

// ------------------------------------------------------------ ICPSequence --
template <typename T>
bool PointMatcher<T>::ICP::setMap(const DataPoints& inputCloud) {
    // ICP.cpp:464-508
    if (!matcher) throw std::runtime_error("You must setup a matcher before running ICP");
    if (!inspector) throw std::runtime_error("You must setup an inspector before running ICP");
    auto t = std::chrono::steady_clock::now();
    const int dim = inputCloud.rows;
    const int64_t ptCount = inputCloud.n;
    if (ptCount == 0) return false;  // "Ignoring attempt to create a map from an empty cloud"
    if (dim != 3 && dim != 4) throw std::runtime_error("clouds must be 2-D or 3-D (3 or 4 homogeneous rows)");
    if (dev.sharded())
        for (const auto& f : referenceDataPointsFilters)
            if (f->usesRandState())
                throw ConfigurationError(f->className + " draws from the process's rand() state: it cannot run on "
                                         "the reading shards of a multi-rank ICP");
    // the new map is built in locals and committed only once it is indexed:
    // a filter or Matcher::init that throws leaves the previous map (or none),
    // and mapIndexed_ false — the device reference may be half replaced
    mapIndexed_ = false;
    DataPoints map(inputCloud);
    // the mean of the map BEFORE the reference filters (ICP.cpp:490-497; ICP::compute
    // filters first), sequential sums in T as prepare
    TransformationParameters T_map((size_t)dim * dim, (T)0);
    for (int i = 0; i < dim; ++i) T_map[i * dim + i] = 1;
    for (int r = 0; r < dim - 1; ++r) {
        T s = 0;
        for (int64_t j = 0; j < ptCount; ++j) s = s + map.features[j * dim + r];
        const T mean = s / (T)ptCount;
        T_map[r * dim + dim - 1] = mean;
        for (int64_t j = 0; j < ptCount; ++j) map.features[j * dim + r] = map.features[j * dim + r] - mean;
    }
    for (auto& f : referenceDataPointsFilters) f->device = dev.device;
    referenceDataPointsFilters.init();
    referenceDataPointsFilters.apply(map);
    if (map.n <= 0) throw ConvergenceError("empty reference");
    dev.ensure();
    matcher->init(dev, map);  // ICP.cpp:503 (the grid stays on the device)
    map_ = std::move(map);
    T_map_ = std::move(T_map);
    mapIndexed_ = true;
    referencePreprocessingDuration = since<T>(t);  // (SetMapDuration)
    prefilteredReferencePtsCount = map_.n;
    return true;
}

template <typename T>
void PointMatcher<T>::ICP::clearMap() {
    map_ = DataPoints();
    T_map_.clear();
    mapIndexed_ = false;
}

template <typename T>
typename PointMatcher<T>::DataPoints PointMatcher<T>::ICP::getPrefilteredMap() const {
    DataPoints g(map_);
    if (hasMap()) {
        const int dim = map_.rows;
        for (int r = 0; r < dim - 1; ++r) {
            const T m = T_map_[r * dim + dim - 1];
            for (int64_t j = 0; j < g.n; ++j) g.features[j * dim + r] = g.features[j * dim + r] + m;
        }
    }
    return g;
}

template <typename T>
void PointMatcher<T>::ICP::reinitMap() {
    if (!hasMap() || !matcher) return;
    dev.ensure();
    matcher->init(dev, map_);
    mapIndexed_ = true;
}

template <typename T>
bool PointMatcher<T>::ICP::prepareSequence(const DataPoints& readingIn, const TransformationParameters& T_init) {
    if (!hasMap()) return false;  // "Ignoring attempt to perform ICP with an empty map"
    if (!matcher) throw std::runtime_error("You must setup a matcher before running ICP");
    if (!errorMinimizer) throw std::runtime_error("You must setup an error minimizer before running ICP");
    if (!inspector) throw std::runtime_error("You must setup an inspector before running ICP");
    if (dev.sharded())
        for (const auto& f : readingDataPointsFilters)
            if (f->usesRandState())
                throw ConfigurationError(f->className + " draws from the process's rand() state: it cannot run on "
                                         "the reading shards of a multi-rank ICP");
    if (dev.sharded())
        for (const auto& f : readingStepDataPointsFilters)
            if (f->usesRandState())
                throw ConfigurationError(f->className + " draws from the process's rand() state: it cannot run on "
                                         "the reading shards of a multi-rank ICP");
    for (auto& f : readingDataPointsFilters) f->device = dev.device;
    if (!mapIndexed_) reinitMap();  // (a plain compute replaced the device's reference)
    T_refIn_refMean_ = T_map_;
    prepareReading(readingIn, T_init);
    return true;
}

template <typename T>
typename PointMatcher<T>::TransformationParameters PointMatcher<T>::ICP::computeSequence(
    const DataPoints& reading, const TransformationParameters& T_init) {
    if (!prepareSequence(reading, T_init)) {
        const int dim = reading.rows;
        TransformationParameters I((size_t)dim * dim, (T)0);
        for (int i = 0; i < dim; ++i) I[i * dim + i] = 1;
        return I;
    }
    while (iterate(1 << 30)) {
    }
    return finish();
}

template <typename T>
bool PointMatcher<T>::ICP::step() {
    return iterate(1);
}

// every module's device form, or false (ICP.cpp:371-430 then runs through the
// module calls)
template <typename T>
bool PointMatcher<T>::ICP::loopConfig(pmx_loop_cfg& cfg) const {
    std::memset(&cfg, 0, sizeof(cfg));
    if (!matcher->loopConfig(cfg) || !errorMinimizer->loopConfig(cfg)) return false;
    if (outlierFilters.size() > 8 || transformationCheckers.size() > 8) return false;
    cfg.n_filters = (int)outlierFilters.size();
    for (size_t i = 0; i < outlierFilters.size(); ++i)
        if (!outlierFilters[i]->loopConfig(cfg, (int)i)) return false;
    cfg.n_checkers = (int)transformationCheckers.size();
    for (size_t i = 0; i < transformationCheckers.size(); ++i)
        if (!transformationCheckers[i]->loopConfig(cfg, (int)i)) return false;
    cfg.keep_trace = keepTrace ? 1 : 0;
    return true;
}

template <typename T>
bool PointMatcher<T>::ICP::iterate(int n) {
    if (!iterate_ || n <= 0) return iterate_;
    if (loopMode_ == 0) {  // first iterations after prepare: pick the mode
        loopMode_ = -1;
        pmx_loop_cfg cfg;
        // (step filters re-upload the reading every iteration: module calls)
        if (deviceLoop && readingStepDataPointsFilters.empty() && loopConfig(cfg)) {
            const int rc = pmx_loop_begin(dev.ctx, &cfg, T_iter_.data());
            if (rc == PMX_OK)
                loopMode_ = 1;
            else if (rc != PMX_E_BAD_PARAM)  // (BAD_PARAM: a configuration the loop does not take)
                dev.check(rc);
        }
    }
    if (loopMode_ < 0) {
        for (int i = 0; i < n && iterate_; ++i) stepModules();
        return iterate_;
    }
    pmx_loop_status st;
    std::memset(&st, 0, sizeof(st));
    const int rc = pmx_loop_run(dev.ctx, n, &st);
    if (rc != PMX_OK && st.error == 0) dev.check(rc);  // HIP / RCCL / state failure
    // mirror the device loop's state into the modules (what the per-module
    // calls would have left there)
    const int dim = rows_;
    const int64_t fresh = st.iterations - loopIters_;
    if (keepTrace && fresh > 0) {
        std::vector<T> buf((size_t)fresh * dim * dim);
        dev.check(pmx_loop_trace(dev.ctx, (int)loopIters_, (int)fresh, buf.data()));
        for (int64_t i = 0; i < fresh; ++i)
            trace.emplace_back(buf.begin() + i * dim * dim, buf.begin() + (i + 1) * dim * dim);
    }
    iterationCount += fresh;
    for (auto& f : outlierFilters) f->loopAdvance(fresh);
    loopIters_ = st.iterations;
    matcher->visitCounter += (uint64_t)(st.point_count_touched - loopTouched_);  // MatchersImpl.cpp:98
    loopTouched_ = st.point_count_touched;
    if (st.last.kept > 0) errorMinimizer->setStats(st.last);
    for (size_t i = 0; i < transformationCheckers.size(); ++i) {
        auto& cv = transformationCheckers[i]->conditionVariables;
        for (size_t j = 0; j < cv.size() && j < 2; ++j) cv[j] = (T)st.cond[i][j];
    }
    for (int i = 0; i < dim * dim; ++i) T_iter_[(size_t)i] = (T)st.T_iter[i];
    if (st.reason == 1) maxNumIterationsReached = true;
    if (st.done) iterate_ = false;
    if (rc != PMX_OK) dev.check(rc);  // the exception the loop raised
    return iterate_;
}

template <typename T>
bool PointMatcher<T>::ICP::stepModules() {
    // one pass of the loop body, ICP.cpp:371-430
    if (!iterate_) return false;
    const int dim = rows_;
    if (std::fabs((T)1 - dense::det_rot(T_iter_.data(), dim)) > (T)0.001)  // TransformationsImpl.cpp:62-63
        throw TransformationError("RigidTransformation: Error, rotation matrix is not orthogonal.");
    if (!readingStepDataPointsFilters.empty()) {  // ICP.cpp:373-377
        DataPoints stepReading(stepBase_);
        readingStepDataPointsFilters.apply(stepReading);
        TransformationParameters I((size_t)dim * dim, (T)0);
        for (int i = 0; i < dim; ++i) I[(size_t)i * dim + i] = 1;
        dev.check(pmx_set_reading(dev.ctx, stepReading.features.data(), dim, stepReading.n, I.data()));
        matcher->initReading(dev, stepReading);
    }
    const Matches matches = matcher->findClosests(dev, T_iter_);
    outlierFilters.compute(dev, matches);
    const TransformationParameters dT = errorMinimizer->compute(dev, dim);
    matcher->visitCounter += (uint64_t)errorMinimizer->lastVisited;  // MatchersImpl.cpp:98
    dense::matmul(dT.data(), T_iter_.data(), dim, T_iter_.data());
    try {
        transformationCheckers.check(T_iter_, dim, iterate_);
    } catch (const MaxNumIterationsReached&) {
        iterate_ = false;
        maxNumIterationsReached = true;
    }
    ++iterationCount;
    if (keepTrace) trace.push_back(T_iter_);
    return iterate_;
}

template <typename T>
typename PointMatcher<T>::TransformationParameters PointMatcher<T>::ICP::finish() {
    convergenceDuration = since<T>(t0_);
    const int dim = rows_;
    TransformationParameters tmp((size_t)dim * dim), out((size_t)dim * dim);
    dense::matmul(T_refIn_refMean_.data(), T_iter_.data(), dim, tmp.data());
    dense::matmul(tmp.data(), T_refMean_dataIn_.data(), dim, out.data());
    return out;  // ICP.cpp:448
}

template struct PointMatcher<float>;
template struct PointMatcher<double>;

}  // namespace pm
