// pm_icp.h — PointMatcher<T> restated for the device-resident GPU path.
//
// The class layout follows pointmatcher/PointMatcher.h (Matcher :470-485,
// OutlierFilter :496-514, ErrorMinimizer :527-569, TransformationChecker
// :580-610, ICPChainBase / ICP :652-764) and the loop of
// pointmatcher/ICP.cpp:265-449.  The differences are the ones device
// residency forces:
//   * Matches and OutlierWeights live in HBM (inside the pmx_ctx the ICP
//     object owns); host copies are made lazily (Matches::mirror()).
//   * The step transform is not applied to a host copy of the reading
//     (ICP.cpp:373-381): it is passed to the matcher and fused into the match
//     kernel; the minimiser kernels re-apply it bit-identically.
//   * Plugins receive the device context explicitly.
#pragma once

#include <array>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "pm_core.h"
#include "pmx.h"

namespace pm {

// device handle shared by the modules of one ICP object
struct Device {
    pmx_ctx* ctx = nullptr;
    int device = 0;
    int dtype = PMX_F32;
    int nranks = 1;
    int rank = 0;
    std::vector<unsigned char> uid;  // RCCL unique id of a sharded ICP (pmx_comm_init)
    // or the caller's host collectives (pmx_comm_init_host)
    pmx_allreduce_fn host_ar = nullptr;
    pmx_allgather_fn host_ag = nullptr;
    void* host_user = nullptr;
    bool sharded() const { return !uid.empty() || host_ar != nullptr; }
    ~Device();
    void ensure();
    void check(int rc) const;  // PMX_E_* -> reference exception types
};

template <typename T>
struct PointMatcher {
    typedef pm::DataPoints<T> DataPoints;
    typedef std::vector<T> TransformationParameters;  // rows x rows, row-major
    typedef Parametrizable::Parameters Parameters;
    typedef Parametrizable::ParametersDoc ParametersDoc;

    // Matches (PointMatcher.h:371-391): k x N squared distances + ids, on the
    // device; mirror() copies them to the host.
    struct Matches {
        Device* dev = nullptr;
        int knn = 0;
        int64_t n = 0;
        mutable bool mirrored = false;
        mutable std::vector<T> dists;
        mutable std::vector<int32_t> ids;
        void mirror() const;
        T getDistsQuantile(T quantile) const;  // Matches.cpp:60-87 (host, on the mirror)
    };

    // ---------------------------------------------------------- Matcher --
    struct Matcher : Parametrizable {
        uint64_t visitCounter = 0;
        Matcher() {}
        Matcher(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~Matcher() {}
        void resetVisitCount() { visitCounter = 0; }
        uint64_t getVisitCount() const { return visitCounter; }
        // centre (may be null): rows - 1 values the matcher subtracts per axis
        // in T (ICP.cpp:299's centring done with the upload, on the device);
        // mean_out (may be null, then centre is ignored): the matcher
        // computes the reference mean itself (ICP.cpp:291-292, on a host
        // thread while the cloud uploads), centres by it and writes it here
        virtual void init(Device& dev, const DataPoints& filteredReference, const T* centre = nullptr,
                          T* mean_out = nullptr) = 0;
        // the reading's inputs of the match, once per compute after the
        // reading upload (KDTreeVarDistMatcher: its per-point radii)
        virtual void initReading(Device&, const DataPoints&) {}
        virtual Matches findClosests(Device& dev, const TransformationParameters& T_iter) = 0;
        // device loop (pmx_loop_*): describe this module in cfg, or return
        // false to keep the per-module calls (the default for any plugin)
        virtual bool loopConfig(pmx_loop_cfg&) const { return false; }
    };

    // ---------------------------------------------------- OutlierFilter --
    struct OutlierFilter : Parametrizable {
        OutlierFilter() {}
        OutlierFilter(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~OutlierFilter() {}
        // multiply this filter's weights into the device weights
        // (chain_pos 0 assigns) — OutlierFilter.cpp:90-99
        virtual void compute(Device& dev, const Matches& m, int chain_pos) = 0;
        virtual bool loopConfig(pmx_loop_cfg&, int /*chain_pos*/) const { return false; }
        // the device loop ran `iterations` more calls of this filter (its
        // per-call state, as the per-module calls would have left it)
        virtual void loopAdvance(int64_t /*iterations*/) {}
    };
    struct OutlierFilters : std::vector<std::shared_ptr<OutlierFilter>> {
        void compute(Device& dev, const Matches& m);  // OutlierFilter.cpp:63-103
    };

    // --------------------------------------------------- ErrorMinimizer --
    struct ErrorMinimizer : Parametrizable {
        // ErrorElements statistics (ErrorMinimizer.cpp:133-192)
        T pointUsedRatio = -1;
        T weightedPointUsedRatio = -1;
        int64_t nbRejectedMatches = -1;
        int64_t nbRejectedPoints = -1;
        int64_t keptPoints = 0;
        int64_t lastVisited = 0;  // pair evaluations of the iteration's match
        ErrorMinimizer() {}
        ErrorMinimizer(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~ErrorMinimizer() {}
        virtual TransformationParameters compute(Device& dev, int rows) = 0;
        virtual bool loopConfig(pmx_loop_cfg&) const { return false; }
        T getPointUsedRatio() const { return pointUsedRatio; }
        T getWeightedPointUsedRatio() const { return weightedPointUsedRatio; }
        virtual T getOverlap() const { return weightedPointUsedRatio; }
        void setStats(const pmx_stats& st);
    };

    // --------------------------------------------- TransformationChecker --
    struct TransformationChecker : Parametrizable {
        std::vector<T> limits, conditionVariables;
        std::vector<std::string> limitNames, conditionVariableNames;
        TransformationChecker() {}
        TransformationChecker(const std::string& n, const ParametersDoc& d, const Parameters& p)
            : Parametrizable(n, d, p) {}
        virtual ~TransformationChecker() {}
        virtual void init(const TransformationParameters& T_, int rows, bool& iterate) = 0;
        virtual void check(const TransformationParameters& T_, int rows, bool& iterate) = 0;
        virtual bool loopConfig(pmx_loop_cfg&, int /*pos*/) const { return false; }
    };
    struct TransformationCheckers : std::vector<std::shared_ptr<TransformationChecker>> {
        void init(const TransformationParameters& T_, int rows, bool& iterate);
        void check(const TransformationParameters& T_, int rows, bool& iterate);
    };
    struct MaxNumIterationsReached {};

    // ---------------------------------------- data filters / inspector / logger --
    struct DataPointsFilter : Parametrizable {
        DataPointsFilter() {}
        DataPointsFilter(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~DataPointsFilter() {}
        virtual void init() {}
        virtual void inPlaceFilter(DataPoints& cloud) = 0;
        // true when the result depends on the process's C library rand()
        // state (RandomSampling, FixStepSampling): such a filter cannot run
        // on the shards of a multi-rank ICP (each rank would draw from its own
        // state and restart its counting at the shard's first point)
        virtual bool usesRandState() const { return false; }
        int device = 0;  // HIP device of the ICP that applies the filter (GPU filters)
    };
    struct DataPointsFilters : std::vector<std::shared_ptr<DataPointsFilter>> {
        void init() {
            for (auto& f : *this) f->init();
        }
        void apply(DataPoints& c) {
            for (auto& f : *this) f->inPlaceFilter(c);
        }
    };
    struct Inspector : Parametrizable {
        Inspector() {}
        Inspector(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~Inspector() {}
    };
    struct Logger : Parametrizable {
        Logger() {}
        Logger(const std::string& n, const ParametersDoc& d, const Parameters& p) : Parametrizable(n, d, p) {}
        virtual ~Logger() {}
    };

    // ---------------------------------------------------------- registry --
    Registrar<Matcher> MatcherRegistrar;
    Registrar<OutlierFilter> OutlierFilterRegistrar;
    Registrar<ErrorMinimizer> ErrorMinimizerRegistrar;
    Registrar<TransformationChecker> TransformationCheckerRegistrar;
    Registrar<DataPointsFilter> DataPointsFilterRegistrar;
    Registrar<Inspector> InspectorRegistrar;
    Registrar<Logger> LoggerRegistrar;
    PointMatcher();
    static const PointMatcher& get();

    // --------------------------------------------------------------- ICP --
    struct ICP {
        DataPointsFilters readingDataPointsFilters, readingStepDataPointsFilters, referenceDataPointsFilters;
        std::shared_ptr<Matcher> matcher;
        OutlierFilters outlierFilters;
        std::shared_ptr<ErrorMinimizer> errorMinimizer;
        TransformationCheckers transformationCheckers;
        std::shared_ptr<Inspector> inspector;
        std::shared_ptr<Logger> logger;
        Device dev;

        ICP(int device = 0);
        void cleanup();
        void setDefault();                       // ICP.cpp:99-113
        void loadFromYaml(const std::string& text);  // ICP.cpp:116-167

        TransformationParameters operator()(const DataPoints& reading, const DataPoints& reference);
        TransformationParameters compute(const DataPoints& reading, const DataPoints& reference,
                                         const TransformationParameters& T_init);  // ICP.cpp:265-313

        // the loop of computeWithTransformedReference (ICP.cpp:317-449) in three
        // phases, so a caller can time the iterations alone
        void prepare(const DataPoints& reading, const DataPoints& reference, const TransformationParameters& T_init);
        bool step();                          // one iteration; false when a checker stopped
        // up to n iterations; false when a checker stopped.  When every module
        // has a device form (loopConfig) the iterations run as the
        // device-resident loop (pmx_loop_*: solve, T_iter update and checkers
        // on the GPU, no host round trip per iteration); PMX_DEVICE_LOOP=0 or
        // deviceLoop = false keeps the per-module calls.
        bool iterate(int n);
        bool deviceLoop = true;
        TransformationParameters finish();    // T_refIn_refMean * T_iter * T_refMean_dataIn

        // ICPSequence (PointMatcher.h:730-764, ICP.cpp:455-609): a map kept
        // resident on the device (centred, filtered and indexed once by
        // setMap); every compute matches a new reading against it.
        bool setMap(const DataPoints& map);   // ICP.cpp:464-508 (false: empty cloud, ignored)
        void clearMap();                      // ICP.cpp:512-517
        bool hasMap() const { return map_.n > 0; }   // ICP.cpp:457-460
        DataPoints getPrefilteredMap() const;        // ICP.cpp:543-554 (global coordinates)
        const DataPoints& getPrefilteredInternalMap() const { return map_; }  // ICP.cpp:564-567
        // ICPSequence::compute (ICP.cpp:595-609): identity without a map
        TransformationParameters computeSequence(const DataPoints& reading, const TransformationParameters& T_init);
        // its first phase (then iterate / finish as after prepare); false without a map
        bool prepareSequence(const DataPoints& reading, const TransformationParameters& T_init);
        // the map's matcher again after a chain reload (ICPSequence::setDefault /
        // loadFromYaml, ICP.cpp:520-539)
        void reinitMap();

        // statistics (Inspector::addStat names, ICP.cpp:305-307, 363-365, 432-436)
        int64_t iterationCount = 0;
        bool maxNumIterationsReached = false;
        double convergenceDuration = 0, referencePreprocessingDuration = 0, readingPreprocessingDuration = 0;
        int64_t prefilteredReadingPtsCount = 0, prefilteredReferencePtsCount = 0;
        std::vector<TransformationParameters> trace;  // T_iter after each iteration
        bool keepTrace = false;
        bool getMaxNumIterationsReached() const { return maxNumIterationsReached; }

      private:
        bool stepModules();                   // ICP.cpp:371-430 through the module calls
        bool loopConfig(pmx_loop_cfg& cfg) const;
        void prepareReading(const DataPoints& readingIn, const TransformationParameters& T_init);
        DataPoints stepBase_;                 // the reading in <refMean> (readingStepDataPointsFilters)
        DataPoints map_;                      // the map in <refMean>, filtered (mapPointCloud)
        TransformationParameters T_map_;      // its T_refIn_refMean
        bool mapIndexed_ = false;             // the device holds the map (no other reference since)
        int loopMode_ = 0;                    // 0 undecided, 1 device loop, -1 module calls
        int64_t loopIters_ = 0, loopTouched_ = 0;
        int rows_ = 0;
        bool iterate_ = false;
        TransformationParameters T_refIn_refMean_, T_refMean_dataIn_, T_iter_;
        std::chrono::steady_clock::time_point t0_;
    };
};

// DataPoints::load for .csv / .vtk (pm_io.cpp, IO.cpp:374-389)
template <typename T>
DataPoints<T> load_cloud(const std::string& path);

}  // namespace pm
