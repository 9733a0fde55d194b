// pm_core.h — host-side support restated from libpointmatcher for the GPU ICP:
// exceptions, string parameters with bounds (Parametrizable), the name ->
// factory registry (Registrar), a block-YAML subset parser, the DataPoints
// container and the small dense kit (Eigen 3.3 algorithms the reference's
// minimisers and checkers rely on).
//
// Reference interfaces mirrored (paths relative to the libpointmatcher root):
//   exceptions        pointmatcher/PointMatcher.h:83-100, 148-151,
//                     Parametrizable.h:101-104, Registrar.h:69-72, ICP.cpp:158-166
//   Parametrizable    pointmatcher/Parametrizable.h:98-175, Parametrizable.cpp:170-240
//   Registrar         pointmatcher/Registrar.h:75-218, Registrar.cpp:10-31
//   DataPoints        pointmatcher/PointMatcher.h:207-358 (features (D+1) x N,
//                     descriptors stacked by label; here stored point-major)
#pragma once

#include <cmath>
#include <cstdint>
#include <functional>
#include <limits>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../common/pmx_dense.h"

namespace pm {

// ------------------------------------------------------------- exceptions --
struct ConvergenceError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct TransformationError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct InvalidParameter : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct InvalidElement : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct InvalidModuleType : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct ConfigurationError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------- YAML --
// Minimal block YAML: maps, sequences ("- "), plain scalars, '#' comments,
// empty values (null).  Enough for libpointmatcher chain files
// (doc/Configuration.md, examples/data/*.yaml).
struct YNode {
    enum Kind { Null, Scalar, Map, Seq } kind = Null;
    std::string scalar;
    std::vector<std::pair<std::string, YNode>> map;  // insertion order
    std::vector<YNode> seq;
    const YNode* find(const std::string& key) const {
        for (auto& kv : map)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    size_t size() const { return kind == Map ? map.size() : kind == Seq ? seq.size() : 0; }
};
YNode parse_yaml(const std::string& text);

// --------------------------------------------------------- Parametrizable --
// lexical_cast with the reference's special cases for "inf", "-inf", "nan"
// (Parametrizable.h:48-64)
template <typename S>
S lexical_cast(const std::string& s);

struct Parametrizable {
    typedef bool (*LexicalComparison)(const std::string&, const std::string&);
    struct ParameterDoc {
        std::string name, doc, defaultValue, minValue, maxValue;
        LexicalComparison comp;
    };
    typedef std::vector<ParameterDoc> ParametersDoc;
    typedef std::map<std::string, std::string> Parameters;

    template <typename S>
    static bool Comp(const std::string& a, const std::string& b) {
        return lexical_cast<S>(a) < lexical_cast<S>(b);
    }
    static bool FalseComp(const std::string&, const std::string&) { return false; }

    std::string className;
    ParametersDoc parametersDoc;
    Parameters parameters;
    std::set<std::string> parametersUsed;

    Parametrizable() : className("unknown") {}
    Parametrizable(const std::string& className, const ParametersDoc& doc, const Parameters& params);
    virtual ~Parametrizable() {}
    std::string getParamValueString(const std::string& name);
    template <typename S>
    S get(const std::string& name) {
        return lexical_cast<S>(getParamValueString(name));
    }
};

// ParameterDoc helpers: bounded (name, doc, default, min, max, comp) or free
inline Parametrizable::ParameterDoc PDoc(const std::string& n, const std::string& d, const std::string& def,
                                         const std::string& mn, const std::string& mx,
                                         Parametrizable::LexicalComparison c) {
    return {n, d, def, mn, mx, c};
}
inline Parametrizable::ParameterDoc PDoc(const std::string& n, const std::string& d, const std::string& def) {
    return {n, d, def, "", "", &Parametrizable::FalseComp};
}

// --------------------------------------------------------------- Registrar --
template <typename Interface>
struct Registrar {
    typedef std::function<std::shared_ptr<Interface>(const Parametrizable::Parameters&)> Factory;
    struct Entry {
        Factory make;
        bool hasParams;
        std::string description;
    };
    std::map<std::string, Entry> classes;

    void reg(const std::string& name, Factory f, bool hasParams, const std::string& desc = "") {
        classes[name] = Entry{f, hasParams, desc};
    }
    bool has(const std::string& name) const { return classes.count(name) != 0; }

    // Registrar::create + GenericClassDescriptor(NoParam)::createInstance
    // (Registrar.h:98-135, 169-181)
    std::shared_ptr<Interface> create(const std::string& name,
                                      const Parametrizable::Parameters& params = Parametrizable::Parameters()) const {
        auto it = classes.find(name);
        if (it == classes.end())
            throw InvalidElement("Trying to instanciate unknown element " + name + " from registrar");
        if (!it->second.hasParams) {
            for (const auto& p : params)
                throw InvalidParameter("Parameter " + p.first + " was set but module " + name +
                                       " dos not use any parameter");
            return it->second.make(params);
        }
        std::shared_ptr<Interface> inst = it->second.make(params);
        for (const auto& p : params)
            if (inst->parametersUsed.find(p.first) == inst->parametersUsed.end())
                throw InvalidParameter("Parameter " + p.first + " for module " + name + " was set but is not used");
        return inst;
    }
    // getNameParamsFromYAML (Registrar.cpp:12-31)
    std::shared_ptr<Interface> createFromYAML(const YNode& module) const {
        std::string name;
        Parametrizable::Parameters params;
        if (module.size() != 1) {
            name = module.scalar;
        } else {
            name = module.map[0].first;
            const YNode& p = module.map[0].second;
            for (const auto& kv : p.map) params[kv.first] = kv.second.scalar;
        }
        return create(name, params);
    }
};

// -------------------------------------------------------------- DataPoints --
template <typename T>
struct DataPoints {
    struct Label {
        std::string text;
        int span;
    };
    int rows = 0;    // D + 1 (homogeneous row last)
    int64_t n = 0;   // number of points
    std::vector<T> features;  // point-major: features[i * rows + r]
    std::vector<Label> featureLabels;
    std::vector<Label> descriptorLabels;
    int descDim = 0;
    std::vector<T> descriptors;  // point-major: descriptors[i * descDim + r]
    // A borrowed cloud (the C ABI's prepare / setMap with the caller's arrays,
    // pm_capi.cpp): the features / descriptors are read in place, not copied
    // (1M points: 44 MB of host copies and first-touch page faults, ~3 ms of
    // setup).  Any copy of a DataPoints owns its data (the filter chains
    // mutate copies), and every mutator materialises first; read through
    // feat() / desc().
    const T* ext = nullptr;
    const T* extDesc = nullptr;

    DataPoints() = default;
    DataPoints(DataPoints&&) = default;
    DataPoints& operator=(DataPoints&&) = default;
    DataPoints(const DataPoints& o) { *this = o; }
    DataPoints& operator=(const DataPoints& o) {
        if (this == &o) return *this;
        rows = o.rows;
        n = o.n;
        featureLabels = o.featureLabels;
        descriptorLabels = o.descriptorLabels;
        descDim = o.descDim;
        if (o.ext)
            features.assign(o.ext, o.ext + (size_t)rows * (size_t)n);
        else
            features = o.features;
        if (o.extDesc)
            descriptors.assign(o.extDesc, o.extDesc + (size_t)descDim * (size_t)n);
        else
            descriptors = o.descriptors;
        ext = extDesc = nullptr;
        return *this;
    }
    const T* feat() const { return ext ? ext : features.data(); }
    const T* desc() const { return extDesc ? extDesc : descriptors.data(); }
    void materialize() {
        if (ext) features.assign(ext, ext + (size_t)rows * (size_t)n);
        if (extDesc) descriptors.assign(extDesc, extDesc + (size_t)descDim * (size_t)n);
        ext = extDesc = nullptr;
    }

    int64_t getNbPoints() const { return n; }
    int getEuclideanDim() const { return rows - 1; }
    int getHomogeneousDim() const { return rows; }
    bool descriptorExists(const std::string& name) const {
        for (auto& l : descriptorLabels)
            if (l.text == name) return true;
        return false;
    }
    // copy of one descriptor (span x n, point-major) — getDescriptorViewByName
    std::vector<T> descriptor(const std::string& name, int* span = nullptr) const {
        int off = 0;
        for (auto& l : descriptorLabels) {
            if (l.text == name) {
                std::vector<T> out((size_t)l.span * n);
                const T* d = desc();
                for (int64_t i = 0; i < n; ++i)
                    for (int r = 0; r < l.span; ++r) out[i * l.span + r] = d[i * descDim + off + r];
                if (span) *span = l.span;
                return out;
            }
            off += l.span;
        }
        throw InvalidElement("DataPoints::getDescriptorViewByName(): descriptor " + name + " not found");
    }
    // allocateDescriptors + the view assignment of a data filter: overwrite an
    // existing label of the same span, else append (PointMatcher.h:281-296)
    void setDescriptor(const std::string& name, int span, const T* data) {
        materialize();
        int off = 0;
        for (auto& l : descriptorLabels) {
            if (l.text == name && l.span == span) {
                for (int64_t i = 0; i < n; ++i)
                    for (int r = 0; r < span; ++r) descriptors[i * descDim + off + r] = data[i * span + r];
                return;
            }
            off += l.span;
        }
        addDescriptor(name, span, data);
    }
    void addDescriptor(const std::string& name, int span, const T* data) {
        materialize();
        std::vector<T> nd((size_t)(descDim + span) * n);
        for (int64_t i = 0; i < n; ++i) {
            for (int r = 0; r < descDim; ++r) nd[i * (descDim + span) + r] = descriptors[i * descDim + r];
            for (int r = 0; r < span; ++r) nd[i * (descDim + span) + descDim + r] = data[i * span + r];
        }
        descriptors.swap(nd);
        descDim += span;
        descriptorLabels.push_back({name, span});
    }
};

// ------------------------------------------------------------- dense kit --
// The Eigen 3.3 algorithms of the minimisers and checkers live in
// csrc/common/pmx_dense.h, shared with the device-resident ICP loop.
namespace dense {
using namespace ::pmx_dense;
}  // namespace dense
}  // namespace pm
