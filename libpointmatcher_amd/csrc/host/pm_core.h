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
                for (int64_t i = 0; i < n; ++i)
                    for (int r = 0; r < l.span; ++r) out[i * l.span + r] = descriptors[i * descDim + off + r];
                if (span) *span = l.span;
                return out;
            }
            off += l.span;
        }
        throw InvalidElement("DataPoints::getDescriptorViewByName(): descriptor " + name + " not found");
    }
    void addDescriptor(const std::string& name, int span, const T* data) {
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
// Row-major n x n arrays (n <= 6).  Eigen 3.3 algorithms (not vendored in the
// reference); sequential summation order.
namespace dense {

template <typename T>
T eps() {
    return std::numeric_limits<T>::epsilon();
}
template <typename T>
T tiny() {
    return std::numeric_limits<T>::min();
}
template <typename T>
T dot(const T* x, const T* y, int n) {
    T s = 0;
    for (int i = 0; i < n; ++i) s = s + x[i] * y[i];
    return s;
}

// LLT<Lower> unblocked (Eigen/src/Cholesky/LLT.h); the reference ignores a
// failed decomposition, so does this
template <typename T>
void llt(const T* A, int n, T* L) {
    for (int i = 0; i < n * n; ++i) L[i] = 0;
    for (int r = 0; r < n; ++r)
        for (int c = 0; c <= r; ++c) L[r * n + c] = A[r * n + c];
    for (int k = 0; k < n; ++k) {
        T x = L[k * n + k];
        if (k > 0) x = x - dot(&L[k * n], &L[k * n], k);
        if (x <= (T)0) return;
        x = std::sqrt(x);
        L[k * n + k] = x;
        for (int i = k + 1; i < n; ++i) {
            T v = L[i * n + k];
            if (k > 0) v = v - dot(&L[i * n], &L[k * n], k);
            L[i * n + k] = v / x;
        }
    }
}
template <typename T>
void llt_solve(const T* L, int n, const T* b, T* x) {
    T y[6];
    for (int i = 0; i < n; ++i) {
        T s = b[i];
        for (int j = 0; j < i; ++j) s = s - L[i * n + j] * y[j];
        y[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        T s = y[i];
        for (int j = i + 1; j < n; ++j) s = s - L[j * n + i] * x[j];
        x[i] = s / L[i * n + i];
    }
}

// Householder reflector on v[0], v[stride], ... (makeHouseholderInPlace)
template <typename T>
void make_householder(T* v, int stride, int m, T& tau, T& beta) {
    T tail = 0;
    for (int i = 1; i < m; ++i) tail = tail + v[i * stride] * v[i * stride];
    const T c0 = v[0];
    if (m == 1 || tail <= tiny<T>()) {
        tau = 0;
        beta = c0;
        for (int i = 1; i < m; ++i) v[i * stride] = 0;
        return;
    }
    T b = std::sqrt(c0 * c0 + tail);
    if (c0 >= (T)0) b = -b;
    for (int i = 1; i < m; ++i) v[i * stride] = v[i * stride] / (c0 - b);
    tau = (b - c0) / b;
    beta = b;
}

// applyHouseholderOnTheLeft to rows r0..r0+m, columns c0..c0+nc of M (ld n)
template <typename T>
void householder_left(T* M, int n, int r0, int m, int c0, int nc, const T* ess, int es, T tau) {
    if (m == 1) {
        for (int c = 0; c < nc; ++c) M[r0 * n + c0 + c] = M[r0 * n + c0 + c] * ((T)1 - tau);
        return;
    }
    if (tau == (T)0) return;
    for (int c = 0; c < nc; ++c) {
        T t = 0;
        for (int i = 1; i < m; ++i) t = t + ess[(i - 1) * es] * M[(r0 + i) * n + c0 + c];
        t = t + M[r0 * n + c0 + c];
        M[r0 * n + c0 + c] = M[r0 * n + c0 + c] - tau * t;
        for (int i = 1; i < m; ++i) M[(r0 + i) * n + c0 + c] = M[(r0 + i) * n + c0 + c] - tau * ess[(i - 1) * es] * t;
    }
}

// FullPivHouseholderQR (Eigen/src/QR/FullPivHouseholderQR.h)
template <typename T>
struct FullPivQR {
    int n = 0;
    T qr[36];
    T hcoeffs[6];
    int rowtr[6], coltr[6], perm[6];
    int nonzero = 0;
    T maxpivot = 0;

    void compute(const T* A, int nn) {
        n = nn;
        for (int i = 0; i < n * n; ++i) qr[i] = A[i];
        const T precision = eps<T>() * (T)n;
        maxpivot = 0;
        nonzero = n;
        T biggest = 0;
        for (int k = 0; k < n; ++k) {
            int br = k, bc = k;
            T best = -1;
            for (int c = k; c < n; ++c)
                for (int r = k; r < n; ++r) {
                    const T v = std::fabs(qr[r * n + c]);
                    if (v > best) {
                        best = v;
                        br = r;
                        bc = c;
                    }
                }
            if (k == 0) biggest = best;
            if (best <= biggest * precision) {
                nonzero = k;
                for (int i = k; i < n; ++i) {
                    rowtr[i] = i;
                    coltr[i] = i;
                    hcoeffs[i] = 0;
                }
                break;
            }
            rowtr[k] = br;
            coltr[k] = bc;
            if (k != br)
                for (int c = k; c < n; ++c) std::swap(qr[k * n + c], qr[br * n + c]);
            if (k != bc)
                for (int r = 0; r < n; ++r) std::swap(qr[r * n + k], qr[r * n + bc]);
            T tau, beta;
            make_householder(&qr[k * n + k], n, n - k, tau, beta);
            hcoeffs[k] = tau;
            qr[k * n + k] = beta;
            if (std::fabs(beta) > maxpivot) maxpivot = std::fabs(beta);
            householder_left(qr, n, k, n - k, k + 1, n - k - 1, &qr[(k + 1) * n + k], n, tau);
        }
        for (int i = 0; i < n; ++i) perm[i] = i;
        for (int k = 0; k < n; ++k) std::swap(perm[k], perm[coltr[k]]);
    }
    int rank() const {
        const T thr = std::fabs(maxpivot) * ((T)n * eps<T>());
        int r = 0;
        for (int i = 0; i < nonzero; ++i) r += std::fabs(qr[i * n + i]) > thr;
        return r;
    }
    void matrixQ(T* Q) const {
        for (int i = 0; i < n * n; ++i) Q[i] = 0;
        for (int i = 0; i < n; ++i) Q[i * n + i] = 1;
        for (int k = n - 1; k >= 0; --k) {
            householder_left(Q, n, k, n - k, k, n - k, &qr[(k + 1) * n + k], n, hcoeffs[k]);
            const int t = rowtr[k];
            if (t != k)
                for (int c = 0; c < n; ++c) std::swap(Q[k * n + c], Q[t * n + c]);
        }
    }
};

// two-sided Jacobi SVD of a square matrix (Eigen/src/SVD/JacobiSVD.h):
// A = U diag(S) V^T, S descending
template <typename T>
void make_jacobi(T x, T y, T z, T& c, T& s) {
    const T deno = (T)2 * std::fabs(y);
    if (deno < tiny<T>()) {
        c = 1;
        s = 0;
        return;
    }
    const T tau = (x - z) / deno;
    const T w = std::sqrt(tau * tau + (T)1);
    const T t = tau > (T)0 ? (T)1 / (tau + w) : (T)1 / (tau - w);
    const T sign_t = t > (T)0 ? (T)1 : (T)-1;
    const T nn = (T)1 / std::sqrt(t * t + (T)1);
    s = -sign_t * (y / std::fabs(y)) * std::fabs(t) * nn;
    c = nn;
}
template <typename T>
void rot_left(T* M, int n, int p, int q, T c, T s) {
    for (int i = 0; i < n; ++i) {
        const T xi = M[p * n + i], yi = M[q * n + i];
        M[p * n + i] = c * xi + s * yi;
        M[q * n + i] = -s * xi + c * yi;
    }
}
template <typename T>
void rot_right(T* M, int n, int p, int q, T c, T s) {
    const T ct = c, st = -s;
    for (int i = 0; i < n; ++i) {
        const T xi = M[i * n + p], yi = M[i * n + q];
        M[i * n + p] = ct * xi + st * yi;
        M[i * n + q] = -st * xi + ct * yi;
    }
}
template <typename T>
int jacobi_svd(const T* A, int n, T* U, T* S, T* V) {
    T W[36];
    const T precision = (T)2 * eps<T>();
    T scale = 0;
    for (int i = 0; i < n * n; ++i) scale = std::max(scale, (T)std::fabs(A[i]));
    if (scale == (T)0) scale = 1;
    for (int i = 0; i < n * n; ++i) W[i] = A[i] / scale;
    for (int i = 0; i < n * n; ++i) U[i] = V[i] = 0;
    for (int i = 0; i < n; ++i) U[i * n + i] = V[i * n + i] = 1;
    T maxDiag = 0;
    for (int i = 0; i < n; ++i) maxDiag = std::max(maxDiag, (T)std::fabs(W[i * n + i]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
        finished = true;
        for (int p = 1; p < n; ++p)
            for (int q = 0; q < p; ++q) {
                const T thr = std::max(tiny<T>(), precision * maxDiag);
                if (std::fabs(W[p * n + q]) > thr || std::fabs(W[q * n + p]) > thr) {
                    finished = false;
                    const T m00 = W[p * n + p], m01 = W[p * n + q], m10 = W[q * n + p], m11 = W[q * n + q];
                    const T t = m00 + m11, d = m10 - m01;
                    T c1, s1;
                    if (std::fabs(d) < tiny<T>()) {
                        s1 = 0;
                        c1 = 1;
                    } else {
                        const T u = t / d;
                        const T tmp = std::sqrt((T)1 + u * u);
                        s1 = (T)1 / tmp;
                        c1 = u / tmp;
                    }
                    const T n00 = c1 * m00 + s1 * m10, n01 = c1 * m01 + s1 * m11;
                    const T n11 = -s1 * m01 + c1 * m11;
                    T cr, sr;
                    make_jacobi(n00, n01, n11, cr, sr);
                    const T cl = c1 * cr - s1 * (-sr);
                    const T sl = c1 * (-sr) + s1 * cr;
                    rot_left(W, n, p, q, cl, sl);
                    rot_right(U, n, p, q, cl, -sl);
                    rot_right(W, n, p, q, cr, sr);
                    rot_right(V, n, p, q, cr, sr);
                    maxDiag = std::max(maxDiag, std::max((T)std::fabs(W[p * n + p]), (T)std::fabs(W[q * n + q])));
                }
            }
    }
    for (int i = 0; i < n; ++i) {
        const T a = W[i * n + i];
        S[i] = std::fabs(a);
        if (a < (T)0)
            for (int r = 0; r < n; ++r) U[r * n + i] = -U[r * n + i];
    }
    for (int i = 0; i < n; ++i) S[i] = S[i] * scale;
    int nonzero = n;
    for (int i = 0; i < n; ++i) {
        int pos = i;
        T mx = S[i];
        for (int j = i + 1; j < n; ++j)
            if (S[j] > mx) {
                mx = S[j];
                pos = j;
            }
        if (mx == (T)0) {
            nonzero = i;
            break;
        }
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < n; ++r) {
                std::swap(U[r * n + i], U[r * n + pos]);
                std::swap(V[r * n + i], V[r * n + pos]);
            }
        }
    }
    return nonzero;
}
template <typename T>
void svd_solve(const T* A, int n, const T* b, T* x) {
    T U[36], S[6], V[36], tmp[6];
    const int nz = jacobi_svd(A, n, U, S, V);
    T thr = std::max(S[0] * ((T)n * eps<T>()), tiny<T>());
    int rank = nz;
    while (rank > 0 && S[rank - 1] < thr) --rank;
    for (int i = 0; i < rank; ++i) {
        T s = 0;
        for (int r = 0; r < n; ++r) s = s + U[r * n + i] * b[r];
        tmp[i] = s / S[i];
    }
    for (int r = 0; r < n; ++r) {
        T s = 0;
        for (int i = 0; i < rank; ++i) s = s + V[r * n + i] * tmp[i];
        x[r] = s;
    }
}

// solvePossiblyUnderdeterminedLinearSystem (ErrorMinimizers/PointToPlane.cpp:108-161)
template <typename T>
void solve_underdetermined(const T* A, const T* b, int n, T* x) {
    FullPivQR<T> qr;
    qr.compute(A, n);
    const int rank = qr.rank();
    if (rank == n) {
        T L[36];
        llt(A, n, L);
        llt_solve(L, n, b, x);
        return;
    }
    T Q[36], Q1t[36], QA[36], R1[36];
    qr.matrixQ(Q);
    for (int r = 0; r < rank; ++r)
        for (int c = 0; c < n; ++c) Q1t[r * n + c] = Q[c * n + r];
    for (int r = 0; r < rank; ++r)
        for (int c = 0; c < n; ++c) {
            T s = 0;
            for (int k = 0; k < n; ++k) s = s + Q1t[r * n + k] * A[k * n + c];
            QA[r * n + c] = s;
        }
    for (int r = 0; r < rank; ++r)
        for (int c = 0; c < n; ++c) R1[r * n + c] = QA[r * n + qr.perm[c]];
    T RRt[36], Qb[6], y[6], L[36], xp[6];
    for (int i = 0; i < rank; ++i)
        for (int j = 0; j < rank; ++j) RRt[i * rank + j] = dot(&R1[i * n], &R1[j * n], n);
    for (int i = 0; i < rank; ++i) Qb[i] = dot(&Q1t[i * n], b, n);
    llt(RRt, rank, L);
    llt_solve(L, rank, Qb, y);
    for (int c = 0; c < n; ++c) {
        T s = 0;
        for (int r = 0; r < rank; ++r) s = s + ((c >= r) ? R1[r * n + c] : (T)0) * y[r];
        xp[c] = s;
    }
    for (int i = 0; i < n; ++i) x[qr.perm[i]] = xp[i];
    T dn = 0, bn = 0, an = 0;
    for (int r = 0; r < n; ++r) {
        const T ax = dot(&A[r * n], x, n);
        const T d = b[r] - ax;
        dn = dn + d * d;
        bn = bn + b[r] * b[r];
        an = an + ax * ax;
    }
    if (!(dn <= (T)1e-5 * (T)1e-5 * std::min(bn, an))) {
        // "QR solution was too inaccurate": double-precision JacobiSVD
        double Ad[36], bd[6], xd[6];
        for (int i = 0; i < n * n; ++i) Ad[i] = (double)A[i];
        for (int i = 0; i < n; ++i) bd[i] = (double)b[i];
        svd_solve<double>(Ad, n, bd, xd);
        for (int i = 0; i < n; ++i) x[i] = (T)xd[i];
    }
}

// AngleAxis::toRotationMatrix (Eigen/src/Geometry/AngleAxis.h)
template <typename T>
void angle_axis(T angle, const T* axis, T* R) {
    const T s = std::sin(angle), c = std::cos(angle);
    T sa[3], c1a[3];
    for (int i = 0; i < 3; ++i) {
        sa[i] = s * axis[i];
        c1a[i] = ((T)1 - c) * axis[i];
    }
    T tmp;
    tmp = c1a[0] * axis[1];
    R[1] = tmp - sa[2];
    R[3] = tmp + sa[2];
    tmp = c1a[0] * axis[2];
    R[2] = tmp + sa[1];
    R[6] = tmp - sa[1];
    tmp = c1a[1] * axis[2];
    R[5] = tmp - sa[0];
    R[7] = tmp + sa[0];
    for (int i = 0; i < 3; ++i) R[i * 3 + i] = c1a[i] * axis[i] + c;
}

// Quaternion(Matrix3) (Eigen/src/Geometry/Quaternion.h) -> (x, y, z, w)
template <typename T>
void quat_from_matrix(const T* m, T* q) {
    T t = (m[0] + m[4]) + m[8];
    if (t > (T)0) {
        t = std::sqrt(t + (T)1);
        q[3] = (T)0.5 * t;
        t = (T)0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[i * 3 + i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        t = std::sqrt(((m[i * 3 + i] - m[j * 3 + j]) - m[k * 3 + k]) + (T)1);
        q[i] = (T)0.5 * t;
        t = (T)0.5 / t;
        q[3] = (m[k * 3 + j] - m[j * 3 + k]) * t;
        q[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
        q[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
    }
}
// QuaternionBase::angularDistance: 2 atan2(|d.vec|, |d.w|), d = a * conj(b)
template <typename T>
T angular_distance(const T* a, const T* b) {
    const T bx = -b[0], by = -b[1], bz = -b[2], bw = b[3];
    const T w = a[3] * bw - a[0] * bx - a[1] * by - a[2] * bz;
    const T x = a[3] * bx + a[0] * bw + a[1] * bz - a[2] * by;
    const T y = a[3] * by + a[1] * bw + a[2] * bx - a[0] * bz;
    const T z = a[3] * bz + a[2] * bw + a[0] * by - a[1] * bx;
    const T vn = std::sqrt((x * x + y * y) + z * z);
    return (T)2 * std::atan2(vn, (T)std::fabs(w));
}

// C = A * B, n x n, sequential inner sums
template <typename T>
void matmul(const T* A, const T* B, int n, T* C) {
    T tmp[16];
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) {
            T s = A[r * n] * B[c];
            for (int k = 1; k < n; ++k) s = s + A[r * n + k] * B[k * n + c];
            tmp[r * n + c] = s;
        }
    for (int i = 0; i < n * n; ++i) C[i] = tmp[i];
}

template <typename T>
T det_rot(const T* M, int rows) {
    if (rows == 4)
        return M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) +
               M[2] * (M[4] * M[9] - M[5] * M[8]);
    return M[0] * M[4] - M[1] * M[3];
}

}  // namespace dense
}  // namespace pm
