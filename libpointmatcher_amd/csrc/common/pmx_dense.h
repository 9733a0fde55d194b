// pmx_dense.h — the small dense kit of the ICP step (Eigen 3.3 algorithms the
// reference's minimisers and checkers rely on), compiled for the host chain
// (g++) and for the device-resident ICP loop (hipcc, one lane).
//
// Row-major n x n arrays (n <= 6), sequential summation order.  Restated
// from Eigen 3.3 (not vendored in the reference): LLT (Cholesky/LLT.h),
// FullPivHouseholderQR (QR/FullPivHouseholderQR.h), two-sided JacobiSVD
// (SVD/JacobiSVD.h), AngleAxis (Geometry/AngleAxis.h), Quaternion from a
// rotation matrix and angularDistance (Geometry/Quaternion.h); and the
// reference's own solvePossiblyUnderdeterminedLinearSystem
// (ErrorMinimizers/PointToPlane.cpp:108-161) and transform constructions
// (PointToPlane.cpp:245-312, PointToPoint.cpp:61-101).
#pragma once

#include <cmath>
#include <limits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PMX_HD __host__ __device__
#else
#define PMX_HD
#endif
// full unrolling on the device: with the sizes constant after inlining, every
// array index becomes static and the arrays stay in VGPRs (a single lane
// walking scratch memory is ~10x slower)
#if defined(__HIP_DEVICE_COMPILE__)
#define PMX_UNROLL _Pragma("unroll")
#else
#define PMX_UNROLL
#endif

namespace pmx_dense {

using std::acos;
using std::atan2;
using std::cos;
using std::fabs;
using std::sin;
using std::sqrt;

template <typename T>
PMX_HD inline T eps() {
    return std::numeric_limits<T>::epsilon();
}
template <typename T>
PMX_HD inline T tiny() {
    return std::numeric_limits<T>::min();
}
template <typename T>
PMX_HD inline T vmax(T a, T b) {
    return a < b ? b : a;  // std::max
}
template <typename T>
PMX_HD inline T vmin(T a, T b) {
    return b < a ? b : a;  // std::min
}
template <typename T>
PMX_HD inline void vswap(T& a, T& b) {
    T t = a;
    a = b;
    b = t;
}
template <typename T>
PMX_HD inline T dot(const T* x, const T* y, int n) {
    T s = 0;
    PMX_UNROLL
    for (int i = 0; i < 6; ++i)  // (n <= 6; a fixed bound unrolls on the device)
        if (i < n) s = s + x[i] * y[i];
    return s;
}

// LLT<Lower> unblocked (Eigen/src/Cholesky/LLT.h); the reference ignores a
// failed decomposition, so does this
template <typename T>
PMX_HD void llt(const T* A, int n, T* L) {
    PMX_UNROLL
    for (int i = 0; i < n * n; ++i) L[i] = 0;
    PMX_UNROLL
    for (int r = 0; r < n; ++r)
        PMX_UNROLL
        for (int c = 0; c < n; ++c)
            if (c <= r) L[r * n + c] = A[r * n + c];
    bool failed = false;  // (a flag rather than a return keeps the loop unrollable)
    PMX_UNROLL
    for (int k = 0; k < n; ++k) {
        if (failed) continue;
        T x = L[k * n + k];
        if (k > 0) x = x - dot(&L[k * n], &L[k * n], k);
        if (x <= (T)0) {
            failed = true;
            continue;
        }
        x = sqrt(x);
        L[k * n + k] = x;
        PMX_UNROLL
        for (int i = 0; i < n; ++i) {
            if (i <= k) continue;
            T v = L[i * n + k];
            if (k > 0) v = v - dot(&L[i * n], &L[k * n], k);
            L[i * n + k] = v / x;
        }
    }
}
template <typename T>
PMX_HD void llt_solve(const T* L, int n, const T* b, T* x) {
    // inner loops run over fixed bounds with a guard so that the device
    // unroller sees constant trip counts (same operation order)
    T y[6];
    PMX_UNROLL
    for (int i = 0; i < n; ++i) {
        T s = b[i];
        PMX_UNROLL
        for (int j = 0; j < n; ++j)
            if (j < i) s = s - L[i * n + j] * y[j];
        y[i] = s / L[i * n + i];
    }
    PMX_UNROLL
    for (int i = n - 1; i >= 0; --i) {
        T s = y[i];
        PMX_UNROLL
        for (int j = 0; j < n; ++j)
            if (j > i) s = s - L[j * n + i] * x[j];
        x[i] = s / L[i * n + i];
    }
}

// Householder reflector on v[0], v[stride], ... (makeHouseholderInPlace)
template <typename T>
PMX_HD void make_householder(T* v, int stride, int m, T& tau, T& beta) {
    T tail = 0;
    PMX_UNROLL
    for (int i = 1; i < m; ++i) tail = tail + v[i * stride] * v[i * stride];
    const T c0 = v[0];
    if (m == 1 || tail <= tiny<T>()) {
        tau = 0;
        beta = c0;
        PMX_UNROLL
        for (int i = 1; i < m; ++i) v[i * stride] = 0;
        return;
    }
    T b = sqrt(c0 * c0 + tail);
    if (c0 >= (T)0) b = -b;
    PMX_UNROLL
    for (int i = 1; i < m; ++i) v[i * stride] = v[i * stride] / (c0 - b);
    tau = (b - c0) / b;
    beta = b;
}

// applyHouseholderOnTheLeft to rows r0..r0+m, columns c0..c0+nc of M (ld n)
template <typename T>
PMX_HD void householder_left(T* M, int n, int r0, int m, int c0, int nc, const T* ess, int es, T tau) {
    if (m == 1) {
        PMX_UNROLL
        for (int c = 0; c < nc; ++c) M[r0 * n + c0 + c] = M[r0 * n + c0 + c] * ((T)1 - tau);
        return;
    }
    if (tau == (T)0) return;
    PMX_UNROLL
    for (int c = 0; c < nc; ++c) {
        T t = 0;
        PMX_UNROLL
        for (int i = 1; i < m; ++i) t = t + ess[(i - 1) * es] * M[(r0 + i) * n + c0 + c];
        t = t + M[r0 * n + c0 + c];
        M[r0 * n + c0 + c] = M[r0 * n + c0 + c] - tau * t;
        PMX_UNROLL
        for (int i = 1; i < m; ++i) M[(r0 + i) * n + c0 + c] = M[(r0 + i) * n + c0 + c] - tau * ess[(i - 1) * es] * t;
    }
}

// FullPivHouseholderQR (Eigen/src/QR/FullPivHouseholderQR.h)
template <typename T>
struct FullPivQR {
    int n = 0;
    T qr[36];
    T hcoeffs[6];
    int rowtr[6], coltr[6];
    int nonzero = 0;
    T maxpivot = 0;

    PMX_HD void compute(const T* A, int nn) {
        n = nn;
        PMX_UNROLL
        for (int i = 0; i < n * n; ++i) qr[i] = A[i];
        const T precision = eps<T>() * (T)n;
        maxpivot = 0;
        nonzero = n;
        T biggest = 0;
        bool dead = false;  // (a flag rather than a break keeps the k loop unrollable)
        PMX_UNROLL
        for (int k = 0; k < n; ++k) {
            if (dead) continue;
            int br = k, bc = k;
            T best = -1;
            PMX_UNROLL
            for (int c = k; c < n; ++c)
                PMX_UNROLL
                for (int r = k; r < n; ++r) {
                    const T v = fabs(qr[r * n + c]);
                    if (v > best) {
                        best = v;
                        br = r;
                        bc = c;
                    }
                }
            if (k == 0) biggest = best;
            if (best <= biggest * precision) {
                nonzero = k;
                PMX_UNROLL
                for (int i = k; i < n; ++i) {
                    rowtr[i] = i;
                    coltr[i] = i;
                    hcoeffs[i] = 0;
                }
                dead = true;
                continue;
            }
            rowtr[k] = br;
            coltr[k] = bc;
            // swaps written with static indices (the compare selects the row /
            // column) so that qr stays in registers on the device
            PMX_UNROLL
            for (int r2 = k + 1; r2 < n; ++r2) {
                const bool sw = r2 == br;
                PMX_UNROLL
                for (int c = k; c < n; ++c) {
                    const T a = qr[k * n + c], b = qr[r2 * n + c];
                    qr[k * n + c] = sw ? b : a;
                    qr[r2 * n + c] = sw ? a : b;
                }
            }
            PMX_UNROLL
            for (int c2 = k + 1; c2 < n; ++c2) {
                const bool sw = c2 == bc;
                PMX_UNROLL
                for (int r = 0; r < n; ++r) {
                    const T a = qr[r * n + k], b = qr[r * n + c2];
                    qr[r * n + k] = sw ? b : a;
                    qr[r * n + c2] = sw ? a : b;
                }
            }
            T tau, beta;
            make_householder(&qr[k * n + k], n, n - k, tau, beta);
            hcoeffs[k] = tau;
            qr[k * n + k] = beta;
            if (fabs(beta) > maxpivot) maxpivot = fabs(beta);
            householder_left(qr, n, k, n - k, k + 1, n - k - 1, &qr[(k + 1) * n + k], n, tau);
        }
    }
    // colsPermutation (only the rank-deficient path needs it)
    PMX_HD void permutation(int* perm) const {
        for (int i = 0; i < n; ++i) perm[i] = i;
        for (int k = 0; k < n; ++k) vswap(perm[k], perm[coltr[k]]);
    }
    PMX_HD int rank() const {
        const T thr = fabs(maxpivot) * ((T)n * eps<T>());
        int r = 0;
        PMX_UNROLL
        for (int i = 0; i < n; ++i)
            if (i < nonzero) r += fabs(qr[i * n + i]) > thr;
        return r;
    }
    PMX_HD void matrixQ(T* Q) const {
        for (int i = 0; i < n * n; ++i) Q[i] = 0;
        for (int i = 0; i < n; ++i) Q[i * n + i] = 1;
        for (int k = n - 1; k >= 0; --k) {
            householder_left(Q, n, k, n - k, k, n - k, &qr[(k + 1) * n + k], n, hcoeffs[k]);
            const int t = rowtr[k];
            if (t != k)
                for (int c = 0; c < n; ++c) vswap(Q[k * n + c], Q[t * n + c]);
        }
    }
};

// two-sided Jacobi SVD of a square matrix (Eigen/src/SVD/JacobiSVD.h):
// A = U diag(S) V^T, S descending
template <typename T>
PMX_HD void make_jacobi(T x, T y, T z, T& c, T& s) {
    const T deno = (T)2 * fabs(y);
    if (deno < tiny<T>()) {
        c = 1;
        s = 0;
        return;
    }
    const T tau = (x - z) / deno;
    const T w = sqrt(tau * tau + (T)1);
    const T t = tau > (T)0 ? (T)1 / (tau + w) : (T)1 / (tau - w);
    const T sign_t = t > (T)0 ? (T)1 : (T)-1;
    const T nn = (T)1 / sqrt(t * t + (T)1);
    s = -sign_t * (y / fabs(y)) * fabs(t) * nn;
    c = nn;
}
template <typename T>
PMX_HD void rot_left(T* M, int n, int p, int q, T c, T s) {
    for (int i = 0; i < n; ++i) {
        const T xi = M[p * n + i], yi = M[q * n + i];
        M[p * n + i] = c * xi + s * yi;
        M[q * n + i] = -s * xi + c * yi;
    }
}
template <typename T>
PMX_HD void rot_right(T* M, int n, int p, int q, T c, T s) {
    const T ct = c, st = -s;
    for (int i = 0; i < n; ++i) {
        const T xi = M[i * n + p], yi = M[i * n + q];
        M[i * n + p] = ct * xi + st * yi;
        M[i * n + q] = -st * xi + ct * yi;
    }
}
template <typename T>
PMX_HD int jacobi_svd(const T* A, int n, T* U, T* S, T* V) {
    T W[36];
    const T precision = (T)2 * eps<T>();
    T scale = 0;
    for (int i = 0; i < n * n; ++i) scale = vmax(scale, (T)fabs(A[i]));
    if (scale == (T)0) scale = 1;
    for (int i = 0; i < n * n; ++i) W[i] = A[i] / scale;
    for (int i = 0; i < n * n; ++i) U[i] = V[i] = 0;
    for (int i = 0; i < n; ++i) U[i * n + i] = V[i * n + i] = 1;
    T maxDiag = 0;
    for (int i = 0; i < n; ++i) maxDiag = vmax(maxDiag, (T)fabs(W[i * n + i]));
    bool finished = false;
    for (int sweep = 0; !finished && sweep < 100; ++sweep) {
        finished = true;
        for (int p = 1; p < n; ++p)
            for (int q = 0; q < p; ++q) {
                const T thr = vmax(tiny<T>(), precision * maxDiag);
                if (fabs(W[p * n + q]) > thr || fabs(W[q * n + p]) > thr) {
                    finished = false;
                    const T m00 = W[p * n + p], m01 = W[p * n + q], m10 = W[q * n + p], m11 = W[q * n + q];
                    const T t = m00 + m11, d = m10 - m01;
                    T c1, s1;
                    if (fabs(d) < tiny<T>()) {
                        s1 = 0;
                        c1 = 1;
                    } else {
                        const T u = t / d;
                        const T tmp = sqrt((T)1 + u * u);
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
                    maxDiag = vmax(maxDiag, vmax((T)fabs(W[p * n + p]), (T)fabs(W[q * n + q])));
                }
            }
    }
    for (int i = 0; i < n; ++i) {
        const T a = W[i * n + i];
        S[i] = fabs(a);
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
        for (int j = i + 1; j < n; ++j)  // (static indices: see FullPivQR)
            if (j == pos) {
                vswap(S[i], S[j]);
                for (int r = 0; r < n; ++r) {
                    vswap(U[r * n + i], U[r * n + j]);
                    vswap(V[r * n + i], V[r * n + j]);
                }
            }
    }
    return nonzero;
}
template <typename T>
PMX_HD void svd_solve(const T* A, int n, const T* b, T* x) {
    T U[36], S[6], V[36], tmp[6];
    const int nz = jacobi_svd(A, n, U, S, V);
    T thr = vmax(S[0] * ((T)n * eps<T>()), tiny<T>());
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

// The full-rank branch: FullPivHouseholderQR(A).isInvertible() -> LLT solve
// (PointToPlane.cpp:116-118, 159).  Returns false (x untouched) when A is
// rank-deficient.
template <typename T>
PMX_HD bool solve_full_rank(const T* A, const T* b, int n, T* x) {
    FullPivQR<T> qr;
    qr.compute(A, n);
    if (qr.rank() != n) return false;
    T L[36];
    llt(A, n, L);
    llt_solve(L, n, b, x);
    return true;
}

// The rank-deficient branch (PointToPlane.cpp:119-156): minimal-norm solution
// of the rank-r reduced system, double JacobiSVD when that is inaccurate.
template <typename T>
PMX_HD void solve_rank_deficient(const T* A, const T* b, int n, T* x) {
    FullPivQR<T> qr;
    qr.compute(A, n);
    const int rank = qr.rank();
    int perm[6];
    qr.permutation(perm);
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
        for (int c = 0; c < n; ++c) R1[r * n + c] = QA[r * n + perm[c]];
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
    for (int i = 0; i < n; ++i) x[perm[i]] = xp[i];
    T dn = 0, bn = 0, an = 0;
    for (int r = 0; r < n; ++r) {
        const T ax = dot(&A[r * n], x, n);
        const T d = b[r] - ax;
        dn = dn + d * d;
        bn = bn + b[r] * b[r];
        an = an + ax * ax;
    }
    if (!(dn <= (T)1e-5 * (T)1e-5 * vmin(bn, an))) {
        // "QR solution was too inaccurate": double-precision JacobiSVD
        double Ad[36], bd[6], xd[6];
        for (int i = 0; i < n * n; ++i) Ad[i] = (double)A[i];
        for (int i = 0; i < n; ++i) bd[i] = (double)b[i];
        svd_solve<double>(Ad, n, bd, xd);
        for (int i = 0; i < n; ++i) x[i] = (T)xd[i];
    }
}

// solvePossiblyUnderdeterminedLinearSystem (ErrorMinimizers/PointToPlane.cpp:108-161)
template <typename T>
PMX_HD void solve_underdetermined(const T* A, const T* b, int n, T* x) {
    if (!solve_full_rank(A, b, n, x)) solve_rank_deficient(A, b, n, x);
}

// AngleAxis::toRotationMatrix (Eigen/src/Geometry/AngleAxis.h)
template <typename T>
PMX_HD void angle_axis(T angle, const T* axis, T* R) {
    const T s = sin(angle), c = cos(angle);
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
PMX_HD void quat_from_matrix(const T* m, T* q) {
    T t = (m[0] + m[4]) + m[8];
    if (t > (T)0) {
        t = sqrt(t + (T)1);
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
        t = sqrt(((m[i * 3 + i] - m[j * 3 + j]) - m[k * 3 + k]) + (T)1);
        q[i] = (T)0.5 * t;
        t = (T)0.5 / t;
        q[3] = (m[k * 3 + j] - m[j * 3 + k]) * t;
        q[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
        q[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
    }
}
// QuaternionBase::angularDistance: 2 atan2(|d.vec|, |d.w|), d = a * conj(b)
template <typename T>
PMX_HD T angular_distance(const T* a, const T* b) {
    const T bx = -b[0], by = -b[1], bz = -b[2], bw = b[3];
    const T w = a[3] * bw - a[0] * bx - a[1] * by - a[2] * bz;
    const T x = a[3] * bx + a[0] * bw + a[1] * bz - a[2] * by;
    const T y = a[3] * by + a[1] * bw + a[2] * bx - a[0] * bz;
    const T z = a[3] * bz + a[2] * bw + a[0] * by - a[1] * bx;
    const T vn = sqrt((x * x + y * y) + z * z);
    return (T)2 * atan2(vn, (T)fabs(w));
}

// C = A * B, n x n, sequential inner sums
template <typename T>
PMX_HD void matmul(const T* A, const T* B, int n, T* C) {
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
PMX_HD T det_rot(const T* M, int rows) {
    if (rows == 4)
        return M[0] * (M[5] * M[10] - M[6] * M[9]) - M[1] * (M[4] * M[10] - M[6] * M[8]) +
               M[2] * (M[4] * M[9] - M[5] * M[8]);
    return M[0] * M[4] - M[1] * M[3];
}

// PointToPlane: the rigid step from the solved x (PointToPlane.cpp:245-312):
// 3-D x = (rotation vector, translation) -> AngleAxis + t (identity rotation
// when NaN, PointToPlane.cpp:286-292); 2-D x = (angle, tx, ty)
template <typename T>
PMX_HD void p2plane_transform(int rows, const T* x, T* out) {
    for (int i = 0; i < rows * rows; ++i) out[i] = 0;
    if (rows == 4) {
        const T z = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
        const T ang = sqrt(z);
        T axis[3];
        if (z > (T)0) {
            const T sq = sqrt(z);
            for (int i = 0; i < 3; ++i) axis[i] = x[i] / sq;
        } else {
            for (int i = 0; i < 3; ++i) axis[i] = x[i];
        }
        T R[9];
        angle_axis(ang, axis, R);
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) out[r * 4 + c] = R[r * 3 + c];
            out[r * 4 + 3] = x[3 + r];
        }
        out[15] = 1;
        bool nan = false;
        for (int i = 0; i < 16; ++i)
            if (out[i] != out[i]) nan = true;
        if (nan)
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) out[r * 4 + c] = r == c ? (T)1 : (T)0;
    } else {
        const T s = sin(x[0]), c = cos(x[0]);
        const T m[9] = {c, -s, x[1], s, c, x[2], 0, 0, 1};
        for (int i = 0; i < 9; ++i) out[i] = m[i];
    }
}

// PointToPoint: R = U V^T (reflection fixed on the last column of V),
// t = mean_q - R mean_p, from the D x D cross-covariance m (PointToPoint.cpp:61-101)
template <typename T>
PMX_HD void p2point_transform(int rows, const T* m, const T* mp, const T* mq, T* out) {
    const int D = rows - 1;
    T U[9], S[3], V[9], R[9] = {}, Vt[9];
    jacobi_svd(m, D, U, S, V);
    for (int r = 0; r < D; ++r)
        for (int c = 0; c < D; ++c) Vt[r * D + c] = V[c * D + r];
    for (int pass = 0; pass < 2; ++pass) {
        for (int r = 0; r < D; ++r)
            for (int c = 0; c < D; ++c) {
                T s = 0;
                for (int k = 0; k < D; ++k) s = s + U[r * D + k] * Vt[k * D + c];
                R[r * D + c] = s;
            }
        const T det = D == 3 ? R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                                   R[2] * (R[3] * R[7] - R[4] * R[6])
                             : R[0] * R[3] - R[1] * R[2];
        if (pass == 1 || !(det < (T)0)) break;
        for (int c = 0; c < D; ++c) Vt[(D - 1) * D + c] = -Vt[(D - 1) * D + c];
    }
    for (int i = 0; i < rows * rows; ++i) out[i] = 0;
    for (int r = 0; r < D; ++r) {
        T s = 0;
        for (int c = 0; c < D; ++c) s = s + R[r * D + c] * mp[c];
        for (int c = 0; c < D; ++c) out[r * rows + c] = R[r * D + c];
        out[r * rows + D] = mq[r] - s;
    }
    out[D * rows + D] = 1;
}

}  // namespace pmx_dense
