// ORACLE (test infrastructure only -- never linked into the product path).
//
// Small dense kernels restated from the published algorithms the reference gets from its
// vendored Eigen 3.3.4 (admm_anderson_xzu/deps/Eigen3):
//   * two-sided Jacobi SVD with the real 2x2 Jacobi step, scaling by max|F|, threshold
//     max(DBL_MIN, 2*eps*maxDiag), sign fix and descending sort
//     (Eigen/src/SVD/JacobiSVD.h:660-786, Eigen/src/misc/RealSvd2x2.h:19-49,
//      Eigen/src/Jacobi/Jacobi.h:83-114) -- used by TetEnergyTerm::prox
//     (admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:74-96) and TriEnergyTerm::prox (:74-105).
//     The 3x2 case reduces to 2x2 by a Householder QR first (R-SVD, JacobiSVD.h:86-97).
//   * complete orthogonal decomposition solve for the Anderson normal equations:
//     column-pivoted Householder QR with LAPACK norm downdating
//     (Eigen/src/QR/ColPivHouseholderQR.h:482-579), rank threshold eps*size*|maxpivot|
//     (:255-263,378-384), the RZ step and the min-norm solve
//     (Eigen/src/QR/CompleteOrthogonalDecomposition.h:410-525), reflectors as
//     Eigen/src/Householder/Householder.h:65-131.
#pragma once
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------- Jacobi rotations
struct Rot { double c = 1, s = 0; };

// J such that J^T [[x y][y z]] J is diagonal (Jacobi.h:83-114, real case)
inline Rot make_jacobi(double x, double y, double z) {
    Rot r;
    double deno = 2.0 * std::fabs(y);
    if (deno < DBL_MIN) return r;
    double tau = (x - z) / deno;
    double w = std::sqrt(tau * tau + 1.0);
    double t = tau > 0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    double sign_t = t > 0 ? 1.0 : -1.0;
    double n = 1.0 / std::sqrt(t * t + 1.0);
    r.s = -sign_t * (y / std::fabs(y)) * std::fabs(t) * n;
    r.c = n;
    return r;
}
inline Rot rot_mul(const Rot& a, const Rot& b) { return Rot{a.c * b.c - a.s * b.s, a.c * b.s + a.s * b.c}; }
inline Rot rot_t(const Rot& a) { return Rot{a.c, -a.s}; }

// row-major N x N helpers: M[r*N+c]
template <int N> inline void rot_left(double* M, int p, int q, const Rot& j) {   // rows p,q
    for (int i = 0; i < N; ++i) {
        double x = M[p * N + i], y = M[q * N + i];
        M[p * N + i] = j.c * x + j.s * y;
        M[q * N + i] = -j.s * x + j.c * y;
    }
}
template <int N> inline void rot_right(double* M, int p, int q, const Rot& j) {  // cols p,q by J
    Rot t = rot_t(j);
    for (int i = 0; i < N; ++i) {
        double x = M[i * N + p], y = M[i * N + q];
        M[i * N + p] = t.c * x + t.s * y;
        M[i * N + q] = -t.s * x + t.c * y;
    }
}

// real 2x2 Jacobi SVD step on the (p,q) block (RealSvd2x2.h:19-49)
template <int N> inline void real_2x2(const double* W, int p, int q, Rot* jl, Rot* jr) {
    double m00 = W[p * N + p], m01 = W[p * N + q], m10 = W[q * N + p], m11 = W[q * N + q];
    Rot r1;
    double t = m00 + m11, d = m10 - m01;
    if (std::fabs(d) < DBL_MIN) { r1.s = 0; r1.c = 1; }
    else { double u = t / d; double tmp = std::sqrt(1.0 + u * u); r1.s = 1.0 / tmp; r1.c = u / tmp; }
    // m.applyOnTheLeft(0,1,r1)
    double a00 = r1.c * m00 + r1.s * m10, a01 = r1.c * m01 + r1.s * m11;
    double a10 = -r1.s * m00 + r1.c * m10, a11 = -r1.s * m01 + r1.c * m11;
    (void)a10;
    *jr = make_jacobi(a00, a01, a11);
    *jl = rot_mul(r1, rot_t(*jr));
}

// Two-sided Jacobi SVD of a square N x N (row-major) matrix A: A = U diag(S) V^T
template <int N> inline void jacobi_svd_square(const double* A, double* U, double* S, double* V) {
    double scale = 0;
    for (int i = 0; i < N * N; ++i) scale = std::max(scale, std::fabs(A[i]));
    if (scale == 0) scale = 1;
    double W[N * N];
    for (int i = 0; i < N * N; ++i) W[i] = A[i] / scale;
    for (int i = 0; i < N * N; ++i) { U[i] = (i / N == i % N); V[i] = (i / N == i % N); }
    const double precision = 2.0 * DBL_EPSILON, considerAsZero = DBL_MIN;
    double maxDiag = 0;
    for (int i = 0; i < N; ++i) maxDiag = std::max(maxDiag, std::fabs(W[i * N + i]));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 64) {
        finished = true; ++sweeps;
        for (int p = 1; p < N; ++p)
            for (int q = 0; q < p; ++q) {
                double thr = std::max(considerAsZero, precision * maxDiag);
                if (std::fabs(W[p * N + q]) > thr || std::fabs(W[q * N + p]) > thr) {
                    finished = false;
                    Rot jl, jr;
                    real_2x2<N>(W, p, q, &jl, &jr);
                    rot_left<N>(W, p, q, jl);
                    rot_right<N>(U, p, q, rot_t(jl));
                    rot_right<N>(W, p, q, jr);
                    rot_right<N>(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(std::fabs(W[p * N + p]), std::fabs(W[q * N + q])));
                }
            }
    }
    for (int i = 0; i < N; ++i) {
        double a = W[i * N + i];
        S[i] = std::fabs(a);
        if (a < 0) for (int r = 0; r < N; ++r) U[r * N + i] = -U[r * N + i];
    }
    for (int i = 0; i < N; ++i) S[i] *= scale;
    for (int i = 0; i < N; ++i) {
        int pos = i;
        for (int k = i + 1; k < N; ++k) if (S[k] > S[pos]) pos = k;
        if (S[pos] == 0) break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < N; ++r) { std::swap(U[r * N + i], U[r * N + pos]); std::swap(V[r * N + i], V[r * N + pos]); }
        }
    }
}

inline double det3(const double* F /*row-major*/) {
    return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
}

// 3x2 (row-major, F[r*2+c]) SVD: Householder QR to 2x2 then Jacobi. U is 3x3, V 2x2.
inline void svd_3x2(const double* F, double* U, double* S, double* V) {
    double scale = 0;
    for (int i = 0; i < 6; ++i) scale = std::max(scale, std::fabs(F[i]));
    if (scale == 0) scale = 1;
    double A[6];
    for (int i = 0; i < 6; ++i) A[i] = F[i] / scale;
    // Q = H1 H2 (Householder), R upper 2x2
    double Q[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 2; ++k) {
        double c0 = A[k * 2 + k], tail = 0;
        for (int r = k + 1; r < 3; ++r) tail += A[r * 2 + k] * A[r * 2 + k];
        if (tail <= DBL_MIN) continue;
        double beta = std::sqrt(c0 * c0 + tail);
        if (c0 >= 0) beta = -beta;
        double v[3] = {0, 0, 0};
        v[k] = 1.0;
        for (int r = k + 1; r < 3; ++r) v[r] = A[r * 2 + k] / (c0 - beta);
        double tau = (beta - c0) / beta;
        for (int c = k; c < 2; ++c) {  // A = (I - tau v v^T) A
            double d = 0;
            for (int r = k; r < 3; ++r) d += v[r] * A[r * 2 + c];
            for (int r = k; r < 3; ++r) A[r * 2 + c] -= tau * v[r] * d;
        }
        for (int r = 0; r < 3; ++r) {  // Q = Q (I - tau v v^T)
            double d = 0;
            for (int c = k; c < 3; ++c) d += Q[r * 3 + c] * v[c];
            for (int c = k; c < 3; ++c) Q[r * 3 + c] -= tau * d * v[c];
        }
    }
    double R[4] = {A[0], A[1], 0.0, A[3]}, U2[4], V2[4];
    jacobi_svd_square<2>(R, U2, S, V2);
    for (int i = 0; i < 2; ++i) S[i] *= scale;
    for (int r = 0; r < 3; ++r) {
        U[r * 3 + 0] = Q[r * 3 + 0] * U2[0] + Q[r * 3 + 1] * U2[2];
        U[r * 3 + 1] = Q[r * 3 + 0] * U2[1] + Q[r * 3 + 1] * U2[3];
        U[r * 3 + 2] = Q[r * 3 + 2];
    }
    for (int i = 0; i < 4; ++i) V[i] = V2[i];
}

// ---------------------------------------------------------------- COD least squares
// Solves M theta = b for the small square (n x n, column-major M[c*n+r]) normal-equation
// matrix of Anderson acceleration with Eigen's CompleteOrthogonalDecomposition semantics.
inline void cod_solve(int n, const double* Min, const double* b, double* theta) {
    std::vector<double> qr(Min, Min + n * n), hc(n, 0.0), normsU(n), normsD(n);
    auto QR = [&](int r, int c) -> double& { return qr[(size_t)c * n + r]; };
    std::vector<int> transp(n);
    for (int k = 0; k < n; ++k) {
        double s = 0;
        for (int r = 0; r < n; ++r) s += QR(r, k) * QR(r, k);
        normsD[k] = normsU[k] = std::sqrt(s);
    }
    double maxn = 0;
    for (int k = 0; k < n; ++k) maxn = std::max(maxn, normsU[k]);
    (void)maxn;
    const double ddt = std::sqrt(DBL_EPSILON);
    double maxpivot = 0;
    for (int k = 0; k < n; ++k) {
        int big = k;
        for (int j = k + 1; j < n; ++j) if (normsU[j] > normsU[big]) big = j;
        transp[k] = big;
        if (big != k) {
            for (int r = 0; r < n; ++r) std::swap(QR(r, k), QR(r, big));
            std::swap(normsU[k], normsU[big]);
            std::swap(normsD[k], normsD[big]);
        }
        // Householder on column k rows k..n-1
        double c0 = QR(k, k), tail = 0;
        for (int r = k + 1; r < n; ++r) tail += QR(r, k) * QR(r, k);
        double beta, tau;
        if (tail <= DBL_MIN) { tau = 0; beta = c0; for (int r = k + 1; r < n; ++r) QR(r, k) = 0; }
        else {
            beta = std::sqrt(c0 * c0 + tail);
            if (c0 >= 0) beta = -beta;
            for (int r = k + 1; r < n; ++r) QR(r, k) /= (c0 - beta);
            tau = (beta - c0) / beta;
        }
        hc[k] = tau;
        QR(k, k) = beta;
        maxpivot = std::max(maxpivot, std::fabs(beta));
        if (tau != 0) {
            for (int c = k + 1; c < n; ++c) {
                double t = QR(k, c);
                for (int r = k + 1; r < n; ++r) t += QR(r, k) * QR(r, c);
                QR(k, c) -= tau * t;
                for (int r = k + 1; r < n; ++r) QR(r, c) -= tau * QR(r, k) * t;
            }
        }
        for (int j = k + 1; j < n; ++j) {
            if (normsU[j] != 0) {
                double t = std::fabs(QR(k, j)) / normsU[j];
                t = (1.0 + t) * (1.0 - t);
                t = t < 0 ? 0 : t;
                double r2 = normsU[j] / normsD[j];
                double t2 = t * r2 * r2;
                if (t2 <= ddt) {
                    double s = 0;
                    for (int r = k + 1; r < n; ++r) s += QR(r, j) * QR(r, j);
                    normsD[j] = normsU[j] = std::sqrt(s);
                } else normsU[j] *= std::sqrt(t);
            }
        }
    }
    std::vector<int> perm(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    for (int k = 0; k < n; ++k) std::swap(perm[k], perm[transp[k]]);
    // rank with threshold eps * size * |maxpivot|
    double thr = std::fabs(maxpivot) * DBL_EPSILON * n;
    int rank = 0;
    for (int i = 0; i < n; ++i) rank += std::fabs(QR(i, i)) > thr;
    std::vector<double> zc(n, 0.0);
    if (rank < n) {   // RZ: [R11 R12] = [T11 0] Z
        for (int k = rank - 1; k >= 0; --k) {
            if (k != rank - 1) for (int r = 0; r <= k; ++r) std::swap(QR(r, k), QR(r, rank - 1));
            // row k, entries at columns rank-1 .. n-1 (length n-rank+1), head = QR(k, rank-1)
            int len = n - rank + 1;
            double c0 = QR(k, rank - 1), tail = 0;
            for (int c = rank; c < n; ++c) tail += QR(k, c) * QR(k, c);
            double beta, tau;
            if (tail <= DBL_MIN) { tau = 0; beta = c0; for (int c = rank; c < n; ++c) QR(k, c) = 0; }
            else {
                beta = std::sqrt(c0 * c0 + tail);
                if (c0 >= 0) beta = -beta;
                for (int c = rank; c < n; ++c) QR(k, c) /= (c0 - beta);
                tau = (beta - c0) / beta;
            }
            zc[k] = tau;
            QR(k, rank - 1) = beta;
            if (k > 0 && tau != 0 && len > 1) {
                // apply on the right to rows 0..k-1 of columns [rank-1, rank..n-1]
                for (int r = 0; r < k; ++r) {
                    double t = QR(r, rank - 1);
                    for (int c = rank; c < n; ++c) t += QR(r, c) * QR(k, c);
                    QR(r, rank - 1) -= tau * t;
                    for (int c = rank; c < n; ++c) QR(r, c) -= tau * t * QR(k, c);
                }
            }
            if (k != rank - 1) for (int r = 0; r <= k; ++r) std::swap(QR(r, k), QR(r, rank - 1));
        }
    }
    if (rank == 0) { for (int i = 0; i < n; ++i) theta[i] = 0; return; }
    std::vector<double> c(b, b + n);
    for (int k = 0; k < rank; ++k) {   // c = H_{rank-1}..H_0 c  (Q^T c with setLength(rank))
        if (hc[k] == 0) continue;
        double t = c[k];
        for (int r = k + 1; r < n; ++r) t += QR(r, k) * c[r];
        c[k] -= hc[k] * t;
        for (int r = k + 1; r < n; ++r) c[r] -= hc[k] * QR(r, k) * t;
    }
    std::vector<double> y(n, 0.0);
    for (int i = rank - 1; i >= 0; --i) {
        double s = c[i];
        for (int j = i + 1; j < rank; ++j) s -= QR(i, j) * y[j];
        y[i] = s / QR(i, i);
    }
    if (rank < n) {   // y = Z^T [y; 0]
        for (int k = 0; k < rank; ++k) {
            if (k != rank - 1) std::swap(y[k], y[rank - 1]);
            if (zc[k] != 0) {
                double t = y[rank - 1];
                for (int cc = rank; cc < n; ++cc) t += QR(k, cc) * y[cc];
                y[rank - 1] -= zc[k] * t;
                for (int cc = rank; cc < n; ++cc) y[cc] -= zc[k] * QR(k, cc) * t;
            }
            if (k != rank - 1) std::swap(y[k], y[rank - 1]);
        }
    }
    for (int i = 0; i < n; ++i) theta[perm[i]] = y[i];
}

}  // namespace oracle
