// ORACLE (test infrastructure only -- never linked into the product path).
//
// Restatement of the hyperelastic per-tet proximal solve of the reference:
//   HyperElasticTet::prox (admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:151-162) minimising
//   f(F) = vol * (Psi(F) + k/2 |F - v|^2) with the vendored mcloptlib L-BFGS
//   (deps/mcloptlib/include/MCL/LBFGS.hpp:135-305: history m = 6, eps = 1e-6 relative
//   gradient test, past = 1 / delta = 1e-16 objective test, max_iters = 100, Armijo
//   backtracking with ftol = 1e-4, factor 0.5, first step 1/|d| then 1).
//   Energies: NeoHookean (TetEnergyTerm.cpp:206-251), StVK (:256-307).
#pragma once
#include <cmath>
#include <stdexcept>

namespace oracle {

enum { MAT_LINEAR = 0, MAT_NEOHOOKEAN = 1, MAT_STVK = 2 };

// F(r,c) = x[c*3 + r]  (Eigen column-major Map<Matrix3d>)
inline double Fget(const double* x, int r, int c) { return x[c * 3 + r]; }

inline double det3cm(const double* x) {
    auto F = [&](int r, int c) { return Fget(x, r, c); };
    return F(0, 0) * (F(1, 1) * F(2, 2) - F(1, 2) * F(2, 1)) - F(0, 1) * (F(1, 0) * F(2, 2) - F(1, 2) * F(2, 0)) +
           F(0, 2) * (F(1, 0) * F(2, 1) - F(1, 1) * F(2, 0));
}

// energy density Psi(F)
inline double psi(int mat, double mu, double lambda, const double* x) {
    if (mat == MAT_NEOHOOKEAN) {
        double J = det3cm(x);
        double I1 = 0;
        for (int i = 0; i < 9; ++i) I1 += x[i] * x[i];
        double I3 = J * J;
        double lI3 = std::log(I3);
        return 0.5 * mu * (I1 - lI3 - 3.0) + 0.125 * lambda * lI3 * lI3;
    }
    // StVK: E = 1/2 (F^T F - I); mu tr(E^T E) + lambda/2 tr(E)^2
    double E[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Fget(x, k, r) * Fget(x, k, c);
            E[c * 3 + r] = 0.5 * (s - (r == c ? 1.0 : 0.0));
        }
    double tr = E[0] + E[4] + E[8], ee = 0;
    for (int i = 0; i < 9; ++i) ee += E[i] * E[i];
    return mu * ee + 0.5 * lambda * tr * tr;
}

// dPsi/dF into g (column-major 9)
inline void psi_grad(int mat, double mu, double lambda, const double* x, double* g) {
    if (mat == MAT_NEOHOOKEAN) {
        // mu (F - F^-T) + lambda log(J) F^-T
        auto F = [&](int r, int c) { return Fget(x, r, c); };
        double J = det3cm(x);
        double cof[9];  // cofactor matrix C(r,c); F^-T = C / J
        cof[0 * 3 + 0] = F(1, 1) * F(2, 2) - F(1, 2) * F(2, 1);
        cof[0 * 3 + 1] = -(F(1, 0) * F(2, 2) - F(1, 2) * F(2, 0));
        cof[0 * 3 + 2] = F(1, 0) * F(2, 1) - F(1, 1) * F(2, 0);
        cof[1 * 3 + 0] = -(F(0, 1) * F(2, 2) - F(0, 2) * F(2, 1));
        cof[1 * 3 + 1] = F(0, 0) * F(2, 2) - F(0, 2) * F(2, 0);
        cof[1 * 3 + 2] = -(F(0, 0) * F(2, 1) - F(0, 1) * F(2, 0));
        cof[2 * 3 + 0] = F(0, 1) * F(1, 2) - F(0, 2) * F(1, 1);
        cof[2 * 3 + 1] = -(F(0, 0) * F(1, 2) - F(0, 2) * F(1, 0));
        cof[2 * 3 + 2] = F(0, 0) * F(1, 1) - F(0, 1) * F(1, 0);
        double invJ = 1.0 / J, lJ = std::log(J);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                double FinvT = cof[r * 3 + c] * invJ;
                g[c * 3 + r] = mu * (F(r, c) - FinvT) + lambda * lJ * FinvT;
            }
        return;
    }
    // StVK: F (2 mu E + lambda tr(E) I)
    double E[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Fget(x, k, r) * Fget(x, k, c);
            E[c * 3 + r] = 0.5 * (s - (r == c ? 1.0 : 0.0));
        }
    double tr = E[0] + E[4] + E[8];
    double P[9];
    for (int i = 0; i < 9; ++i) P[i] = 2.0 * mu * E[i];
    P[0] += lambda * tr; P[4] += lambda * tr; P[8] += lambda * tr;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0;
            for (int k = 0; k < 3; ++k) s += Fget(x, r, k) * P[c * 3 + k];
            g[c * 3 + r] = s;
        }
}

struct ProxProblem {
    int mat;
    double mu, lambda, k, vol;
    double v[9];
    // returns vol*value, grad = vol*(dPsi + k (x - v))   (NHProx::gradient, TetEnergyTerm.cpp:235-244)
    double eval(const double* x, double* grad) const {
        psi_grad(mat, mu, lambda, x, grad);
        double q = 0;
        for (int i = 0; i < 9; ++i) {
            double d = v[i] - x[i];
            q += d * d;
            grad[i] = vol * (grad[i] + k * (x[i] - v[i]));
        }
        return vol * (psi(mat, mu, lambda, x) + 0.5 * k * q);
    }
};

inline double dot9(const double* a, const double* b) { double s = 0; for (int i = 0; i < 9; ++i) s += a[i] * b[i]; return s; }
inline double nrm9(const double* a) { return std::sqrt(dot9(a, a)); }

// LBFGS<double,9>::minimize; returns the iteration count k (1 = early exit).
inline int lbfgs_minimize(const ProxProblem& P, double* x) {
    const int m = 6, max_iters = 100, max_ls = 2000;
    const double eps = 1e-6, delta = 1e-16, ftol = 1e-4, min_step = 1e-20, max_step = 1e20;
    double s[6][9], y[6][9], ys_h[6], alpha[6], g[9], gp[9], xp[9], drt[9];
    double fx = P.eval(x, g);
    double xnorm = nrm9(x), gnorm = nrm9(g);
    double fpast = fx;
    if (gnorm <= eps * std::max(xnorm, 1.0)) return 1;
    for (int i = 0; i < 9; ++i) drt[i] = -g[i];
    double step = 1.0 / nrm9(drt);
    int k = 1, end = 0;
    for (;;) {
        for (int i = 0; i < 9; ++i) { xp[i] = x[i]; gp[i] = g[i]; }
        // backtracking Armijo line search
        {
            const double fx_init = fx, dg_init = dot9(g, drt), dg_test = ftol * dg_init;
            for (int it = 0; it < max_ls; ++it) {
                for (int i = 0; i < 9; ++i) x[i] = xp[i] + step * drt[i];
                fx = P.eval(x, g);
                if (!(fx > fx_init + step * dg_test)) break;   // Armijo met (NaN counts as met)
                if (step < min_step) throw std::runtime_error("the line search step became smaller than the minimum value allowed");
                if (step > max_step) throw std::runtime_error("the line search step became larger than the maximum value allowed");
                step *= 0.5;
            }
        }
        xnorm = nrm9(x); gnorm = nrm9(g);
        if (gnorm <= eps * std::max(xnorm, 1.0)) return k;
        if (k >= 1 && std::fabs(fpast - fx) < delta) return k;
        fpast = fx;
        if (k >= max_iters) return k;
        for (int i = 0; i < 9; ++i) { s[end][i] = x[i] - xp[i]; y[end][i] = g[i] - gp[i]; }
        double ys = dot9(y[end], s[end]), yy = dot9(y[end], y[end]);
        ys_h[end] = ys;
        for (int i = 0; i < 9; ++i) drt[i] = -g[i];
        int bound = std::min(m, k);
        end = (end + 1) % m;
        int j = end;
        for (int i = 0; i < bound; ++i) {
            j = (j + m - 1) % m;
            alpha[j] = dot9(s[j], drt) / ys_h[j];
            for (int t = 0; t < 9; ++t) drt[t] -= alpha[j] * y[j][t];
        }
        for (int t = 0; t < 9; ++t) drt[t] *= ys / yy;
        for (int i = 0; i < bound; ++i) {
            double beta = dot9(y[j], drt) / ys_h[j];
            for (int t = 0; t < 9; ++t) drt[t] += (alpha[j] - beta) * s[j][t];
            j = (j + 1) % m;
        }
        step = 1.0;
        ++k;
    }
}

}  // namespace oracle
