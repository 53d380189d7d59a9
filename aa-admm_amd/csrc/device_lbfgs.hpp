// Hyperelastic per-tet proximal solve, device side (one tet per thread, registers).
//
// Same algorithm as the reference's HyperElasticTet::prox
// (admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:151-162) with the vendored mcloptlib
// L-BFGS<double,9> (deps/mcloptlib/include/MCL/LBFGS.hpp:135-305): history 6, relative
// gradient test 1e-6*max(|x|,1), objective-change test 1e-16, at most 100 iterations,
// Armijo backtracking (ftol 1e-4, factor 0.5), first step 1/|g| then 1. Energies:
//   NeoHookean  Psi = mu/2 (I1 - log I3 - 3) + lambda/8 (log I3)^2   (TetEnergyTerm.cpp:206-251)
//   StVK        Psi = mu tr(E^T E) + lambda/2 tr(E)^2, E = (F^T F - I)/2  (:256-307)
// f(F) = vol (Psi(F) + k/2 |F - v|^2). A line-search step below 1e-20 raises the error flag
// (the reference throws std::runtime_error there).
#pragma once
#include <hip/hip_runtime.h>

namespace aa {
namespace dev {

__device__ __forceinline__ double det3cm(const double* x) {  // column-major F(r,c) = x[c*3+r]
    return x[0] * (x[4] * x[8] - x[7] * x[5]) - x[3] * (x[1] * x[8] - x[7] * x[2]) + x[6] * (x[1] * x[5] - x[4] * x[2]);
}

// Psi and dPsi/dF (column-major)
__device__ __forceinline__ double hyper_psi_grad(int mat, double mu, double lambda, const double* x, double* g) {
    if (mat == 1) {
        const double J = det3cm(x);
        double cof[9];  // cofactor matrix, column-major: cof(r,c) at [c*3+r]; F^-T = cof / J
        cof[0] = x[4] * x[8] - x[7] * x[5];
        cof[3] = -(x[1] * x[8] - x[7] * x[2]);
        cof[6] = x[1] * x[5] - x[4] * x[2];
        cof[1] = -(x[3] * x[8] - x[6] * x[5]);
        cof[4] = x[0] * x[8] - x[6] * x[2];
        cof[7] = -(x[0] * x[5] - x[3] * x[2]);
        cof[2] = x[3] * x[7] - x[6] * x[4];
        cof[5] = -(x[0] * x[7] - x[6] * x[1]);
        cof[8] = x[0] * x[4] - x[3] * x[1];
        const double invJ = 1.0 / J, lJ = log(J);
        double I1 = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            I1 += x[i] * x[i];
            const double finvt = cof[i] * invJ;
            g[i] = mu * (x[i] - finvt) + lambda * lJ * finvt;
        }
        // log I3 = log J^2 = 2 log J for J > 0 (one log fewer per evaluation; equal to rounding);
        // an inverted element keeps the reference's log(J^2) (finite) next to its NaN gradient
        const double lI3 = J > 0.0 ? 2.0 * lJ : log(J * J);
        return 0.5 * mu * (I1 - lI3 - 3.0) + 0.125 * lambda * lI3 * lI3;
    }
    // StVK
    double E[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            E[c * 3 + r] = 0.5 * ((x[r * 3 + 0] * x[c * 3 + 0] + x[r * 3 + 1] * x[c * 3 + 1] + x[r * 3 + 2] * x[c * 3 + 2]) -
                                  (r == c ? 1.0 : 0.0));
    const double tr = E[0] + E[4] + E[8];
    double ee = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) ee += E[i] * E[i];
    double P[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) P[i] = 2.0 * mu * E[i];
    P[0] += lambda * tr; P[4] += lambda * tr; P[8] += lambda * tr;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c)
            g[c * 3 + r] = x[0 * 3 + r] * P[c * 3 + 0] + x[1 * 3 + r] * P[c * 3 + 1] + x[2 * 3 + r] * P[c * 3 + 2];
    return mu * ee + 0.5 * lambda * tr * tr;
}

__device__ __forceinline__ double hyper_eval(int mat, double mu, double lambda, double k, double vol, const double* v,
                                             const double* x, double* g) {
    const double psi = hyper_psi_grad(mat, mu, lambda, x, g);
    double q = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const double d = v[i] - x[i];
        q += d * d;
        g[i] = vol * (g[i] + k * (x[i] - v[i]));
    }
    return vol * (psi + 0.5 * k * q);
}

__device__ __forceinline__ double d9(const double* a, const double* b) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) s += a[i] * b[i];
    return s;
}

// The L-BFGS of mcloptlib (LBFGS.hpp:205-305) as a resumable per-lane state machine, so a
// persistent kernel can run one outer iteration per trip for whichever elements its lanes hold
// (k_local_z_hq) and the plain kernel can run it to completion (hyper_prox). The history is a
// shift register (slot 0 = newest) instead of mcloptlib's ring buffer: every index is a
// compile-time constant, so s, y stay in registers (the ring buffer's dynamic indices put 864 B
// per thread in scratch). The two-loop recursion visits the pairs in the same order (newest ->
// oldest, then back), so the arithmetic is the reference's.
// AA_LBFGS_RHO (default 1): each pair keeps rho = 1 / y.s, computed once when it is pushed, and
// the two-loop recursion multiplies by it (alpha = rho s.d, beta = rho y.d) instead of dividing by
// y.s at every use -- 2 divisions per iteration instead of 13 (a division is ~8 dependent fp64
// instructions incl. a quarter-rate v_rcp_f64). mcloptlib divides (LBFGS.hpp:272-287); the
// quotients differ from the products by at most an ulp, inside the L-BFGS's own 1e-6 gradient
// tolerance (TetEnergyTerm.cpp:151-162), which is what the reference goldens are held to.
#ifndef AA_LBFGS_RHO
#define AA_LBFGS_RHO 1
#endif
struct HyperLbfgs {
    static constexpr int M = 6;
    double s[M][9], yv[M][9], ysh[M], g[9], drt[9];   // ysh: y.s, or rho = 1 / y.s (AA_LBFGS_RHO)
    double fx, fpast, step;
    int k_it;

    // x: in = v (start point). true: x already satisfies the gradient test (no iteration)
    __device__ __forceinline__ bool start(int mat, double mu, double lambda, double k, double vol, const double* v,
                                          double* x) {
        fx = hyper_eval(mat, mu, lambda, k, vol, v, x, g);
        const double xnorm = sqrt(d9(x, x)), gnorm = sqrt(d9(g, g));
        fpast = fx;
        k_it = 1;
        if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) return true;
#pragma unroll
        for (int i = 0; i < 9; ++i) drt[i] = -g[i];
        step = 1.0 / sqrt(d9(drt, drt));
        return false;
    }

    // one outer iteration: Armijo line search, stopping tests, history push, two-loop direction.
    // true when finished (converged, stalled, capped or a collapsed line search: *fail = 1)
    __device__ __forceinline__ bool iterate(int mat, double mu, double lambda, double k, double vol, const double* v,
                                            double* x, int* fail, int /*head: unused*/ = 0) {
        double xp[9], gp[9], alpha[M];
#pragma unroll
        for (int i = 0; i < 9; ++i) { xp[i] = x[i]; gp[i] = g[i]; }
        {
            const double fx_init = fx, dg_test = 1e-4 * d9(g, drt);
            for (int it = 0; it < 2000; ++it) {
#pragma unroll
                for (int i = 0; i < 9; ++i) x[i] = xp[i] + step * drt[i];
                fx = hyper_eval(mat, mu, lambda, k, vol, v, x, g);
                if (!(fx > fx_init + step * dg_test)) break;
                if (step < 1e-20 || step > 1e20) { *fail = 1; return true; }
                step *= 0.5;
            }
        }
        const double xnorm = sqrt(d9(x, x)), gnorm = sqrt(d9(g, g));
        if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) return true;
        if (fabs(fpast - fx) < 1e-16) return true;
        fpast = fx;
        if (k_it >= 100) return true;
#pragma unroll
        for (int q = M - 1; q > 0; --q) {   // push (s, y) into slot 0
            ysh[q] = ysh[q - 1];
#pragma unroll
            for (int i = 0; i < 9; ++i) { s[q][i] = s[q - 1][i]; yv[q][i] = yv[q - 1][i]; }
        }
        double ys = 0, yy = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double si = x[i] - xp[i], yi = g[i] - gp[i];
            s[0][i] = si; yv[0][i] = yi;
            ys += yi * si; yy += yi * yi;
        }
        ysh[0] = AA_LBFGS_RHO ? 1.0 / ys : ys;
#pragma unroll
        for (int i = 0; i < 9; ++i) drt[i] = -g[i];
        const int bound = k_it < M ? k_it : M;
#pragma unroll
        for (int q = 0; q < M; ++q) {
            if (q < bound) {
                alpha[q] = AA_LBFGS_RHO ? d9(s[q], drt) * ysh[q] : d9(s[q], drt) / ysh[q];
#pragma unroll
                for (int t = 0; t < 9; ++t) drt[t] -= alpha[q] * yv[q][t];
            }
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) drt[t] *= ys / yy;
#pragma unroll
        for (int q = M - 1; q >= 0; --q) {
            if (q < bound) {
                const double beta = AA_LBFGS_RHO ? d9(yv[q], drt) * ysh[q] : d9(yv[q], drt) / ysh[q];
#pragma unroll
                for (int t = 0; t < 9; ++t) drt[t] += (alpha[q] - beta) * s[q][t];
            }
        }
        step = 1.0;
        ++k_it;
        return false;
    }
};

// HyperLbfgs with the y half of the history (and y.s) in LDS: a ring of M slots per lane, 10
// doubles each (y, y.s), lane-interleaved (entry j of the lane at lds[j * stride], stride = the
// block's lanes: a wave's 64 lanes read 64 consecutive doubles, conflict-free). The s half stays
// a register shift register. That takes 120 of the ~400 registers per lane out of the VGPR/AGPR
// file: the AGPR spill traffic (v_accvgpr_read/write around every use of the history, a VALU
// instruction each) and the y half of the shift (54 moves per iteration) go away. Slot of pair q
// (0 = newest) = (head - q) mod M; the same operands in the same order as HyperLbfgs, so the
// results are bit-identical.
struct HyperLbfgsLds {
    static constexpr int M = 6, E = 10;
    double s[M][9], g[9], drt[9];
    double fx, fpast, step;
    int k_it, head;
    double* yl;   // this lane's ring: entry (slot, i) at yl[(slot * E + i) * stride]
    int stride;

    __device__ __forceinline__ void bind(double* lane_base, int lanes) { yl = lane_base; stride = lanes; }

    __device__ __forceinline__ bool start(int mat, double mu, double lambda, double k, double vol, const double* v,
                                          double* x) {
        fx = hyper_eval(mat, mu, lambda, k, vol, v, x, g);
        const double xnorm = sqrt(d9(x, x)), gnorm = sqrt(d9(g, g));
        fpast = fx;
        k_it = 1;
        head = M - 1;
        if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) return true;
#pragma unroll
        for (int i = 0; i < 9; ++i) drt[i] = -g[i];
        step = 1.0 / sqrt(d9(drt, drt));
        return false;
    }

    __device__ __forceinline__ bool iterate(int mat, double mu, double lambda, double k, double vol, const double* v,
                                            double* x, int* fail, int /*head: unused*/ = 0) {
        double xp[9], gp[9], alpha[M];
#pragma unroll
        for (int i = 0; i < 9; ++i) { xp[i] = x[i]; gp[i] = g[i]; }
        {
            const double fx_init = fx, dg_test = 1e-4 * d9(g, drt);
            for (int it = 0; it < 2000; ++it) {
#pragma unroll
                for (int i = 0; i < 9; ++i) x[i] = xp[i] + step * drt[i];
                fx = hyper_eval(mat, mu, lambda, k, vol, v, x, g);
                if (!(fx > fx_init + step * dg_test)) break;
                if (step < 1e-20 || step > 1e20) { *fail = 1; return true; }
                step *= 0.5;
            }
        }
        const double xnorm = sqrt(d9(x, x)), gnorm = sqrt(d9(g, g));
        if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) return true;
        if (fabs(fpast - fx) < 1e-16) return true;
        fpast = fx;
        if (k_it >= 100) return true;
#pragma unroll
        for (int q = M - 1; q > 0; --q)
#pragma unroll
            for (int i = 0; i < 9; ++i) s[q][i] = s[q - 1][i];
        head = head == M - 1 ? 0 : head + 1;
        double* yh = yl + (size_t)head * E * stride;
        double ys = 0, yy = 0;
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double si = x[i] - xp[i], yi = g[i] - gp[i];
            s[0][i] = si; yh[i * stride] = yi;
            ys += yi * si; yy += yi * yi;
        }
        yh[9 * stride] = AA_LBFGS_RHO ? 1.0 / ys : ys;   // as HyperLbfgs
#pragma unroll
        for (int i = 0; i < 9; ++i) drt[i] = -g[i];
        const int bound = k_it < M ? k_it : M;
        int sl = head;
#pragma unroll
        for (int q = 0; q < M; ++q) {
            if (q < bound) {
                const double* yq = yl + (size_t)sl * E * stride;
                alpha[q] = AA_LBFGS_RHO ? d9(s[q], drt) * yq[9 * stride] : d9(s[q], drt) / yq[9 * stride];
#pragma unroll
                for (int t = 0; t < 9; ++t) drt[t] -= alpha[q] * yq[t * stride];
            }
            sl = sl == 0 ? M - 1 : sl - 1;
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) drt[t] *= ys / yy;
        // sl is now (head - M) mod M = head: walk back up from the oldest pair
        sl = head == M - 1 ? 0 : head + 1;
#pragma unroll
        for (int q = M - 1; q >= 0; --q) {
            if (q < bound) {
                const double* yq = yl + (size_t)sl * E * stride;
                double yd = 0;
#pragma unroll
                for (int t = 0; t < 9; ++t) yd += yq[t * stride] * drt[t];
                const double beta = AA_LBFGS_RHO ? yd * yq[9 * stride] : yd / yq[9 * stride];
#pragma unroll
                for (int t = 0; t < 9; ++t) drt[t] += (alpha[q] - beta) * s[q][t];
            }
            sl = sl == M - 1 ? 0 : sl + 1;
        }
        step = 1.0;
        ++k_it;
        return false;
    }
};

// ---------------------------------------------------------------- two lanes per element
// HyperLbfgs with every 9-vector split over a lane PAIR (lanes 2j, 2j+1 of a wave; h = lane & 1):
// lane h holds components 5h .. 5h+4 (h = 1: components 5..8 and a zero pad). The history then
// takes 6 x 2 x 5 doubles per lane instead of 6 x 2 x 9, so the state fits 256 registers and a
// SIMD holds two waves instead of one (k_local_z_hq2, AA_LQ_SPLIT). Dot products are the two
// lanes' partial sums added across the pair (DPP quad_perm swap: a + b on one lane, b + a on the
// other, the same IEEE sum), so every decision -- Armijo, stopping tests, k_it -- is identical on
// both lanes and the pair never diverges. The energy is evaluated on the full F, gathered from
// both halves and computed redundantly on each lane. Same algorithm and constants as HyperLbfgs
// (mcloptlib LBFGS.hpp:205-305, TetEnergyTerm.cpp:151-162); the 9-term sums are now two partial
// sums added, so results differ from HyperLbfgs by rounding only (within the L-BFGS's own 1e-6
// gradient tolerance).
__device__ __forceinline__ double pair_swap(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), 0xB1, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double pair_sum(double a) { return a + pair_swap(a); }

constexpr int kHalf = 5;
__device__ __forceinline__ double d5(const double* a, const double* b) {
    double s = 0;
#pragma unroll
    for (int i = 0; i < kHalf; ++i) s += a[i] * b[i];
    return pair_sum(s);
}

// the element's full F from the two halves (h: this lane's half)
__device__ __forceinline__ void pair_full(int h, const double* x, double* F) {
#pragma unroll
    for (int j = 0; j < kHalf; ++j) {
        const double o = pair_swap(x[j]);
        F[j] = h ? o : x[j];
        if (j < 4) F[5 + j] = h ? x[j] : o;
    }
}

// Psi (full F, redundantly on both lanes) and this lane's half of dPsi/dF: the NeoHookean
// gradient mu (F - F^-T) + lambda log J F^-T needs only the own components' cofactors, so the
// other half is never formed (registers: the state must fit 256 per lane)
__device__ __forceinline__ double hyper_psi_grad2(int h, int mat, double mu, double lambda, const double* x, double* go) {
    if (mat != 1) {   // StVK: the full gradient, then this lane's half
        double G[9];
        const double psi = hyper_psi_grad(mat, mu, lambda, x, G);
#pragma unroll
        for (int j = 0; j < kHalf; ++j) go[j] = j < 4 ? (h ? G[5 + j] : G[j]) : (h ? 0.0 : G[4]);
        return psi;
    }
    const double J = det3cm(x);
    // cofactors, column-major cof(r,c) at [c*3+r] (as hyper_psi_grad)
    const double c0 = x[4] * x[8] - x[7] * x[5], c5 = -(x[0] * x[7] - x[6] * x[1]);
    const double c3 = -(x[1] * x[8] - x[7] * x[2]), c6 = x[1] * x[5] - x[4] * x[2];
    const double c1 = -(x[3] * x[8] - x[6] * x[5]), c7 = -(x[0] * x[5] - x[3] * x[2]);
    const double c2 = x[3] * x[7] - x[6] * x[4], c8 = x[0] * x[4] - x[3] * x[1];
    const double c4 = x[0] * x[8] - x[6] * x[2];
    const double invJ = 1.0 / J, lJ = log(J);
    double I1 = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) I1 += x[i] * x[i];
    const double co[kHalf] = {h ? c5 : c0, h ? c6 : c1, h ? c7 : c2, h ? c8 : c3, c4};
#pragma unroll
    for (int j = 0; j < kHalf; ++j) {
        const double xi = j < 4 ? (h ? x[5 + j] : x[j]) : x[4];
        const double finvt = co[j] * invJ;
        go[j] = (h && j == 4) ? 0.0 : mu * (xi - finvt) + lambda * lJ * finvt;
    }
    const double lI3 = J > 0.0 ? 2.0 * lJ : log(J * J);
    return 0.5 * mu * (I1 - lI3 - 3.0) + 0.125 * lambda * lI3 * lI3;
}

__device__ __forceinline__ double hyper_eval2(int h, int mat, double mu, double lambda, double k, double vol,
                                              const double* v, const double* x, double* g) {
    double F[9], go[kHalf];
    pair_full(h, x, F);
    const double psi = hyper_psi_grad2(h, mat, mu, lambda, F, go);
    double q = 0;
#pragma unroll
    for (int j = 0; j < kHalf; ++j) {
        const double d = v[j] - x[j];
        q += d * d;
        g[j] = vol * (go[j] + k * (x[j] - v[j]));
    }
    q = pair_sum(q);
    return vol * (psi + 0.5 * k * q);
}

// One EVALUATION per call (trip): a fresh element's start evaluation, or one trial point of the
// Armijo line search, followed -- when the trial is accepted -- by the stopping tests, the new
// (s, y) pair and the two-loop direction. A single call site of the energy keeps the kernel's
// register footprint at the state's own size. The history shifts when a line search begins and
// slot 0 holds (x_prev, g_prev) during it; the pair (x - x_prev, g - g_prev) is formed in place on
// acceptance (an element that stops never reads its history again). Per element the sequence of
// evaluations, tests and updates is HyperLbfgs's (LBFGS.hpp:205-305: backtracking until
// f <= f0 + 1e-4 step g.d, a step outside [1e-20, 1e20] fails; the 2000-trial cap of the line
// search cannot bind before that).
struct HyperLbfgs2 {
    static constexpr int M = 6, H = kHalf;
    double s[M][H], yv[M][H], rho[M], g[H], drt[H];   // rho = 1 / y.s (AA_LBFGS_RHO) or y.s
    double fpast, step, dg_test;   // fpast: the last accepted f (also the line search's f0)
    int k_it;
    bool fresh;

    __device__ __forceinline__ void begin() { fresh = true; }

    // shift the history, slot 0 = (x, g): the line search from x along drt starts (its f0 is
    // fpast: the start's f, or the f just accepted)
    __device__ __forceinline__ void begin_search(const double* x) {
#pragma unroll
        for (int q = M - 1; q > 0; --q) {
            rho[q] = rho[q - 1];
#pragma unroll
            for (int i = 0; i < H; ++i) { s[q][i] = s[q - 1][i]; yv[q][i] = yv[q - 1][i]; }
        }
#pragma unroll
        for (int i = 0; i < H; ++i) { s[0][i] = x[i]; yv[0][i] = g[i]; }
        dg_test = 1e-4 * d5(g, drt);
    }

    // v: the prox target; x: in/out (the point, v on a fresh element). true = the element is done
    __device__ __forceinline__ bool trip(int h, int mat, double mu, double lambda, double k, double vol,
                                         const double* v, double* x, int* fail) {
        if (!fresh) {
#pragma unroll
            for (int i = 0; i < H; ++i) x[i] = s[0][i] + step * drt[i];
        }
        const double f = hyper_eval2(h, mat, mu, lambda, k, vol, v, x, g);
        if (fresh) {   // LBFGS.hpp: start
            fresh = false;
            const double xnorm = sqrt(d5(x, x)), gnorm = sqrt(d5(g, g));
            fpast = f;
            k_it = 1;
            if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) { k_it = 0; return true; }   // (k_it 0: no iteration)
#pragma unroll
            for (int i = 0; i < H; ++i) drt[i] = -g[i];
            step = 1.0 / sqrt(d5(drt, drt));
            begin_search(x);
            return false;
        }
        if (f > fpast + step * dg_test) {   // trial rejected: backtrack (f0 = fpast, see begin_search)
            if (step < 1e-20 || step > 1e20) { *fail = 1; return true; }
            step *= 0.5;
            return false;
        }
        const double xnorm = sqrt(d5(x, x)), gnorm = sqrt(d5(g, g));
        if (gnorm <= 1e-6 * fmax(xnorm, 1.0)) return true;
        if (fabs(fpast - f) < 1e-16) return true;
        fpast = f;
        if (k_it >= 100) return true;
        double ys = 0, yy = 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const double si = x[i] - s[0][i], yi = g[i] - yv[0][i];
            s[0][i] = si; yv[0][i] = yi;
            ys += yi * si; yy += yi * yi;
        }
        ys = pair_sum(ys);
        yy = pair_sum(yy);
        rho[0] = AA_LBFGS_RHO ? 1.0 / ys : ys;
#pragma unroll
        for (int i = 0; i < H; ++i) drt[i] = -g[i];
        const int bound = k_it < M ? k_it : M;
        double alpha[M];
#pragma unroll
        for (int q = 0; q < M; ++q) {
            if (q < bound) {
                alpha[q] = AA_LBFGS_RHO ? d5(s[q], drt) * rho[q] : d5(s[q], drt) / rho[q];
#pragma unroll
                for (int t = 0; t < H; ++t) drt[t] -= alpha[q] * yv[q][t];
            }
        }
#pragma unroll
        for (int t = 0; t < H; ++t) drt[t] *= ys / yy;
#pragma unroll
        for (int q = M - 1; q >= 0; --q) {
            if (q < bound) {
                const double beta = AA_LBFGS_RHO ? d5(yv[q], drt) * rho[q] : d5(yv[q], drt) / rho[q];
#pragma unroll
                for (int t = 0; t < H; ++t) drt[t] += (alpha[q] - beta) * s[q][t];
            }
        }
        step = 1.0;
        ++k_it;
        begin_search(x);
        return false;
    }
};

// x: in = v (start point), out = prox. Returns iterations; sets *fail on a collapsed line search.
__device__ __forceinline__ int hyper_prox(int mat, double mu, double lambda, double k, double vol, const double* v,
                                          double* x, int* fail) {
    HyperLbfgs L;
    if (L.start(mat, mu, lambda, k, vol, v, x)) return 1;
    while (!L.iterate(mat, mu, lambda, k, vol, v, x, fail)) {}
    return L.k_it;
}

}  // namespace dev
}  // namespace aa
