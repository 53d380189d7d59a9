// Per-element proximal operators, device side (one element per thread, all in registers).
//
// Semantics follow the reference element plugins:
//   TriEnergyTerm::prox   (UX variant) admm_anderson_hard_zxu/src/TriEnergyTerm.cpp:74-105
//                          z = U clamp((1+S)/2) V^T
//   TriEnergyTerm::prox   (Z variant)  admm_anderson_xzu/src/TriEnergyTerm.cpp:77-108
//                          z = (U[I;0]V^T + F)/2 then per-column norm clamp
//   TetEnergyTerm::prox   admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:74-96
//                          z = (U diag(1,1,det F<1e-16 ? -1 : 1) V^T + F)/2
//   TetEnergyTerm::get_gradient (Z variant, admm_anderson_xzu/src/TetEnergyTerm.cpp:156-165)
//
// The reference uses Eigen::JacobiSVD. The 3x2 SVD here is the exact one-rotation one-sided
// Jacobi (the projection z = sum_i f(s_i) u_i v_i^T is invariant to the SVD's sign and order
// freedom, so only rounding differs); the 3x3 SVD is a register-resident two-sided Jacobi with
// Eigen's 2x2 step, stopping rule and descending sort, so that the det-flip picks the same
// singular pair. The 3x3 path is compiled without FMA contraction (Eigen's x86 build has none):
// for a (near-)singular F the null-space pair, hence U diag(1,1,-1) V^T, is decided by rounding,
// and only the same operation-by-operation rounding reproduces the reference's choice there.
#pragma once
#include <hip/hip_runtime.h>

#include "elastic_kernels.hpp"

namespace aa {
namespace dev {

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ------------------------------------------------------------------ triangles (3x2)
// z: column-major 3x2 (z[c*3+r]); mode 1 = UX (hard_zxu), 0 = Z (xzu)
__device__ __forceinline__ void tri_prox(const double* z, double* out, int mode, double lmin, double lmax) {
    const double* f0 = z;
    const double* f1 = z + 3;
    const double a = dot3(f0, f0), b = dot3(f1, f1), c = dot3(f0, f1);
    double cs = 1.0, sn = 0.0;
    if (c != 0.0) {
        const double zeta = (b - a) / (2.0 * c);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        cs = 1.0 / sqrt(1.0 + t * t);
        sn = cs * t;
    }
    double g0[3], g1[3];
    for (int r = 0; r < 3; ++r) { g0[r] = cs * f0[r] - sn * f1[r]; g1[r] = sn * f0[r] + cs * f1[r]; }
    double s0 = sqrt(dot3(g0, g0)), s1 = sqrt(dot3(g1, g1));
    double u0[3], u1[3];
    if (s0 > 0) { for (int r = 0; r < 3; ++r) u0[r] = g0[r] / s0; }
    else { u0[0] = 1; u0[1] = 0; u0[2] = 0; }
    if (s1 > 0) { for (int r = 0; r < 3; ++r) u1[r] = g1[r] / s1; }
    else {  // rank-deficient: any unit vector orthogonal to u0 (Eigen's choice is arbitrary too)
        double e[3] = {0, 0, 0};
        int k = fabs(u0[0]) <= fabs(u0[1]) ? (fabs(u0[0]) <= fabs(u0[2]) ? 0 : 2) : (fabs(u0[1]) <= fabs(u0[2]) ? 1 : 2);
        e[k] = 1;
        double d = dot3(e, u0);
        for (int r = 0; r < 3; ++r) u1[r] = e[r] - d * u0[r];
        double l = sqrt(dot3(u1, u1));
        for (int r = 0; r < 3; ++r) u1[r] /= l;
    }
    const double v0[2] = {cs, -sn}, v1[2] = {sn, cs};
    if (mode == 1) {
        double sg0 = (1.0 + s0) / 2.0, sg1 = (1.0 + s1) / 2.0;
        if (lmin > 0.0 || lmax < 99.0) {
            const double l0 = sg0, l1 = sg1;
            if (l0 < lmin) sg0 = lmin;
            if (l1 < lmin) sg1 = lmin;
            if (l0 > lmax) sg0 = lmax;
            if (l1 > lmax) sg1 = lmax;
        }
        for (int cc = 0; cc < 2; ++cc)
            for (int r = 0; r < 3; ++r) out[cc * 3 + r] = u0[r] * sg0 * v0[cc] + u1[r] * sg1 * v1[cc];
    } else {
        for (int cc = 0; cc < 2; ++cc)
            for (int r = 0; r < 3; ++r) out[cc * 3 + r] = 0.5 * ((u0[r] * v0[cc] + u1[r] * v1[cc]) + z[cc * 3 + r]);
        if (lmin > 0.0 || lmax < 99.0) {
            const double l0 = sqrt(dot3(out, out)), l1 = sqrt(dot3(out + 3, out + 3));
            if (l0 < lmin) for (int i = 0; i < 3; ++i) out[i] *= lmin / l0;
            if (l1 < lmin) for (int i = 3; i < 6; ++i) out[i] *= lmin / l1;
            if (l0 > lmax) for (int i = 0; i < 3; ++i) out[i] *= lmax / l0;
            if (l1 > lmax) for (int i = 3; i < 6; ++i) out[i] *= lmax / l1;
        }
    }
}

// ------------------------------------------------------------------ tets (3x3)
struct Rot2 { double c, s; };

__device__ __forceinline__ Rot2 jacobi_rot(double x, double y, double z) {  // J^T [[x y][y z]] J diagonal
#pragma clang fp contract(off)
    Rot2 r{1.0, 0.0};
    const double deno = 2.0 * fabs(y);
    if (deno < 2.2250738585072014e-308) return r;
    const double tau = (x - z) / deno;
    const double w = sqrt(tau * tau + 1.0);
    const double t = tau > 0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    const double sign_t = t > 0 ? 1.0 : -1.0;
    const double n = 1.0 / sqrt(t * t + 1.0);
    r.s = -sign_t * (y > 0 ? 1.0 : -1.0) * fabs(t) * n;
    r.c = n;
    return r;
}

// W, U, V row-major 3x3 in registers; one Eigen-style 2x2 step on pair (P,Q)
template <int P, int Q>
__device__ __forceinline__ bool jacobi_pair(double (&W)[9], double (&U)[9], double (&V)[9], double& maxDiag) {
#pragma clang fp contract(off)
    const double thr = fmax(2.2250738585072014e-308, 2.0 * 2.220446049250313e-16 * maxDiag);
    if (!(fabs(W[P * 3 + Q]) > thr || fabs(W[Q * 3 + P]) > thr)) return false;
    // real 2x2 Jacobi SVD of [[W_pp W_pq][W_qp W_qq]]
    const double m00 = W[P * 3 + P], m01 = W[P * 3 + Q], m10 = W[Q * 3 + P], m11 = W[Q * 3 + Q];
    Rot2 r1;
    const double t = m00 + m11, d = m10 - m01;
    if (fabs(d) < 2.2250738585072014e-308) { r1.s = 0; r1.c = 1; }
    else { const double u = t / d; const double tmp = sqrt(1.0 + u * u); r1.s = 1.0 / tmp; r1.c = u / tmp; }
    const double a00 = r1.c * m00 + r1.s * m10, a01 = r1.c * m01 + r1.s * m11, a11 = -r1.s * m01 + r1.c * m11;
    const Rot2 jr = jacobi_rot(a00, a01, a11);
    const Rot2 jl{r1.c * jr.c + r1.s * jr.s, r1.c * (-jr.s) + r1.s * jr.c};  // r1 * jr^T
    // W = jl applied on the left to rows P,Q
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = W[P * 3 + i], y = W[Q * 3 + i];
        W[P * 3 + i] = jl.c * x + jl.s * y;
        W[Q * 3 + i] = -jl.s * x + jl.c * y;
    }
    // U = U * jl^T  (columns P,Q): apply_rotation(col_p, col_q, (jl^T)^T = jl)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = U[i * 3 + P], y = U[i * 3 + Q];
        U[i * 3 + P] = jl.c * x + jl.s * y;
        U[i * 3 + Q] = -jl.s * x + jl.c * y;
    }
    // W = W * jr, V = V * jr  (columns): apply_rotation(col_p, col_q, jr^T)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double x = W[i * 3 + P], y = W[i * 3 + Q];
        W[i * 3 + P] = jr.c * x - jr.s * y;
        W[i * 3 + Q] = jr.s * x + jr.c * y;
        const double vx = V[i * 3 + P], vy = V[i * 3 + Q];
        V[i * 3 + P] = jr.c * vx - jr.s * vy;
        V[i * 3 + Q] = jr.s * vx + jr.c * vy;
    }
    maxDiag = fmax(maxDiag, fmax(fabs(W[P * 3 + P]), fabs(W[Q * 3 + Q])));
    return true;
}

// F row-major 3x3 -> U S V^T, S descending (Eigen JacobiSVD semantics, square case)
__device__ __forceinline__ void svd3(const double (&F)[9], double (&U)[9], double (&S)[3], double (&V)[9]) {
#pragma clang fp contract(off)
    double scale = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) scale = fmax(scale, fabs(F[i]));
    if (scale == 0) scale = 1;
    double W[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) { W[i] = F[i] / scale; U[i] = (i % 4 == 0) ? 1.0 : 0.0; V[i] = U[i]; }
    double maxDiag = fmax(fabs(W[0]), fmax(fabs(W[4]), fabs(W[8])));
    for (int sweep = 0; sweep < 32; ++sweep) {
        bool any = jacobi_pair<1, 0>(W, U, V, maxDiag);
        any |= jacobi_pair<2, 0>(W, U, V, maxDiag);
        any |= jacobi_pair<2, 1>(W, U, V, maxDiag);
        if (!any) break;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double a = W[i * 4];
        S[i] = fabs(a) * scale;
        if (a < 0) { U[0 * 3 + i] = -U[0 * 3 + i]; U[1 * 3 + i] = -U[1 * 3 + i]; U[2 * 3 + i] = -U[2 * 3 + i]; }
    }
    // selection sort, descending, first max wins (Eigen maxCoeff)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        int pos = i;
#pragma unroll
        for (int k = i + 1; k < 3; ++k) if (S[k] > S[pos]) pos = k;
        if (pos != i) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if (k == pos) {
                    double t = S[i]; S[i] = S[k]; S[k] = t;
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        double tu = U[r * 3 + i]; U[r * 3 + i] = U[r * 3 + k]; U[r * 3 + k] = tu;
                        double tv = V[r * 3 + i]; V[r * 3 + i] = V[r * 3 + k]; V[r * 3 + k] = tv;
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ double det3rm(const double (&F)[9]) {
#pragma clang fp contract(off)
    return F[0] * (F[4] * F[8] - F[5] * F[7]) - F[1] * (F[3] * F[8] - F[5] * F[6]) + F[2] * (F[3] * F[7] - F[4] * F[6]);
}

// z column-major 9 -> out column-major 9
__device__ __forceinline__ void tet_linear_prox(const double* z, double* out) {
#pragma clang fp contract(off)
    double F[9], U[9], S[3], V[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) F[r * 3 + c] = z[c * 3 + r];
    svd3(F, U, S, V);
    const double s2 = det3rm(F) < 1e-16 ? -1.0 : 1.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double p = U[r * 3 + 0] * V[c * 3 + 0] + U[r * 3 + 1] * V[c * 3 + 1] + U[r * 3 + 2] * s2 * V[c * 3 + 2];
            out[c * 3 + r] = 0.5 * (p + z[c * 3 + r]);
        }
}

// k*vol*(F - U V^T)   (Z variant get_gradient of the linear tet)
__device__ __forceinline__ void tet_linear_grad(const double* z, double kvol, double* g) {
#pragma clang fp contract(off)
    double F[9], U[9], S[3], V[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) F[r * 3 + c] = z[c * 3 + r];
    svd3(F, U, S, V);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double p = U[r * 3 + 0] * V[c * 3 + 0] + U[r * 3 + 1] * V[c * 3 + 1] + U[r * 3 + 2] * V[c * 3 + 2];
            g[c * 3 + r] = kvol * (F[r * 3 + c] - p);
        }
}

// (1/w) * ((w x + u) - c) of an identity-reduction row, without FMA contraction (c = -w x_pin for
// a pinned node, whose x enters through c: the same sum)
__device__ inline void collision_candidate(const double* x, const double* u, double w, double* q) {
#pragma clang fp contract(off)
    const double iw = 1.0 / w;
    for (int i = 0; i < 3; ++i) q[i] = iw * (w * x[i] + u[i]);
}

// Collision::prox (admm_anderson_hard_zxu/src/CollisionEnergyTerm.hpp:79-91): the candidate q is
// tested against every passive obstacle in insertion order; an obstacle replaces the running
// (dx, point) when its signed distance is <= the current one (PassiveObject.hpp's `if (dx >
// p.dx) return;`), and q moves to the closest surface point when the final dx < 0. The
// signed-distance functions restate PassiveObject.hpp:32-136 with the reference's operation
// order (no FMA contraction, Eigen's norm / normalize: division by sqrt of the squared norm).
// Obstacle table: obs[0] = count, then kObsStride doubles each: type, parameters.
__device__ inline void collision_prox(const double* q, const double* obs, double* out) {
#pragma clang fp contract(off)
    double best = 1.79769313486231570815e+308;   // std::numeric_limits<double>::max()
    double pt[3] = {0.0, 0.0, 0.0};
    const int n = obs ? (int)obs[0] : 0;
    auto sq3 = [](double a, double b, double c) { return (a * a + b * b) + c * c; };   // squaredNorm
    for (int k = 0; k < n; ++k) {
        const double* o = obs + 1 + k * kObsStride;
        const int type = (int)o[0];
        double dx, p0, p1, p2;
        if (type == OBS_FLOOR) {                      // Floor(y)                   :32-45
            dx = q[1] - o[1];
            p0 = q[0]; p1 = o[1]; p2 = q[2];
        } else if (type == OBS_SLIDE_FLOOR) {         // SlideFloor(center, normal) :47-62
            const double l0 = q[0] - o[1], l1 = q[1] - o[2], l2 = q[2] - o[3];
            dx = l0 * o[4] + l1 * o[5] + l2 * o[6];
            p0 = q[0] - dx * o[4]; p1 = q[1] - dx * o[5]; p2 = q[2] - dx * o[6];
        } else if (type == OBS_SPHERE) {              // Sphere(center, rad)        :64-80
            double d0 = q[0] - o[1], d1 = q[1] - o[2], d2 = q[2] - o[3];
            const double z2 = sq3(d0, d1, d2), nrm = sqrt(z2);
            dx = nrm - o[4];
            if (dx > best) continue;
            if (z2 > 0.0) { d0 /= nrm; d1 /= nrm; d2 /= nrm; }
            p0 = o[1] + d0 * o[4]; p1 = o[2] + d1 * o[4]; p2 = o[3] + d2 * o[4];
        } else if (type == OBS_PLANE_HALF_SPHERE) {   // PlaneAndHalfSphere         :82-116
            const double dc = sqrt(sq3(q[0] - o[1], 0.0, q[2] - o[3])) - o[4];
            if (dc > 0) {
                dx = q[1] - o[2];
                p0 = q[0]; p1 = o[2]; p2 = q[2];
            } else {
                const double dpl = q[1] - o[2];
                double d0 = q[0] - o[1], d1 = q[1] - o[2], d2 = q[2] - o[3];
                const double z2 = sq3(d0, d1, d2), nrm = sqrt(z2);
                dx = dpl > 0 ? nrm + o[4] : o[4] - nrm;
                if (dx > best) continue;
                if (z2 > 0.0) { d0 /= nrm; d1 /= nrm; d2 /= nrm; }
                p0 = o[1] + d0 * o[4]; p1 = o[2] + d1 * o[4]; p2 = o[3] + d2 * o[4];
            }
        } else {                                      // Cylinder(center, rad), axis z :118-136
            double d0 = q[0] - o[1], d1 = q[1] - o[2], d2 = 0.0 - o[3];
            const double z2 = sq3(d0, d1, d2), nrm = sqrt(z2);
            dx = nrm - o[4];
            if (dx > best) continue;
            if (z2 > 0.0) { d0 /= nrm; d1 /= nrm; d2 /= nrm; }
            p0 = o[1] + d0 * o[4] + 0.0; p1 = o[2] + d1 * o[4] + 0.0; p2 = o[3] + d2 * o[4] + q[2];
        }
        if (dx > best) continue;
        best = dx;
        pt[0] = p0; pt[1] = p1; pt[2] = p2;
    }
    if (best < 0) { out[0] = pt[0]; out[1] = pt[1]; out[2] = pt[2]; }
    else { out[0] = q[0]; out[1] = q[1]; out[2] = q[2]; }
}

}  // namespace dev
}  // namespace aa
