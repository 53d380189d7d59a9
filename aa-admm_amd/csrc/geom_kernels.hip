// HIP kernels of the Geometry (ALM) hot path (gfx950, wave64, fp64).
//
// One thread per constraint: the K point positions are gathered (24 B each, the point array
// stays L2/MALL resident), transformed (mean-centring / subtract-first / identity), projected
// in registers, and the thread writes its z columns (SoA, coalesced) and its K rows of the
// global right-hand side (slot rows, gathered per point by a fixed-order CSR pass: no atomics,
// deterministic). Projections (Geometry/Constraint.h):
//   plane  -- best-fit plane through the (mean-centred) columns: one-sided Jacobi on the three
//             coordinate rows (relative accuracy, same left singular vectors as the reference's
//             Eigen JacobiSVD), normal = the row rotation of the smallest row norm;
//   angle  -- the closed-form rotation of Constraint.h:243-291;
//   edge   -- v |v|^-1 L;   closeness -- identity (Constraint.h:319-322 never overrides);
//   closest point on a reference surface -- stackless traversal of a depth-first BVH with exact
//             box pruning, warm-started from the previous iteration's triangle.
#include <cstdlib>

#include "common.hpp"
#include "geom_kernels.hpp"

namespace aa {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

__device__ __forceinline__ double block_sum(double v, double* sm) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sm[wid] = v;
    __syncthreads();
    double r = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += sm[i];
    __syncthreads();
    return r;
}

__device__ __forceinline__ bool gated(const Ctrl* c) { return c && c->done; }

// a thread's share of nb partials in index order, loads issued 8 at a time (as in elastic_kernels)
__device__ __forceinline__ double thread_sum_strided(const double* red, int nb) {
    double a = 0;
    int i = threadIdx.x;
    const int st = blockDim.x;
    for (; i + 7 * st < nb; i += 8 * st) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = red[i + q * st];
#pragma unroll
        for (int q = 0; q < 8; ++q) a += v[q];
    }
    for (; i < nb; i += st) a += red[i];
    return a;
}

// ------------------------------------------------------------------ transforms (Constraint.h:73-94)
// out: 3*cols values, column-major (column c at out[3c..3c+2])
template <int T, int K>
__device__ __forceinline__ void transform(const GeoGroupDev& g, int e, const double* __restrict__ x, double* out) {
    double p[3 * K];
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const int v = g.idx[(size_t)a * g.count + e];
        p[3 * a] = x[3 * (size_t)v]; p[3 * a + 1] = x[3 * (size_t)v + 1]; p[3 * a + 2] = x[3 * (size_t)v + 2];
    }
    if constexpr (T == GEO_ANGLE || T == GEO_EDGE) {          // SUBTRACT_FIRST
#pragma unroll
        for (int a = 1; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) out[3 * (a - 1) + d] = p[3 * a + d] - p[d];
    } else if constexpr (T == GEO_PLANE) {                     // MEAN_CENTERING
        double m[3] = {0, 0, 0};
#pragma unroll
        for (int a = 0; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) m[d] += p[3 * a + d];
#pragma unroll
        for (int d = 0; d < 3; ++d) m[d] /= K;
#pragma unroll
        for (int a = 0; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) out[3 * a + d] = p[3 * a + d] - m[d];
    } else {                                                   // IDENTITY
#pragma unroll
        for (int i = 0; i < 3 * K; ++i) out[i] = p[i];
    }
}

// rhs slot rows: y_a = s * (T^T q)_a
template <int T, int K>
__device__ __forceinline__ void write_slots(const GeoGroupDev& g, int e, const double* q, double s, double* __restrict__ y) {
    double* yr = y + 3 * (size_t)(g.slot0 + (long long)e * K);
    if constexpr (T == GEO_ANGLE || T == GEO_EDGE) {
        double f[3] = {0, 0, 0};
#pragma unroll
        for (int a = 1; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) { f[d] -= q[3 * (a - 1) + d]; yr[3 * a + d] = s * q[3 * (a - 1) + d]; }
#pragma unroll
        for (int d = 0; d < 3; ++d) yr[d] = s * f[d];
    } else if constexpr (T == GEO_PLANE) {
        double m[3] = {0, 0, 0};
#pragma unroll
        for (int a = 0; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) m[d] += q[3 * a + d];
#pragma unroll
        for (int d = 0; d < 3; ++d) m[d] /= K;
#pragma unroll
        for (int a = 0; a < K; ++a)
#pragma unroll
            for (int d = 0; d < 3; ++d) yr[3 * a + d] = s * (q[3 * a + d] - m[d]);
    } else {
#pragma unroll
        for (int i = 0; i < 3 * K; ++i) yr[i] = s * q[i];
    }
}

// ------------------------------------------------------------------ projections
// best-fit plane normal of the columns of P (3 x K): one-sided Jacobi over the coordinate rows
template <int K>
__device__ void plane_project(double* v) {
    double R[3][K], W[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int a = 0; a < K; ++a) R[d][a] = v[3 * a + d];
    for (int sweep = 0; sweep < 30; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int pr = 0; pr < 3; ++pr) {
            const int p = pr == 2 ? 1 : 0, q = pr == 0 ? 1 : 2;
            double a = 0, b = 0, gg = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) { a += R[p][k] * R[p][k]; b += R[q][k] * R[q][k]; gg += R[p][k] * R[q][k]; }
            if (fabs(gg) > 1e-15 * sqrt(a * b) && gg != 0.0) {
                rotated = true;
                const double zeta = (b - a) / (2.0 * gg);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const double rp = R[p][k], rq = R[q][k];
                    R[p][k] = c * rp - s * rq;
                    R[q][k] = s * rp + c * rq;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double wp = W[p][k], wq = W[q][k];
                    W[p][k] = c * wp - s * wq;
                    W[q][k] = s * wp + c * wq;
                }
            }
        }
        if (!rotated) break;
    }
    double nr[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        double s = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) s += R[d][k] * R[d][k];
        nr[d] = s;
    }
    int i = 0;
    if (nr[1] < nr[i]) i = 1;
    if (nr[2] < nr[i]) i = 2;
    double n0 = W[i][0], n1 = W[i][1], n2 = W[i][2];
    const double l = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
    if (l > 0) { n0 /= l; n1 /= l; n2 /= l; }
#pragma unroll
    for (int a = 0; a < K; ++a) {
        const double dp = n0 * v[3 * a] + n1 * v[3 * a + 1] + n2 * v[3 * a + 2];
        v[3 * a] -= n0 * dp; v[3 * a + 1] -= n1 * dp; v[3 * a + 2] -= n2 * dp;
    }
}

// AngleConstraint::project_impl (Constraint.h:243-291), v = (v1, v2) in place
__device__ void angle_project(double* v, double min_r, double max_r) {
    const double min_a = fmax(0.0, min_r), max_a = fmin(M_PI, max_r);
    const double min_cos = fmin(fmax(cos(min_a), -1.0), 1.0), max_cos = fmin(fmax(cos(max_a), -1.0), 1.0);
    const double v1s = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double v2s = v[3] * v[3] + v[4] * v[4] + v[5] * v[5];
    const double v1n = sqrt(v1s), v2n = sqrt(v2s);
    double u1[3] = {v[0], v[1], v[2]}, u2[3] = {v[3], v[4], v[5]};
    if (v1s > 0) { const double r = 1.0 / sqrt(v1s); u1[0] *= r; u1[1] *= r; u1[2] *= r; }
    if (v2s > 0) { const double r = 1.0 / sqrt(v2s); u2[0] *= r; u2[1] *= r; u2[2] *= r; }
    const double cg = fmin(fmax(u1[0] * u2[0] + u1[1] * u2[1] + u1[2] * u2[2], -1.0), 1.0);
    if (!((1.0 - fabs(cg) > 1e-14) && (cg > min_cos || cg < max_cos))) return;
    const double gamma = acos(cg);
    double eta = cg > min_cos ? (min_a - gamma) : (gamma - max_a);
    eta = fmax(eta, 0.0);
    double theta = 0.5 * atan2(v2s * sin(2 * eta), v1s + v2s * cos(2 * eta));
    theta = fmax(0.0, fmin(eta, theta));
    const double phi = eta - theta;
    double w3[3], w4[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) { w3[d] = u2[d] - u1[d] * cg; w4[d] = u1[d] - u2[d] * cg; }
    const double l3 = w3[0] * w3[0] + w3[1] * w3[1] + w3[2] * w3[2];
    const double l4 = w4[0] * w4[0] + w4[1] * w4[1] + w4[2] * w4[2];
    const double s3 = (l3 > 0 ? 1.0 / sqrt(l3) : 1.0) * (cg > min_cos ? -1.0 : 1.0);
    const double s4 = (l4 > 0 ? 1.0 / sqrt(l4) : 1.0) * (cg > min_cos ? -1.0 : 1.0);
    const double ct = cos(theta), st = sin(theta), cp = cos(phi), sp = sin(phi);
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        v[d] = (u1[d] * ct + w3[d] * s3 * st) * (v1n * ct);
        v[3 + d] = (u2[d] * cp + w4[d] * s4 * sp) * (v2n * cp);
    }
}

// Ericson closest point on a triangle (igl point_simplex_squared_distance.cpp:40-108). Every
// product-sum is an explicit fma and contraction is off, so the bits do not depend on how the
// compiler fuses the inlined code at each call site (the one-lane and the group traversal must
// agree bit for bit).
__device__ __forceinline__ double dot3(double ax, double ay, double az, double bx, double by, double bz) {
#pragma clang fp contract(off)
    return fma(ax, bx, fma(ay, by, az * bz));
}
__device__ __forceinline__ double dist2(double px, double py, double pz, double qx, double qy, double qz) {
#pragma clang fp contract(off)
    const double dx = px - qx, dy = py - qy, dz = pz - qz;
    return fma(dx, dx, fma(dy, dy, dz * dz));
}
__device__ __forceinline__ void closest_on_tri(const double* t, double px, double py, double pz, double& cx,
                                               double& cy, double& cz) {
#pragma clang fp contract(off)
    const double ax = t[0], ay = t[1], az = t[2], bx = t[3], by = t[4], bz = t[5], qx = t[6], qy = t[7], qz = t[8];
    const double abx = bx - ax, aby = by - ay, abz = bz - az, acx = qx - ax, acy = qy - ay, acz = qz - az;
    const double apx = px - ax, apy = py - ay, apz = pz - az;
    const double d1 = dot3(abx, aby, abz, apx, apy, apz), d2 = dot3(acx, acy, acz, apx, apy, apz);
    if (d1 <= 0.0 && d2 <= 0.0) { cx = ax; cy = ay; cz = az; return; }
    const double bpx = px - bx, bpy = py - by, bpz = pz - bz;
    const double d3 = dot3(abx, aby, abz, bpx, bpy, bpz), d4 = dot3(acx, acy, acz, bpx, bpy, bpz);
    if (d3 >= 0.0 && d4 <= d3) { cx = bx; cy = by; cz = bz; return; }
    const double vc = fma(d1, d4, -(d3 * d2));
    if (!(ax == bx && ay == by && az == bz) && vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) {
        const double v = d1 / (d1 - d3);
        cx = fma(v, abx, ax); cy = fma(v, aby, ay); cz = fma(v, abz, az); return;
    }
    const double cpx = px - qx, cpy = py - qy, cpz = pz - qz;
    const double d5 = dot3(abx, aby, abz, cpx, cpy, cpz), d6 = dot3(acx, acy, acz, cpx, cpy, cpz);
    if (d6 >= 0.0 && d5 <= d6) { cx = qx; cy = qy; cz = qz; return; }
    const double vb = fma(d5, d2, -(d1 * d6));
    if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) {
        const double w = d2 / (d2 - d6);
        cx = fma(w, acx, ax); cy = fma(w, acy, ay); cz = fma(w, acz, az); return;
    }
    const double va = fma(d3, d6, -(d5 * d4));
    if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
        const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        cx = fma(w, qx - bx, bx); cy = fma(w, qy - by, by); cz = fma(w, qz - bz, bz); return;
    }
    const double denom = 1.0 / (va + vb + vc);
    const double v = vb * denom, w = vc * denom;
    cx = fma(acx, w, fma(abx, v, ax)); cy = fma(acy, w, fma(aby, v, ay)); cz = fma(acz, w, fma(abz, v, az));
}

// Branch-free: max(lo - v, v - hi, 0) is the distance outside [lo, hi] bit for bit (one of the two
// differences is positive at most, and it is the one the comparisons would pick). The ternary
// form compiled to branches with each field's load sunk into its branch -- a load and a wait per
// field, serialised -- which made the greedy descent (a third of C5's queries) a long chain.
__device__ __forceinline__ double box_d2(const BvhNode& nd, double px, double py, double pz) {
    const double l0 = nd.lo[0], l1 = nd.lo[1], l2 = nd.lo[2], h0 = nd.hi[0], h1 = nd.hi[1], h2 = nd.hi[2];
    const double tx = fmax(fmax(l0 - px, px - h0), 0.0);
    const double ty = fmax(fmax(l1 - py, py - h1), 0.0);
    const double tz = fmax(fmax(l2 - pz, pz - h2), 0.0);
#ifdef AA_CP_NO_AABB
    const double b = 0.0 * (tx + ty + tz);
#else
    const double b = tx * tx + ty * ty + tz * tz;
#endif
    // oriented-box lower bound: the distances of (n.p, t1.p, t2.p) outside the node's ranges
    // (the axes are orthonormal to fp32 accuracy: shrunk by 4e-6 to stay below)
    auto outside = [](double v, float lo, float hi) { return fmax(fmax((double)lo - v, v - (double)hi), 0.0); };
    const double t = outside((double)nd.nrm[0] * px + (double)nd.nrm[1] * py + (double)nd.nrm[2] * pz, nd.dlo, nd.dhi);
    const double u1 = outside((double)nd.t1[0] * px + (double)nd.t1[1] * py + (double)nd.t1[2] * pz, nd.t1lo, nd.t1hi);
    const double u2 = outside((double)nd.t2[0] * px + (double)nd.t2[1] * py + (double)nd.t2[2] * pz, nd.t2lo, nd.t2hi);
    const double sl = (t * t + u1 * u1 + u2 * u2) * (1.0 - 4e-6);
    return b > sl ? b : sl;
}

// The same lower bound in fp32 arithmetic for the traversal's prune tests (AA_CP_F32=1, the
// default): the query is rounded to fp32 once, and every per-axis distance is shrunk by
// eps = 8 u (|qx| + |qy| + |qz|) (u = 2^-24), which covers the rounding of the query and of the
// fp32 dot products (|n_i| <= 1), so the bound stays below the true distance -- it only prunes
// less. No conversions per node, half the registers per operand. The greedy descent keeps the
// fp64 bound: its left / right choice picks the seed triangle, which decides ties. Single-lane
// traversal only (C5 z 1 366 -> 1 195 us); the group traversal measured slower with it (C3).
#ifndef AA_CP_F32
#define AA_CP_F32 1
#endif
struct QueryF { float x, y, z, eps; };
__device__ __forceinline__ QueryF query_f(double px, double py, double pz) {
    QueryF q;
    q.x = (float)px; q.y = (float)py; q.z = (float)pz;
    q.eps = 8.0f * 5.9604645e-8f * 1.0001f * (fabsf(q.x) + fabsf(q.y) + fabsf(q.z));
    return q;
}
__device__ __forceinline__ double box_d2f(const BvhNode& nd, const QueryF& q) {
    auto outside = [&](float v, float lo, float hi) { return fmaxf(fmaxf(fmaxf(lo - v, v - hi), 0.0f) - q.eps, 0.0f); };
    const float tx = outside(q.x, nd.lo[0], nd.hi[0]), ty = outside(q.y, nd.lo[1], nd.hi[1]),
                tz = outside(q.z, nd.lo[2], nd.hi[2]);
    const float t = outside(nd.nrm[0] * q.x + nd.nrm[1] * q.y + nd.nrm[2] * q.z, nd.dlo, nd.dhi);
    const float u1 = outside(nd.t1[0] * q.x + nd.t1[1] * q.y + nd.t1[2] * q.z, nd.t1lo, nd.t1hi);
    const float u2 = outside(nd.t2[0] * q.x + nd.t2[1] * q.y + nd.t2[2] * q.z, nd.t2lo, nd.t2hi);
    const float b = tx * tx + ty * ty + tz * tz, sl = t * t + u1 * u1 + u2 * u2;
    return (double)fmaxf(b, sl) * (1.0 - 4e-6);   // fp32 squares and sums: a few ulp
}
#if AA_CP_F32
#define CP_PRUNE_BOUND(nd) box_d2f((nd), Q)
#else
#define CP_PRUNE_BOUND(nd) box_d2((nd), px, py, pz)
#endif

// (warm distance / warm triangle's first edge)^2 up to which the warm bound is used alone: the
// greedy root-to-leaf descent (a chain of dependent node loads) only runs for points that slid
// farther than ~8 edges from their previous triangle (and on cold starts). Measured (round 2):
// always descending C3 995 / C5 157 it/s, never 1 056 / 154, 64 -> 1 056 / 158; 4 and 16 in between.
#ifndef AA_WARM_TIGHT
#define AA_WARM_TIGHT 64.0
#endif
// share of a wave's live lanes that must hold a leaf before the wave tests leaf triangles
// (0 = one loop: test as soon as any lane reaches a leaf); see bvh_closest
#ifndef AA_BVH_HOLD_PCT
#define AA_BVH_HOLD_PCT 50
#endif

#ifdef AA_CP_STATS
// diagnostics build only (-DAA_CP_STATS): per-query traversal counts of bvh_closest
__device__ unsigned long long g_cp_stats[64];
#define CP_STAT(i, v) atomicAdd(&g_cp_stats[(i)], (unsigned long long)(v))
#endif
// exact closest point on the surface. Stackless depth-first traversal over escape links
// (`skip` = the node after a subtree): no per-lane stack, so no scratch memory. The upper
// bound comes from `warm` (the previous iteration's triangle: points move little between ALM
// iterations) or, on a cold start, from a greedy descent to the nearest-box leaf; boxes that
// cannot beat it are skipped whole. Strictly smaller distances replace the best, so the result
// is the exact minimum (ties resolved toward the warm / first-found triangle).
__device__ int bvh_closest(const SurfDev& S, double px, double py, double pz, int warm, double& cx, double& cy,
                           double& cz) {
    double best = INFINITY;
    int best_t = -1;
    cx = px; cy = py; cz = pz;
    if (S.n_nodes == 0) return -1;
#ifdef AA_CP_STATS
    unsigned nbox = 0, ntri = 0;
    double e2s = 0;
#define CP_BOX() (++nbox)
#define CP_TRI() (++ntri)
#else
#define CP_BOX() ((void)0)
#define CP_TRI() ((void)0)
#endif
    auto test_tri = [&](int t) {
        CP_TRI();
        double qx, qy, qz;
        closest_on_tri(S.tris[t].v, px, py, pz, qx, qy, qz);
        const double d2 = dist2(px, py, pz, qx, qy, qz);
        if (d2 < best) { best = d2; best_t = t; cx = qx; cy = qy; cz = qz; }
    };
    bool tight = false;
    if (warm >= 0 && warm < S.n_tris) {
        test_tri(warm);
        const double* v = S.tris[warm].v;
        const double e2 = (v[3] - v[0]) * (v[3] - v[0]) + (v[4] - v[1]) * (v[4] - v[1]) + (v[5] - v[2]) * (v[5] - v[2]);
        tight = best <= AA_WARM_TIGHT * e2;
#ifdef AA_CP_STATS
        e2s = e2;
#endif
    }
    if (!tight)
    {   // greedy descent to the nearest-box leaf: a tight bound even when the point slid far
        // from its previous triangle (the warm bound alone then lets the traversal open every
        // box within that distance)
        // the chosen child's record comes with the pair just loaded: one dependent load per level
        int i = 0;
        BvhNode nd = S.nodes[0];
        for (;;) {
            if (bvh_count(nd) > 0) {
                for (int t = nd.a; t < nd.a + bvh_count(nd); ++t) test_tri(t);
                break;
            }
            const BvhNode cl = S.nodes[i + 1], cr = S.nodes[nd.a];   // both children's loads issued together
            const double dl = box_d2(cl, px, py, pz), dr = box_d2(cr, px, py, pz);
            CP_BOX(); CP_BOX();
            if (dl <= dr) { i = i + 1; nd = cl; } else { i = nd.a; nd = cr; }
        }
    }
    const int seed = best_t;
    [[maybe_unused]] const QueryF Q = query_f(px, py, pz);
    int i = 0;
#if AA_BVH_HOLD_PCT > 0
    // Two-phase ("while-while") schedule of the same per-lane traversal: a lane that reaches a
    // leaf whose box passes parks on it while the other lanes keep walking inner nodes; the
    // wave tests leaf triangles only once at least AA_BVH_HOLD_PCT % of its live lanes hold a
    // leaf (or none walks any more). Each lane visits the same nodes and tests the same
    // triangles in the same order as the one-loop form below -- only the interleaving across
    // the wave changes -- so the result is bit-identical. What changes is the SIMD use of the
    // triangle tests: in one loop, every step where any lane sits on a leaf runs the whole
    // (divergent) triangle body for the wave.
    int hold_a = -1, hold_n = 0;
    bool done = S.n_nodes <= 0;
    for (;;) {
        for (;;) {
            if (!done && hold_a < 0) {
                const BvhNode nd = S.nodes[i];
                CP_BOX();
                if (CP_PRUNE_BOUND(nd) < best) {
                    const int nc = bvh_count(nd);
                    if (nc > 0) { hold_a = nd.a; hold_n = nc; i = bvh_skip(nd); }
                    else i = i + 1;
                } else {
                    i = bvh_skip(nd);
                }
                if (hold_a < 0 && i >= S.n_nodes) done = true;
            }
            const unsigned long long live = __ballot(!done), held = __ballot(hold_a >= 0);
            const int nl = __popcll(live), nh = __popcll(held);
            if (nh == nl || (nh > 0 && 100 * nh >= AA_BVH_HOLD_PCT * nl)) break;
        }
        if (__ballot(!done) == 0ull) break;
        if (hold_a >= 0) {
            for (int t = hold_a; t < hold_a + hold_n; ++t)
                if (t != seed) test_tri(t);
            hold_a = -1;
            if (i >= S.n_nodes) done = true;
        }
    }
#else
    while (i < S.n_nodes) {
        const BvhNode nd = S.nodes[i];
        CP_BOX();
        if (CP_PRUNE_BOUND(nd) < best) {
            const int nc = bvh_count(nd);
            if (nc > 0) {
                for (int t = nd.a; t < nd.a + nc; ++t)
                    if (t != seed) test_tri(t);
                i = bvh_skip(nd);
            } else {
                i = i + 1;
            }
        } else {
            i = bvh_skip(nd);
        }
    }
#endif
#ifdef AA_CP_STATS
    {
        auto lg = [](double v) { int b = 0; while (v >= 2.0 && b < 15) { v *= 0.5; ++b; } return b; };
        CP_STAT(0, 1); CP_STAT(1, nbox); CP_STAT(2, ntri); CP_STAT(3, tight ? 1 : 0); CP_STAT(4, best_t != warm ? 1 : 0);
        CP_STAT(8 + lg((double)nbox), 1);
        // distance / warm edge length, log2 buckets from 2^-12
        if (e2s > 0) { double r = sqrt(best / e2s) * 4096.0; CP_STAT(24 + lg(r), 1); }
        // oracle: the same walk started with the final distance as the bound (what a perfect
        // seed would leave to test)
        unsigned ob = 0, ot = 0;
        for (int k = 0; k < S.n_nodes;) {
            const BvhNode nd = S.nodes[k];
            ++ob;
            if (CP_PRUNE_BOUND(nd) < best) {
                const int nc = bvh_count(nd);
                if (nc > 0) { ot += nc; k = bvh_skip(nd); } else k = k + 1;
            } else {
                k = bvh_skip(nd);
            }
        }
        CP_STAT(40, ob); CP_STAT(41, ot);
    }
#endif
#undef CP_BOX
#undef CP_TRI
    return best_t;
}

// The same query run by a group of G lanes (G = 4 or 8, aligned within the wave) over the
// collapsed tree S.wide: each step the G lanes load and test the G children of one node at once
// (one dependent load per log2(G) levels of the binary tree), a leaf's <= 4 triangles are tested
// one per lane, and the children that pass are visited nearest first through a per-query stack
// in LDS (stk_i / stk_d, kCpStack entries; the host checks (G - 1) x depth fits). A query then
// costs about 1 / log2(G) of the dependent node loads of bvh_closest and G lanes' worth of
// occupancy, which is what a latency-bound traversal with few queries per SIMD lacks.
// Same result as bvh_closest: the seed / descent part is bvh_closest's own (every lane alike),
// giving t0; bvh_closest then keeps t0 if no triangle is strictly closer, else the first
// triangle in its depth-first order -- the smallest leaf-order index -- among the closest ones.
// Here the visit order differs, so a tie is broken explicitly by that rule (t0 first, then the
// smaller index), and a box whose bound EQUALS the best distance is still opened.
template <int G>
__device__ int bvh_closest_grp(const SurfDev& S, double px, double py, double pz, int warm, int* __restrict__ stk_i,
                               float* __restrict__ stk_d, double& cx, double& cy, double& cz) {
    const int lane = threadIdx.x & 63, base = lane & ~(G - 1), j = lane - base;
    const unsigned long long gm = ((1ull << G) - 1ull) << base;
    double best = INFINITY;
    int best_t = -1;
    cx = px; cy = py; cz = pz;
    if (S.n_nodes == 0) return -1;
    auto test_tri = [&](int t) {
        double qx, qy, qz;
        closest_on_tri(S.tris[t].v, px, py, pz, qx, qy, qz);
        const double d2 = dist2(px, py, pz, qx, qy, qz);
        if (d2 < best) { best = d2; best_t = t; cx = qx; cy = qy; cz = qz; }
    };
    bool tight = false;
    if (warm >= 0 && warm < S.n_tris) {
        test_tri(warm);
        const double* v = S.tris[warm].v;
        const double e2 = (v[3] - v[0]) * (v[3] - v[0]) + (v[4] - v[1]) * (v[4] - v[1]) + (v[5] - v[2]) * (v[5] - v[2]);
        tight = best <= AA_WARM_TIGHT * e2;
    }
    if (!tight) {
        int i = 0;
        BvhNode nd = S.nodes[0];
        for (;;) {
            if (bvh_count(nd) > 0) {
                for (int t = nd.a; t < nd.a + bvh_count(nd); ++t) test_tri(t);
                break;
            }
            const BvhNode cl = S.nodes[i + 1], cr = S.nodes[nd.a];   // both children's loads issued together
            const double dl = box_d2(cl, px, py, pz), dr = box_d2(cr, px, py, pz);
            if (dl <= dr) { i = i + 1; nd = cl; } else { i = nd.a; nd = cr; }
        }
    }
    const int t0 = best_t;
    int cur = 0, sp = 0;
    for (;;) {
        const BvhNode rec = S.wide[(size_t)cur * G + j];
        const bool valid = rec.a >= 0;
        const int cnt = bvh_count(rec);
        const double d = valid ? box_d2(rec, px, py, pz) : INFINITY;   // fp64 here: measured faster (C3)
        // leaf children: one after the other, a triangle per lane, group arg-min by (distance, index)
        for (unsigned long long lm = __ballot(valid && cnt > 0 && d <= best) & gm; lm; lm &= lm - 1) {
            const int src = __ffsll((long long)lm) - 1;
            if (!(__shfl(d, src) <= best)) continue;   // group-uniform
            const int ak = __shfl(rec.a, src), nk = __shfl(cnt, src);
            double qd = INFINITY, qx = 0, qy = 0, qz = 0;
            int qt = 0x7fffffff;
            for (int k = j; k < nk; k += G) {   // ascending index: strict < keeps the first
                double rx, ry, rz;
                closest_on_tri(S.tris[ak + k].v, px, py, pz, rx, ry, rz);
                const double rd = dist2(px, py, pz, rx, ry, rz);
                if (rd < qd) { qd = rd; qt = ak + k; qx = rx; qy = ry; qz = rz; }
            }
#pragma unroll
            for (int off = G / 2; off > 0; off >>= 1) {
                const double od = __shfl_xor(qd, off, G), ox = __shfl_xor(qx, off, G), oy = __shfl_xor(qy, off, G),
                             oz = __shfl_xor(qz, off, G);
                const int ot = __shfl_xor(qt, off, G);
                if (od < qd || (od == qd && ot < qt)) { qd = od; qt = ot; qx = ox; qy = oy; qz = oz; }
            }
            if (qd < best || (qd == best && best_t != t0 && qt < best_t)) {
                best = qd; best_t = qt; cx = qx; cy = qy; cz = qz;
            }
        }
        // inner children: descend into the nearest, push the others (farthest deepest)
        const bool inner = valid && cnt == 0 && d <= best;
        const unsigned long long im = __ballot(inner) & gm;
        const int ni = __popcll(im);
        if (ni == 0) {
            bool next = false;
            while (sp > 0) {
                --sp;
                if ((double)stk_d[sp] <= best) { cur = stk_i[sp]; next = true; break; }
            }
            if (!next) break;
            continue;
        }
        int rank = 0;   // position in descending distance (ties: lower lane first)
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const double dk = __shfl(d, base + k);
            if (((im >> (base + k)) & 1ull) && (dk > d || (dk == d && k < j))) ++rank;
        }
        if (inner && rank < ni - 1) {
            float f = (float)d;   // rounded down: the pop test never drops a box it should open
            if ((double)f > d) f = nextafterf(f, -INFINITY);
            stk_i[sp + rank] = rec.a;
            stk_d[sp + rank] = f;
        }
        const unsigned long long nm = __ballot(inner && rank == ni - 1) & gm;
        cur = __shfl(rec.a, __ffsll((long long)nm) - 1);
        sp += ni - 1;
    }
    return best_t;
}

// ------------------------------------------------------------------ z step
// One constraint: v = T(x) (+u), z = P(v); PLAIN (GeometrySolver<3>): soft groups combine
// z = a v + (1 - a) P(v) (Constraint::project_and_combine, Constraint.h:118-130) and the
// return value is this constraint's |T(x) - z|^2 (GeometrySolver::get_ADMM_residual,
// GeometrySolver.h:459-461); ALM: returns 0.
// G > 1: the element's closest-point query runs on a group of G lanes (bvh_closest_grp, stack
// stk_i / stk_d); every lane of the group computes the transform alike, the first one writes.
template <int T, int K, bool PLAIN, int G = 1>
__device__ __forceinline__ double geo_z_one(const GeoGroupDev& g, int e, const double* __restrict__ x,
                                            const double* __restrict__ u, double* __restrict__ z,
                                            double* __restrict__ y, int* stk_i = nullptr, float* stk_d = nullptr) {
    const bool writer = G == 1 || (threadIdx.x & (G - 1)) == 0;
    constexpr int C = (T == GEO_ANGLE || T == GEO_EDGE) ? K - 1 : K;
    double v[3 * C], uu[3 * C];
    double t[PLAIN ? 3 * C : 1];
    // the loads that do not depend on the point positions first (u, the parameters, the warm
    // triangle): issued after the transform's gathers, each one had added a round trip
    if (g.hard) {
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) uu[i] = u[g.uoff + (size_t)i * g.count + e];
    }
    double pr0 = 0.0, pr1 = 0.0;
    if constexpr (T == GEO_ANGLE) { pr0 = g.prm[e]; pr1 = g.prm[(size_t)g.count + e]; }
    else if constexpr (T == GEO_EDGE) pr0 = g.prm[e];
    [[maybe_unused]] int w0 = -1;
    if constexpr (T == GEO_POINT_TO_REF || T == GEO_REF_SURFACE) w0 = g.warm ? g.warm[e] : -1;
    transform<T, K>(g, e, x, v);
    if constexpr (PLAIN) {
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) t[i] = v[i];
    }
    if (g.hard) {
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) v[i] += uu[i];
    }
    if constexpr (T == GEO_PLANE) {
        plane_project<K>(v);
    } else if constexpr (T == GEO_ANGLE) {
        angle_project(v, pr0, pr1);
    } else if constexpr (T == GEO_EDGE) {
        const double L = pr0;
        const double s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        const double r = s2 > 0 ? L / sqrt(s2) : L;
        v[0] *= r; v[1] *= r; v[2] *= r;
    } else if constexpr (T == GEO_POINT_TO_REF || T == GEO_REF_SURFACE) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double qx, qy, qz;
            int tr;
            if constexpr (G > 1) tr = bvh_closest_grp<G>(g.surf, v[3 * c], v[3 * c + 1], v[3 * c + 2], w0, stk_i, stk_d, qx, qy, qz);
            else tr = bvh_closest(g.surf, v[3 * c], v[3 * c + 1], v[3 * c + 2], w0, qx, qy, qz);
            if (g.warm && writer) g.warm[e] = tr;
            v[3 * c] = qx; v[3 * c + 1] = qy; v[3 * c + 2] = qz;
        }
    }   // CLOSENESS: identity
    double part = 0;
    if constexpr (PLAIN) {   // every plain group carries u (g.hard == 1)
        if (g.comb_a > 0) {
            const double a = g.comb_a, b = 1.0 - g.comb_a;
#pragma unroll
            for (int i = 0; i < 3 * C; ++i) v[i] = (t[i] + uu[i]) * a + v[i] * b;
        }
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) { const double r = t[i] - v[i]; part += r * r; }
    }
    if (!writer) return part;
    if (g.hard) {
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) { z[g.uoff + (size_t)i * g.count + e] = v[i]; uu[i] = v[i] - uu[i]; }
        write_slots<T, K>(g, e, uu, g.yscale, y);
    } else {
        write_slots<T, K>(g, e, v, g.yscale, y);
    }
    return part;
}

template <int T, int K>
__global__ __launch_bounds__(kBlock) void k_geo_z(GeoGroupDev g, const double* __restrict__ x,
                                                  const double* __restrict__ u, double* __restrict__ z,
                                                  double* __restrict__ y, const Ctrl* ctrl) {
    if (gated(ctrl)) return;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= g.count) return;
    (void)geo_z_one<T, K, false>(g, e, x, u, z, y);
}

// single-point closest-point groups (PointToRef / ReferenceSurface, K = 1) with G lanes per
// constraint (bvh_closest_grp)
template <int T, int G>
__global__ __launch_bounds__(kBlock) void k_geo_z_cp(GeoGroupDev g, const double* __restrict__ x,
                                                     const double* __restrict__ u, double* __restrict__ z,
                                                     double* __restrict__ y, const Ctrl* ctrl) {
    if (gated(ctrl)) return;
    __shared__ int stk_i[kBlock / G * kCpStack];
    __shared__ float stk_d[kBlock / G * kCpStack];
    const int e = (int)((blockIdx.x * (long long)blockDim.x + threadIdx.x) / G);
    if (e >= g.count) return;   // whole groups
    const int q = threadIdx.x / G;
    (void)geo_z_one<T, 1, false, G>(g, e, x, u, z, y, stk_i + q * kCpStack, stk_d + q * kCpStack);
}

// GeometrySolver z-update with the residual's block partials; gate 1 = only after a residual
// increase (the recomputation that follows the swap to the un-accelerated iterate)
template <int T, int K>
__global__ __launch_bounds__(kBlock) void k_geo_zp(GeoGroupDev g, const double* __restrict__ x,
                                                   const double* __restrict__ u, double* __restrict__ z,
                                                   double* __restrict__ y, const Ctrl* ctrl, double* red, int red_off,
                                                   int gate) {
    if (gated(ctrl) || (gate && !ctrl->reject)) return;
    __shared__ double sm[kBlock / 64];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double part = 0;
    if (e < g.count) part = geo_z_one<T, K, true>(g, e, x, u, z, y);
    if (red) {
        const double sum = block_sum(part, sm);
        if (threadIdx.x == 0) red[red_off + blockIdx.x] = sum;
    }
}

// PlaneConstraint with any number of points (faces of valence > kGeoMaxK; PlanarityOpt.cpp:235-246
// adds one per polygon face). The same arithmetic as plane_project<K> / write_slots<PLANE, K> in
// the same order, with the 3 x K working rows kept in this constraint's own rhs slot rows
// (scratch, overwritten by the final slot values) instead of registers.
template <bool PLAIN>
__global__ __launch_bounds__(kBlock) void k_geo_z_plane_dyn(GeoGroupDev g, const double* __restrict__ x,
                                                            const double* __restrict__ u, double* __restrict__ z,
                                                            double* __restrict__ y, const Ctrl* ctrl, double* red,
                                                            int red_off, int gate) {
    if (gated(ctrl) || (gate && !ctrl->reject)) return;
    __shared__ double sm[kBlock / 64];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double part = 0;
    if (e < g.count) {
        const int K = g.K;
        double* yr = y + 3 * (size_t)(g.slot0 + (long long)e * K);
        auto pt = [&](int a, int d) { return x[3 * (size_t)g.idx[(size_t)a * g.count + e] + d]; };
        auto uat = [&](int a, int d) { return u[g.uoff + (size_t)(3 * a + d) * g.count + e]; };
        double m[3] = {0, 0, 0};
        for (int a = 0; a < K; ++a)
            for (int d = 0; d < 3; ++d) m[d] += pt(a, d);
        for (int d = 0; d < 3; ++d) m[d] /= K;
        for (int a = 0; a < K; ++a)
            for (int d = 0; d < 3; ++d) {
                double v = pt(a, d) - m[d];
                if (g.hard) v += uat(a, d);
                yr[3 * a + d] = v;
            }
        double W[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        for (int sweep = 0; sweep < 30; ++sweep) {
            bool rotated = false;
            for (int pr = 0; pr < 3; ++pr) {
                const int p = pr == 2 ? 1 : 0, q = pr == 0 ? 1 : 2;
                double aa = 0, bb = 0, gg = 0;
                for (int k = 0; k < K; ++k) {
                    const double rp = yr[3 * k + p], rq = yr[3 * k + q];
                    aa += rp * rp; bb += rq * rq; gg += rp * rq;
                }
                if (fabs(gg) > 1e-15 * sqrt(aa * bb) && gg != 0.0) {
                    rotated = true;
                    const double zeta = (bb - aa) / (2.0 * gg);
                    const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                    const double c = 1.0 / sqrt(1.0 + tt * tt), sn = c * tt;
                    for (int k = 0; k < K; ++k) {
                        const double rp = yr[3 * k + p], rq = yr[3 * k + q];
                        yr[3 * k + p] = c * rp - sn * rq;
                        yr[3 * k + q] = sn * rp + c * rq;
                    }
                    for (int k = 0; k < 3; ++k) {
                        const double wp = W[p][k], wq = W[q][k];
                        W[p][k] = c * wp - sn * wq;
                        W[q][k] = sn * wp + c * wq;
                    }
                }
            }
            if (!rotated) break;
        }
        double nr[3];
        for (int d = 0; d < 3; ++d) {
            double sq = 0;
            for (int k = 0; k < K; ++k) sq += yr[3 * k + d] * yr[3 * k + d];
            nr[d] = sq;
        }
        int i = 0;
        if (nr[1] < nr[i]) i = 1;
        if (nr[2] < nr[i]) i = 2;
        double n0 = W[i][0], n1 = W[i][1], n2 = W[i][2];
        const double l = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
        if (l > 0) { n0 /= l; n1 /= l; n2 /= l; }
        double qm[3] = {0, 0, 0};
        for (int a = 0; a < K; ++a) {
            double t[3], uu[3] = {0, 0, 0}, v[3];
            for (int d = 0; d < 3; ++d) {
                t[d] = pt(a, d) - m[d];
                if (g.hard) uu[d] = uat(a, d);
                v[d] = g.hard ? t[d] + uu[d] : t[d];
            }
            const double dp = n0 * v[0] + n1 * v[1] + n2 * v[2];
            double q[3] = {v[0] - n0 * dp, v[1] - n1 * dp, v[2] - n2 * dp};
            if constexpr (PLAIN) {
                if (g.comb_a > 0)
                    for (int d = 0; d < 3; ++d) q[d] = v[d] * g.comb_a + q[d] * (1.0 - g.comb_a);
                for (int d = 0; d < 3; ++d) { const double r = t[d] - q[d]; part += r * r; }
            }
            for (int d = 0; d < 3; ++d) {
                if (g.hard) { z[g.uoff + (size_t)(3 * a + d) * g.count + e] = q[d]; q[d] -= uu[d]; }
                yr[3 * a + d] = q[d];
                qm[d] += q[d];
            }
        }
        for (int d = 0; d < 3; ++d) qm[d] /= K;
        for (int a = 0; a < K; ++a)
            for (int d = 0; d < 3; ++d) yr[3 * a + d] = g.yscale * (yr[3 * a + d] - qm[d]);
    }
    if (red) {
        const double sum = block_sum(part, sm);
        if (threadIdx.x == 0) red[red_off + blockIdx.x] = sum;
    }
}

// ------------------------------------------------------------------ dual update + residual partials
template <int T, int K>
__global__ __launch_bounds__(kBlock) void k_geo_u(GeoGroupDev g, const double* __restrict__ xnew,
                                                  const double* __restrict__ xcur, const double* __restrict__ z,
                                                  const double* __restrict__ u, double* __restrict__ unew,
                                                  const Ctrl* ctrl, double* red, int red_off) {
    if (gated(ctrl)) return;
    __shared__ double sm[kBlock / 64];
    constexpr int C = (T == GEO_ANGLE || T == GEO_EDGE) ? K - 1 : K;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double part = 0;
    if (e < g.count) {
        double dn[3 * C], dp[3 * C];
        transform<T, K>(g, e, xnew, dn);
        transform<T, K>(g, e, xcur, dp);
#pragma unroll
        for (int i = 0; i < 3 * C; ++i) {
            const size_t o = g.uoff + (size_t)i * g.count + e;
            const double zz = z[o];
            const double r = dn[i] - zz, d = dn[i] - dp[i];
            part += r * r + d * d;
            unew[o] = u[o] + r;
        }
    }
    const double s = block_sum(part, sm);
    if (threadIdx.x == 0) red[red_off + blockIdx.x] = s;
}

// k_geo_u of a plane group with any number of points (same arithmetic and order as transform<PLANE, K>)
__global__ __launch_bounds__(kBlock) void k_geo_u_plane_dyn(GeoGroupDev g, const double* __restrict__ xnew,
                                                            const double* __restrict__ xcur, const double* __restrict__ z,
                                                            const double* __restrict__ u, double* __restrict__ unew,
                                                            const Ctrl* ctrl, double* red, int red_off) {
    if (gated(ctrl)) return;
    __shared__ double sm[kBlock / 64];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double part = 0;
    if (e < g.count) {
        const int K = g.K;
        double mn[3] = {0, 0, 0}, mp[3] = {0, 0, 0};
        for (int a = 0; a < K; ++a) {
            const size_t v = 3 * (size_t)g.idx[(size_t)a * g.count + e];
            for (int d = 0; d < 3; ++d) { mn[d] += xnew[v + d]; mp[d] += xcur[v + d]; }
        }
        for (int d = 0; d < 3; ++d) { mn[d] /= K; mp[d] /= K; }
        for (int a = 0; a < K; ++a) {
            const size_t v = 3 * (size_t)g.idx[(size_t)a * g.count + e];
            for (int d = 0; d < 3; ++d) {
                const size_t o = g.uoff + (size_t)(3 * a + d) * g.count + e;
                const double dn = xnew[v + d] - mn[d], dpv = xcur[v + d] - mp[d];
                const double r = dn - z[o], dd = dn - dpv;
                part += r * r + dd * dd;
                unew[o] = u[o] + r;
            }
        }
    }
    const double sum = block_sum(part, sm);
    if (threadIdx.x == 0) red[red_off + blockIdx.x] = sum;
}

// ------------------------------------------------------------------ rhs gather
// one lane per point COMPONENT: lanes 3j, 3j+1, 3j+2 of a wave sum x, y, z of point 21 w + j
// (lane 63 idles), so one load instruction reads 21 slot rows whole instead of 64 rows a third
// each; every component is summed in slot order, as with a lane per point (bit for bit)
#ifndef AA_RHS_CHUNK
#define AA_RHS_CHUNK 1
#endif
__global__ __launch_bounds__(kBlock) void k_geo_rhs(int n, const int* __restrict__ ptr, const int* __restrict__ slots,
                                                    const double* __restrict__ y, const double* __restrict__ rf,
                                                    double* __restrict__ b, const Ctrl* ctrl) {
    if (gated(ctrl)) return;
    const int lane = threadIdx.x & 63;
    if (lane == 63) return;
    const long long w = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long i = w * 21 + lane / 3;
    const int c = lane % 3;
    if (i >= n) return;
    const size_t o = 3 * (size_t)i + c;
    double sum = rf[o];
    const int k0 = ptr[i], k1 = ptr[i + 1];
#if AA_RHS_CHUNK
    // chunks of 8 slots: the 8 slot ids, then the 8 rows, each group issued together (ids clamped
    // to the last slot, the extra terms adding 0) -- two round trips per chunk instead of two per
    // slot; the same sum order
    for (int k = k0; k < k1; k += 8) {
        int id[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) id[m] = slots[min(k + m, k1 - 1)];
        __builtin_amdgcn_sched_barrier(0);
        double g[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) g[m] = y[3 * (size_t)id[m] + c];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 8; ++m) sum += k + m < k1 ? g[m] : 0.0;
    }
#else
    for (int k = k0; k < k1; ++k) sum += y[3 * (size_t)slots[k] + c];
#endif
    b[o] = sum;
}

// ------------------------------------------------------------------ control
__global__ __launch_bounds__(kBlock) void k_geo_control(Ctrl* ctrl, const double* red, int nb, int accel,
                                                        double* hist_comb, unsigned long long* hist_clock) {
    if (ctrl->done) return;
    __shared__ double sm[kBlock / 64];
    double a = thread_sum_strided(red, nb);
    a = block_sum(a, sm);
    if (threadIdx.x != 0) return;
    const double comb = a;
    ctrl->comb = comb;
    ctrl->iters_run += 1;
    const bool accept = !accel || ctrl->alm_reset || comb < ctrl->prev_prim;
    if (accept) {
        const int k = ctrl->nrec;
        if (k < ctrl->cap) { hist_comb[k] = comb; hist_clock[k] = wall_clock64(); }
        ctrl->nrec = k + 1;
        ctrl->prev_prim = comb;
        ctrl->alm_reset = 0;
        ctrl->reject = 0;
        ctrl->aa_skip = 0;
        if (ctrl->nrec >= ctrl->max_iter) ctrl->done = 1;
        // run-to-epsilon (GeomSolver::set_stop): the commented-out test of ALMGeometrySolver.h:258
        // and / or a level relative to the first accepted iteration's comb
        const double c0 = k < ctrl->cap ? hist_comb[0] : comb;
        if ((ctrl->eps_abs > 0.0 && comb < ctrl->eps_abs) || (ctrl->eps_rel > 0.0 && comb <= ctrl->eps_rel * c0)) {
            ctrl->eps_hit = 1;
            ctrl->done = 1;
        }
    } else {
        ctrl->reject = 1;
        ctrl->nrej += 1;
        ctrl->alm_reset = 1;
        ctrl->aa_iter = 0;   // accelerator->reset (AndersonAcceleration.h:73-91)
        ctrl->aa_col = 0;
        ctrl->aa_skip = 1;
    }
}

// GeometrySolver::solve_ADMM decisions (GeometrySolver.h:180-231): op 0 after the z-update --
// residual = |Dx - z| from the partials; with Anderson, a residual above the previous one
// flags the swap to the un-accelerated iterate (reject; the history is NOT reset: replace);
// otherwise the iteration is recorded. op 1 (only when flagged) records the recomputed
// residual. Recording ends the loop after max_iter iterations, else prev = residual.
__global__ __launch_bounds__(kBlock) void k_plain_control(Ctrl* ctrl, const double* red, int nb, int accel, int op,
                                                          double* hist_comb, unsigned long long* hist_clock) {
    if (ctrl->done || (op == 1 && !ctrl->reject)) return;
    __shared__ double sm[kBlock / 64];
    double a = thread_sum_strided(red, nb);
    a = block_sum(a, sm);
    if (threadIdx.x != 0) return;
    const double res = sqrt(a);
    if (op == 0) {
        ctrl->reject = (accel && res > ctrl->prev_prim) ? 1 : 0;
        if (ctrl->reject) { ctrl->nrej += 1; return; }
    }
    ctrl->comb = res;
    const int k = ctrl->nrec;
    if (k < ctrl->cap) { hist_comb[k] = res; hist_clock[k] = wall_clock64(); }
    ctrl->nrec = k + 1;
    ctrl->iters_run += 1;
    if (ctrl->nrec >= ctrl->max_iter) ctrl->done = 1;
    else ctrl->prev_prim = res;
}

__global__ void k_geo_start(Ctrl* ctrl, unsigned long long* clock0) {
    (void)ctrl;
    *clock0 = wall_clock64();
}

__global__ __launch_bounds__(kBlock) void k_geo_restore(double* __restrict__ cu, double* __restrict__ cx,
                                                        double* __restrict__ aacur, const double* __restrict__ du,
                                                        const double* __restrict__ dx, long long nu, long long nx,
                                                        const Ctrl* ctrl) {
    if (ctrl->done || !ctrl->reject) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nu + nx; i += (long long)gridDim.x * blockDim.x) {
        if (i < nu) { const double v = du[i]; cu[i] = v; if (aacur) aacur[i] = v; }
        else { const double v = dx[i - nu]; cx[i - nu] = v; if (aacur) aacur[i] = v; }
    }
}

__global__ __launch_bounds__(kBlock) void k_closest(SurfDev S, const double* __restrict__ p, double* __restrict__ c, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double qx, qy, qz;
    bvh_closest(S, p[3 * (size_t)i], p[3 * (size_t)i + 1], p[3 * (size_t)i + 2], -1, qx, qy, qz);
    c[3 * (size_t)i] = qx; c[3 * (size_t)i + 1] = qy; c[3 * (size_t)i + 2] = qz;
}

template <int G>
__global__ __launch_bounds__(kBlock) void k_closest_grp(SurfDev S, const double* __restrict__ p, double* __restrict__ c, int n) {
    __shared__ int stk_i[kBlock / G * kCpStack];
    __shared__ float stk_d[kBlock / G * kCpStack];
    const int i = (int)((blockIdx.x * (long long)blockDim.x + threadIdx.x) / G);
    if (i >= n) return;
    const int q = threadIdx.x / G;
    double qx, qy, qz;
    bvh_closest_grp<G>(S, p[3 * (size_t)i], p[3 * (size_t)i + 1], p[3 * (size_t)i + 2], -1, stk_i + q * kCpStack,
                       stk_d + q * kCpStack, qx, qy, qz);
    if ((threadIdx.x & (G - 1)) == 0) { c[3 * (size_t)i] = qx; c[3 * (size_t)i + 1] = qy; c[3 * (size_t)i + 2] = qz; }
}

// test hook: Constraint::project_impl of plane (any k) / angle / edge on transformed points
template <int K>
__device__ void test_plane(double* v) { plane_project<K>(v); }

__global__ void k_test_geo_project(int type, int k, double p0, double p1, const double* __restrict__ in, int n,
                                   double* __restrict__ out) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const int C = (type == GEO_ANGLE || type == GEO_EDGE) ? k - 1 : k;
    double v[3 * kGeoMaxK];
    for (int i = 0; i < 3 * C; ++i) v[i] = in[(size_t)e * 3 * C + i];
    if (type == GEO_PLANE) {
        switch (k) {
            case 3: test_plane<3>(v); break;
            case 4: test_plane<4>(v); break;
            case 5: test_plane<5>(v); break;
            case 6: test_plane<6>(v); break;
            case 7: test_plane<7>(v); break;
            default: test_plane<8>(v); break;
        }
    } else if (type == GEO_ANGLE) {
        angle_project(v, p0, p1);
    } else if (type == GEO_EDGE) {
        const double s2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        const double r = s2 > 0 ? p0 / sqrt(s2) : p0;
        v[0] *= r; v[1] *= r; v[2] *= r;
    }
    for (int i = 0; i < 3 * C; ++i) out[(size_t)e * 3 * C + i] = v[i];
}

inline int grid_for(long long n) { long long b = (n + kBlock - 1) / kBlock; return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048); }

}  // namespace

// ============================================================================ launchers
#define GEO_DISPATCH(KERNEL, ...)                                                                          \
    switch (g.type) {                                                                                      \
        case GEO_PLANE:                                                                                    \
            switch (g.K) {                                                                                 \
                case 3: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 3>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                case 4: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 4>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                case 5: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 5>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                case 6: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 6>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                case 7: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 7>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                case 8: hipLaunchKernelGGL((KERNEL<GEO_PLANE, 8>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
                default: throw Error(ERR_ARG, "plane constraint with < 3 points");                       \
            }                                                                                              \
            break;                                                                                         \
        case GEO_ANGLE: hipLaunchKernelGGL((KERNEL<GEO_ANGLE, 3>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
        case GEO_EDGE: hipLaunchKernelGGL((KERNEL<GEO_EDGE, 2>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
        case GEO_CLOSENESS: hipLaunchKernelGGL((KERNEL<GEO_CLOSENESS, 1>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
        case GEO_POINT_TO_REF: hipLaunchKernelGGL((KERNEL<GEO_POINT_TO_REF, 1>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
        case GEO_REF_SURFACE: hipLaunchKernelGGL((KERNEL<GEO_REF_SURFACE, 1>), grid, dim3(kBlock), 0, s, __VA_ARGS__); break; \
        default: throw Error(ERR_ARG, "unknown constraint type");                                        \
    }

void launch_geo_z(const GeoGroupDev& g, const double* x, const double* u, double* z, double* y, const Ctrl* ctrl,
                  hipStream_t s) {
    if (g.count == 0) return;
    const dim3 grid(blocks_for(g.count));
    // Group traversal only where one lane per query leaves the chip short of waves: below about
    // 5 waves per SIMD (256 CUs x 4 SIMDs x 64 lanes x 5 = 327 680 queries) the traversal is a
    // latency chain with nothing to hide it (C3, 101 k queries: z 236 -> 194 us); above, the
    // single-lane traversal already fills the SIMDs and the group's redundant seed test and
    // shuffles cost more than they save (C5, 500 k: 493 -> 507 ms per solve). AA_CP_GROUP_MAX
    // overrides the bound.
    static const long long cp_max = std::getenv("AA_CP_GROUP_MAX") ? std::atoll(std::getenv("AA_CP_GROUP_MAX")) : 327680;
    const bool cp = (g.type == GEO_POINT_TO_REF || g.type == GEO_REF_SURFACE) && g.K == 1 && g.surf.wide_g > 0 &&
                    g.count < cp_max;
    if (cp) {   // G lanes per query
        const int G = g.surf.wide_g;
        const dim3 gg(blocks_for((long long)g.count * G));
        if (g.type == GEO_POINT_TO_REF) {
            if (G == 8) hipLaunchKernelGGL((k_geo_z_cp<GEO_POINT_TO_REF, 8>), gg, dim3(kBlock), 0, s, g, x, u, z, y, ctrl);
            else hipLaunchKernelGGL((k_geo_z_cp<GEO_POINT_TO_REF, 4>), gg, dim3(kBlock), 0, s, g, x, u, z, y, ctrl);
        } else {
            if (G == 8) hipLaunchKernelGGL((k_geo_z_cp<GEO_REF_SURFACE, 8>), gg, dim3(kBlock), 0, s, g, x, u, z, y, ctrl);
            else hipLaunchKernelGGL((k_geo_z_cp<GEO_REF_SURFACE, 4>), gg, dim3(kBlock), 0, s, g, x, u, z, y, ctrl);
        }
    } else if (g.type == GEO_PLANE && g.K > kGeoMaxK) {
        hipLaunchKernelGGL(k_geo_z_plane_dyn<false>, grid, dim3(kBlock), 0, s, g, x, u, z, y, ctrl, nullptr, 0, 0);
    } else {
        GEO_DISPATCH(k_geo_z, g, x, u, z, y, ctrl)
    }
    AA_CHECK_LAUNCH();
}

void launch_geo_z_plain(const GeoGroupDev& g, const double* x, const double* u, double* z, double* y, const Ctrl* ctrl,
                        double* red, int red_off, int gate, hipStream_t s) {
    if (g.count == 0) return;
    const dim3 grid(blocks_for(g.count));
    if (g.type == GEO_PLANE && g.K > kGeoMaxK) {
        hipLaunchKernelGGL(k_geo_z_plane_dyn<true>, grid, dim3(kBlock), 0, s, g, x, u, z, y, ctrl, red, red_off, gate);
    } else {
        GEO_DISPATCH(k_geo_zp, g, x, u, z, y, ctrl, red, red_off, gate)
    }
    AA_CHECK_LAUNCH();
}

void launch_plain_control(Ctrl* ctrl, const double* red, int nb, int accel, int op, double* hist_comb,
                          unsigned long long* hist_clock, hipStream_t s) {
    hipLaunchKernelGGL(k_plain_control, dim3(1), dim3(kBlock), 0, s, ctrl, red, nb, accel, op, hist_comb, hist_clock);
    AA_CHECK_LAUNCH();
}

int geo_u_blocks(int count) { return blocks_for(count); }

void launch_geo_u(const GeoGroupDev& g, const double* xnew, const double* xcur, const double* z, const double* u,
                  double* unew, const Ctrl* ctrl, double* red, int red_off, hipStream_t s) {
    if (g.count == 0 || !g.hard) return;
    const dim3 grid(blocks_for(g.count));
    if (g.type == GEO_PLANE && g.K > kGeoMaxK)
        hipLaunchKernelGGL(k_geo_u_plane_dyn, grid, dim3(kBlock), 0, s, g, xnew, xcur, z, u, unew, ctrl, red, red_off);
    else
        GEO_DISPATCH(k_geo_u, g, xnew, xcur, z, u, unew, ctrl, red, red_off)
    AA_CHECK_LAUNCH();
}

void launch_geo_rhs(int n, const int* ptr, const int* slots, const double* y, const double* rhs_fixed, double* b,
                    const Ctrl* ctrl, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_geo_rhs, dim3(blocks_for(64 * ((n + 20) / 21LL))), dim3(kBlock), 0, s, n, ptr, slots, y, rhs_fixed, b, ctrl);
    AA_CHECK_LAUNCH();
}

void launch_geo_control(Ctrl* ctrl, const double* red, int nb, int accel, double* hist_comb,
                        unsigned long long* hist_clock, hipStream_t s) {
    hipLaunchKernelGGL(k_geo_control, dim3(1), dim3(kBlock), 0, s, ctrl, red, nb, accel, hist_comb, hist_clock);
    AA_CHECK_LAUNCH();
}

void launch_geo_start(Ctrl* ctrl, unsigned long long* clock0, hipStream_t s) {
    hipLaunchKernelGGL(k_geo_start, dim3(1), dim3(1), 0, s, ctrl, clock0);
    AA_CHECK_LAUNCH();
}

void launch_geo_restore(double* cu, double* cx, double* aacur, const double* du, const double* dx, long long nu,
                        long long nx, const Ctrl* ctrl, hipStream_t s) {
    hipLaunchKernelGGL(k_geo_restore, dim3(grid_for(nu + nx)), dim3(kBlock), 0, s, cu, cx, aacur, du, dx, nu, nx, ctrl);
    AA_CHECK_LAUNCH();
}

#ifdef AA_CP_STATS
void cp_stats_dump() {
    unsigned long long h[64];
    AA_HIP(hipDeviceSynchronize());
    AA_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_cp_stats), sizeof(h)));
    fprintf(stderr, "CP_STATS queries %llu box %llu tri %llu tight %llu moved %llu\nCP_BOX_HIST", h[0], h[1], h[2], h[3], h[4]);
    for (int i = 0; i < 16; ++i) fprintf(stderr, " %llu", h[8 + i]);
    fprintf(stderr, "\nCP_DIST_HIST");
    for (int i = 0; i < 16; ++i) fprintf(stderr, " %llu", h[24 + i]);
    fprintf(stderr, "\nCP_ORACLE box %llu tri %llu\n", h[40], h[41]);
    const unsigned long long z[64] = {};
    AA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_cp_stats), z, sizeof(z)));
}
#endif

void launch_closest(const SurfDev& sd, const double* p, double* c, int n, hipStream_t s) {
    if (n == 0) return;
    if (sd.wide_g == 8) hipLaunchKernelGGL(k_closest_grp<8>, dim3(blocks_for(8LL * n)), dim3(kBlock), 0, s, sd, p, c, n);
    else if (sd.wide_g == 4) hipLaunchKernelGGL(k_closest_grp<4>, dim3(blocks_for(4LL * n)), dim3(kBlock), 0, s, sd, p, c, n);
    else hipLaunchKernelGGL(k_closest, dim3(blocks_for(n)), dim3(kBlock), 0, s, sd, p, c, n);
    AA_CHECK_LAUNCH();
}

void launch_test_geo_project(int type, int k, const double* prm2, const double* in, int n, double* out, hipStream_t s) {
    if (n <= 0) return;
    if (type == GEO_PLANE && (k < 3 || k > kGeoMaxK)) throw Error(ERR_ARG, "test hook: plane k must be 3..8 (register path)");
    if (type == GEO_ANGLE && k != 3) throw Error(ERR_ARG, "test hook: angle k = 3");
    if (type == GEO_EDGE && k != 2) throw Error(ERR_ARG, "test hook: edge k = 2");
    if (type != GEO_PLANE && type != GEO_ANGLE && type != GEO_EDGE) throw Error(ERR_ARG, "test hook: plane, angle or edge");
    hipLaunchKernelGGL(k_test_geo_project, dim3((n + 63) / 64), dim3(64), 0, s, type, k, prm2[0], prm2[1], in, n, out);
    AA_CHECK_LAUNCH();
}

}  // namespace aa
