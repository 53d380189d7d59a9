// Device data structures and kernel launchers of the Geometry (ALM) hot path
// (the reference's ALMGeometrySolver<3>, Geometry/ALMGeometrySolver.h:163-461).
#pragma once
#include <hip/hip_runtime.h>

#include "elastic_kernels.hpp"   // Ctrl, Seg2, Anderson launchers

namespace aa {

// constraint types (Geometry/Constraint.h) -- must match include/aa_admm.h AA_CON_*
enum GeoType { GEO_PLANE = 0, GEO_ANGLE = 1, GEO_EDGE = 2, GEO_CLOSENESS = 3, GEO_POINT_TO_REF = 4, GEO_REF_SURFACE = 5 };
constexpr int kGeoMaxK = 8;   // planes up to this valence run in registers; larger ones in slot-row scratch

// Bounding-volume hierarchy over one reference triangle surface (closest-point queries of
// PointToRefSurfaceConstraint / ReferenceSurfceConstraint). Nodes in depth-first order:
// the left child of node i is i+1; `a` is the right child (inner) or the first triangle
// (leaf), `b` = -(triangle count) for a leaf, 0 otherwise; `skip` is the first node after
// this node's subtree (the escape link of a stackless traversal).
// 64-B BVH node: box in fp32 rounded OUTWARD (never prunes a box the fp64 box would keep),
// a = right child (inner) or first triangle (leaf), sn = escape link (node after the subtree,
// low 29 bits) | leaf triangle count << 29 (0 = inner), and a slab: the subtree's mean unit
// normal n and the range [dlo, dhi] of n . v over its vertices (rounded outward). The slab
// bounds the distance to every triangle of the subtree from below like the box does, and is
// far tighter for sloped, thin patches seen from afar (a point well off the surface).
// With the two tangent axes t1, t2 (principal directions of the subtree's vertices in the plane
// normal to n) and their ranges the slab becomes an oriented box: a point far above a flat
// patch has the same normal distance to every patch around its foot point, and only the
// tangent ranges tell those patches apart. 128 B, one cache line.
struct alignas(128) BvhNode {
    float lo[3], hi[3];
    int a;
    unsigned sn;
    float nrm[3], dlo, dhi;
    float t1[3], t1lo, t1hi;
    float t2[3], t2lo, t2hi;
};
static_assert(sizeof(BvhNode) == 128, "BvhNode is one 128-B line");
__host__ __device__ inline int bvh_skip(const BvhNode& n) { return (int)(n.sn & 0x1fffffffu); }
__host__ __device__ inline int bvh_count(const BvhNode& n) { return (int)(n.sn >> 29); }
struct BvhTri { double v[9]; };   // triangle corners, stored in leaf order
// The same tree collapsed to `wide_g` (4 or 8) children per node for the group traversal
// (wide_g lanes per query, see bvh_closest_grp): node w's children are the records
// wide[w * wide_g + k], copies of the BvhNode of a descendant log2(wide_g) levels down (or of a
// leaf met earlier), with `a` = the child's wide node (inner) or its first triangle (leaf) and
// sn = triangle count << 29 (0 = inner); unused slots have a = -1. wide_g = 0: not built.
constexpr int kCpStack = 64;   // per-query traversal stack entries of the group traversal
struct SurfDev {
    const BvhNode* nodes;
    const BvhTri* tris;
    int n_nodes, n_tris;
    const BvhNode* wide = nullptr;
    int wide_g = 0;
};

// One homogeneous block of constraints (same type / index count / weight / hard-soft).
struct GeoGroupDev {
    int type, K, cols, hard;
    int count;
    double sw;            // weight_ = sqrt(weight) (Constraint.h:64-69)
    double yscale;        // scale of the rhs contribution: rho (hard) / weight (soft)
    double comb_a;        // GeometrySolver soft groups: rho / (weight + rho) (project_and_combine); else 0
    long long uoff;       // hard: u / z offset, SoA [(c*3 + d)][count]
    long long slot0;      // first rhs slot of this group: slot(e, a) = slot0 + e*K + a
    const int* idx;       // [K][count] internal point ids
    const double* prm;    // [P][count]   EDGE length; ANGLE min, max; else unused
    int* warm;            // [count] last closest triangle (closest-point groups), may be null
    SurfDev surf;
};

// z-step of one group: Dx = T(x) (+u for hard), z = P(Dx) (x sqrt(w) for soft); writes z
// (hard) and the rhs slot rows y[slot] = yscale * T^T (z - u)  (hard)  /  w T^T P(Dx)  (soft)
void launch_geo_z(const GeoGroupDev& g, const double* x, const double* u, double* z, double* y, const Ctrl* ctrl,
                  hipStream_t s);
// GeometrySolver<3> z-update (Geometry/GeometrySolver.h:423-439): every group carries u (hard = 1),
// soft groups combine z = a v + (1 - a) P(v) (comb_a = a); block partials of |T(x) - z|^2 into
// red[red_off + block]; gate 1 = run only when ctrl->reject (the recomputation after a swap)
void launch_geo_z_plain(const GeoGroupDev& g, const double* x, const double* u, double* z, double* y, const Ctrl* ctrl,
                        double* red, int red_off, int gate, hipStream_t s);
// GeometrySolver decisions: op 0 = residual check (reject flag / record), op 1 = record the
// recomputed residual after a swap (see k_plain_control)
void launch_plain_control(Ctrl* ctrl, const double* red, int nb, int accel, int op, double* hist_comb,
                          unsigned long long* hist_clock, hipStream_t s);
// b = rhs_fixed + sum of the slot rows of each point (fixed order)
void launch_geo_rhs(int n, const int* ptr, const int* slots, const double* y, const double* rhs_fixed, double* b,
                    const Ctrl* ctrl, hipStream_t s);
// hard groups: Dn = T(x_new), Dp = T(x_cur); u_new = u + Dn - z; partial sums of
// |Dn - z|^2 + |Dn - Dp|^2 (the combined residual, ALMGeometrySolver.h:452-461)
void launch_geo_u(const GeoGroupDev& g, const double* xnew, const double* xcur, const double* z, const double* u,
                  double* unew, const Ctrl* ctrl, double* red, int red_off, hipStream_t s);
int geo_u_blocks(int count);
// accept / reject (ALMGeometrySolver.h:215-263): comb from the partials; on accept record
// (comb, device clock), nrec++, done when nrec >= max_iter; on reject reject = 1, Anderson
// reset (aa_iter = aa_col = 0) and aa_skip = 1.
void launch_geo_control(Ctrl* ctrl, const double* red, int nb, int accel, double* hist_comb,
                        unsigned long long* hist_clock, hipStream_t s);
// prologue: ctrl fields, clock origin
void launch_geo_start(Ctrl* ctrl, unsigned long long* clock0, hipStream_t s);
// reject restore: (cur_u, cur_x) = (def_u, def_x) and the Anderson current iterate alike (gate: reject)
void launch_geo_restore(double* cu, double* cx, double* aacur, const double* du, const double* dx, long long nu,
                        long long nx, const Ctrl* ctrl, hipStream_t s);
// closest points of `n` points (test hook / soft-energy evaluation)
void launch_closest(const SurfDev& sd, const double* p, double* c, int n, hipStream_t s);
#ifdef AA_CP_STATS
void cp_stats_dump();   // diagnostics build: print and reset the traversal counters
#endif

// test hook (aa_test_geom_project): project_impl of n constraints of one type on transformed points
void launch_test_geo_project(int type, int k, const double* prm2, const double* in, int n, double* out, hipStream_t s);

}  // namespace aa
