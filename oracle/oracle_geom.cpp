// ORACLE -- test infrastructure only (see oracle.h). Plain C++ restatement, no Eigen/igl/OpenMesh.
//
// Restates the Geometry ALM hot path of the reference:
//   ALMGeometrySolver<3>::setup_ADMM   Geometry/ALMGeometrySolver.h:81-161
//   ALMGeometrySolver<3>::solve_ADMM   Geometry/ALMGeometrySolver.h:163-283 (+ helpers :411-461)
//   Constraint<3>::apply_transform / project / add_constraint   Geometry/Constraint.h:73-159
//   EdgeLength :194-218, Angle :220-296, Closeness :299-326 (its `proj_impl` typo makes the
//   projection the identity), PointToRefSurface :328-349, ReferenceSurfce :351-394, Plane :396-414
//   LinearRegularization::add_* / get_regularization_system   Geometry/LinearRegularization.h:47-147
//   AndersonAcceleration (Geometry/AndersonAcceleration.h:93-211) -- oracle_common.hpp
//   igl::AABB::squared_distance + point_simplex_squared_distance (Ericson, "Real-time collision
//   detection" ch. 5; Geometry/external/igl/point_simplex_squared_distance.cpp:40-108) -- a
//   median-split AABB tree with exact pruning (same closest point; ties only to rounding).
// The SimplicialLDLT of the global matrix (Geometry/SPDSolver.h:67-90) is an envelope Cholesky
// under reverse Cuthill-McKee (same solution to rounding). The best-fit plane normal (Eigen
// JacobiSVD with FullPivHouseholderQR preconditioner, ComputeFullU) is restated as a Householder
// QR of P^T followed by the Jacobi SVD of R^T (oracle_svd.hpp): the same left singular vectors.
//
// I/O: the AAGEOM01 scene / AAGEOMR1 result files of oracle/ref_drivers/ref_geom_driver.cpp.
#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "oracle.h"
#include "oracle_common.hpp"
#include "oracle_svd.hpp"

namespace oracle {
namespace {

enum { PLANE = 0, ANGLE = 1, EDGE = 2, CLOSENESS = 3, POINT_TO_REF = 4, REF_SURFACE = 5 };
enum { MEAN_CENTERING, SUBTRACT_FIRST, IDENTITY };

struct V3 { double x, y, z; };
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 mul(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// ------------------------------------------------------------------ closest point on a triangle mesh
struct TriSurface {
    std::vector<double> V;
    std::vector<int> F;
    struct Node { double lo[3], hi[3]; int left, right, tri; };
    std::vector<Node> nodes;

    V3 vert(int i) const { return {V[3 * i], V[3 * i + 1], V[3 * i + 2]}; }

    int build(std::vector<int>& ids, int b, int e) {
        Node nd;
        for (int d = 0; d < 3; ++d) { nd.lo[d] = DBL_MAX; nd.hi[d] = -DBL_MAX; }
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a)
                for (int d = 0; d < 3; ++d) {
                    const double v = V[3 * F[3 * ids[i] + a] + d];
                    nd.lo[d] = std::min(nd.lo[d], v); nd.hi[d] = std::max(nd.hi[d], v);
                }
        nd.left = nd.right = nd.tri = -1;
        const int me = (int)nodes.size();
        nodes.push_back(nd);
        if (e - b == 1) { nodes[me].tri = ids[b]; return me; }
        int ax = 0;
        double ext = -1;
        for (int d = 0; d < 3; ++d) if (nd.hi[d] - nd.lo[d] > ext) { ext = nd.hi[d] - nd.lo[d]; ax = d; }
        auto cen = [&](int t) { double s = 0; for (int a = 0; a < 3; ++a) s += V[3 * F[3 * t + a] + ax]; return s; };
        const int mid = (b + e) / 2;
        std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e, [&](int p, int q) { return cen(p) < cen(q); });
        const int l = build(ids, b, mid), r = build(ids, mid, e);
        nodes[me].left = l; nodes[me].right = r;
        return me;
    }
    void init() {
        std::vector<int> ids(F.size() / 3);
        std::iota(ids.begin(), ids.end(), 0);
        nodes.clear();
        if (!ids.empty()) build(ids, 0, (int)ids.size());
    }
    // Ericson, closest point on triangle (igl point_simplex_squared_distance.cpp:40-108)
    static V3 closest_on_tri(V3 p, V3 a, V3 b, V3 c) {
        const V3 ab = sub(b, a), ac = sub(c, a), ap = sub(p, a);
        const double d1 = dot(ab, ap), d2 = dot(ac, ap);
        if (d1 <= 0.0 && d2 <= 0.0) return a;
        const V3 bp = sub(p, b);
        const double d3 = dot(ab, bp), d4 = dot(ac, bp);
        if (d3 >= 0.0 && d4 <= d3) return b;
        const double vc = d1 * d4 - d3 * d2;
        if (!(a.x == b.x && a.y == b.y && a.z == b.z))
            if (vc <= 0.0 && d1 >= 0.0 && d3 <= 0.0) { const double v = d1 / (d1 - d3); return add(a, mul(ab, v)); }
        const V3 cp = sub(p, c);
        const double d5 = dot(ab, cp), d6 = dot(ac, cp);
        if (d6 >= 0.0 && d5 <= d6) return c;
        const double vb = d5 * d2 - d1 * d6;
        if (vb <= 0.0 && d2 >= 0.0 && d6 <= 0.0) { const double w = d2 / (d2 - d6); return add(a, mul(ac, w)); }
        const double va = d3 * d6 - d5 * d4;
        if (va <= 0.0 && (d4 - d3) >= 0.0 && (d5 - d6) >= 0.0) {
            const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
            return add(b, mul(sub(c, b), w));
        }
        const double denom = 1.0 / (va + vb + vc);
        const double v = vb * denom, w = vc * denom;
        return add(add(a, mul(ab, v)), mul(ac, w));
    }
    double box_d2(const Node& nd, V3 p) const {
        const double q[3] = {p.x, p.y, p.z};
        double s = 0;
        for (int d = 0; d < 3; ++d) {
            const double t = q[d] < nd.lo[d] ? nd.lo[d] - q[d] : (q[d] > nd.hi[d] ? q[d] - nd.hi[d] : 0.0);
            s += t * t;
        }
        return s;
    }
    void search(int ni, V3 p, double& best, V3& bc) const {
        const Node& nd = nodes[ni];
        if (nd.tri >= 0) {
            const int t = nd.tri;
            const V3 c = closest_on_tri(p, vert(F[3 * t]), vert(F[3 * t + 1]), vert(F[3 * t + 2]));
            const V3 dv = sub(p, c);
            const double d2 = dot(dv, dv);
            if (d2 < best) { best = d2; bc = c; }
            return;
        }
        const double dl = box_d2(nodes[nd.left], p), dr = box_d2(nodes[nd.right], p);
        if (dl <= dr) {
            if (dl < best) search(nd.left, p, best, bc);
            if (dr < best) search(nd.right, p, best, bc);
        } else {
            if (dr < best) search(nd.right, p, best, bc);
            if (dl < best) search(nd.left, p, best, bc);
        }
    }
    V3 closest(V3 p) const {
        double best = std::numeric_limits<double>::infinity();
        V3 c = p;
        if (!nodes.empty()) search(0, p, best, c);
        return c;
    }
};

// ------------------------------------------------------------------ constraints
struct Con {
    int type, transform, k;
    double sw;                 // weight_ = sqrt(weight)   (Constraint.h:64-69)
    double prm[3];
    int surf;
    std::vector<int> idx;
    int idO = -1;
    int cols() const { return transform == SUBTRACT_FIRST ? k - 1 : k; }
};

// x and Dx are 3 x N column-major ([col*3 + d])
void apply_transform(const Con& c, const double* x, double* Dx) {
    if (c.transform == SUBTRACT_FIRST) {
        const double* f = x + 3 * (size_t)c.idx[0];
        for (int i = 1; i < c.k; ++i)
            for (int d = 0; d < 3; ++d) Dx[3 * (size_t)(c.idO + i - 1) + d] = x[3 * (size_t)c.idx[i] + d] - f[d];
    } else {
        for (int i = 0; i < c.k; ++i)
            for (int d = 0; d < 3; ++d) Dx[3 * (size_t)(c.idO + i) + d] = x[3 * (size_t)c.idx[i] + d];
        if (c.transform == MEAN_CENTERING) {
            double mean[3] = {0, 0, 0};
            for (int i = 0; i < c.k; ++i) for (int d = 0; d < 3; ++d) mean[d] += Dx[3 * (size_t)(c.idO + i) + d];
            for (int d = 0; d < 3; ++d) mean[d] /= c.k;
            for (int i = 0; i < c.k; ++i) for (int d = 0; d < 3; ++d) Dx[3 * (size_t)(c.idO + i) + d] -= mean[d];
        }
    }
}

// best-fit plane normal of the mean-centred points P (3 x k): U[:,2] of the SVD
V3 plane_normal(const double* P, int k) {
    double A[9];   // row-major 3x3 whose left singular vectors equal those of P
    if (k == 3) {
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) A[r * 3 + c] = P[3 * c + r];
    } else {
        // Householder QR of P^T (k x 3): P^T = Q R  =>  P = R^T Q^T, same left singular vectors as R^T
        std::vector<double> M((size_t)k * 3);
        for (int i = 0; i < k; ++i) for (int d = 0; d < 3; ++d) M[(size_t)i * 3 + d] = P[3 * i + d];
        for (int j = 0; j < 3 && j < k; ++j) {
            double nrm = 0;
            for (int i = j; i < k; ++i) nrm += M[i * 3 + j] * M[i * 3 + j];
            nrm = std::sqrt(nrm);
            if (nrm == 0) continue;
            const double alpha = M[j * 3 + j] > 0 ? -nrm : nrm;
            std::vector<double> v(k, 0.0);
            for (int i = j; i < k; ++i) v[i] = M[i * 3 + j];
            v[j] -= alpha;
            double vv = 0;
            for (int i = j; i < k; ++i) vv += v[i] * v[i];
            if (vv == 0) continue;
            for (int c = j; c < 3; ++c) {
                double s = 0;
                for (int i = j; i < k; ++i) s += v[i] * M[i * 3 + c];
                s = 2 * s / vv;
                for (int i = j; i < k; ++i) M[i * 3 + c] -= s * v[i];
            }
        }
        for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) A[r * 3 + c] = (c <= r) ? M[c * 3 + r] : 0.0;  // R^T
    }
    double U[9], S[3], Vv[9];
    jacobi_svd_square<3>(A, U, S, Vv);
    V3 n{U[0 * 3 + 2], U[1 * 3 + 2], U[2 * 3 + 2]};
    const double l = std::sqrt(dot(n, n));
    if (l > 0) n = mul(n, 1.0 / l);
    return n;
}

void project_impl(const Con& c, const std::vector<TriSurface>& surf, const double* in, double* out) {
    const int nc = c.cols();
    switch (c.type) {
        case EDGE: {   // Constraint.h:211-214 (Eigen normalized(): unchanged if |v| == 0)
            V3 v{in[0], in[1], in[2]};
            const double z = dot(v, v);
            if (z > 0) v = mul(v, 1.0 / std::sqrt(z));
            out[0] = v.x * c.prm[0]; out[1] = v.y * c.prm[0]; out[2] = v.z * c.prm[0];
            break;
        }
        case ANGLE: {   // Constraint.h:243-291
            for (int i = 0; i < 6; ++i) out[i] = in[i];
            const double min_a = std::max(0.0, c.prm[0]), max_a = std::min(M_PI, c.prm[1]);
            const double min_cos = std::min(std::max(std::cos(min_a), -1.0), 1.0);
            const double max_cos = std::min(std::max(std::cos(max_a), -1.0), 1.0);
            const V3 v1{in[0], in[1], in[2]}, v2{in[3], in[4], in[5]};
            const double eps = 1e-14;
            const double v1s = dot(v1, v1), v2s = dot(v2, v2);
            const double v1n = std::sqrt(v1s), v2n = std::sqrt(v2s);
            const V3 u1 = v1s > 0 ? mul(v1, 1.0 / std::sqrt(v1s)) : v1;
            const V3 u2 = v2s > 0 ? mul(v2, 1.0 / std::sqrt(v2s)) : v2;
            const double cg = std::min(std::max(dot(u1, u2), -1.0), 1.0);
            if ((1.0 - std::fabs(cg) > eps) && (cg > min_cos || cg < max_cos)) {
                const double gamma = std::acos(cg);
                double eta = cg > min_cos ? (min_a - gamma) : (gamma - max_a);
                eta = std::max(eta, 0.0);
                double theta = 0.5 * std::atan2(v2s * std::sin(2 * eta), v1s + v2s * std::cos(2 * eta));
                theta = std::max(0.0, std::min(eta, theta));
                const double phi = eta - theta;
                V3 w3 = sub(u2, mul(u1, cg)), w4 = sub(u1, mul(u2, cg));
                double l3 = dot(w3, w3), l4 = dot(w4, w4);
                if (l3 > 0) w3 = mul(w3, 1.0 / std::sqrt(l3));
                if (l4 > 0) w4 = mul(w4, 1.0 / std::sqrt(l4));
                if (cg > min_cos) { w3 = mul(w3, -1.0); w4 = mul(w4, -1.0); }
                const V3 p1 = mul(add(mul(u1, std::cos(theta)), mul(w3, std::sin(theta))), v1n * std::cos(theta));
                const V3 p2 = mul(add(mul(u2, std::cos(phi)), mul(w4, std::sin(phi))), v2n * std::cos(phi));
                out[0] = p1.x; out[1] = p1.y; out[2] = p1.z;
                out[3] = p2.x; out[4] = p2.y; out[5] = p2.z;
            }
            break;
        }
        case PLANE: {   // Constraint.h:405-413
            const V3 n = plane_normal(in, nc);
            for (int i = 0; i < nc; ++i) {
                const V3 p{in[3 * i], in[3 * i + 1], in[3 * i + 2]};
                const V3 q = sub(p, mul(n, dot(n, p)));
                out[3 * i] = q.x; out[3 * i + 1] = q.y; out[3 * i + 2] = q.z;
            }
            break;
        }
        case POINT_TO_REF:
        case REF_SURFACE: {   // Constraint.h:340-345, 377-383
            for (int i = 0; i < nc; ++i) {
                const V3 q = surf[c.surf].closest({in[3 * i], in[3 * i + 1], in[3 * i + 2]});
                out[3 * i] = q.x; out[3 * i + 1] = q.y; out[3 * i + 2] = q.z;
            }
            break;
        }
        default:   // CLOSENESS (identity: Constraint.h:319-322 overrides a non-virtual name) and base
            for (int i = 0; i < 3 * nc; ++i) out[i] = in[i];
    }
}

// Constraint::project (Constraint.h:96-116)
void project(const Con& c, const std::vector<TriSurface>& surf, const double* Dx, double* z, bool weighted) {
    const size_t o = 3 * (size_t)c.idO;
    project_impl(c, surf, Dx + o, z + o);
    if (weighted)
        for (int i = 0; i < 3 * c.cols(); ++i) z[o + i] *= c.sw;
}

// Constraint::add_constraint (Constraint.h:132-159) as (row, point, coef) triplets
void add_rows(Con& c, bool weighted, int& idO, std::vector<std::vector<std::pair<int, double>>>& rows) {
    c.idO = idO;
    const double w = weighted ? c.sw : 1.0;
    const int k = c.k;
    if (c.transform == MEAN_CENTERING) {
        const double c1 = (1.0 - 1.0 / k) * w, c2 = -w / k;
        for (int i = 0; i < k; ++i) {
            std::vector<std::pair<int, double>> r;
            for (int j = 0; j < k; ++j) r.push_back({c.idx[j], i == j ? c1 : c2});
            rows.push_back(r); ++idO;
        }
    } else if (c.transform == SUBTRACT_FIRST) {
        for (int i = 1; i < k; ++i) { rows.push_back({{c.idx[0], -w}, {c.idx[i], w}}); ++idO; }
    } else {
        for (int i = 0; i < k; ++i) { rows.push_back({{c.idx[i], w}}); ++idO; }
    }
}

struct Reader {
    FILE* f;
    template <typename T> T get() {
        T v;
        if (fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("scene: short read");
        return v;
    }
    template <typename T> void arr(std::vector<T>& out, size_t n) {
        out.resize(n);
        if (n && fread(out.data(), sizeof(T), n, f) != n) throw std::runtime_error("scene: short read");
    }
};

// GeometrySolver<3>::solve_ADMM (Geometry/GeometrySolver.h:153-252) + ADMM_init_variables
// (:356-382) and the private updates (:423-461). D = [D_hard ; D_soft] (unweighted rows).
int run_plain(std::vector<Con>& hard, std::vector<Con>& soft, const std::vector<TriSurface>& surf,
              const std::vector<std::vector<std::pair<int, double>>>& Dh,
              const std::vector<std::vector<std::pair<int, double>>>& Ds, const std::vector<double>& rhs_fixed,
              const std::vector<int>& perm, Envelope& chol, int n, double rho, int max_iter, int m,
              const std::vector<double>& x0, const char* out_path, double setup_s) {
    const int Zh = 3 * (int)Dh.size(), Z = Zh + 3 * (int)Ds.size();
    std::vector<double> x1(x0), x2(x0), u1(Z, 0.0), u2(Z, 0.0), Dx(Z), Dxu(Z), z(Z), b(3 * (size_t)n);
    std::vector<double>*cx = &x1, *dx = &x2, *cu = &u1, *du = &u2;
    auto compute_Dx = [&](const std::vector<double>& x) {
        for (auto& c : hard) apply_transform(c, x.data(), Dx.data());
        for (auto& c : soft) { Con cc = c; cc.idO += Zh / 3; apply_transform(cc, x.data(), Dx.data()); }
    };
    auto z_update = [&]() {
        for (int i = 0; i < Z; ++i) Dxu[i] = Dx[i] + (*cu)[i];
        for (auto& c : hard) project(c, surf, Dxu.data(), z.data(), false);
        for (auto& c : soft) {   // project_and_combine (Constraint.h:118-130)
            Con cc = c; cc.idO += Zh / 3;
            project(cc, surf, Dxu.data(), z.data(), false);
            const double w = c.sw * c.sw, a = rho / (w + rho);
            const size_t o = 3 * (size_t)cc.idO;
            for (int i = 0; i < 3 * c.cols(); ++i) z[o + i] = Dxu[o + i] * a + z[o + i] * (1 - a);
        }
    };
    auto x_update = [&]() {   // default_x = A^-1 (rhs_fixed + rho D^T (z - u))
        b = rhs_fixed;
        int row = 0;
        for (auto* D : {&Dh, &Ds})
            for (auto& rr : *D) {
                for (auto& e : rr)
                    for (int d = 0; d < 3; ++d) b[3 * (size_t)e.first + d] += rho * e.second * (z[3 * (size_t)row + d] - (*cu)[3 * (size_t)row + d]);
                ++row;
            }
        std::vector<double> bp(3 * (size_t)n);
        for (int i = 0; i < n; ++i) for (int d = 0; d < 3; ++d) bp[3 * (size_t)perm[i] + d] = b[3 * (size_t)i + d];
        chol.solve3(bp.data());
        for (int i = 0; i < n; ++i) for (int d = 0; d < 3; ++d) (*dx)[3 * (size_t)i + d] = bp[3 * (size_t)perm[i] + d];
    };
    auto u_update = [&]() { for (int i = 0; i < Z; ++i) (*du)[i] = (*cu)[i] + Dx[i] - z[i]; };
    auto residual = [&]() { double s = 0; for (int i = 0; i < Z; ++i) { const double r = Dx[i] - z[i]; s += r * r; } return std::sqrt(s); };
    // ADMM_init_variables
    compute_Dx(*cx); z_update(); x_update(); compute_Dx(*dx); u_update();
    *cx = *dx; *cu = *du;
    Anderson aa;
    std::vector<double> g((size_t)Z + 3 * (size_t)n), o(g.size());
    auto pack = [&](const std::vector<double>& u, const std::vector<double>& x) {
        std::copy(u.begin(), u.end(), g.begin());
        std::copy(x.begin(), x.end(), g.begin() + Z);
    };
    if (m > 0) { pack(*cu, *cx); aa.init(m, (int)g.size(), Z, g.data()); }
    std::vector<double> comb_hist, time_hist;
    double prev = std::numeric_limits<double>::max();
    int iter_count = 0, x_updates = 0;
    auto tl = std::chrono::steady_clock::now();
    for (;;) {
        z_update();
        double cur = residual();
        if (m > 0 && cur > prev) {   // swap to the un-accelerated iterate, accelerator->replace
            std::swap(cx, dx); std::swap(cu, du);
            pack(*cu, *cx); aa.replace(g.data());
            compute_Dx(*cx); z_update(); cur = residual();
        }
        ++iter_count;
        comb_hist.push_back(cur);
        time_hist.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - tl).count());
        if (iter_count >= max_iter) break;
        prev = cur;
        x_update(); ++x_updates;
        compute_Dx(*dx);
        u_update();
        if (m > 0) {
            pack(*du, *dx);
            aa.compute(g.data(), o.data());
            std::copy(o.begin(), o.begin() + Z, cu->begin());
            std::copy(o.begin() + Z, o.end(), cx->begin());
        } else { std::swap(du, cu); std::swap(dx, cx); }
        compute_Dx(*cx);
    }
    const double loop_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tl).count();
    FILE* o2 = fopen(out_path, "wb");
    if (!o2) throw std::runtime_error("cannot open output");
    fwrite("AAGEOMR1", 1, 8, o2);
    const int nrec = (int)comb_hist.size();
    fwrite(&nrec, 4, 1, o2);
    fwrite(comb_hist.data(), 8, nrec, o2);
    fwrite(time_hist.data(), 8, nrec, o2);
    fwrite(cx->data(), 8, 3 * (size_t)n, o2);   // get_solution() = *current_x_ (GeometrySolver.h:254-256)
    fwrite(&setup_s, 8, 1, o2);
    fwrite(&loop_s, 8, 1, o2);
    fwrite(&x_updates, 4, 1, o2);
    fclose(o2);
    return 0;
}

// plain = true: GeometrySolver<3> (Geometry/GeometrySolver.h:85-263) instead of the ALM solver --
// all constraint rows unweighted and scaled by rho, u on every column, soft constraints
// projected with project_and_combine (Constraint.h:118-130), residual |Dx - z| after the z-update,
// Anderson on (u, x) with u the effective part, `replace` (no history reset) on a residual increase
int run(const char* scene_path, const char* out_path, bool plain) {
    FILE* f = fopen(scene_path, "rb");
    if (!f) throw std::runtime_error("cannot open scene");
    Reader r{f};
    char magic[8];
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "AAGEOM01", 8) != 0) throw std::runtime_error("bad magic");
    const int n = r.get<int>();
    std::vector<double> x0, refp;
    r.arr(x0, 3 * (size_t)n);
    r.arr(refp, 3 * (size_t)n);
    const int n_surf = r.get<int>();
    std::vector<TriSurface> surf(n_surf);
    for (auto& s : surf) {
        const int nv = r.get<int>(), nf = r.get<int>();
        r.arr(s.V, 3 * (size_t)nv);
        r.arr(s.F, 3 * (size_t)nf);
        s.init();
    }
    std::vector<Con> hard, soft;
    const int n_groups = r.get<int>();
    for (int gi = 0; gi < n_groups; ++gi) {
        const int is_hard = r.get<int>(), type = r.get<int>(), k = r.get<int>(), count = r.get<int>();
        const double weight = r.get<double>();
        const int npar = r.get<int>();
        std::vector<int> idx;
        std::vector<double> prm;
        r.arr(idx, (size_t)count * k);
        r.arr(prm, (size_t)count * npar);
        auto mk = [&](int c, int kk, const int* id) {
            Con con;
            con.type = type; con.k = kk; con.sw = std::sqrt(weight);
            con.transform = type == PLANE ? MEAN_CENTERING : (type == ANGLE || type == EDGE) ? SUBTRACT_FIRST : IDENTITY;
            for (int j = 0; j < 3; ++j) con.prm[j] = j < npar ? prm[(size_t)c * npar + j] : 0.0;
            con.surf = (type == POINT_TO_REF || type == REF_SURFACE) ? (int)con.prm[0] : -1;
            con.idx.assign(id, id + kk);
            (is_hard ? hard : soft).push_back(con);
        };
        if (type == REF_SURFACE) mk(0, count, idx.data());   // one constraint over all points
        else for (int c = 0; c < count; ++c) mk(c, k, &idx[(size_t)c * k]);
    }
    // regularisation rows (LinearRegularization.h:47-117)
    struct Reg { std::vector<int> idx; std::vector<double> coef; double tgt[3]; };
    std::vector<Reg> regs;
    const int n_reg = r.get<int>();
    for (int i = 0; i < n_reg; ++i) {
        const int kind = r.get<int>(), k = r.get<int>();
        const double w = r.get<double>();
        std::vector<int> idx;
        std::vector<double> coef, tgt;
        r.arr(idx, k);
        r.arr(coef, k);
        r.arr(tgt, 3);
        Reg g;
        const double sw = std::sqrt(w);
        g.idx = idx;
        g.tgt[0] = g.tgt[1] = g.tgt[2] = 0;
        if (kind == 2) {
            g.coef = {sw};
            for (int d = 0; d < 3; ++d) g.tgt[d] = tgt[d] * sw;
        } else {
            for (int j = 0; j < k; ++j) g.coef.push_back(coef[j] * sw);
            if (kind == 1) {
                double t[3] = {0, 0, 0};
                for (int j = 0; j < k; ++j) for (int d = 0; d < 3; ++d) t[d] += refp[3 * (size_t)idx[j] + d] * coef[j];
                for (int d = 0; d < 3; ++d) g.tgt[d] = t[d] * sw;
            }
        }
        regs.push_back(g);
    }
    const double rho = r.get<double>();
    const int max_iter = r.get<int>(), m = r.get<int>();
    fclose(f);

    auto t0 = std::chrono::steady_clock::now();
    // ---- setup_ADMM
    std::vector<std::vector<std::pair<int, double>>> Dh, Ds;
    int zc = 0, sc = 0;
    for (auto& c : hard) add_rows(c, false, zc, Dh);
    for (auto& c : soft) add_rows(c, !plain, sc, Ds);
    // global = rho Dh^T Dh + Ds^T Ds + L^T L (scalar n x n), rhs_fixed = L^T b
    std::vector<std::vector<std::pair<int, double>>> Arows(n);
    auto accum = [&](const std::vector<std::pair<int, double>>& row, double s) {
        for (auto& a : row) for (auto& b : row) Arows[a.first].push_back({b.first, s * a.second * b.second});
    };
    for (auto& row : Dh) accum(row, rho);
    for (auto& row : Ds) accum(row, plain ? rho : 1.0);
    std::vector<double> rhs_fixed(3 * (size_t)n, 0.0);
    for (auto& g : regs) {
        std::vector<std::pair<int, double>> row;
        for (size_t j = 0; j < g.idx.size(); ++j) row.push_back({g.idx[j], g.coef[j]});
        accum(row, 1.0);
        for (auto& a : row) for (int d = 0; d < 3; ++d) rhs_fixed[3 * (size_t)a.first + d] += a.second * g.tgt[d];
    }
    std::vector<std::vector<int>> adj(n);
    for (int i = 0; i < n; ++i) for (auto& e : Arows[i]) if (e.first != i) adj[i].push_back(e.first);
    for (auto& l : adj) { std::sort(l.begin(), l.end()); l.erase(std::unique(l.begin(), l.end()), l.end()); }
    std::vector<int> order = rcm_order(adj, std::vector<int>(n, 0));
    std::vector<int> perm(n);   // old -> new
    for (int i = 0; i < n; ++i) perm[order[i]] = i;
    Envelope chol;
    chol.n = n;
    chol.first.assign(n, 0);
    for (int i = 0; i < n; ++i) {
        int fi = perm[i];
        for (auto& e : Arows[i]) fi = std::min(fi, perm[e.first]);
        chol.first[perm[i]] = fi;
    }
    chol.start.assign(n + 1, 0);
    for (int i = 0; i < n; ++i) chol.start[i + 1] = chol.start[i] + (size_t)(i - chol.first[i] + 1);
    chol.L.assign(chol.start[n], 0.0);
    for (int i = 0; i < n; ++i)
        for (auto& e : Arows[i]) {
            const int pi = perm[i], pj = perm[e.first];
            if (pj <= pi) chol.at(pi, pj) += e.second;
        }
    chol.factor();
    const int Zh = 3 * zc, Zs = 3 * sc;
    auto t1 = std::chrono::steady_clock::now();

    if (plain) return run_plain(hard, soft, surf, Dh, Ds, rhs_fixed, perm, chol, n, rho, max_iter, m, x0, out_path,
                                std::chrono::duration<double>(t1 - t0).count());
    // ---- solve_ADMM
    const bool accel = m > 0;
    std::vector<double> cur_x(x0), def_x(x0), new_x(3 * (size_t)n), cur_u(Zh, 0.0), def_u(Zh, 0.0), new_u(Zh);
    std::vector<double> Dxh(Zh), Dxs(Zs), zh(Zh), zs(Zs), prev(Zh), b(3 * (size_t)n);
    Anderson aa;
    std::vector<double> g((size_t)Zh + 3 * (size_t)n), o((size_t)Zh + 3 * (size_t)n);
    auto pack = [&](const std::vector<double>& u, const std::vector<double>& x, std::vector<double>& out) {
        std::copy(u.begin(), u.end(), out.begin());
        std::copy(x.begin(), x.end(), out.begin() + Zh);
    };
    if (accel) { pack(cur_u, cur_x, g); aa.init(m, (int)g.size(), (int)g.size(), g.data()); }
    std::vector<double> comb_hist, time_hist;
    double prev_res = std::numeric_limits<double>::max();
    bool reset = false;
    int iter_count = 0;
    auto solve_x = [&](const std::vector<double>& xin) {
        (void)xin;
        // rhs = rhs_fixed + rho Dh^T (zh - u) + Ds^T zs  (ALMGeometrySolver.h:442-450)
        b = rhs_fixed;
        int row = 0;
        for (auto& rr : Dh) {
            for (auto& e : rr) for (int d = 0; d < 3; ++d) b[3 * (size_t)e.first + d] += rho * e.second * (zh[3 * (size_t)row + d] - cur_u[3 * (size_t)row + d]);
            ++row;
        }
        row = 0;
        for (auto& rr : Ds) {
            for (auto& e : rr) for (int d = 0; d < 3; ++d) b[3 * (size_t)e.first + d] += e.second * zs[3 * (size_t)row + d];
            ++row;
        }
        std::vector<double> bp(3 * (size_t)n);
        for (int i = 0; i < n; ++i) for (int d = 0; d < 3; ++d) bp[3 * (size_t)perm[i] + d] = b[3 * (size_t)i + d];
        chol.solve3(bp.data());
        for (int i = 0; i < n; ++i) for (int d = 0; d < 3; ++d) new_x[3 * (size_t)i + d] = bp[3 * (size_t)perm[i] + d];
    };
    int x_updates = 0;
    auto tl = std::chrono::steady_clock::now();
    for (;;) {
        for (auto& c : hard) apply_transform(c, cur_x.data(), Dxh.data());
        for (auto& c : soft) apply_transform(c, cur_x.data(), Dxs.data());
        prev = Dxh;
        for (int i = 0; i < Zh; ++i) Dxh[i] += cur_u[i];
        for (auto& c : hard) project(c, surf, Dxh.data(), zh.data(), false);
        for (auto& c : soft) project(c, surf, Dxs.data(), zs.data(), true);
        solve_x(cur_x);
        ++x_updates;
        for (auto& c : hard) apply_transform(c, new_x.data(), Dxh.data());
        for (int i = 0; i < Zh; ++i) new_u[i] = cur_u[i] + Dxh[i] - zh[i];
        double r1 = 0, r2 = 0;
        for (int i = 0; i < Zh; ++i) { const double a = Dxh[i] - zh[i], c2 = Dxh[i] - prev[i]; r1 += a * a; r2 += c2 * c2; }
        const double res = r1 + r2;
        const bool accept = !accel || reset || res < prev_res;
        if (accept) {
            def_x = new_x; def_u = new_u;
            ++iter_count;
            comb_hist.push_back(res);
            time_hist.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - tl).count());
            prev_res = res;
            reset = false;
            if (accel) {
                pack(new_u, new_x, g);
                aa.compute(g.data(), o.data());
                std::copy(o.begin(), o.begin() + Zh, cur_u.begin());
                std::copy(o.begin() + Zh, o.end(), cur_x.begin());
            } else { cur_u = new_u; cur_x = new_x; }
        } else {
            cur_u = def_u; cur_x = def_x;
            reset = true;
            if (accel) { pack(cur_u, cur_x, g); aa.reset(g.data()); }
        }
        if (iter_count >= max_iter) break;
    }
    auto t2 = std::chrono::steady_clock::now();
    FILE* o2 = fopen(out_path, "wb");
    if (!o2) throw std::runtime_error("cannot open output");
    fwrite("AAGEOMR1", 1, 8, o2);
    const int nrec = (int)comb_hist.size();
    fwrite(&nrec, 4, 1, o2);
    fwrite(comb_hist.data(), 8, nrec, o2);
    fwrite(time_hist.data(), 8, nrec, o2);
    fwrite(def_x.data(), 8, 3 * (size_t)n, o2);
    const double setup_s = std::chrono::duration<double>(t1 - t0).count(), loop_s = std::chrono::duration<double>(t2 - t1).count();
    fwrite(&setup_s, 8, 1, o2);
    fwrite(&loop_s, 8, 1, o2);
    fwrite(&x_updates, 4, 1, o2);
    fclose(o2);
    return 0;
}

}  // namespace
}  // namespace oracle

extern "C" int oracle_geom_run_file(const char* scene_path, const char* out_path, char* err, int err_cap) {
    return oracle_geom_run_file_mode(scene_path, out_path, 0, err, err_cap);
}

extern "C" int oracle_geom_run_file_mode(const char* scene_path, const char* out_path, int plain, char* err,
                                         int err_cap) {
    try {
        return oracle::run(scene_path, out_path, plain != 0);
    } catch (const std::exception& e) {
        if (err && err_cap > 0) { std::strncpy(err, e.what(), err_cap - 1); err[err_cap - 1] = 0; }
        return -1;
    }
}

extern "C" void oracle_closest_point(const double* V, int nv, const int* F, int nf, const double* P, int np, double* out) {
    oracle::TriSurface s;
    s.V.assign(V, V + 3 * (size_t)nv);
    s.F.assign(F, F + 3 * (size_t)nf);
    s.init();
    for (int i = 0; i < np; ++i) {
        const oracle::V3 c = s.closest({P[3 * i], P[3 * i + 1], P[3 * i + 2]});
        out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
    }
}

extern "C" void oracle_geom_project(int type, int k, const double* params, const double* in, double* out) {
    oracle::Con c;
    c.type = type; c.k = k; c.sw = 1.0; c.surf = -1; c.idO = 0;
    c.transform = type == oracle::PLANE ? oracle::MEAN_CENTERING : (type == oracle::ANGLE || type == oracle::EDGE) ? oracle::SUBTRACT_FIRST : oracle::IDENTITY;
    for (int j = 0; j < 3; ++j) c.prm[j] = params ? params[j] : 0.0;
    std::vector<oracle::TriSurface> none;
    oracle::project_impl(c, none, in, out);
}
