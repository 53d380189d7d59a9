// Host orchestration of the Geometry (ALM) hot path (see geom.hpp).
//
// Reference call stack being replaced:
//   ALMGeometrySolver<3>::add_hard_constraint / add_soft_constraint / add_*laplacian / add_closeness
//                                              Geometry/ALMGeometrySolver.h:286-318
//   ALMGeometrySolver<3>::setup_ADMM           Geometry/ALMGeometrySolver.h:81-161
//   ALMGeometrySolver<3>::solve_ADMM           Geometry/ALMGeometrySolver.h:163-283
// Every ALM iteration is enqueued on one HIP stream; the accept/reject decision of the
// reference (comb < prev, reset, Anderson reset) is taken by a device control kernel that
// gates the following kernels, so the loop runs as replays of captured hipGraphs with one
// host synchronisation per launch of the passes still needed (GeomSolver::solve).
#include "geom.hpp"

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>

#include "dense_gpu.hpp"
#include "spd_direct.hpp"

namespace aa {

namespace {

int n_params(int type) {
    switch (type) {
        case GEO_EDGE: return 1;
        case GEO_ANGLE: return 2;
        case GEO_CLOSENESS: return 3;
        case GEO_POINT_TO_REF: case GEO_REF_SURFACE: return 1;
        default: return 0;
    }
}
int cols_of(int type, int K) { return (type == GEO_ANGLE || type == GEO_EDGE) ? K - 1 : K; }

// rows of one constraint's reduction block D_c (cols x K), Constraint::add_constraint
// (Geometry/Constraint.h:132-159), weight w folded in
std::vector<double> reduction_block(int type, int K, double w) {
    const int C = cols_of(type, K);
    std::vector<double> D((size_t)C * K, 0.0);
    if (type == GEO_PLANE) {
        const double c1 = (1.0 - 1.0 / K) * w, c2 = -w / K;
        for (int i = 0; i < K; ++i) for (int j = 0; j < K; ++j) D[(size_t)i * K + j] = i == j ? c1 : c2;
    } else if (type == GEO_ANGLE || type == GEO_EDGE) {
        for (int i = 1; i < K; ++i) { D[(size_t)(i - 1) * K] = -w; D[(size_t)(i - 1) * K + i] = w; }
    } else {
        for (int i = 0; i < K; ++i) D[(size_t)i * K + i] = w;
    }
    return D;
}

// median-split BVH, leaves of <= 4 triangles, depth-first node order
struct BvhBuilder {
    const double* V;
    const int* F;
    std::vector<int> ids;
    std::vector<double> cen;
    std::vector<BvhNode>* nodes;
    std::vector<BvhTri>* tris;
    int leaf = 4;            // triangles per leaf (AA_CP_LEAF, 1..7)
    bool split_t1 = false;   // split along the principal tangent axis (AA_CP_SPLIT=t1)
    static float down(double v) {   // largest float <= v
        float f = (float)v;
        if ((double)f > v) f = std::nextafter(f, -INFINITY);
        return f;
    }
    static float up(double v) {     // smallest float >= v
        float f = (float)v;
        if ((double)f < v) f = std::nextafter(f, INFINITY);
        return f;
    }
    int build(int b, int e) {
        BvhNode nd{};
        double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        double clo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, chi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int i = b; i < e; ++i) {
            const int t = ids[i];
            for (int a = 0; a < 3; ++a)
                for (int d = 0; d < 3; ++d) {
                    const double v = V[3 * (size_t)F[3 * (size_t)t + a] + d];
                    lo[d] = std::min(lo[d], v); hi[d] = std::max(hi[d], v);
                }
            for (int d = 0; d < 3; ++d) { clo[d] = std::min(clo[d], cen[3 * (size_t)t + d]); chi[d] = std::max(chi[d], cen[3 * (size_t)t + d]); }
        }
        for (int d = 0; d < 3; ++d) { nd.lo[d] = down(lo[d]); nd.hi[d] = up(hi[d]); }
        {   // slab: area-weighted mean normal of the subtree, range of n . v over its vertices
            double N[3] = {0, 0, 0};
            for (int i = b; i < e; ++i) {
                const double* A = V + 3 * (size_t)F[3 * (size_t)ids[i]];
                const double* Bv = V + 3 * (size_t)F[3 * (size_t)ids[i] + 1];
                const double* C = V + 3 * (size_t)F[3 * (size_t)ids[i] + 2];
                const double u[3] = {Bv[0] - A[0], Bv[1] - A[1], Bv[2] - A[2]}, w[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
                N[0] += u[1] * w[2] - u[2] * w[1]; N[1] += u[2] * w[0] - u[0] * w[2]; N[2] += u[0] * w[1] - u[1] * w[0];
            }
            const double l = std::sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
            for (int d = 0; d < 3; ++d) nd.nrm[d] = l > 0 ? (float)(N[d] / l) : 0.0f;
            double dl = DBL_MAX, dh = -DBL_MAX;
            for (int i = b; i < e; ++i)
                for (int a = 0; a < 3; ++a) {
                    const double* P = V + 3 * (size_t)F[3 * (size_t)ids[i] + a];
                    const double dd = (double)nd.nrm[0] * P[0] + (double)nd.nrm[1] * P[1] + (double)nd.nrm[2] * P[2];
                    dl = std::min(dl, dd); dh = std::max(dh, dd);
                }
            if (l > 0) { nd.dlo = down(dl); nd.dhi = up(dh); }
            else { nd.dlo = -FLT_MAX; nd.dhi = FLT_MAX; }   // degenerate patch: no slab bound
            // tangent axes: the principal directions of the vertices projected on the plane
            // normal to the (fp32) n, then their ranges (AA_CP_OBB=0: unbounded, slab only)
            for (int d = 0; d < 3; ++d) { nd.t1[d] = nd.t2[d] = 0.0f; }
            nd.t1lo = nd.t2lo = -FLT_MAX; nd.t1hi = nd.t2hi = FLT_MAX;
            static const bool obb = !(std::getenv("AA_CP_OBB") && std::getenv("AA_CP_OBB")[0] == '0');
            if (l > 0 && obb) {
                const double n[3] = {nd.nrm[0], nd.nrm[1], nd.nrm[2]};
                const double nl = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                const double nn[3] = {n[0] / nl, n[1] / nl, n[2] / nl};
                // any unit e1 normal to n, e2 = n x e1
                const int k = std::fabs(nn[0]) < 0.6 ? 0 : (std::fabs(nn[1]) < 0.6 ? 1 : 2);
                double e1[3] = {0, 0, 0};
                e1[k] = 1.0;
                const double pr = e1[0] * nn[0] + e1[1] * nn[1] + e1[2] * nn[2];
                for (int d = 0; d < 3; ++d) e1[d] -= pr * nn[d];
                const double el = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
                for (int d = 0; d < 3; ++d) e1[d] /= el;
                const double e2[3] = {nn[1] * e1[2] - nn[2] * e1[1], nn[2] * e1[0] - nn[0] * e1[2], nn[0] * e1[1] - nn[1] * e1[0]};
                double m1 = 0, m2 = 0, c11 = 0, c22 = 0, c12 = 0, cnt = 0;
                for (int i = b; i < e; ++i)
                    for (int a = 0; a < 3; ++a) {
                        const double* P = V + 3 * (size_t)F[3 * (size_t)ids[i] + a];
                        const double x1 = e1[0] * P[0] + e1[1] * P[1] + e1[2] * P[2], x2 = e2[0] * P[0] + e2[1] * P[1] + e2[2] * P[2];
                        m1 += x1; m2 += x2; c11 += x1 * x1; c22 += x2 * x2; c12 += x1 * x2; cnt += 1;
                    }
                m1 /= cnt; m2 /= cnt;
                c11 = c11 / cnt - m1 * m1; c22 = c22 / cnt - m2 * m2; c12 = c12 / cnt - m1 * m2;
                const double th = 0.5 * std::atan2(2.0 * c12, c11 - c22);
                const double a1[3] = {std::cos(th) * e1[0] + std::sin(th) * e2[0], std::cos(th) * e1[1] + std::sin(th) * e2[1],
                                      std::cos(th) * e1[2] + std::sin(th) * e2[2]};
                const double a2[3] = {nn[1] * a1[2] - nn[2] * a1[1], nn[2] * a1[0] - nn[0] * a1[2], nn[0] * a1[1] - nn[1] * a1[0]};
                for (int d = 0; d < 3; ++d) { nd.t1[d] = (float)a1[d]; nd.t2[d] = (float)a2[d]; }
                double l1 = DBL_MAX, h1 = -DBL_MAX, l2 = DBL_MAX, h2 = -DBL_MAX;
                for (int i = b; i < e; ++i)
                    for (int a = 0; a < 3; ++a) {
                        const double* P = V + 3 * (size_t)F[3 * (size_t)ids[i] + a];
                        const double x1 = (double)nd.t1[0] * P[0] + (double)nd.t1[1] * P[1] + (double)nd.t1[2] * P[2];
                        const double x2 = (double)nd.t2[0] * P[0] + (double)nd.t2[1] * P[1] + (double)nd.t2[2] * P[2];
                        l1 = std::min(l1, x1); h1 = std::max(h1, x1); l2 = std::min(l2, x2); h2 = std::max(h2, x2);
                    }
                nd.t1lo = down(l1); nd.t1hi = up(h1); nd.t2lo = down(l2); nd.t2hi = up(h2);
            }
        }
        const int me = (int)nodes->size();
        if (me >= (1 << 29)) throw Error(ERR_ARG, "add_ref_surface: too many BVH nodes");
        nodes->push_back(nd);
        if (e - b <= leaf) {
            (*nodes)[me].a = (int)tris->size();
            (*nodes)[me].sn = (unsigned)(me + 1) | ((unsigned)(e - b) << 29);
            for (int i = b; i < e; ++i) {
                BvhTri tr;
                for (int a = 0; a < 3; ++a)
                    for (int d = 0; d < 3; ++d) tr.v[3 * a + d] = V[3 * (size_t)F[3 * (size_t)ids[i] + a] + d];
                tris->push_back(tr);
            }
            return me;
        }
        const int mid = (b + e) / 2;
        if (split_t1 && (nd.t1hi - nd.t1lo) < FLT_MAX) {   // median along the principal tangent axis
            const double a1[3] = {nd.t1[0], nd.t1[1], nd.t1[2]};
            auto key = [&](int p) { return a1[0] * cen[3 * (size_t)p] + a1[1] * cen[3 * (size_t)p + 1] + a1[2] * cen[3 * (size_t)p + 2]; };
            std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e, [&](int p, int q) { return key(p) < key(q); });
        } else {   // median along the longest axis of the centroids' box
            int ax = 0;
            for (int d = 1; d < 3; ++d) if (chi[d] - clo[d] > chi[ax] - clo[ax]) ax = d;
            std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e,
                             [&](int p, int q) { return cen[3 * (size_t)p + ax] < cen[3 * (size_t)q + ax]; });
        }
        build(b, mid);
        const int r = build(mid, e);
        (*nodes)[me].a = r;
        (*nodes)[me].sn = (unsigned)nodes->size();
        return me;
    }
};

// The BVH collapsed to G children per node (layout: SurfDev::wide). Returns the number of
// wide levels below the root (the group traversal's stack holds at most (G - 1) per level).
int build_wide(const std::vector<BvhNode>& N, int G, std::vector<BvhNode>& W) {
    W.clear();
    int depth = 0;
    // descendants of n log2(G) levels down, left to right; a leaf met earlier stands for itself
    auto expand = [&](int n) {
        std::vector<int> c{n};
        for (int l = 1; l < G; l <<= 1) {
            std::vector<int> nx;
            for (int i : c) {
                if (bvh_count(N[i]) > 0) nx.push_back(i);
                else { nx.push_back(i + 1); nx.push_back(N[i].a); }
            }
            c.swap(nx);
        }
        return c;
    };
    std::function<int(int, int)> make = [&](int n, int level) -> int {
        const int w = (int)(W.size() / G);
        W.resize(W.size() + G);
        depth = std::max(depth, level);
        const std::vector<int> c = expand(n);
        for (int k = 0; k < G; ++k) {
            BvhNode r{};
            r.a = -1;
            if (k < (int)c.size()) {
                r = N[c[k]];
                if (bvh_count(r) > 0) r.sn = (unsigned)bvh_count(r) << 29;
                else { r.sn = 0; r.a = make(c[k], level + 1); }
            }
            W[(size_t)w * G + k] = r;
        }
        return w;
    };
    if (!N.empty()) make(0, 1);
    return depth;
}

}  // namespace

GeomSolver::~GeomSolver() {
    drop_graph();
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    if (side_) (void)hipStreamDestroy(side_);
    for (auto& kv : kstats_)
        for (auto e : kv.second.ev) (void)hipEventDestroy(e);
}

void GeomSolver::drop_graph() {
    for (int i = 0; i < kNChunks; ++i) {
        if (gexec_[i]) (void)hipGraphExecDestroy(gexec_[i]);
        if (graph_[i]) (void)hipGraphDestroy(graph_[i]);
        gexec_[i] = nullptr;
        graph_[i] = nullptr;
    }
}

int GeomSolver::add_ref_surface(const double* V3, int nv, const int* F3, int nf) {
    if (nv <= 0 || nf <= 0 || !V3 || !F3) throw Error(ERR_ARG, "add_ref_surface: empty surface");
    for (long long i = 0; i < 3LL * nf; ++i)
        if (F3[i] < 0 || F3[i] >= nv) throw Error(ERR_ARG, "add_ref_surface: face index out of range");
    Surface S;
    BvhBuilder B;
    B.V = V3; B.F = F3;
    B.ids.resize(nf);
    std::iota(B.ids.begin(), B.ids.end(), 0);
    B.cen.resize(3 * (size_t)nf);
    for (int t = 0; t < nf; ++t)
        for (int d = 0; d < 3; ++d)
            B.cen[3 * (size_t)t + d] = (V3[3 * (size_t)F3[3 * t] + d] + V3[3 * (size_t)F3[3 * t + 1] + d] + V3[3 * (size_t)F3[3 * t + 2] + d]) / 3.0;
    B.nodes = &S.nodes;
    B.tris = &S.tris;
    if (const char* ev = std::getenv("AA_CP_LEAF")) B.leaf = std::min(7, std::max(1, std::atoi(ev)));
    if (const char* ev = std::getenv("AA_CP_SPLIT")) B.split_t1 = std::string(ev) == "t1";
    S.nodes.reserve(nf);
    S.tris.reserve(nf);
    B.build(0, nf);
    S.dnodes.upload(S.nodes, s());
    S.dtris.upload(S.tris, s());
    {   // group traversal (AA_CP_GROUP = lanes per query: 4 or 8; 0 = one lane per query)
        const char* ev = std::getenv("AA_CP_GROUP");
        const int G = ev ? std::atoi(ev) : 4;
        if (G == 4 || G == 8) {
            const int depth = build_wide(S.nodes, G, S.wide);
            if ((G - 1) * depth <= kCpStack) {
                S.wide_g = G;
                S.dwide.upload(S.wide, s());
            } else {
                S.wide.clear();   // too deep for the stack: one lane per query
            }
        }
    }
    AA_HIP(hipStreamSynchronize(s()));
    surfs_.push_back(std::move(S));
    return (int)surfs_.size() - 1;
}

// add_hard_constraint / add_soft_constraint of `count` constraints of one type
// (ALMGeometrySolver.h:286-294; constructors Constraint.h:194-414)
void GeomSolver::add_constraints(int hard, int type, const int* idx, int k, int count, double weight,
                                 const double* params) {
    if (setup_done_) throw Error(ERR_STATE, "constraints must be added before setup_ADMM");
    if (count < 0) throw Error(ERR_ARG, "add_constraints: negative count");
    if (count == 0) return;
    if (type < GEO_PLANE || type > GEO_REF_SURFACE) throw Error(ERR_ARG, "add_constraints: unknown constraint type");
    const int want = type == GEO_ANGLE ? 3 : type == GEO_EDGE ? 2 : type == GEO_PLANE ? k : 1;
    if (k != want) throw Error(ERR_ARG, "add_constraints: wrong number of indices for this constraint type");
    if (type == GEO_PLANE && k < 3) throw Error(ERR_ARG, "add_constraints: plane constraints need at least 3 points");
    if (!(weight >= 0.0)) throw Error(ERR_ARG, "add_constraints: weight must be >= 0");
    const int P = n_params(type);
    if (P && !params) throw Error(ERR_ARG, "add_constraints: this constraint type needs parameters");
    if (!idx && type != GEO_REF_SURFACE) throw Error(ERR_ARG, "add_constraints: null indices");
    int surf = -1;
    if (type == GEO_POINT_TO_REF || type == GEO_REF_SURFACE) {
        surf = (int)params[0];
        for (int c = 1; c < count; ++c)
            if ((int)params[(size_t)c * P] != surf) throw Error(ERR_ARG, "add_constraints: one reference surface per call");
        if (surf < 0 || surf >= (int)surfs_.size()) throw Error(ERR_ARG, "add_constraints: unknown reference surface");
    }
    const auto key = std::make_tuple(hard ? 1 : 0, type, k, weight, surf);
    auto it = group_of_.find(key);
    if (it == group_of_.end()) {
        HostGroup g;
        g.hard = hard ? 1 : 0; g.type = type; g.K = k; g.weight = weight; g.surf = surf;
        hgroups_.push_back(g);
        it = group_of_.emplace(key, (int)hgroups_.size() - 1).first;
    }
    HostGroup& g = hgroups_[it->second];
    for (int c = 0; c < count; ++c) {
        for (int a = 0; a < k; ++a) {
            const int v = idx ? idx[(size_t)c * k + a] : c;
            if (v < 0) throw Error(ERR_ARG, "add_constraints: negative point index");
            g.idx.push_back(v);
        }
        for (int p = 0; p < P; ++p) g.prm.push_back(params[(size_t)c * P + p]);
    }
}

// LinearRegularization::add_laplacian_helper (Geometry/LinearRegularization.h:119-141)
void GeomSolver::add_laplacian(const int* idx, const double* coefs, int k, double weight, const double* ref_points3) {
    if (setup_done_) throw Error(ERR_STATE, "regularization must be added before setup_ADMM");
    if (k <= 0 || !idx || !coefs) throw Error(ERR_ARG, "add_laplacian: bad input");
    Reg r;
    const double sw = std::sqrt(weight);
    double t[3] = {0, 0, 0};
    for (int i = 0; i < k; ++i) {
        if (idx[i] < 0) throw Error(ERR_ARG, "add_laplacian: negative point index");
        r.idx.push_back(idx[i]);
        r.coef.push_back(coefs[i] * sw);
        if (ref_points3)
            for (int d = 0; d < 3; ++d) t[d] += ref_points3[3 * (size_t)idx[i] + d] * coefs[i];
    }
    for (int d = 0; d < 3; ++d) r.tgt[d] = t[d] * sw;
    regs_.push_back(r);
}

// LinearRegularization::add_closeness (LinearRegularization.h:75-89)
void GeomSolver::add_closeness(int idx, double weight, const double* target3) {
    if (setup_done_) throw Error(ERR_STATE, "regularization must be added before setup_ADMM");
    if (idx < 0 || !target3) throw Error(ERR_ARG, "add_closeness: bad input");
    Reg r;
    const double sw = std::sqrt(weight);
    r.idx.push_back(idx);
    r.coef.push_back(sw);
    for (int d = 0; d < 3; ++d) r.tgt[d] = target3[d] * sw;
    regs_.push_back(r);
}

// setup_ADMM (ALMGeometrySolver.h:81-161): global = rho D_h^T D_h + D_s^T D_s + L^T L and
// rhs_fixed = L^T b. The factorisation needs point positions for the nested-dissection order,
// so it happens at the first solve (and is reused by later solves).
void GeomSolver::setup(int n_points, double penalty, int spd_solver_type) {
    if (setup_done_) throw Error(ERR_STATE, "setup_ADMM called twice");
    if (n_points <= 0) throw Error(ERR_ARG, "setup_ADMM: n_points must be positive");
    if (hgroups_.empty()) throw Error(ERR_ARG, "setup_ADMM: no constraints");
    if (spd_solver_type != AA_SPD_LDLT && spd_solver_type != AA_SPD_LLT)
        throw Error(ERR_ARG, "setup_ADMM: unsupported SPD solver type");
    auto t0 = std::chrono::steady_clock::now();
    n_ = n_points;
    rho_ = penalty;
    // the reference builds the hard rows, then the soft rows (ALMGeometrySolver.h:97-129) and
    // sums rho D_h^T D_h + D_s^T D_s + L^T L in that order: keep that order whatever the order
    // of the add_*_constraint calls (so the C++ facade and the bindings assemble identically)
    std::stable_partition(hgroups_.begin(), hgroups_.end(), [](const decltype(hgroups_)::value_type& g) { return g.hard; });
    group_of_.clear();
    for (size_t gi = 0; gi < hgroups_.size(); ++gi) {
        const auto& g = hgroups_[gi];
        group_of_.emplace(std::make_tuple(g.hard, g.type, g.K, g.weight, g.surf), (int)gi);
    }
    arows_.assign(n_, {});
    for (auto& g : hgroups_) {
        for (int v : g.idx) if (v >= n_) throw Error(ERR_ARG, "constraint references a point index >= n_points");
        // ALM: soft rows weighted, hard rows x rho; GeometrySolver: every row unweighted, x rho
        // (GeometrySolver.h:100-119)
        const double w = (g.hard || plain_) ? 1.0 : std::sqrt(g.weight);
        const double scale = (g.hard || plain_) ? rho_ : 1.0;
        const std::vector<double> D = reduction_block(g.type, g.K, w);
        const int C = cols_of(g.type, g.K), K = g.K;
        std::vector<double> DtD((size_t)K * K, 0.0);
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b) {
                double sacc = 0;
                for (int r = 0; r < C; ++r) sacc += D[(size_t)r * K + a] * D[(size_t)r * K + b];
                DtD[(size_t)a * K + b] = scale * sacc;
            }
        const int cnt = g.count();
        for (int c = 0; c < cnt; ++c) {
            const int* id = &g.idx[(size_t)c * K];
            for (int a = 0; a < K; ++a)
                for (int b = 0; b < K; ++b)
                    if (DtD[(size_t)a * K + b] != 0.0) arows_[id[a]].push_back({id[b], DtD[(size_t)a * K + b]});
        }
    }
    rhs_fixed_user_.assign(3 * (size_t)n_, 0.0);
    for (auto& r : regs_) {
        for (int v : r.idx) if (v >= n_) throw Error(ERR_ARG, "regularization references a point index >= n_points");
        for (size_t a = 0; a < r.idx.size(); ++a) {
            for (size_t b = 0; b < r.idx.size(); ++b) arows_[r.idx[a]].push_back({r.idx[b], r.coef[a] * r.coef[b]});
            for (int d = 0; d < 3; ++d) rhs_fixed_user_[3 * (size_t)r.idx[a] + d] += r.coef[a] * r.tgt[d];
        }
    }
    for (int i = 0; i < n_; ++i) {
        auto& row = arows_[i];
        std::stable_sort(row.begin(), row.end(), [](const std::pair<int, double>& a, const std::pair<int, double>& b) { return a.first < b.first; });
        size_t w = 0;
        for (size_t k = 0; k < row.size();) {
            size_t k2 = k;
            double v = 0;
            while (k2 < row.size() && row[k2].first == row[k].first) v += row[k2++].second;
            row[w++] = {row[k].first, v};
            k = k2;
        }
        row.resize(w);
        bool diag = false;
        for (auto& e : row) if (e.first == i && e.second > 0) diag = true;
        if (!diag) throw Error(ERR_NUMERIC, "Error: SPD solver initialization failed (a point has no constraint)");
    }
    setup_done_ = true;
    factored_ = false;
    rt_ = aa_geom_runtime{};
    rt_.n_points = n_;
    rt_.setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void GeomSolver::set_comm(Comm* c) {
    if (factored_) throw Error(ERR_STATE, "set_comm after the first solve_ADMM is not supported");
    comm_ = c;
    rank_ = c ? c->rank() : 0;
}

void GeomSolver::factor_and_upload(const double* init_x3) {
    auto t0 = std::chrono::steady_clock::now();
    drop_graph();
    // nested-dissection order over the matrix graph, bisected on the initial point positions
    std::vector<int> aptr(n_ + 1, 0), aj;
    const bool parted = comm_ && comm_->size() > 1;
    std::vector<std::vector<int>> cl;
    if (parted) {
        // partitioned: every constraint's points must land in one part (plus separators), but
        // D^T D need not couple them all (an angle constraint's two side points have no matrix
        // entry): dissect the graph with each constraint's points made a clique. Separators of
        // this supergraph also separate the matrix graph, so the tree stays a valid elimination
        // order for the factor.
        cl.resize(n_);
        for (auto& g : hgroups_)
            for (int c = 0; c < g.count(); ++c)
                for (int a = 0; a < g.K; ++a)
                    for (int b = 0; b < g.K; ++b)
                        if (a != b) cl[g.idx[(size_t)c * g.K + a]].push_back(g.idx[(size_t)c * g.K + b]);
    }
    for (int i = 0; i < n_; ++i) {
        const size_t s0 = aj.size();
        for (auto& e : arows_[i]) if (e.first != i) aj.push_back(e.first);
        if (parted) {
            aj.insert(aj.end(), cl[i].begin(), cl[i].end());
            std::sort(aj.begin() + s0, aj.end());
            aj.erase(std::unique(aj.begin() + s0, aj.end()), aj.end());
            std::vector<int>().swap(cl[i]);
        }
        aptr[i + 1] = (int)aj.size();
    }
    // partitioned: the top bisections (P parts) are forced; part r (a contiguous
    // range of points) belongs to rank r, the separators ("top") are shared
    const int P = comm_ ? comm_->size() : 1;
    // the shared top separators as one dense root split over the ranks (AA_TOP_DENSE=0: one
    // supernode per separator, replicated on every rank -- the round-1 layout)
    const bool top_dense = !(std::getenv("AA_TOP_DENSE") && std::getenv("AA_TOP_DENSE")[0] == '0');
    // ... and each part's own upper levels amalgamated into one dense supernode of up to this many
    // rows (AA_PART_TOP_ROWS)
    const int part_top_rows = std::getenv("AA_PART_TOP_ROWS") ? std::atoi(std::getenv("AA_PART_TOP_ROWS"))
                                                              : DirectSolver::kPartTopRows;
    const int nd_leaf = default_nd_leaf(n_);
    if (P > 1) {   // every rank must have been handed the same problem
        double h[4] = {(double)n_, (double)hgroups_.size(), 0, 0};
        for (auto& g : hgroups_) h[2] += (double)g.idx.size();
        for (int i = 0; i < 3 * n_; ++i) h[3] += init_x3[i];
        double r[4] = {h[0], h[1], h[2], h[3]};
        comm_->allreduce_sum_host(r, 4);
        for (int i = 0; i < 4; ++i)
            if (std::fabs(r[i] - P * h[i]) > 1e-12 * std::fabs(P * h[i]))
                throw Error(ERR_ARG, "solve_ADMM: the ranks were given different problems");
    }
    NdTree tree = nested_dissection(n_, init_x3, aptr, aj, nd_leaf, P > 1 ? 0 : DirectSolver::top_rows(n_), P > 1 ? P : 0, top_dense,
                                     part_top_rows);
    top_beg_ = P > 1 ? tree.top_beg : n_;
    own_beg_ = P > 1 ? tree.part_beg[rank_] : 0;
    own_end_ = P > 1 ? tree.part_end[rank_] : n_;
    int2user_ = tree.perm;
    user2int_.assign(n_, -1);
    for (int q = 0; q < n_; ++q) user2int_[int2user_[q]] = q;
    CsrMatrix A;
    A.n = n_;
    A.ptr.assign(n_ + 1, 0);
    for (int q = 0; q < n_; ++q) {
        std::vector<std::pair<int, double>> r;
        for (auto& e : arows_[int2user_[q]]) r.push_back({user2int_[e.first], e.second});
        std::sort(r.begin(), r.end(), [](const std::pair<int, double>& a, const std::pair<int, double>& b) { return a.first < b.first; });
        for (auto& e : r) { A.col.push_back(e.first); A.val.push_back(e.second); }
        A.ptr[q + 1] = (int)A.col.size();
    }
    SupernodalFactor F;
    try {
        auto pf = make_part_factor(P > 1 ? comm_ : nullptr, rank_, s());   // no rank factors another's part
        F = factor_on_device(A, tree, s(), pf.get());
    } catch (const Error&) {
        throw;   // device / allocation failures keep their own status
    } catch (const std::runtime_error& e) {
        throw Error(ERR_NUMERIC, std::string("Error: SPD solver initialization failed: ") + e.what());
    }
    // surface meshes: their supernodes above the subtree cut are small and many, split-K tiles
    // from p > 64 / R > 128 on (C3 solve 375 -> 270 us, C5 695 -> 559 us; the elastic 3D and
    // cloth configs are faster with the default thresholds)
    solver_.build(F, s(), P > 1 ? &tree.part : nullptr, rank_, top_beg_, comm_, 1, false, 64, 128);
    rt_.nnz_factor = (long long)F.nnz_L;

    // constraint ownership (partitioned): a constraint touching a point of part r belongs to
    // rank r (it cannot touch another part); constraints on separator points only go
    // round-robin. Every rank computes the same assignment.
    std::vector<HostGroup> owned;
    nbg_ = 0;
    long long zhmax = 0;
    if (P > 1) {
        std::vector<int> qpart(n_, -1);
        for (int r = 0; r < P; ++r) for (int q = tree.part_beg[r]; q < tree.part_end[r]; ++q) qpart[q] = r;
        std::vector<long long> zr(P, 0);
        std::vector<int> br(P, 0);
        long long rr = 0;
        for (auto& hg : hgroups_) {
            const int cnt = hg.count(), K = hg.K, Pn = n_params(hg.type), C = cols_of(hg.type, K);
            std::vector<int> c(P, 0);
            HostGroup lg = hg;
            lg.idx.clear(); lg.prm.clear();
            for (int e = 0; e < cnt; ++e) {
                int o = -1;
                for (int a = 0; a < K && o < 0; ++a) o = qpart[user2int_[hg.idx[(size_t)e * K + a]]];
                if (o < 0) o = (int)(rr++ % P);
                ++c[o];
                if (o != rank_) continue;
                lg.idx.insert(lg.idx.end(), hg.idx.begin() + (size_t)e * K, hg.idx.begin() + (size_t)(e + 1) * K);
                lg.prm.insert(lg.prm.end(), hg.prm.begin() + (size_t)e * Pn, hg.prm.begin() + (size_t)(e + 1) * Pn);
            }
            if (has_u(hg))
                for (int r = 0; r < P; ++r) { br[r] += geo_u_blocks(c[r]); zr[r] += 3LL * C * c[r]; }
            owned.push_back(std::move(lg));
        }
        for (int r = 0; r < P; ++r) { nbg_ = std::max(nbg_, br[r]); zhmax = std::max(zhmax, zr[r]); }
    }
    const std::vector<HostGroup>& dgroups = P > 1 ? owned : hgroups_;

    // device constraint groups (internal point ids), z/u offsets, rhs slots
    groups_.clear();
    groups_.resize(dgroups.size());
    Zh_ = 0; slots_ = 0; red_blocks_ = 0;
    std::vector<std::vector<int>> pslots(n_);
    long long soft_cols = 0, ncons = 0;
    for (size_t gi = 0; gi < dgroups.size(); ++gi) {
        const HostGroup& hg = dgroups[gi];
        DevGroup& dg = groups_[gi];
        const int cnt = hg.count(), K = hg.K, P = n_params(hg.type), C = cols_of(hg.type, K);
        std::vector<int> idx((size_t)K * cnt);
        std::vector<double> prm((size_t)std::max(P, 1) * cnt, 0.0);
        // reference-surface groups run in the nested-dissection order of their points: a wave's
        // 64 queries then sit in one compact patch and their BVH traversals share most nodes
        // (in the caller's order a wave spans a long strip of the mesh)
        std::vector<int> ord(cnt);
        std::iota(ord.begin(), ord.end(), 0);
        if ((hg.type == GEO_POINT_TO_REF || hg.type == GEO_REF_SURFACE) && nd_sort_surf_)
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
                return user2int_[hg.idx[(size_t)a * K]] < user2int_[hg.idx[(size_t)b * K]];
            });
        for (int ee = 0; ee < cnt; ++ee) {
            const int e = ord[ee];
            for (int a = 0; a < K; ++a) {
                const int q = user2int_[hg.idx[(size_t)e * K + a]];
                idx[(size_t)a * cnt + ee] = q;
                pslots[q].push_back((int)(slots_ + (long long)ee * K + a));
            }
            for (int p = 0; p < P; ++p) prm[(size_t)p * cnt + ee] = hg.prm[(size_t)e * P + p];
        }
        dg.idx.upload(idx, s());
        dg.prm.upload(prm, s());
        GeoGroupDev& d = dg.d;
        d.type = hg.type; d.K = K; d.cols = C; d.hard = has_u(hg) ? 1 : 0; d.count = cnt;
        d.sw = std::sqrt(hg.weight);
        d.yscale = d.hard ? rho_ : hg.weight;
        // project_and_combine's a = rho / (w + rho), w = weight_^2 (Constraint.h:125-128)
        d.comb_a = (plain_ && !hg.hard) ? rho_ / (d.sw * d.sw + rho_) : 0.0;
        d.uoff = d.hard ? Zh_ : 0;
        d.slot0 = slots_;
        d.idx = dg.idx.p;
        d.prm = dg.prm.p;
        d.warm = nullptr;
        d.surf = SurfDev{nullptr, nullptr, 0, 0};
        if (hg.surf >= 0) {
            dg.warm.alloc(cnt);
            d.warm = dg.warm.p;
            d.surf = surfs_[hg.surf].dev();
        }
        if (d.hard) { Zh_ += 3LL * C * cnt; red_blocks_ += geo_u_blocks(cnt); }
        if (!hg.hard) soft_cols += (long long)C * cnt;
        slots_ += (long long)K * cnt;
        ncons += cnt;
    }
    if (slots_ > 0x7fffffffLL) throw Error(ERR_ARG, "too many constraint slots for int32 indexing");
    {
        std::vector<int> ptr(n_ + 1, 0), sl;
        for (int q = 0; q < n_; ++q) {
            sl.insert(sl.end(), pslots[q].begin(), pslots[q].end());
            ptr[q + 1] = (int)sl.size();
        }
        slot_ptr_.upload(ptr, s());
        slot_idx_.upload(sl, s());
    }
    std::vector<double> rf(3 * (size_t)n_);
    for (int q = 0; q < n_; ++q)
        for (int d = 0; d < 3; ++d) rf[3 * (size_t)q + d] = rhs_fixed_user_[3 * (size_t)int2user_[q] + d];
    // partitioned: a shared separator row's constant (regularisation) term enters once (rank 0)
    if (P > 1 && rank_ != 0) std::fill(rf.begin() + 3 * (size_t)top_beg_, rf.end(), 0.0);
    if (P == 1) { nbg_ = red_blocks_; zhmax = Zh_; }
    zh_max_ = zhmax;
    aamask_ = AAMask();
    if (P > 1) {   // the x entries this rank owns enter the Anderson dot products
        aamask_.lo1 = 3LL * own_beg_; aamask_.hi1 = 3LL * own_end_;
        aamask_.lo2 = rank_ == 0 ? 3LL * top_beg_ : 0; aamask_.hi2 = rank_ == 0 ? 3LL * n_ : 0;
    }
    rhs_fixed_.upload(rf, s());
    const size_t nx = 3 * (size_t)n_, nu = std::max<size_t>(1, (size_t)Zh_);
    b_.alloc(nx); y_.alloc(std::max<size_t>(3, 3 * (size_t)slots_));
    cur_x_.alloc(nx); new_x_.alloc(nx); def_x_.alloc(nx);
    cur_x_.zero(s()); new_x_.zero(s()); def_x_.zero(s());   // rows of other parts stay finite
    cur_u_.alloc(nu); new_u_.alloc(nu); def_u_.alloc(nu); z_.alloc(nu);
    nbg_ = std::max(1, nbg_);
    red_.alloc(nbg_);   // this rank's partials, padded to the largest rank's block count
    red_.zero(s());
    if (comm_) { red_g_.alloc(nbg_); red_g_.zero(s()); redg_ = red_g_.p; }
    else redg_ = red_.p;
    ctrl_.alloc(1);
    clock0_.alloc(1);
    // constraint groups on parallel branches (ALM loop only; opt-in, AA_GEOM_CONCURRENT=1): the
    // closest-point group stays on the main stream (it dominates), the others run beside it.
    // Measured slower (C5 396 -> 385, C3 1730 -> 1659 it/s): the short groups
    // take CU slots from the closest-point walk, whose occupancy is what hides its latency.
    conc_ = false;
    if (const char* e = std::getenv("AA_GEOM_CONCURRENT")) conc_ = !plain_ && groups_.size() > 1 && e[0] == '1';
    heavy_ = 0;
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
        const GeoGroupDev& d = groups_[gi].d;
        const bool cp = d.type == GEO_POINT_TO_REF || d.type == GEO_REF_SURFACE;
        const GeoGroupDev& h = groups_[heavy_].d;
        const bool hcp = h.type == GEO_POINT_TO_REF || h.type == GEO_REF_SURFACE;
        if ((cp && !hcp) || (cp == hcp && (long long)d.count * d.K > (long long)h.count * h.K)) heavy_ = (int)gi;
    }
    if (conc_) {
        if (!side_) AA_HIP(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
        if (!ev_fork_) AA_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
        if (!ev_join_) AA_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    }
    int khz = 0;
    AA_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx_->device));
    clock_khz_ = khz > 0 ? khz : 100000.0;
    AA_HIP(hipStreamSynchronize(s()));
    factored_ = true;
    cur_m_ = -1;
    rt_.hard_cols = (long long)(Zh_ / 3) - (plain_ ? soft_cols : 0);
    rt_.soft_cols = soft_cols;
    rt_.n_constraints = ncons;
    rt_.factor_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();

    // algorithmic bytes per launch class (DESIGN.md "roofline accounting")
    kstats_.clear();
    double zb = 24.0 * n_, ub = 48.0 * n_;
    for (auto& g : groups_) {
        const GeoGroupDev& d = g.d;
        const double per = 4.0 * d.K + 8.0 * n_params(d.type) + 24.0 * d.K + (d.surf.nodes ? 8.0 : 0.0) +
                           (d.hard ? 48.0 * d.cols : 0.0);
        zb += per * d.count;
        if (d.hard) ub += (4.0 * d.K + 72.0 * d.cols) * d.count;
    }
    kstats_["z"].bytes = zb;
    kstats_["u"].bytes = ub;
    kstats_["rhs"].bytes = 4.0 * (n_ + 1) + 28.0 * (double)slots_ + 48.0 * n_;
    kstats_["solve"].bytes = solver_.bytes_per_solve();
}

void GeomSolver::prepare_m(int m) {
    if (m == cur_m_) return;
    drop_graph();
    const long long dim = Zh_ + 3LL * n_;
    if (m > 0) {
        aa_cur_.alloc(dim);
        aa_dF_.alloc((size_t)m * (plain_ ? std::max<long long>(1, Zh_) : dim)); aa_dF_.zero(s());
        aa_dG_.alloc((size_t)m * dim); aa_dG_.zero(s());
        aa_blocks_ = aa_reduce_blocks(zh_max_ + 3LL * n_);   // the same grid on every rank
        const int mm = aa_window_bucket(m);
        aa_red_.alloc((size_t)aa_blocks_ * (2 + 2 * mm)); aa_red_.zero(s());
        if (comm_) { aa_red_g_.alloc(aa_red_.n); aa_red_g_.zero(s()); aag_ = aa_red_g_.p; }
        else aag_ = aa_red_.p;
        kstats_["aa"].bytes = 8.0 * dim * (2.0 * std::min(m, 32) + 8.0);
    } else {
        aa_cur_.release(); aa_dF_.release(); aa_dG_.release(); aa_red_.release();
        aa_blocks_ = 0;
        kstats_["aa"].bytes = 16.0 * dim * 2;
    }
    cur_m_ = m;
}

void GeomSolver::prologue(const double* init_x3, int max_iter, int m, int cap, double eps_abs, double eps_rel) {
    std::vector<double> x(3 * (size_t)n_);
    for (int q = 0; q < n_; ++q)
        for (int d = 0; d < 3; ++d) x[3 * (size_t)q + d] = init_x3[3 * (size_t)int2user_[q] + d];
    cur_x_.upload(x, s());
    def_x_.upload(x, s());
    cur_u_.zero(s());
    def_u_.zero(s());
    if (m > 0) {
        AA_HIP(hipMemsetAsync(aa_cur_.p, 0, (size_t)Zh_ * 8, s()));
        AA_HIP(hipMemcpyAsync(aa_cur_.p + Zh_, cur_x_.p, x.size() * 8, hipMemcpyDeviceToDevice, s()));
    }
    for (auto& g : groups_)
        if (g.d.warm) AA_HIP(hipMemsetAsync(g.d.warm, 0xff, (size_t)g.d.count * sizeof(int), s()));
    cap = std::max(1, cap);
    if (cap > hist_cap_) {
        drop_graph();   // the captured chunk holds the old history pointers
        hist_cap_ = cap;
        hist_comb_.alloc(cap);
        hist_clock_.alloc(cap);
    }
    Ctrl c;
    std::memset(&c, 0, sizeof(c));
    c.prev_prim = DBL_MAX;
    c.cap = hist_cap_;
    c.max_iter = max_iter;
    c.aa_m = m;
    c.aa_active = m > 0 ? 1 : 0;
    c.eps_abs = eps_abs;
    c.eps_rel = eps_rel;
    AA_HIP(hipMemcpyAsync(ctrl_.p, &c, sizeof(Ctrl), hipMemcpyHostToDevice, s()));
    if (plain_) {
        // GeometrySolver::ADMM_init_variables (GeometrySolver.h:356-382): one z / x / u update
        // from (init_x, 0), then current = default; the accelerator starts from it
        const long long nx = 3LL * n_;
        for (auto& g : groups_) launch_geo_z_plain(g.d, cur_x_.p, cur_u_.p, z_.p, y_.p, ctrl_.p, nullptr, 0, 0, s());
        launch_geo_rhs(n_, slot_ptr_.p, slot_idx_.p, y_.p, rhs_fixed_.p, b_.p, ctrl_.p, s());
        solver_.solve(b_.p, new_x_.p, ctrl_.p, 0, s());
        enqueue_u_update(red_.p, s());
        if (Zh_) launch_copy(cur_u_.p, new_u_.p, Zh_, ctrl_.p, 0, s());
        launch_copy(cur_x_.p, new_x_.p, nx, ctrl_.p, 0, s());
        if (m > 0) {
            if (Zh_) launch_copy(aa_cur_.p, new_u_.p, Zh_, ctrl_.p, 0, s());
            launch_copy(aa_cur_.p + Zh_, new_x_.p, nx, ctrl_.p, 0, s());
        }
    }
    launch_geo_start(ctrl_.p, clock0_.p, s());
}

void GeomSolver::fork() {
    AA_HIP(hipEventRecord(ev_fork_, s()));
    AA_HIP(hipStreamWaitEvent(side_, ev_fork_, 0));
}

void GeomSolver::join() {
    AA_HIP(hipEventRecord(ev_join_, side_));
    AA_HIP(hipStreamWaitEvent(s(), ev_join_, 0));
}

// ADMM_u_update (+ the ALM residual partials): u_new = u + T(x_new) - z on every group with u
// (each group's partials at its own block offset; with conc_, the groups beside the heaviest
// on the side stream)
void GeomSolver::enqueue_u_update(double* red, hipStream_t st) {
    const bool br = conc_ && st == s() && !instrument_;
    if (br) fork();
    int off = 0;
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
        auto& g = groups_[gi];
        if (!g.d.hard) continue;
        launch_geo_u(g.d, new_x_.p, cur_x_.p, z_.p, cur_u_.p, new_u_.p, ctrl_.p, red, off,
                     br && (int)gi != heavy_ ? side_ : st);
        off += geo_u_blocks(g.d.count);
    }
    if (br) join();
}

// one pass of the while-loop body of GeometrySolver::solve_ADMM (Geometry/GeometrySolver.h:180-251)
void GeomSolver::enqueue_iteration_plain(int m) {
    Ctrl* c = ctrl_.p;
    const long long nx = 3LL * n_;
    auto z_update = [&](int gate) {
        int off = 0;
        for (auto& g : groups_) {
            launch_geo_z_plain(g.d, cur_x_.p, cur_u_.p, z_.p, y_.p, c, red_.p, off, gate, s());
            off += geo_u_blocks(g.d.count);
        }
        if (comm_) comm_->allreduce_sum(red_.p, red_g_.p, (size_t)nbg_, s());
    };
    ev_mark("z");
    z_update(0);                                                                         // ADMM_z_update
    ev_mark("z");
    launch_plain_control(c, redg_, nbg_, m > 0, 0, hist_comb_.p, hist_clock_.p, s());  // residual, reset test
    if (m > 0) {   // residual increased: swap to the un-accelerated (u, x), accelerator->replace, redo
        launch_geo_restore(cur_u_.p, cur_x_.p, aa_cur_.p, new_u_.p, new_x_.p, Zh_, nx, c, s());
        z_update(1);
        launch_plain_control(c, redg_, nbg_, 1, 1, hist_comb_.p, hist_clock_.p, s());
    }
    ev_mark("rhs");
    launch_geo_rhs(n_, slot_ptr_.p, slot_idx_.p, y_.p, rhs_fixed_.p, b_.p, c, s());     // ADMM_x_update
    ev_mark("rhs");
    ev_mark("solve");
    solver_.solve(b_.p, new_x_.p, c, 0, s());
    ev_mark("solve");
    ev_mark("u");
    enqueue_u_update(red_.p, s());                                                       // ADMM_u_update
    ev_mark("u");
    ev_mark("aa");
    if (m > 0) {   // aa->compute(default_u, default_x, current_u, current_x): u is the effective part
        Seg2 G{new_u_.p, Zh_, new_x_.p, nx};
        Seg2 none{nullptr, 0, nullptr, 0};
        Seg2 out{cur_u_.p, Zh_, cur_x_.p, nx};
        launch_aa_reduce(G, aa_cur_.p, Zh_, aa_dF_.p, aa_dG_.p, c, aa_red_.p, aa_blocks_, none, m, s(), nullptr,
                         nullptr, 0, nullptr, nullptr, nullptr, aamask_);
        if (comm_) comm_->allreduce_sum(aa_red_.p, aa_red_g_.p, aa_red_.n, s());
        launch_aa_solve(c, aag_, aa_blocks_, m, s());
        launch_aa_mix(G, aa_cur_.p, Zh_, aa_dF_.p, aa_dG_.p, c, out, m, s());
        if (instrument_ && n_mk_log_ < (int)(mk_log_.n / 2)) {
            AA_HIP(hipMemcpyAsync(mk_log_.p + 2 * n_mk_log_, &c->aa_mk, sizeof(int), hipMemcpyDeviceToDevice, s()));
            AA_HIP(hipMemcpyAsync(mk_log_.p + 2 * n_mk_log_ + 1, &c->aa_skip, sizeof(int), hipMemcpyDeviceToDevice, s()));
            ++n_mk_log_;
        }
    } else {   // swap(default, current)
        if (Zh_) launch_copy(cur_u_.p, new_u_.p, Zh_, c, 0, s());
        launch_copy(cur_x_.p, new_x_.p, nx, c, 0, s());
    }
    ev_mark("aa");
}

// one chunk of loop passes
void GeomSolver::enqueue_chunk(int chunk, int m) {
    for (int i = 0; i < chunk; ++i) enqueue_iteration(m);
}

void GeomSolver::ev_mark(const char* name) {
    if (!instrument_) return;
    hipEvent_t e;
    AA_HIP(hipEventCreate(&e));
    AA_HIP(hipEventRecord(e, s()));
    kstats_[name].ev.push_back(e);
}

// one pass of the while-loop body of solve_ADMM (ALMGeometrySolver.h:197-267)
void GeomSolver::enqueue_iteration(int m) {
    if (plain_) return enqueue_iteration_plain(m);
    Ctrl* c = ctrl_.p;
    const long long nx = 3LL * n_;
    ev_mark("z");
    const bool br = conc_ && !instrument_;
    if (br) fork();
    for (size_t gi = 0; gi < groups_.size(); ++gi)                                      // ADMM_z_update
        launch_geo_z(groups_[gi].d, cur_x_.p, cur_u_.p, z_.p, y_.p, c, br && (int)gi != heavy_ ? side_ : s());
    if (br) join();
    ev_mark("z");
    ev_mark("rhs");
    launch_geo_rhs(n_, slot_ptr_.p, slot_idx_.p, y_.p, rhs_fixed_.p, b_.p, c, s());     // ADMM_x_update rhs
    ev_mark("rhs");
    ev_mark("solve");
    solver_.solve(b_.p, new_x_.p, c, 0, s());                                           // SPD_solver_->solve
    ev_mark("solve");
    ev_mark("u");
    enqueue_u_update(red_.p, s());                                                       // ADMM_u_update + residual
    ev_mark("u");
    ev_mark("aa");
    if (comm_) comm_->allreduce_sum(red_.p, red_g_.p, (size_t)nbg_, s());
    launch_geo_control(c, redg_, nbg_, m > 0, hist_comb_.p, hist_clock_.p, s());
    if (m > 0) {
        launch_geo_restore(cur_u_.p, cur_x_.p, aa_cur_.p, def_u_.p, def_x_.p, Zh_, nx, c, s());
        Seg2 G{new_u_.p, Zh_, new_x_.p, nx};
        Seg2 cp{def_u_.p, Zh_, def_x_.p, nx};
        Seg2 out{cur_u_.p, Zh_, cur_x_.p, nx};
        launch_aa_reduce(G, aa_cur_.p, Zh_ + nx, aa_dF_.p, aa_dG_.p, c, aa_red_.p, aa_blocks_, cp, m, s(), nullptr,
                         nullptr, 0, nullptr, nullptr, nullptr, aamask_);
        if (comm_) comm_->allreduce_sum(aa_red_.p, aa_red_g_.p, aa_red_.n, s());
        launch_aa_solve(c, aag_, aa_blocks_, m, s());
        launch_aa_mix(G, aa_cur_.p, Zh_ + nx, aa_dF_.p, aa_dG_.p, c, out, m, s());
        if (instrument_ && n_mk_log_ < (int)(mk_log_.n / 2)) {   // this launch's window / skip flag
            AA_HIP(hipMemcpyAsync(mk_log_.p + 2 * n_mk_log_, &c->aa_mk, sizeof(int), hipMemcpyDeviceToDevice, s()));
            AA_HIP(hipMemcpyAsync(mk_log_.p + 2 * n_mk_log_ + 1, &c->aa_skip, sizeof(int), hipMemcpyDeviceToDevice, s()));
            ++n_mk_log_;
        }
    } else {
        if (Zh_) launch_copy(cur_u_.p, new_u_.p, Zh_, c, 0, s());
        launch_copy(cur_x_.p, new_x_.p, nx, c, 0, s());
    }
    ev_mark("aa");
}

void GeomSolver::fetch_results() {
    Ctrl c;
    AA_HIP(hipMemcpyAsync(&c, ctrl_.p, sizeof(Ctrl), hipMemcpyDeviceToHost, s()));
    AA_HIP(hipStreamSynchronize(s()));
    const int nrec = std::min(c.nrec, hist_cap_);
    h_comb_.resize(nrec);
    h_time_.resize(nrec);
    std::vector<unsigned long long> clk(nrec);
    unsigned long long c0 = 0;
    if (nrec) {
        AA_HIP(hipMemcpy(h_comb_.data(), hist_comb_.p, nrec * 8, hipMemcpyDeviceToHost));
        AA_HIP(hipMemcpy(clk.data(), hist_clock_.p, nrec * 8, hipMemcpyDeviceToHost));
    }
    AA_HIP(hipMemcpy(&c0, clock0_.p, 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < nrec; ++k) h_time_[k] = (double)(clk[k] - c0) / (clock_khz_ * 1e3);
    rt_.iterations = c.iters_run;
    rt_.accepted = c.nrec;
    rt_.rejects = c.nrej;
}

// solve_ADMM (ALMGeometrySolver.h:163-283). rel_residual_eps is accepted for API parity: the
// reference computes its threshold but the stopping test is commented out (:258-263).
void GeomSolver::set_stop(int at_eps, double eps_rel) {
    if (!(eps_rel >= 0.0)) throw Error(ERR_ARG, "set_stop: eps_rel must be >= 0");
    if (plain_ && (at_eps || eps_rel > 0)) throw Error(ERR_ARG, "set_stop: ALMGeometrySolver only");
    stop_eps_ = at_eps != 0;
    stop_rel_ = eps_rel;
}

// z_hard_.cols(): a constraint's columns are its transformed points -- K for the mean-centred
// kinds, K - 1 for the subtract-first ones (angle, edge; Constraint.h:73-94)
long long GeomSolver::hard_cols() const {
    long long n = 0;
    for (const auto& g : hgroups_)
        if (g.hard) n += (long long)g.count() * ((g.type == GEO_ANGLE || g.type == GEO_EDGE) ? g.K - 1 : g.K);
    return n;
}

void GeomSolver::solve(const double* init_x3, double rel_residual_eps, int max_iter, int m) {
    if (!setup_done_) throw Error(ERR_STATE, "Error: solver not initialized yet");
    if (!init_x3) throw Error(ERR_ARG, "solve_ADMM: null init_x");
    if (m < 0 || m > kMaxM) throw Error(ERR_ARG, "solve_ADMM: Anderson window must be in [0, 32]");
    if (max_iter < 0) throw Error(ERR_ARG, "solve_ADMM: max_iter < 0");
    auto t0 = std::chrono::steady_clock::now();
    if (!factored_) factor_and_upload(init_x3);
    prepare_m(m);
    last_init_.assign(init_x3, init_x3 + 3 * (size_t)n_);
    double eps_abs = 0.0;
    if (stop_eps_) {   // residual_eps of ALMGeometrySolver.h:172
        const double cols = (double)hard_cols();
        eps_abs = rel_residual_eps * rel_residual_eps * cols * cols * 2.0;
    }
    prologue(init_x3, max_iter, m, max_iter, eps_abs, stop_rel_);
    const bool may_stop = eps_abs > 0.0 || stop_rel_ > 0.0;
    const int target = std::max(1, max_iter);
    const int chunk = std::min(target, kChunks[0]);
    bool use_graph = !(std::getenv("AA_ADMM_NO_GRAPH") && std::getenv("AA_ADMM_NO_GRAPH")[0] == '1') &&
                     !(comm_ && !comm_->capturable());
    if (graph_m_ != m) { drop_graph(); graph_m_ = m; }
    // n loop passes: replays of the captured 64 / 16 / 4 / 1-pass graphs (each captured on first use)
    auto run_passes = [&](int n) {
        if (!use_graph) { enqueue_chunk(n, m); return; }
        for (int i = 0; i < kNChunks && n > 0; ++i) {
            for (; n >= kChunks[i]; n -= kChunks[i]) {
                if (!gexec_[i]) {
                    bool ok = capture_graph(s(), [&] { enqueue_chunk(kChunks[i], m); }, &graph_[i], &gexec_[i]);
                    if (comm_) {   // the ranks replay or launch eagerly together
                        double f = ok ? 0.0 : 1.0;
                        comm_->allreduce_sum_host(&f, 1);
                        if (f > 0 && ok) ok = false;
                    }
                    if (!ok) { drop_graph(); use_graph = false; enqueue_chunk(n, m); return; }
                }
                AA_HIP(hipGraphLaunch(gexec_[i], s()));
            }
        }
    };
    // A pass accepts at most one iteration and a rejected pass is always followed by an accepted
    // one (alm_reset), so the loop needs between `target` and 2 target passes. Without a
    // run-to-epsilon stop it launches exactly the passes still needed at least -- target, then
    // target - accepted after each check -- so no pass runs gated after the last acceptance (the
    // fixed 64-pass chunks of round 3 ran up to 63 such passes per solve: ~3 % of C3's loop).
    // With a stop (unknown end): two 64-pass chunks in flight, then one per done check.
    // AA_GEOM_EXACT_TAIL=0 restores the fixed chunks for both (A/B).
    static const bool exact_tail = !(std::getenv("AA_GEOM_EXACT_TAIL") && std::getenv("AA_GEOM_EXACT_TAIL")[0] == '0');
    const bool exact = exact_tail && !may_stop;
    const int first = exact ? target : (may_stop ? std::min(2, (target + chunk - 1) / chunk) : (target + chunk - 1) / chunk) * chunk;
    run_passes(first);
    int passes = first;
    for (;;) {
        Ctrl c;
        AA_HIP(hipMemcpyAsync(&c, ctrl_.p, sizeof(Ctrl), hipMemcpyDeviceToHost, s()));
        AA_HIP(hipStreamSynchronize(s()));
        if (c.done) break;
        if (passes > 2 * target + 2 * chunk) throw Error(ERR_NUMERIC, "solve_ADMM: the loop did not terminate");
        const int next = exact ? std::max(1, target - c.nrec) : chunk;
        run_passes(next);
        passes += next;
    }
    fetch_results();
#ifdef AA_CP_STATS
    cp_stats_dump();
#endif
    if (comm_) {   // every rank ends with the full solution: zero what it does not own, sum
        double* sol = solution_buf();
        auto zero = [&](int q0, int q1) {
            if (q1 > q0) AA_HIP(hipMemsetAsync(sol + 3 * (size_t)q0, 0, 24 * (size_t)(q1 - q0), s()));
        };
        zero(0, own_beg_);
        zero(own_end_, top_beg_);
        if (rank_ != 0) zero(top_beg_, n_);
        comm_->allreduce_sum(sol, sol, 3 * (size_t)n_, s());
        AA_HIP(hipStreamSynchronize(s()));
    }
    have_solution_ = true;
    rt_.solve_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// get_solution: ALM (ALMGeometrySolver.h:280-282) = default_x_, the x of the last accepted
// iteration, which is the last x-update since the loop always ends on an acceptance;
// GeometrySolver (GeometrySolver.h:254-256) = *current_x_
void GeomSolver::get_solution(double* x3) const {
    if (!have_solution_) throw Error(ERR_STATE, "get_solution before solve_ADMM");
    std::vector<double> x(3 * (size_t)n_);
    AA_HIP(hipMemcpy(x.data(), plain_ ? cur_x_.p : new_x_.p, x.size() * 8, hipMemcpyDeviceToHost));
    for (int q = 0; q < n_; ++q)
        for (int d = 0; d < 3; ++d) x3[3 * (size_t)int2user_[q] + d] = x[3 * (size_t)q + d];
}

int GeomSolver::history(double* comb, double* time_s, int cap) const {
    const int n = std::min(cap, (int)h_comb_.size());
    for (int i = 0; i < n; ++i) {
        if (comb) comb[i] = h_comb_[i];
        if (time_s) time_s[i] = h_time_[i];
    }
    return (int)h_comb_.size();
}

void GeomSolver::closest_points(int surface, const double* p3, int n, double* out3) {
    if (surface < 0 || surface >= (int)surfs_.size()) throw Error(ERR_ARG, "closest_points: unknown surface");
    if (n <= 0) return;
    DevBuf<double> p, c(3 * (size_t)n);
    p.upload(p3, 3 * (size_t)n, s());
    launch_closest(surfs_[surface].dev(), p.p, c.p, n, s());
    AA_HIP(hipMemcpyAsync(out3, c.p, 24 * (size_t)n, hipMemcpyDeviceToHost, s()));
    AA_HIP(hipStreamSynchronize(s()));
}

double GeomSolver::bench_iterations(int iters) {
    if (!setup_done_ || !factored_ || cur_m_ < 0) throw Error(ERR_STATE, "bench before solve_ADMM");
    for (auto& kv : kstats_) { for (auto e : kv.second.ev) (void)hipEventDestroy(e); kv.second.ev.clear(); }
    prologue(last_init_.data(), 1 << 30, cur_m_, iters + 1);
    mk_log_.alloc(2 * (size_t)std::max(1, iters));
    n_mk_log_ = 0;
    AA_HIP(hipStreamSynchronize(s()));
    instrument_ = true;
    hipEvent_t e0, e1;
    AA_HIP(hipEventCreate(&e0)); AA_HIP(hipEventCreate(&e1));
    AA_HIP(hipEventRecord(e0, s()));
    enqueue_chunk(iters, cur_m_);
    AA_HIP(hipEventRecord(e1, s()));
    AA_HIP(hipEventSynchronize(e1));
    instrument_ = false;
    float ms = 0;
    AA_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    for (auto& kv : kstats_) {
        KStat& k = kv.second;
        k.total_ms = 0; k.launches = 0;
        for (size_t i = 0; i + 1 < k.ev.size(); i += 2) {
            float t = 0;
            AA_HIP(hipEventElapsedTime(&t, k.ev[i], k.ev[i + 1]));
            k.total_ms += t; k.launches += 1;
        }
    }
    if (cur_m_ > 0 && n_mk_log_ > 0) {
        // Anderson bytes of each launch from the window it actually used (mk < m while a window
        // fills or after a reset; an ALM reject skips the step and only restores u, x)
        std::vector<int> lg(2 * (size_t)n_mk_log_);
        AA_HIP(hipMemcpy(lg.data(), mk_log_.p, lg.size() * sizeof(int), hipMemcpyDeviceToHost));
        const double dim = (double)Zh_ + 3.0 * n_;
        double tot = 0;
        for (int k = 0; k < n_mk_log_; ++k)
            tot += lg[2 * k + 1] ? 16.0 * dim : 8.0 * dim * (2.0 * lg[2 * k] + 8.0);
        kstats_["aa"].bytes = tot / n_mk_log_;
    }
    fetch_results();
    return ms;
}

bool GeomSolver::kernel_stats(const std::string& name, double* avg_ms, double* bytes, int* launches) const {
    auto it = kstats_.find(name);
    if (it == kstats_.end()) return false;
    const KStat& k = it->second;
    if (avg_ms) *avg_ms = k.launches ? k.total_ms / k.launches : 0.0;
    if (bytes) *bytes = k.bytes;
    if (launches) *launches = k.launches;
    return true;
}

}  // namespace aa
