// ORACLE -- test infrastructure only (see oracle.h). Plain C++ restatement, no Eigen.
//
// Restates, for both reference variants:
//   Solver::initialize   admm_anderson_hard_zxu/src/Solver.cpp:361-491 (X: admm_anderson_xzu/src/Solver.cpp:373-498)
//   Solver::step         admm_anderson_hard_zxu/src/Solver.cpp:34-234  (X: admm_anderson_xzu/src/Solver.cpp:34-263)
//   EnergyTerm::update_z / update_u / get_all_gradient  (src/EnergyTerm.hpp:155-213)
//   TetEnergyTerm / TriEnergyTerm ctor, get_reduction, prox, get_gradient
//        (admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:32-96, TriEnergyTerm.cpp:30-105;
//         X tri prox admm_anderson_xzu/src/TriEnergyTerm.cpp:77-108)
//   AndersonAcceleration  H/G: admm_anderson_hard_zxu/src/AndersonAcceleration.h:40-211
//                         X:   admm_anderson_xzu/src/AndersonAcceleration.h:138-200,279-295
// The global LDLT (LinearSolver.hpp:79-90) is restated as an envelope Cholesky of the
// scalar matrix A_s (A = A_s (x) I3): same solution to rounding.
#include "oracle.h"
#include "oracle_lbfgs.hpp"
#include "oracle_svd.hpp"
#include "oracle_common.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace oracle {

struct Elem {
    int kind, mat, nv, ncol, dim, off;
    int v[4];        // internal node ids
    double G[3][4];  // F[:,c] = sum_a G[c][a] x_{v_a}
    double w, vol, mu, lambda, k, lmin, lmax;
};

// ------------------------------------------------------------------ element kernels
// column-major 3x3 <-> row-major helpers
inline void cm_to_rm3(const double* z, double* F) { for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) F[r * 3 + c] = z[c * 3 + r]; }

void tet_linear_prox(const double* z, double* out) {
    double F[9], U[9], S[3], V[9];
    cm_to_rm3(z, F);
    jacobi_svd_square<3>(F, U, S, V);
    double s[3] = {1, 1, det3(F) < 1e-16 ? -1.0 : 1.0};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double p = 0;
            for (int k = 0; k < 3; ++k) p += U[r * 3 + k] * s[k] * V[c * 3 + k];
            out[c * 3 + r] = 0.5 * (p + z[c * 3 + r]);
        }
}

void tet_linear_grad(const Elem& e, const double* z, double* g) {  // k vol (F - U V^T)  (X TetEnergyTerm::get_gradient)
    double F[9], U[9], S[3], V[9];
    cm_to_rm3(z, F);
    jacobi_svd_square<3>(F, U, S, V);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double p = 0;
            for (int k = 0; k < 3; ++k) p += U[r * 3 + k] * V[c * 3 + k];
            g[c * 3 + r] = e.k * e.vol * (F[r * 3 + c] - p);
        }
}

void tri_prox_h(const double* z, double lmin, double lmax, double* out) {
    double F[6];  // row-major 3x2 ; z col-major 3x2
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 2; ++c) F[r * 2 + c] = z[c * 3 + r];
    double U[9], S[2], V[4];
    svd_3x2(F, U, S, V);
    double sg[2] = {(1.0 + S[0]) / 2.0, (1.0 + S[1]) / 2.0};
    if (lmin > 0.0 || lmax < 99.0) {
        double l0 = sg[0], l1 = sg[1];
        if (l0 < lmin) sg[0] = lmin;
        if (l1 < lmin) sg[1] = lmin;
        if (l0 > lmax) sg[0] = lmax;
        if (l1 > lmax) sg[1] = lmax;
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 2; ++c)
            out[c * 3 + r] = U[r * 3 + 0] * sg[0] * V[c * 2 + 0] + U[r * 3 + 1] * sg[1] * V[c * 2 + 1];
}

void tri_prox_x(const double* z, double lmin, double lmax, double* out) {
    double F[6];
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 2; ++c) F[r * 2 + c] = z[c * 3 + r];
    double U[9], S[2], V[4];
    svd_3x2(F, U, S, V);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 2; ++c) {
            double p = U[r * 3 + 0] * V[c * 2 + 0] + U[r * 3 + 1] * V[c * 2 + 1];
            out[c * 3 + r] = 0.5 * (p + z[c * 3 + r]);
        }
    if (lmin > 0.0 || lmax < 99.0) {
        double l0 = std::sqrt(out[0] * out[0] + out[1] * out[1] + out[2] * out[2]);
        double l1 = std::sqrt(out[3] * out[3] + out[4] * out[4] + out[5] * out[5]);
        if (l0 < lmin) for (int i = 0; i < 3; ++i) out[i] *= lmin / l0;
        if (l1 < lmin) for (int i = 3; i < 6; ++i) out[i] *= lmin / l1;
        if (l0 > lmax) for (int i = 0; i < 3; ++i) out[i] *= lmax / l0;
        if (l1 > lmax) for (int i = 3; i < 6; ++i) out[i] *= lmax / l1;
    }
}

// ------------------------------------------------------------------ the solver
struct Elastic {
    int n = 0, nf = 0, np = 0, Z = 0;
    oracle_settings st{};
    std::vector<int> int2node, node2int;
    std::vector<double> mass, x, v;  // node-ordered (input order), 3 per node
    std::vector<Elem> el;
    std::vector<double> xpin;        // 3*np, internal pinned order
    Envelope chol;
    double pdt2 = 0;

    // rest3: rest positions the element reductions are built from (create_tets_from_mesh takes
    // the mesh vertices, TetEnergyTerm.hpp:36-51); x3: initial node positions (add_nodes).
    void build(int n_nodes, const double* x3, const double* rest3, const double* masses, int n_groups, const int* g_kind,
               const int* g_mat, const double* g_E, const double* g_nu, const double* g_lmin, const double* g_lmax,
               const int* g_count, const int* g_off, const int* idx, int n_pins, const int* pin_idx) {
        n = n_nodes;
        if (!rest3) rest3 = x3;
        x.assign(x3, x3 + 3 * n);
        v.assign(3 * n, 0.0);
        mass.assign(masses, masses + n);
        std::map<int, int> pins;
        for (int i = 0; i < n_pins; ++i) pins[pin_idx[i]] = i;
        np = (int)pins.size();
        nf = n - np;
        node2int.assign(n, -1);
        // free nodes in reverse Cuthill-McKee order (keeps the envelope factor small); pinned last
        std::vector<std::vector<int>> adj(n);
        for (int g = 0; g < n_groups; ++g) {
            const int nv = g_kind[g] == 0 ? 4 : 3;
            for (int t = 0; t < g_count[g]; ++t) {
                const int* id = idx + g_off[g] + (size_t)t * nv;
                for (int a = 0; a < nv; ++a)
                    for (int b = 0; b < nv; ++b)
                        if (a != b) adj[id[a]].push_back(id[b]);
            }
        }
        for (auto& l : adj) { std::sort(l.begin(), l.end()); l.erase(std::unique(l.begin(), l.end()), l.end()); }
        std::vector<int> order, seen(n, 0);
        for (int i = 0; i < n; ++i) if (pins.count(i)) seen[i] = 1;
        for (;;) {
            int start = -1;
            for (int i = 0; i < n; ++i)
                if (!seen[i] && (start < 0 || adj[i].size() < adj[start].size())) start = i;
            if (start < 0) break;
            size_t head = order.size();
            order.push_back(start); seen[start] = 1;
            while (head < order.size()) {
                int v0 = order[head++];
                std::vector<int> nb;
                for (int u : adj[v0]) if (!seen[u]) { seen[u] = 1; nb.push_back(u); }
                std::sort(nb.begin(), nb.end(), [&](int a, int b) { return adj[a].size() < adj[b].size() || (adj[a].size() == adj[b].size() && a < b); });
                order.insert(order.end(), nb.begin(), nb.end());
            }
        }
        std::reverse(order.begin(), order.end());
        int c = 0;
        for (int i : order) { node2int[i] = c++; int2node.push_back(i); }
        for (auto& kv : pins) { node2int[kv.first] = c++; int2node.push_back(kv.first); }
        Z = 0;
        for (int g = 0; g < n_groups; ++g) {
            const double E = g_E[g], nu = g_nu[g];
            const double mu = E / (2.0 * (1.0 + nu)), lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu));
            const double k = lam + (2.0 / 3.0) * mu;
            const int nv = g_kind[g] == 0 ? 4 : 3;
            for (int t = 0; t < g_count[g]; ++t) {
                const int* id = idx + g_off[g] + (size_t)t * nv;
                Elem e{};
                e.kind = g_kind[g]; e.mat = g_mat[g]; e.nv = nv; e.ncol = nv - 1; e.dim = 3 * (nv - 1);
                e.mu = mu; e.lambda = lam; e.k = k; e.lmin = g_lmin[g]; e.lmax = g_lmax[g];
                const double* P[4];
                for (int a = 0; a < nv; ++a) { e.v[a] = node2int[id[a]]; P[a] = rest3 + 3 * (size_t)id[a]; }
                if (e.kind == 0) {
                    double B[9];  // row-major, columns = edges
                    for (int r = 0; r < 3; ++r) for (int cc = 0; cc < 3; ++cc) B[r * 3 + cc] = P[cc + 1][r] - P[0][r];
                    double cof[9];
                    cof[0] = B[4] * B[8] - B[5] * B[7]; cof[1] = B[5] * B[6] - B[3] * B[8]; cof[2] = B[3] * B[7] - B[4] * B[6];
                    cof[3] = B[2] * B[7] - B[1] * B[8]; cof[4] = B[0] * B[8] - B[2] * B[6]; cof[5] = B[1] * B[6] - B[0] * B[7];
                    cof[6] = B[1] * B[5] - B[2] * B[4]; cof[7] = B[2] * B[3] - B[0] * B[5]; cof[8] = B[0] * B[4] - B[1] * B[3];
                    double det = B[0] * cof[0] + B[1] * cof[1] + B[2] * cof[2];
                    double Binv[9];  // inverse = adj / det, adj = cof^T
                    for (int r = 0; r < 3; ++r) for (int cc = 0; cc < 3; ++cc) Binv[r * 3 + cc] = cof[cc * 3 + r] / det;
                    e.vol = det / 6.0;
                    if (e.vol < 0) throw std::runtime_error("**TetEnergyTerm Error: Inverted initial tet");
                    for (int r = 0; r < 3; ++r) {
                        e.G[r][0] = -Binv[0 * 3 + r] - Binv[1 * 3 + r] - Binv[2 * 3 + r];
                        for (int a = 1; a < 4; ++a) e.G[r][a] = Binv[(a - 1) * 3 + r];
                    }
                } else {
                    double e12[3], e13[3], n1[3], n2[3];
                    for (int r = 0; r < 3; ++r) { e12[r] = P[1][r] - P[0][r]; e13[r] = P[2][r] - P[0][r]; }
                    double l = std::sqrt(e12[0] * e12[0] + e12[1] * e12[1] + e12[2] * e12[2]);
                    for (int r = 0; r < 3; ++r) n1[r] = e12[r] / l;
                    double d = e13[0] * n1[0] + e13[1] * n1[1] + e13[2] * n1[2];
                    for (int r = 0; r < 3; ++r) n2[r] = e13[r] - d * n1[r];
                    l = std::sqrt(n2[0] * n2[0] + n2[1] * n2[1] + n2[2] * n2[2]);
                    for (int r = 0; r < 3; ++r) n2[r] /= l;
                    auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
                    double b00 = dot(n1, e12), b01 = dot(n1, e13), b10 = dot(n2, e12), b11 = dot(n2, e13);
                    double det = b00 * b11 - b01 * b10;
                    double invdet = 1.0 / det;
                    double R[2][2] = {{b11 * invdet, -b01 * invdet}, {-b10 * invdet, b00 * invdet}};
                    e.vol = 0.5 * det;
                    if (e.vol < 0) throw std::runtime_error("**TriEnergyTerm Error: Inverted initial pose");
                    for (int cc = 0; cc < 2; ++cc) {
                        e.G[cc][0] = -R[0][cc] - R[1][cc];
                        e.G[cc][1] = R[0][cc];
                        e.G[cc][2] = R[1][cc];
                    }
                }
                e.w = std::sqrt(k * e.vol);
                if (e.w <= 0) throw std::runtime_error("**EnergyTerm::get_reduction Error: Some weight leq 0");
                e.off = Z;
                Z += e.dim;
                el.push_back(e);
            }
        }
        xpin.assign(3 * (size_t)np, 0.0);
    }

    void set_pins(int n_pins, const int* pin_idx, const double* pts) {
        for (int i = 0; i < n_pins; ++i) {
            int q = node2int[pin_idx[i]] - nf;
            for (int j = 0; j < 3; ++j) xpin[3 * q + j] = pts[3 * i + j];
        }
    }

    void initialize(const oracle_settings& s) {
        st = s;
        const double dt2 = st.dt * st.dt;
        pdt2 = (st.variant == 1 ? st.penalty : 1.0) * dt2;
        // envelope of A_s = M + pdt2 * sum_e w^2 G^T G over free nodes
        chol.n = nf;
        chol.first.resize(nf);
        for (int i = 0; i < nf; ++i) chol.first[i] = i;
        for (auto& e : el)
            for (int a = 0; a < e.nv; ++a)
                for (int b = 0; b < e.nv; ++b)
                    if (e.v[a] < nf && e.v[b] < nf && e.v[b] < e.v[a]) chol.first[e.v[a]] = std::min(chol.first[e.v[a]], e.v[b]);
        chol.start.resize(nf + 1);
        size_t off = 0;
        for (int i = 0; i < nf; ++i) { chol.start[i] = off; off += (size_t)(i - chol.first[i] + 1); }
        chol.L.assign(off, 0.0);
        for (int i = 0; i < nf; ++i) chol.at(i, i) = mass[int2node[i]];
        for (auto& e : el)
            for (int a = 0; a < e.nv; ++a)
                for (int b = 0; b < e.nv; ++b) {
                    int i = e.v[a], j = e.v[b];
                    if (i >= nf || j >= nf || j > i) continue;
                    double s = 0;
                    for (int c = 0; c < e.ncol; ++c) s += e.G[c][a] * e.G[c][b];
                    chol.at(i, j) += pdt2 * e.w * e.w * s;
                }
        chol.factor();
    }

    // full position of internal node q from the free vector xf
    inline const double* pos(const std::vector<double>& xf, int q) const {
        return q < nf ? &xf[3 * (size_t)q] : &xpin[3 * (size_t)(q - nf)];
    }
    // F = P_e x_full (col-major, dim entries)
    void Px(const Elem& e, const std::vector<double>& xf, double* F) const {
        for (int c = 0; c < e.ncol; ++c)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int a = 0; a < e.nv; ++a) s += e.G[c][a] * pos(xf, e.v[a])[j];
                F[3 * c + j] = s;
            }
    }
    // c_e = -w * P_e^{pinned} x_pin
    void Ce(const Elem& e, double* c) const {
        for (int cc = 0; cc < e.ncol; ++cc)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int a = 0; a < e.nv; ++a)
                    if (e.v[a] >= nf) s += e.G[cc][a] * xpin[3 * (size_t)(e.v[a] - nf) + j];
                c[3 * cc + j] = -e.w * s;
            }
    }
    void prox(const Elem& e, const double* vin, double* out) const {
        if (e.kind == 1) {
            if (st.variant == 1) tri_prox_h(vin, e.lmin, e.lmax, out);
            else tri_prox_x(vin, e.lmin, e.lmax, out);
        } else if (e.mat == MAT_LINEAR) tet_linear_prox(vin, out);
        else {
            ProxProblem P{e.mat, e.mu, e.lambda, e.k, e.vol, {}};
            for (int i = 0; i < 9; ++i) { P.v[i] = vin[i]; out[i] = vin[i]; }
            lbfgs_minimize(P, out);
        }
    }
    // EnergyTerm::update_z: z_e = prox(W^-1 (D_e x + u_e - c_e))
    void update_z(const std::vector<double>& xf, std::vector<double>& z, const std::vector<double>& u) const {
        #pragma omp parallel for schedule(dynamic, 64)
        for (size_t t = 0; t < el.size(); ++t) {
            const Elem& e = el[t];
            double F[9], vin[9];
            Px(e, xf, F);
            for (int i = 0; i < e.dim; ++i) vin[i] = F[i] + u[e.off + i] / e.w;
            prox(e, vin, &z[e.off]);
        }
    }
    // EnergyTerm::update_u: u_e += D_e x - W_e z_e - c_e
    void update_u(const std::vector<double>& xf, const std::vector<double>& z, std::vector<double>& u) const {
        for (auto& e : el) {
            double F[9];
            Px(e, xf, F);
            for (int i = 0; i < e.dim; ++i) u[e.off + i] += e.w * F[i] - e.w * z[e.off + i];
        }
    }
    // X AA mode: u = W^-1 grad E(z)
    void grad_u(const std::vector<double>& z, std::vector<double>& u) const {
        for (auto& e : el) {
            double g[9];
            const double* ze = &z[e.off];
            if (e.kind == 1) throw std::runtime_error("**TriEnergyTerm TODO: gradient function");
            if (e.mat == MAT_LINEAR) tet_linear_grad(e, ze, g);
            else {
                psi_grad(e.mat, e.mu, e.lambda, ze, g);
                for (int i = 0; i < 9; ++i) g[i] *= e.vol;
            }
            for (int i = 0; i < 9; ++i) u[e.off + i] = g[i] / e.w;
        }
    }
    // |D x - W z - C|^2
    double prim2(const std::vector<double>& xf, const std::vector<double>& z) const {
        double s = 0;
        for (auto& e : el) {
            double F[9];
            Px(e, xf, F);
            for (int i = 0; i < e.dim; ++i) { double r = e.w * (F[i] - z[e.off + i]); s += r * r; }
        }
        return s;
    }
    // |D (x1 - x0)|^2 (free part only; pinned columns are not in D)
    double dual2(const std::vector<double>& x1, const std::vector<double>& x0) const {
        double s = 0;
        for (auto& e : el)
            for (int c = 0; c < e.ncol; ++c)
                for (int j = 0; j < 3; ++j) {
                    double d = 0;
                    for (int a = 0; a < e.nv; ++a)
                        if (e.v[a] < nf) d += e.G[c][a] * (x1[3 * (size_t)e.v[a] + j] - x0[3 * (size_t)e.v[a] + j]);
                    d *= e.w;
                    s += d * d;
                }
        return s;
    }
    // x = A^-1 (M xbar + pdt2 D^T (W z + C - u))
    void global_solve(const std::vector<double>& Mxbar, const std::vector<double>& z, const std::vector<double>& u,
                      std::vector<double>& xf) {
        xf = Mxbar;
        for (auto& e : el) {
            double c[9];
            Ce(e, c);
            double t[9];
            for (int i = 0; i < e.dim; ++i) t[i] = e.w * z[e.off + i] + c[i] - u[e.off + i];
            for (int a = 0; a < e.nv; ++a) {
                int q = e.v[a];
                if (q >= nf) continue;
                for (int j = 0; j < 3; ++j) {
                    double s = 0;
                    for (int cc = 0; cc < e.ncol; ++cc) s += e.w * e.G[cc][a] * t[3 * cc + j];
                    xf[3 * (size_t)q + j] += pdt2 * s;
                }
            }
        }
        chol.solve3(xf.data());
    }

    struct Rec { std::vector<double> prim, comb; std::vector<int> rej; };

    Rec step() {
        Rec rec;
        const double dt = st.dt;
        const bool aa = st.accel != 0;
        for (int q = 0; q < nf; ++q) {
            int node = int2node[q];
            if (std::fabs(st.gravity) > 0) v[3 * node + 1] += dt * st.gravity;
        }
        std::vector<double> xbar(3 * (size_t)nf), Mxbar(3 * (size_t)nf);
        for (int q = 0; q < nf; ++q)
            for (int j = 0; j < 3; ++j) {
                int node = int2node[q];
                xbar[3 * q + j] = x[3 * node + j] + dt * v[3 * node + j];
                Mxbar[3 * q + j] = mass[node] * xbar[3 * q + j];
            }
        std::vector<double> xf = xbar, z(Z), u(Z, 0.0);
        for (auto& e : el) Px(e, xbar, &z[e.off]);  // z = W^-1 (D xbar - C)
        double prev_prim = 1e20;
        const double eps = 1e-20;
        std::vector<double> final_x;
        if (st.variant == 1) {
            update_z(xf, z, u);
            global_solve(Mxbar, z, u, xf);
            update_u(xf, z, u);
            std::vector<double> du = u, dx = xf, last_x;
            Anderson acc;
            std::vector<double> ux((size_t)Z + 3 * nf), gux(ux.size());
            auto pack = [&](const std::vector<double>& a, const std::vector<double>& b, std::vector<double>& o) {
                std::copy(a.begin(), a.end(), o.begin()); std::copy(b.begin(), b.end(), o.begin() + Z); };
            if (aa && st.aa_m > 0) { pack(u, xf, ux); acc.init(st.aa_m, (int)ux.size(), Z, ux.data()); }
            for (int s = 0; s < st.iters; ++s) {
                update_z(xf, z, u);
                double prim = std::sqrt(prim2(xf, z));
                int rej = 0;
                if (aa && prev_prim < prim) {
                    u = du; xf = dx;
                    pack(u, xf, ux);
                    acc.reset(ux.data());
                    update_z(xf, z, u);
                    prim = std::sqrt(prim2(xf, z));
                    rej = 1;
                }
                last_x = xf;
                prev_prim = prim;
                global_solve(Mxbar, z, u, xf);
                double comb = prim2(xf, z) + dual2(xf, last_x);
                if (comb < eps) break;
                update_u(xf, z, u);
                if (aa) {
                    du = u; dx = xf;
                    pack(du, dx, gux);
                    acc.compute(gux.data(), ux.data());
                    std::copy(ux.begin(), ux.begin() + Z, u.begin());
                    std::copy(ux.begin() + Z, ux.end(), xf.begin());
                }
                rec.prim.push_back(prim); rec.comb.push_back(comb); rec.rej.push_back(rej);
            }
            final_x = aa ? dx : xf;
        } else {
            global_solve(Mxbar, z, u, xf);
            update_z(xf, z, u);
            std::vector<double> dz = z, dx = xf, du = u, last_z;
            Anderson acc;
            acc.init(std::max(st.aa_m, 1), Z, Z, z.data());
            for (int s = 0; s < st.iters; ++s) {
                if (aa) grad_u(z, u);
                else update_u(xf, z, u);
                global_solve(Mxbar, z, u, xf);
                double prim = std::sqrt(prim2(xf, z));
                int rej = 0;
                if (aa && prev_prim < prim) {
                    u = du; xf = dx; z = dz;
                    acc.replace(z.data());
                    update_u(xf, z, u);
                    global_solve(Mxbar, z, u, xf);
                    prim = std::sqrt(prim2(xf, z));
                    rej = 1;
                }
                prev_prim = prim;
                last_z = z;
                double comb;
                if (aa) {
                    dx = xf; du = u;
                    update_z(xf, dz, u);
                    acc.compute(dz.data(), z.data());
                    std::vector<double> cx, cz(Z);
                    global_solve(Mxbar, dz, u, cx);
                    update_z(cx, cz, u);
                    double d2 = 0;
                    for (auto& e : el)
                        for (int i = 0; i < e.dim; ++i) { double r = e.w * (cz[e.off + i] - dz[e.off + i]); d2 += r * r; }
                    comb = d2 + prim2(cx, cz);
                } else {
                    update_z(xf, z, u);
                    double d2 = 0;
                    for (auto& e : el)
                        for (int i = 0; i < e.dim; ++i) { double r = e.w * (z[e.off + i] - last_z[e.off + i]); d2 += r * r; }
                    comb = d2 + prim2(xf, z);
                }
                rec.prim.push_back(prim); rec.comb.push_back(comb); rec.rej.push_back(rej);
                if (comb < eps) break;
            }
            final_x = xf;
        }
        // x_full = S_free x + S_fix x_pin ; v = (x_full - x)/dt
        std::vector<double> nx(3 * (size_t)n);
        for (int q = 0; q < n; ++q) {
            const double* p = pos(final_x, q);
            int node = int2node[q];
            for (int j = 0; j < 3; ++j) nx[3 * node + j] = p[j];
        }
        for (size_t i = 0; i < nx.size(); ++i) { v[i] = (nx[i] - x[i]) * (1.0 / dt); x[i] = nx[i]; }
        return rec;
    }
};

}  // namespace oracle

using namespace oracle;

extern "C" int oracle_elastic_run(int n_nodes, const double* x3, const double* rest3, const double* masses, int n_groups,
                                  const int* g_kind,
                                  const int* g_mat, const double* g_E, const double* g_nu, const double* g_lmin,
                                  const double* g_lmax, const int* g_count, const int* g_off, const int* idx, int n_pins,
                                  const int* pin_idx, const double* pin_pts, const double* pin_vel,
                                  const oracle_settings* st, int n_steps, int cap, int* nrec, double* rec_prim,
                                  double* rec_comb, int* rec_rej, double* out_x3, double* out_v3, double* step_ms,
                                  char* err, int err_cap) {
    try {
        Elastic s;
        s.build(n_nodes, x3, rest3, masses, n_groups, g_kind, g_mat, g_E, g_nu, g_lmin, g_lmax, g_count, g_off, idx, n_pins, pin_idx);
        std::vector<double> pts(pin_pts, pin_pts + 3 * (size_t)n_pins);
        s.set_pins(n_pins, pin_idx, pts.data());
        s.initialize(*st);
        for (int k = 1; k <= n_steps; ++k) {
            for (int i = 0; i < 3 * n_pins; ++i) pts[i] = pin_pts[i] + k * pin_vel[i];
            s.set_pins(n_pins, pin_idx, pts.data());
            auto t0 = std::chrono::steady_clock::now();
            auto r = s.step();
            auto t1 = std::chrono::steady_clock::now();
            if (step_ms) step_ms[k - 1] = std::chrono::duration<double, std::milli>(t1 - t0).count();
            int cnt = std::min((int)r.prim.size(), cap);
            nrec[k - 1] = (int)r.prim.size();
            for (int i = 0; i < cnt; ++i) {
                rec_prim[(size_t)(k - 1) * cap + i] = r.prim[i];
                rec_comb[(size_t)(k - 1) * cap + i] = r.comb[i];
                rec_rej[(size_t)(k - 1) * cap + i] = r.rej[i];
            }
        }
        std::copy(s.x.begin(), s.x.end(), out_x3);
        std::copy(s.v.begin(), s.v.end(), out_v3);
        return 0;
    } catch (const std::exception& e) {
        if (err && err_cap > 0) { strncpy(err, e.what(), err_cap - 1); err[err_cap - 1] = 0; }
        return 1;
    }
}

extern "C" void oracle_svd3(const double* F9, double* U9, double* S3, double* V9) {
    double F[9], U[9], V[9];
    cm_to_rm3(F9, F);
    jacobi_svd_square<3>(F, U, S3, V);
    for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) { U9[c * 3 + r] = U[r * 3 + c]; V9[c * 3 + r] = V[r * 3 + c]; }
}
extern "C" void oracle_tri_prox_h(const double* z6, double lmin, double lmax, double* out6) { tri_prox_h(z6, lmin, lmax, out6); }
extern "C" void oracle_tri_prox_x(const double* z6, double lmin, double lmax, double* out6) { tri_prox_x(z6, lmin, lmax, out6); }
extern "C" void oracle_tet_prox_linear(const double* z9, double* out9) { tet_linear_prox(z9, out9); }
extern "C" int oracle_tet_prox_hyper(int material, double mu, double lambda, double k, double vol, const double* v9, double* out9) {
    ProxProblem P{material, mu, lambda, k, vol, {}};
    for (int i = 0; i < 9; ++i) { P.v[i] = v9[i]; out9[i] = v9[i]; }
    return lbfgs_minimize(P, out9);
}
extern "C" void oracle_cod_solve(int n, const double* M, const double* b, double* theta) { cod_solve(n, M, b, theta); }
