// ORACLE -- test infrastructure only (see oracle.h). Pieces shared by the elastic and the
// geometry restatements: Anderson acceleration (identical arithmetic in the three reference
// copies, admm_anderson_hard_zxu/src/AndersonAcceleration.h:40-211 == Geometry/AndersonAcceleration.h,
// admm_anderson_xzu/src/AndersonAcceleration.h:138-200) and an envelope Cholesky standing in
// for Eigen's SimplicialLDLT (same solution to rounding).
#pragma once
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "oracle_svd.hpp"

namespace oracle {

// ------------------------------------------------------------------ Anderson acceleration
// One class for both bookkeeping styles; the arithmetic of compute_impl is identical in all
// three reference copies.
struct Anderson {
    int m = 0, dim = 0, eff = 0, iter = -1, col = -1;
    std::vector<double> u, F, dF, dG, scale, Mg, theta, G;
    void init(int m_, int dim_, int eff_, const double* u0) {
        m = m_; dim = dim_; eff = eff_;
        u.assign(u0, u0 + dim);
        F.assign(eff, 0.0); dF.assign((size_t)eff * m, 0.0); dG.assign((size_t)dim * m, 0.0);
        scale.assign(m, 0.0); Mg.assign((size_t)m * m, 0.0); theta.assign(m, 0.0); G.assign(dim, 0.0);
        iter = 0; col = 0;
    }
    void reset(const double* u0) { std::copy(u0, u0 + dim, u.begin()); iter = 0; col = 0; }
    void replace(const double* u0) { std::copy(u0, u0 + dim, u.begin()); }
    void compute(const double* g, double* out) {
        std::copy(g, g + dim, G.begin());
        for (int i = 0; i < eff; ++i) F[i] = G[i] - u[i];
        if (iter == 0) {
            for (int i = 0; i < eff; ++i) dF[i] = -F[i];
            for (int i = 0; i < dim; ++i) dG[i] = -G[i];
            u = G;
        } else {
            double* dFj = &dF[(size_t)col * eff];
            double* dGj = &dG[(size_t)col * dim];
            for (int i = 0; i < eff; ++i) dFj[i] += F[i];
            for (int i = 0; i < dim; ++i) dGj[i] += G[i];
            const double eps = 1e-14;
            double nrm = 0;
            for (int i = 0; i < eff; ++i) nrm += dFj[i] * dFj[i];
            double sc = std::max(eps, std::sqrt(nrm));
            scale[col] = sc;
            for (int i = 0; i < eff; ++i) dFj[i] /= sc;
            int mk = std::min(m, iter);
            if (mk == 1) {
                theta[0] = 0;
                double sq = 0;
                for (int i = 0; i < eff; ++i) sq += dFj[i] * dFj[i];
                Mg[0] = sq;
                double dn = std::sqrt(sq);
                if (dn > eps) {
                    double t = 0;
                    for (int i = 0; i < eff; ++i) t += (dFj[i] / dn) * (F[i] / dn);
                    theta[0] = t;
                }
            } else {
                for (int c = 0; c < mk; ++c) {
                    const double* dFc = &dF[(size_t)c * eff];
                    double t = 0;
                    for (int i = 0; i < eff; ++i) t += dFj[i] * dFc[i];
                    Mg[(size_t)c * m + col] = t;   // row col  (column-major m x m)
                    Mg[(size_t)col * m + c] = t;   // column col
                }
                std::vector<double> Mk((size_t)mk * mk), rhs(mk);
                for (int c = 0; c < mk; ++c)
                    for (int r = 0; r < mk; ++r) Mk[(size_t)c * mk + r] = Mg[(size_t)c * m + r];
                for (int c = 0; c < mk; ++c) {
                    const double* dFc = &dF[(size_t)c * eff];
                    double t = 0;
                    for (int i = 0; i < eff; ++i) t += dFc[i] * F[i];
                    rhs[c] = t;
                }
                cod_solve(mk, Mk.data(), rhs.data(), theta.data());
            }
            for (int i = 0; i < dim; ++i) {
                double s = 0;
                for (int c = 0; c < mk; ++c) s += dG[(size_t)c * dim + i] * (theta[c] / scale[c]);
                u[i] = G[i] - s;
            }
            col = (col + 1) % m;
            double* nF = &dF[(size_t)col * eff];
            double* nG = &dG[(size_t)col * dim];
            for (int i = 0; i < eff; ++i) nF[i] = -F[i];
            for (int i = 0; i < dim; ++i) nG[i] = -G[i];
        }
        ++iter;
        std::copy(u.begin(), u.end(), out);
    }
};

// ------------------------------------------------------------------ envelope Cholesky
struct Envelope {
    int n = 0;
    std::vector<int> first;       // first column of row i
    std::vector<size_t> start;    // offset of row i in L
    std::vector<double> L;
    double& at(int i, int j) { return L[start[i] + (j - first[i])]; }
    void factor() {
        for (int i = 0; i < n; ++i) {
            for (int j = first[i]; j <= i; ++j) {
                double s = at(i, j);
                int k0 = std::max(first[i], first[j]);
                for (int k = k0; k < j; ++k) s -= at(i, k) * at(j, k);
                if (j < i) at(i, j) = s / at(j, j);
                else {
                    if (!(s > 0)) throw std::runtime_error("oracle: global matrix not SPD");
                    at(i, i) = std::sqrt(s);
                }
            }
        }
    }
    void solve3(double* b /* n x 3 in place */) {
        for (int i = 0; i < n; ++i)
            for (int c = 0; c < 3; ++c) {
                double s = b[3 * i + c];
                for (int k = first[i]; k < i; ++k) s -= at(i, k) * b[3 * k + c];
                b[3 * i + c] = s / at(i, i);
            }
        for (int i = n - 1; i >= 0; --i)
            for (int c = 0; c < 3; ++c) {
                double xi = b[3 * i + c] / at(i, i);
                b[3 * i + c] = xi;
                for (int k = first[i]; k < i; ++k) b[3 * k + c] -= at(i, k) * xi;
            }
    }
};


// reverse Cuthill-McKee order of the vertices with seen[v] == 0 (keeps the envelope small)
inline std::vector<int> rcm_order(const std::vector<std::vector<int>>& adj, std::vector<int> seen) {
    const int n = (int)adj.size();
    std::vector<int> order;
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
    return order;
}

}  // namespace oracle
