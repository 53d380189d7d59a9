// CPU check of the partitioned global solve.
//
// Builds an SPD matrix with the structure of the elastic global matrix A_s (lumped mass +
// dt^2 * tet-mesh stiffness pattern) on a structured block, orders it by nested dissection
// with the top bisections forced (P parts, P = 1, 2, 3, 4, 8), factors it once, and then runs
// the solve the way P GPUs do, on a PARTIAL right-hand side (own rows complete, top rows split
// between the ranks arbitrarily), each "rank" a thread:
//  * separate top separators (merge_top = false, the round-1 layout): each rank forward-sweeps
//    its own part plus the top, the top rows of the forward results are summed (the
//    all-reduce), and each rank back-substitutes the top and its own part;
//  * one dense top root (merge_top = true, DirectSolver's default): each rank forward-sweeps its
//    own part, the top front is summed, each rank computes its row slice of y_top = Linv f_top
//    (equal triangle areas in blocks of kBlk rows, as DirectSolver::build) and the backward
//    products of those rows (a partial x_top), x_top is summed, each rank back-substitutes its
//    own part.
// The assembled solution must match the unpartitioned solve and A x = b.
//   g++ -O2 -std=c++17 -fopenmp tests/cpp/part_solve.cpp aa-admm_amd/csrc/spd_direct.cpp
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <condition_variable>
#include <cstdio>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../aa-admm_amd/csrc/spd_direct.hpp"

namespace {

struct SumBarrier {   // all-reduce (sum) of equal-length vectors across P threads
    int P, arrived = 0, gen = 0;
    std::vector<double> acc[2];   // by generation parity: a thread already in the next reduce
                                  // must not clear the sum the others are still copying out
    std::mutex mu;
    std::condition_variable cv;
    explicit SumBarrier(int p) : P(p) {}
    void reduce(double* v, size_t n) {
        std::unique_lock<std::mutex> lk(mu);
        const int g = gen;
        std::vector<double>& a = acc[g & 1];
        if (arrived == 0) a.assign(n, 0.0);
        for (size_t i = 0; i < n; ++i) a[i] += v[i];   // order of arrival differs: compare to tolerance
        if (++arrived == P) { arrived = 0; ++gen; cv.notify_all(); }
        else cv.wait(lk, [&] { return gen != g; });
        for (size_t i = 0; i < n; ++i) v[i] = a[i];
    }
};

// restatement of DirectSolver's dense-top partitioned solve (direct_solve.hip, solve_nr)
constexpr int kBlk = 8;   // row block of the split (DirectSolver: kFwdRows = 128; small here so every rank gets rows)
void solve_dense_top(const aa::SupernodalFactor& F, const aa::NdTree& T, int part, int P, std::vector<double>& b,
                     SumBarrier& bar) {
    const int nn = F.n_nodes;
    int top = -1;
    for (int s = 0; s < nn; ++s)
        if (T.part[s] == -1 && F.end[s] > F.beg[s]) { if (top >= 0) std::abort(); top = s; }
    if (top < 0 || F.parent[top] >= 0 || !F.bnd[top].empty()) std::abort();
    auto own = [&](int s) { return T.part[s] == part; };
    std::vector<double> t;
    for (int s = 0; s < nn; ++s) {   // forward over the own part
        if (!own(s)) continue;
        const int b0 = F.beg[s], p = F.end[s] - b0, nb = (int)F.bnd[s].size();
        t.assign((size_t)p * 3, 0.0);
        for (int i = 0; i < p; ++i)
            for (int k = 0; k <= i; ++k)
                for (int c = 0; c < 3; ++c) t[3 * i + c] += F.Linv[s][(size_t)i * p + k] * b[3 * (size_t)(b0 + k) + c];
        for (int i = 0; i < p; ++i) for (int c = 0; c < 3; ++c) b[3 * (size_t)(b0 + i) + c] = t[3 * i + c];
        for (int a = 0; a < nb; ++a)
            for (int j = 0; j < p; ++j)
                for (int c = 0; c < 3; ++c) b[3 * (size_t)F.bnd[s][a] + c] -= F.LBP[s][(size_t)a * p + j] * t[3 * j + c];
    }
    const int tb = F.beg[top], pt = F.end[top] - tb;
    double* f = b.data() + 3 * (size_t)tb;
    bar.reduce(f, 3 * (size_t)pt);   // the summed top front
    // this rank's rows: equal triangle areas in kBlk-row blocks
    const int nblk = (pt + kBlk - 1) / kBlk;
    const double total = 0.5 * pt * (pt + 1.0);
    std::vector<int> cut(P + 1, nblk);
    cut[0] = 0;
    double acc = 0;
    for (int bk = 0, r = 1; bk < nblk && r < P; ++bk) {
        const double r0 = (double)bk * kBlk, r1 = std::min<double>(pt, r0 + kBlk);
        acc += 0.5 * (r1 * (r1 + 1) - r0 * (r0 + 1));
        while (r < P && acc >= total * r / P) cut[r++] = bk + 1;
    }
    const int a0 = std::min(pt, cut[part] * kBlk), a1 = std::min(pt, cut[part + 1] * kBlk);
    const std::vector<double>& L = F.Linv[top];
    std::vector<double> y(3 * (size_t)pt, 0.0), x(3 * (size_t)pt, 0.0);
    for (int i = a0; i < a1; ++i)
        for (int k = 0; k <= i; ++k)
            for (int c = 0; c < 3; ++c) y[3 * i + c] += L[(size_t)i * pt + k] * f[3 * k + c];
    for (int j = 0; j < a1; ++j)
        for (int i = std::max(j, a0); i < a1; ++i)
            for (int c = 0; c < 3; ++c) x[3 * j + c] += L[(size_t)i * pt + j] * y[3 * i + c];
    bar.reduce(x.data(), x.size());   // the summed x_top
    std::copy(x.begin(), x.end(), f);
    for (int s = nn - 1; s >= 0; --s) {   // backward over the own part
        if (!own(s)) continue;
        const int b0 = F.beg[s], p = F.end[s] - b0, nb = (int)F.bnd[s].size();
        t.assign((size_t)p * 3, 0.0);
        for (int j = 0; j < p; ++j)
            for (int c = 0; c < 3; ++c) {
                double v = b[3 * (size_t)(b0 + j) + c];
                for (int a = 0; a < nb; ++a) v -= F.LBP[s][(size_t)a * p + j] * b[3 * (size_t)F.bnd[s][a] + c];
                t[3 * j + c] = v;
            }
        for (int j = 0; j < p; ++j)
            for (int c = 0; c < 3; ++c) {
                double v = 0;
                for (int i = j; i < p; ++i) v += F.Linv[s][(size_t)i * p + j] * t[3 * i + c];
                b[3 * (size_t)(b0 + j) + c] = v;
            }
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int nx = argc > 1 ? std::atoi(argv[1]) : 13, ny = argc > 2 ? std::atoi(argv[2]) : 9,
              nz = argc > 3 ? std::atoi(argv[3]) : 11;
    const int n = nx * ny * nz;
    auto id = [&](int i, int j, int k) { return (i * ny + j) * nz + k; };
    std::vector<double> xyz(3 * (size_t)n);
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < ny; ++j)
            for (int k = 0; k < nz; ++k) {
                const int v = id(i, j, k);
                xyz[3 * v] = 0.1 * i; xyz[3 * v + 1] = 0.1 * j + 0.001 * i; xyz[3 * v + 2] = 0.1 * k;
            }
    // 27-point connectivity (the pattern of a hexahedral/tet block), weights from a seeded rng
    std::mt19937_64 rng(20191015);
    std::uniform_real_distribution<double> U(0.5, 1.5);
    std::vector<std::vector<std::pair<int, double>>> rows(n);
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < ny; ++j)
            for (int k = 0; k < nz; ++k) {
                const int a = id(i, j, k);
                for (int di = 0; di <= 1; ++di)
                    for (int dj = -1; dj <= 1; ++dj)
                        for (int dk = -1; dk <= 1; ++dk) {
                            if (di == 0 && (dj < 0 || (dj == 0 && dk <= 0))) continue;
                            const int i2 = i + di, j2 = j + dj, k2 = k + dk;
                            if (i2 >= nx || j2 < 0 || j2 >= ny || k2 < 0 || k2 >= nz) continue;
                            const int b = id(i2, j2, k2);
                            const double w = U(rng);
                            rows[a].push_back({b, -w}); rows[b].push_back({a, -w});
                            rows[a].push_back({a, w}); rows[b].push_back({b, w});
                        }
                rows[a].push_back({a, 0.05 * U(rng)});   // mass
            }
    std::vector<int> aptr(n + 1, 0), aj;
    for (int v = 0; v < n; ++v) {
        std::vector<int> l;
        for (auto& e : rows[v]) if (e.first != v) l.push_back(e.first);
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
        aj.insert(aj.end(), l.begin(), l.end());
        aptr[v + 1] = (int)aj.size();
    }
    std::vector<double> b0(3 * (size_t)n);
    std::normal_distribution<double> N01;
    for (auto& v : b0) v = N01(rng);

    int fails = 0;
    // (P, dense top, rows of each part's amalgamated upper levels)
    const int cases[][3] = {{1, 0, 0}, {2, 0, 0}, {4, 0, 0}, {8, 0, 0}, {2, 1, 0}, {3, 1, 0}, {4, 1, 0}, {8, 1, 0},
                            {4, 1, 64}, {8, 1, 40}};
    for (const auto& cs : cases) {
        const int P = cs[0];
        const bool dense = cs[1] != 0;
        aa::NdTree T = aa::nested_dissection(n, xyz.data(), aptr, aj, 8, 0, P > 1 ? P : 0, dense, cs[2]);
        std::vector<int> inv(n);
        for (int q = 0; q < n; ++q) inv[T.perm[q]] = q;
        aa::CsrMatrix A;
        A.n = n;
        A.ptr.assign(n + 1, 0);
        for (int q = 0; q < n; ++q) {
            std::vector<std::pair<int, double>> r;
            for (auto& e : rows[T.perm[q]]) r.push_back({inv[e.first], e.second});
            std::sort(r.begin(), r.end());
            for (size_t k = 0; k < r.size();) {
                size_t k2 = k;
                double s = 0;
                while (k2 < r.size() && r[k2].first == r[k].first) s += r[k2++].second;
                A.col.push_back(r[k].first); A.val.push_back(s);
                k = k2;
            }
            A.ptr[q + 1] = (int)A.col.size();
        }
        aa::SupernodalFactor F = aa::multifrontal_cholesky(A, T);
        std::vector<double> b(3 * (size_t)n);
        for (int q = 0; q < n; ++q) for (int c = 0; c < 3; ++c) b[3 * q + c] = b0[3 * T.perm[q] + c];
        std::vector<double> xref = b;
        aa::factor_solve_host(F, xref);
        // residual of the unpartitioned solve
        double rmax = 0, bmax = 0;
        for (int q = 0; q < n; ++q)
            for (int c = 0; c < 3; ++c) {
                double s = 0;
                for (int k = A.ptr[q]; k < A.ptr[q + 1]; ++k) s += A.val[k] * xref[3 * A.col[k] + c];
                rmax = std::max(rmax, std::fabs(s - b[3 * q + c]));
                bmax = std::max(bmax, std::fabs(b[3 * q + c]));
            }
        // partitioned: top rows split with random weights summing to one
        std::vector<std::vector<double>> bp(P, std::vector<double>(3 * (size_t)n, 0.0));
        for (int q = 0; q < n; ++q) {
            int owner = -1;
            for (int pp = 0; pp < P; ++pp) if (q >= T.part_beg[pp] && q < T.part_end[pp]) owner = pp;
            if (owner >= 0) { for (int c = 0; c < 3; ++c) bp[owner][3 * q + c] = b[3 * q + c]; continue; }
            std::vector<double> w(P);
            double ws = 0;
            for (auto& x : w) { x = U(rng); ws += x; }
            for (int pp = 0; pp < P; ++pp) for (int c = 0; c < 3; ++c) bp[pp][3 * q + c] = b[3 * q + c] * w[pp] / ws;
        }
        SumBarrier bar(P);
        // each rank factors only its own part and the top (aa::PartFactor: the top fronts are the
        // sum of the ranks' partial fronts), then solves with its own factor
        std::vector<aa::SupernodalFactor> Fr(P);
        std::vector<std::thread> th;
        for (int pp = 0; pp < P; ++pp)
            th.emplace_back([&, pp] {
                aa::PartFactor pf;
                pf.my_part = pp;
                pf.first = pp == 0;
                pf.reduce_host = [&](double* v, size_t m) { bar.reduce(v, m); };
                Fr[pp] = P > 1 ? aa::multifrontal_cholesky(A, T, nullptr, &pf) : F;
                const aa::SupernodalFactor& Fp = Fr[pp];
                if (dense) solve_dense_top(Fp, T, pp, P, bp[pp], bar);
                else aa::factor_solve_host_part(Fp, P > 1 ? &T : nullptr, P > 1 ? pp : -1, bp[pp],
                                                [&](double* v, size_t m) { bar.reduce(v, m); });
            });
        for (auto& t : th) t.join();
        // own part bit-identical to the whole factorization, other parts not factored, the top
        // the same on every rank and within rounding of the whole factorization's
        bool fac_ok = true;
        double top_rel = 0;
        for (int pp = 0; P > 1 && pp < P; ++pp)
            for (int s = 0; s < F.n_nodes; ++s) {
                if (T.part[s] == pp) fac_ok = fac_ok && Fr[pp].Linv[s] == F.Linv[s] && Fr[pp].LBP[s] == F.LBP[s];
                else if (T.part[s] >= 0) fac_ok = fac_ok && Fr[pp].Linv[s].empty();
                else {
                    fac_ok = fac_ok && Fr[pp].Linv[s] == Fr[0].Linv[s] && Fr[pp].Linv[s].size() == F.Linv[s].size();
                    double mx = 0;
                    for (double v : F.Linv[s]) mx = std::max(mx, std::fabs(v));
                    for (size_t k = 0; k < F.Linv[s].size() && k < Fr[pp].Linv[s].size(); ++k)
                        top_rel = std::max(top_rel, std::fabs(Fr[pp].Linv[s][k] - F.Linv[s][k]) / mx);
                }
            }
        fac_ok = fac_ok && top_rel <= 1e-11;
        double emax = 0, xmax = 0, tdiff = 0;
        for (int q = 0; q < n; ++q) {
            int owner = -1;
            for (int pp = 0; pp < P; ++pp) if (q >= T.part_beg[pp] && q < T.part_end[pp]) owner = pp;
            for (int c = 0; c < 3; ++c) {
                const double xv = bp[owner >= 0 ? owner : 0][3 * q + c];
                emax = std::max(emax, std::fabs(xv - xref[3 * q + c]));
                xmax = std::max(xmax, std::fabs(xref[3 * q + c]));
                if (owner < 0)   // top rows: identical on every rank
                    for (int pp = 1; pp < P; ++pp) tdiff = std::max(tdiff, std::fabs(bp[pp][3 * q + c] - bp[0][3 * q + c]));
            }
        }
        int ntop = 0;
        for (int s = 0; s < F.n_nodes; ++s) ntop += T.part[s] == -1 && F.end[s] > F.beg[s];
        const bool ok = fac_ok && rmax <= 1e-10 * bmax && emax <= 1e-10 * xmax && tdiff == 0.0 && (P == 1 || T.top_beg < n) &&
                        (int)T.part_beg.size() == std::max(1, P) && (!dense || ntop == 1);
        std::printf("part_top_rows=%d ", cs[2]);
        std::printf("parts=%d dense_top=%d n=%d top_rows=%d top_nodes=%d nnzL=%zu |Ax-b|=%.2e |x_part-x|=%.2e top_spread=%.1e "
                    "part_factor_top_rel=%.1e %s\n",
                    P, (int)dense, n, n - T.top_beg, ntop, F.nnz_L, rmax / bmax, emax / xmax, tdiff, top_rel, ok ? "OK" : "FAIL");
        if (!ok) ++fails;
    }
    // a matrix that is not positive definite in ONE part only (one node's diagonal negated): the
    // rank owning it fails in its own subtrees, before the first top front's sum -- every rank
    // must still throw (aa::multifrontal_cholesky agrees on the own-part outcome first) instead
    // of the others waiting forever in the top front's all-reduce
    for (const int P : {2, 4}) {
        aa::NdTree T = aa::nested_dissection(n, xyz.data(), aptr, aj, 8, 0, P, true, 0);
        std::vector<int> inv(n);
        for (int q = 0; q < n; ++q) inv[T.perm[q]] = q;
        aa::CsrMatrix A;
        A.n = n;
        A.ptr.assign(n + 1, 0);
        const int bad = T.part_beg[P - 1] + (T.part_end[P - 1] - T.part_beg[P - 1]) / 2;   // inside the last part
        for (int q = 0; q < n; ++q) {
            std::vector<std::pair<int, double>> r;
            for (auto& e : rows[T.perm[q]]) r.push_back({inv[e.first], e.second});
            std::sort(r.begin(), r.end());
            for (size_t k = 0; k < r.size();) {
                size_t k2 = k;
                double sum = 0;
                while (k2 < r.size() && r[k2].first == r[k].first) sum += r[k2++].second;
                A.col.push_back(r[k].first); A.val.push_back(q == bad && r[k].first == q ? -sum : sum);
                k = k2;
            }
            A.ptr[q + 1] = (int)A.col.size();
        }
        SumBarrier bar(P);
        std::vector<int> threw(P, 0);
        std::vector<std::thread> th;
        for (int pp = 0; pp < P; ++pp)
            th.emplace_back([&, pp] {
                aa::PartFactor pf;
                pf.my_part = pp;
                pf.first = pp == 0;
                pf.reduce_host = [&](double* v, size_t m) { bar.reduce(v, m); };
                try {
                    aa::multifrontal_cholesky(A, T, nullptr, &pf);
                } catch (const std::exception&) {
                    threw[pp] = 1;
                }
            });
        for (auto& t : th) t.join();   // a rank left waiting in a collective would hang here
        int nthrew = 0;
        for (int v : threw) nthrew += v;
        std::printf("singular part: parts=%d ranks_threw=%d %s\n", P, nthrew, nthrew == P ? "SINGULAR_OK" : "SINGULAR_FAIL");
        if (nthrew != P) ++fails;
    }
    return fails ? 1 : 0;
}
