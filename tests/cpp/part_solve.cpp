// CPU check of the partitioned global solve.
//
// Builds an SPD matrix with the structure of the elastic global matrix A_s (lumped mass +
// dt^2 * tet-mesh stiffness pattern) on a structured block, orders it by nested dissection
// with the first L bisections forced (2^L parts), factors it once, and then runs the solve the
// way P GPUs do: each "rank" (a thread here) forward-sweeps its own part plus the shared top
// separators on a PARTIAL right-hand side (own rows complete, top rows split between the
// ranks arbitrarily), the top rows of the forward results are summed (the all-reduce), and
// each rank back-substitutes the top and its own part. The assembled solution must match the
// unpartitioned solve and A x = b.
//   g++ -O2 -std=c++17 -fopenmp tests/cpp/part_solve.cpp aa-admm_amd/csrc/spd_direct.cpp
#include <cmath>
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
    std::vector<double> acc;
    std::mutex mu;
    std::condition_variable cv;
    explicit SumBarrier(int p) : P(p) {}
    void reduce(double* v, size_t n) {
        std::unique_lock<std::mutex> lk(mu);
        if (arrived == 0) acc.assign(n, 0.0);
        for (size_t i = 0; i < n; ++i) acc[i] += v[i];   // order of arrival differs: compare to tolerance
        const int g = gen;
        if (++arrived == P) { arrived = 0; ++gen; cv.notify_all(); }
        else cv.wait(lk, [&] { return gen != g; });
        for (size_t i = 0; i < n; ++i) v[i] = acc[i];
    }
};

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
    for (int L = 0; L <= 3; ++L) {
        const int P = 1 << L;
        aa::NdTree T = aa::nested_dissection(n, xyz.data(), aptr, aj, 8, 0, L);
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
        std::vector<std::thread> th;
        for (int pp = 0; pp < P; ++pp)
            th.emplace_back([&, pp] {
                aa::factor_solve_host_part(F, L > 0 ? &T : nullptr, L > 0 ? pp : -1, bp[pp],
                                           [&](double* v, size_t m) { bar.reduce(v, m); });
            });
        for (auto& t : th) t.join();
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
        const bool ok = rmax <= 1e-10 * bmax && emax <= 1e-10 * xmax && tdiff == 0.0 && (L == 0 || T.top_beg < n);
        std::printf("parts=%d n=%d top_rows=%d nnzL=%zu |Ax-b|=%.2e |x_part-x|=%.2e top_spread=%.1e %s\n", P, n,
                    n - T.top_beg, F.nnz_L, rmax / bmax, emax / xmax, tdiff, ok ? "OK" : "FAIL");
        if (!ok) ++fails;
    }
    return fails ? 1 : 0;
}
