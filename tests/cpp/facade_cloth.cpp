// C++ caller of the drop-in facade (include/aa_admm.hpp), written the way the reference's
// samples drive admm::Solver (samples/Asia2019/windyflag.cpp): a small hanging cloth,
// (u,x)-Anderson m=6. Prints "<iterations> <comb_0> <comb_last> <x of node 1>".
#include <cstdio>
#include <vector>

#include "aa_admm.hpp"

int main() {
    const int nx = 8, ny = 8;
    std::vector<double> v;
    std::vector<int> t;
    auto corner = [&](int i, int j) { return i * (ny + 1) + j; };
    for (int i = 0; i <= nx; ++i) for (int j = 0; j <= ny; ++j) { v.push_back(i * 0.25); v.push_back(j * 0.25); v.push_back(0); }
    const int c0 = (nx + 1) * (ny + 1);
    for (int i = 0; i < nx; ++i) for (int j = 0; j < ny; ++j) { v.push_back((i + 0.5) * 0.25); v.push_back((j + 0.5) * 0.25); v.push_back(0); }
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < ny; ++j) {
            const int a = corner(i, j), b = corner(i + 1, j), c = corner(i + 1, j + 1), d = corner(i, j + 1), e = c0 + i * ny + j;
            const int tri[12] = {d, a, e, a, b, e, b, c, e, c, d, e};
            t.insert(t.end(), tri, tri + 12);
        }
    const int n = (int)v.size() / 3;
    std::vector<double> m(3 * n, 1e-3);
    admm::Solver solver;
    solver.add_nodes(v.data(), m.data(), n);
    admm::Lame lame(50, 0.1);
    lame.limit_min = 0.95;
    lame.limit_max = 1.05;
    admm::create_tris_from_mesh<double, admm::TriEnergyTerm>(solver.energyterms, v.data(), t.data(), (int)t.size() / 3, lame, 0);
    solver.set_pins({corner(0, 0), corner(0, ny)});
    admm::Solver::Settings st;
    st.admm_iters = 30;
    st.acceleration_type = admm::Solver::Settings::ANDERSON;
    st.Anderson_m = 6;
    st.verbose = 0;
    if (!solver.initialize(st)) { std::printf("initialize failed\n"); return 1; }
    solver.step();
    std::vector<double> prim, comb;
    std::vector<int> rej;
    const int k = solver.history(prim, comb, rej);
    std::printf("%d %.17g %.17g %.17g %.17g %.17g\n", k, comb.front(), comb.back(), solver.m_x[3], solver.m_x[4], solver.m_x[5]);
    return 0;
}
