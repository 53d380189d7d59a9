// Headless driver for the REFERENCE admm-elastic solver (test infrastructure only).
//
// Compiled by oracle/Makefile directly against the reference sources under
// /root/reference (Solver.cpp, TetEnergyTerm.cpp, TriEnergyTerm.cpp, ExplicitForce.cpp)
// -- nothing of the reference is copied into this repository. It replaces the GLFW
// `Application` loop of the samples (e.g. admm_anderson_hard_zxu/samples/Asia2019/
// windyflag.cpp:63-183, beams.cpp) with a file-driven loop:
//
//   scene file (written by aa-admm_amd/scenes.py: write_scene) -> admm::Solver
//     add_nodes (Solver.hpp:265-279) with the initial positions, create_tets_from_mesh /
//     create_tris_from_mesh on the rest positions (AASCENE2; AASCENE1: rest = initial)
//     (TetEnergyTerm.hpp:36-51, TriEnergyTerm.hpp:33-47), set_pins (Solver.cpp:280-315),
//     initialize (Solver.cpp:361-491), step() x n_steps (Solver.cpp:34-234)
//   -> result file: per time step the per-iteration (prim, comb, reject) rows that
//      Solver::save() writes (Solver.hpp:130-155) plus the node positions/velocities,
//      then a trailer with the wall-clock ms of each step() (initialize excluded).
//
// Build with -DREF_VARIANT_H for admm_anderson_hard_zxu, without it for admm_anderson_xzu.
#include "Solver.hpp"
#include "TetEnergyTerm.hpp"
#include "TriEnergyTerm.hpp"
#include "ExplicitForce.hpp"
#ifdef REF_VARIANT_H
#include "PassiveObject.hpp"
#endif
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>
#include <sys/stat.h>

namespace {

struct Reader {
    FILE* f;
    template <typename T> T get() {
        T v;
        if (fread(&v, sizeof(T), 1, f) != 1) { fprintf(stderr, "scene: short read\n"); exit(2); }
        return v;
    }
    template <typename T> void arr(std::vector<T>& out, size_t n) {
        out.resize(n);
        if (n && fread(out.data(), sizeof(T), n, f) != n) { fprintf(stderr, "scene: short read\n"); exit(2); }
    }
};

struct Group {
    int kind, material;
    double E, nu, lmin, lmax;
    int count;
    std::vector<int> idx;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s scene.bin out.bin\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("scene"); return 2; }
    Reader r{f};
    char magic[8];
    if (fread(magic, 1, 8, f) != 8 || (memcmp(magic, "AASCENE1", 8) != 0 && memcmp(magic, "AASCENE2", 8) != 0)) {
        fprintf(stderr, "bad magic\n");
        return 2;
    }
    const bool has_rest = magic[7] == '2';   // AASCENE2: rest positions follow the node positions
    const int variant = r.get<int>();
    const int n = r.get<int>();
    std::vector<double> x, rest, m;
    r.arr(x, 3 * (size_t)n);
    if (has_rest) r.arr(rest, 3 * (size_t)n);
    else rest = x;
    r.arr(m, 3 * (size_t)n);
    const int n_groups = r.get<int>();
    std::vector<Group> groups(n_groups);
    for (auto& g : groups) {
        g.kind = r.get<int>(); g.material = r.get<int>();
        g.E = r.get<double>(); g.nu = r.get<double>(); g.lmin = r.get<double>(); g.lmax = r.get<double>();
        g.count = r.get<int>();
        r.arr(g.idx, (size_t)g.count * (g.kind == 0 ? 4 : 3));
    }
    const int n_pins = r.get<int>();
    std::vector<int> pin_idx;
    std::vector<double> pin_pts, pin_vel;
    r.arr(pin_idx, n_pins);
    r.arr(pin_pts, 3 * (size_t)n_pins);
    r.arr(pin_vel, 3 * (size_t)n_pins);
    const double dt = r.get<double>(), gravity = r.get<double>(), penalty = r.get<double>();
    const int iters = r.get<int>(), accel = r.get<int>(), aa_m = r.get<int>(), n_steps = r.get<int>();
    // optional extras (AAEXTRA1): passive obstacles, collision nodes, wind forces
    struct Obs { int type; double p[8]; };
    std::vector<Obs> obstacles;
    std::vector<int> coll;
    std::vector<std::pair<std::vector<int>, std::vector<double>>> winds;
    char emagic[8];
    if (fread(emagic, 1, 8, f) == 8 && memcmp(emagic, "AAEXTRA1", 8) == 0) {
        const int no = r.get<int>();
        for (int k = 0; k < no; ++k) {
            Obs o;
            o.type = r.get<int>();
            for (double& v : o.p) v = r.get<double>();
            obstacles.push_back(o);
        }
        const int nc = r.get<int>();
        r.arr(coll, nc);
        const int nw = r.get<int>();
        for (int k = 0; k < nw; ++k) {
            const int nt = r.get<int>();
            std::vector<int> tr;
            std::vector<double> d;
            r.arr(tr, 3 * (size_t)nt);
            r.arr(d, 3);
            winds.push_back({tr, d});
        }
    }
    fclose(f);
#ifdef REF_VARIANT_H
    if (variant != 1) { fprintf(stderr, "scene asks for the z-AA (X) variant; this is the H build\n"); return 2; }
#else
    if (variant != 0) { fprintf(stderr, "scene asks for the (u,x)-AA (H) variant; this is the X build\n"); return 2; }
    (void)penalty;
#endif

    admm::Solver solver;
    solver.add_nodes<double>(x.data(), m.data(), n);
    for (auto& g : groups) {
        admm::Lame lame(g.E, g.nu);
        lame.limit_min = g.lmin;
        lame.limit_max = g.lmax;
        if (g.kind == 0) {
            if (g.material == 0)
                admm::create_tets_from_mesh<double, admm::TetEnergyTerm>(solver.energyterms, rest.data(), g.idx.data(), g.count, lame, 0);
            else if (g.material == 1)
                admm::create_tets_from_mesh<double, admm::NeoHookeanTet>(solver.energyterms, rest.data(), g.idx.data(), g.count, lame, 0);
            else
                admm::create_tets_from_mesh<double, admm::StVKTet>(solver.energyterms, rest.data(), g.idx.data(), g.count, lame, 0);
        } else {
            admm::create_tris_from_mesh<double, admm::TriEnergyTerm>(solver.energyterms, rest.data(), g.idx.data(), g.count, lame, 0);
        }
    }
    auto pins_at = [&](int k) {
        std::vector<admm::Solver::Vec3> pts(n_pins);
        for (int i = 0; i < n_pins; ++i)
            for (int j = 0; j < 3; ++j) pts[i][j] = pin_pts[3 * i + j] + k * pin_vel[3 * i + j];
        return pts;
    };
    solver.set_pins(pin_idx, pins_at(0));
    // (plinkohit.cpp:81-96, plinkopony.cpp:54-117: add_obstacle + set_collisions with the node
    // positions; windyflag.cpp:104-127: WindForce on the cloth's faces)
#ifdef REF_VARIANT_H
    for (const Obs& o : obstacles) {
        typedef admm::Solver::Vec3 V3;
        std::shared_ptr<admm::PassiveCollision> obj;
        if (o.type == 0) obj = std::make_shared<admm::Floor>(o.p[0]);
        else if (o.type == 1) obj = std::make_shared<admm::SlideFloor>(V3(o.p[0], o.p[1], o.p[2]), V3(o.p[3], o.p[4], o.p[5]));
        else if (o.type == 2) obj = std::make_shared<admm::Sphere>(V3(o.p[0], o.p[1], o.p[2]), o.p[3]);
        else if (o.type == 3) obj = std::make_shared<admm::PlaneAndHalfSphere>(V3(o.p[0], o.p[1], o.p[2]), o.p[3]);
        else obj = std::make_shared<admm::Cylinder>(V3(o.p[0], o.p[1], o.p[2]), o.p[3]);
        solver.add_obstacle(obj);
    }
    if (!coll.empty()) {
        std::vector<admm::Solver::Vec3> pts;
        for (int i : coll) pts.push_back(admm::Solver::Vec3(x[3 * (size_t)i], x[3 * (size_t)i + 1], x[3 * (size_t)i + 2]));
        solver.set_collisions(coll, pts);
    }
#else
    if (!obstacles.empty() || !coll.empty()) { fprintf(stderr, "obstacles / collisions: H variant only\n"); return 2; }
#endif
    for (auto& w : winds) {
        auto wf = std::make_shared<admm::WindForce>(w.first);
        wf->direction = Eigen::Vector3d(w.second[0], w.second[1], w.second[2]);
        solver.ext_forces.push_back(wf);
    }

    admm::Solver::Settings st;
    st.timestep_s = dt;
    st.gravity = gravity;
    st.admm_iters = iters;
    st.verbose = 0;
    st.Anderson_m = aa_m;
    st.acceleration_type = accel ? admm::Solver::Settings::ANDERSON : admm::Solver::Settings::NOACC;
#ifdef REF_VARIANT_H
    st.penalty = penalty;
#endif
    if (!solver.initialize(st)) { fprintf(stderr, "initialize failed\n"); return 1; }

    mkdir("result", 0755);
    const std::string res = accel ? "result/residual-" + std::to_string(aa_m) + ".txt" : "result/residual-no.txt";
    FILE* out = fopen(argv[2], "wb");
    fwrite(&n_steps, sizeof(int), 1, out);
    std::vector<double> step_ms;
    for (int k = 1; k <= n_steps; ++k) {
        solver.set_pins(pin_idx, pins_at(k));
        auto t0 = std::chrono::steady_clock::now();
        try {
            solver.step();
        } catch (const std::exception& e) {
            // the reference's own abort (e.g. mcloptlib LBFGS.hpp:192-199): the steps done so far
            // are already in `out`; report the step and stop (exit 3) so callers keep them
            fprintf(stderr, "REF_ABORT step %d: %s\n", k, e.what());
            fclose(out);
            return 3;
        }
        step_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        std::vector<double> prim, comb;
        std::vector<int> rej;
        std::ifstream in(res);
        std::string line;
        while (std::getline(in, line)) {
            if (line.empty()) continue;
            std::istringstream ls(line);
            double t, p, c;
            int rj = 0;
            ls >> t >> p >> c;
            if (!(ls >> rj)) rj = 0;
            prim.push_back(p); comb.push_back(c); rej.push_back(rj);
        }
        int nrec = (int)prim.size();
        fwrite(&nrec, sizeof(int), 1, out);
        fwrite(prim.data(), sizeof(double), nrec, out);
        fwrite(comb.data(), sizeof(double), nrec, out);
        fwrite(rej.data(), sizeof(int), nrec, out);
        fwrite(solver.m_x.data(), sizeof(double), 3 * (size_t)n, out);
        fwrite(solver.m_v.data(), sizeof(double), 3 * (size_t)n, out);
        fflush(out);
    }
    fwrite(step_ms.data(), sizeof(double), step_ms.size(), out);   // trailer: wall ms of each step()
    fclose(out);
    return 0;
}
