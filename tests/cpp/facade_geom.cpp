// A reference-style Geometry caller written against include/aa_geometry.hpp (the drop-in
// facade of Geometry/ALMGeometrySolver.h + Constraint.h): it reads a scene in the
// oracle's AAGEOM01 format (aa-admm_amd/geom_scenes.py write_geom_scene), builds the
// constraints as optimize_mesh does (new PointToRefSurfaceConstraint / PlaneConstraint /
// AngleConstraint / EdgeLengthConstraint ..., add_*laplacian, add_closeness), runs
// setup_ADMM + solve_ADMM and writes function_values_ and get_solution() to a binary file.
//   facade_geom scene.bin out.bin [eps] [plain]
// "plain" drives GeometrySolver<3> (Geometry/GeometrySolver.h) instead of ALMGeometrySolver<3>.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <vector>

#include "aa_geometry.hpp"

namespace {
struct Reader {
    std::ifstream f;
    explicit Reader(const char* p) : f(p, std::ios::binary) { if (!f) throw std::runtime_error("cannot open scene"); }
    template <class T> T get() { T v; f.read(reinterpret_cast<char*>(&v), sizeof(T)); return v; }
    template <class T> std::vector<T> vec(size_t n) {
        std::vector<T> v(n);
        if (n) f.read(reinterpret_cast<char*>(v.data()), n * sizeof(T));
        return v;
    }
};
}  // namespace

template <class Solver>
int run(int argc, char** argv) {
    Reader r(argv[1]);
    char magic[8];
    r.f.read(magic, 8);
    if (std::memcmp(magic, "AAGEOM01", 8) != 0) { std::fprintf(stderr, "bad scene\n"); return 2; }
    const int n = r.get<int>();
    Matrix3X x0(n), ref(n);
    auto xv = r.vec<double>(3 * (size_t)n), rv = r.vec<double>(3 * (size_t)n);
    std::memcpy(x0.data(), xv.data(), xv.size() * 8);
    std::memcpy(ref.data(), rv.data(), rv.size() * 8);
    const int nsurf = r.get<int>();
    std::vector<std::shared_ptr<TriMeshAABB>> surf;
    for (int s = 0; s < nsurf; ++s) {
        const int nv = r.get<int>(), nf = r.get<int>();
        auto V = r.vec<double>(3 * (size_t)nv);
        auto F = r.vec<int>(3 * (size_t)nf);
        surf.push_back(std::make_shared<TriMeshAABB>(V, F));
    }
    Solver solver;
    const int ng = r.get<int>();
    for (int gi = 0; gi < ng; ++gi) {
        const int hard = r.get<int>(), type = r.get<int>(), k = r.get<int>(), count = r.get<int>();
        const double w = r.get<double>();
        const int npar = r.get<int>();
        auto idx = r.vec<int>((size_t)count * k);
        auto prm = r.vec<double>((size_t)count * npar);
        auto add = [&](Constraint<3>* c) { hard ? solver.add_hard_constraint(c) : solver.add_soft_constraint(c); };
        if (type == AA_CON_REF_SURFACE) {   // one constraint over points 0..count-1 (WireMeshOpt.cpp:255-259)
            const TriMeshAABB& sf = *surf[(int)prm[0]];
            Matrix3X V((int)(sf.V_.size() / 3));
            Matrix3Xi F((int)(sf.F_.size() / 3));
            std::memcpy(V.data(), sf.V_.data(), sf.V_.size() * 8);
            std::memcpy(F.data(), sf.F_.data(), sf.F_.size() * 4);
            add(new ReferenceSurfceConstraint(count, w, V, F));
            continue;
        }
        for (int i = 0; i < count; ++i) {
            const int* id = &idx[(size_t)i * k];
            const double* p = npar ? &prm[(size_t)i * npar] : nullptr;
            switch (type) {
                case AA_CON_PLANE: add(new PlaneConstraint(std::vector<int>(id, id + k), w)); break;
                case AA_CON_ANGLE: add(new AngleConstraint<3>(id[0], id[1], id[2], w, p[0], p[1])); break;
                case AA_CON_EDGE: add(new EdgeLengthConstraint<3>(id[0], id[1], w, p[0])); break;
                case AA_CON_CLOSENESS: add(new ClosenessConstraint<3>(id[0], w, p)); break;
                case AA_CON_POINT_TO_REF: add(new PointToRefSurfaceConstraint(id[0], w, surf[(int)p[0]])); break;
                default: std::fprintf(stderr, "unknown constraint type %d\n", type); return 2;
            }
        }
    }
    const int nreg = r.get<int>();
    for (int i = 0; i < nreg; ++i) {
        const int kind = r.get<int>(), len = r.get<int>();
        const double w = r.get<double>();
        auto idx = r.vec<int>(len);
        auto coef = r.vec<double>(len);
        auto tgt = r.vec<double>(3);
        if (kind == 2) solver.add_closeness(idx[0], w, tgt.data());
        else if (kind == 1) solver.add_relative_laplacian(idx, coef, w, ref);
        else solver.add_laplacian(idx, coef, w);
    }
    const double penalty = r.get<double>();
    const int iters = r.get<int>(), m = r.get<int>();
    if (!solver.setup_ADMM(n, penalty, LDLT_SOLVER)) { std::fprintf(stderr, "setup_ADMM failed: %s\n", aa_last_error()); return 1; }
    const double eps = argc > 3 ? std::atof(argv[3]) : 1e-10;
    solver.solve_ADMM(x0, eps, iters, m);
    std::ofstream o(argv[2], std::ios::binary);
    const int nf = (int)solver.function_values_.size();
    o.write(reinterpret_cast<const char*>(&nf), 4);
    o.write(reinterpret_cast<const char*>(solver.function_values_.data()), 8 * (size_t)nf);
    o.write(reinterpret_cast<const char*>(solver.get_solution().data()), 24 * (size_t)n);
    std::printf("%d %.17g %.17g\n", nf, nf ? solver.function_values_[0] : 0.0, nf ? solver.function_values_.back() : 0.0);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) { std::fprintf(stderr, "usage: facade_geom scene.bin out.bin [eps] [plain]\n"); return 2; }
    if (argc > 4 && std::strcmp(argv[4], "plain") == 0) return run<GeometrySolver<3>>(argc, argv);
    return run<ALMGeometrySolver<3>>(argc, argv);
}
