// Headless driver for the REFERENCE Geometry ALM solver (test infrastructure only).
//
// Compiled by oracle/Makefile against the reference sources where they lie under
// /root/reference/Geometry (ALMGeometrySolver.h, Constraint.h, LinearRegularization.h,
// AndersonAcceleration.h, SPDSolver.h, TriMeshAABB.h + vendored Eigen / igl / OpenMesh) --
// nothing of the reference is copied here. It replaces the mesh-reading `main`s of
// Geometry/PlanarityOpt.cpp:289-332 and Geometry/WireMeshOpt.cpp:341-443 with a file-driven
// setup so that any constraint set (written by aa-admm_amd/geom_scenes.py) can be solved:
//
//   AAGEOM01 scene -> ALMGeometrySolver<3>
//     add_soft_constraint / add_hard_constraint (ALMGeometrySolver.h:288-294) with
//       PlaneConstraint, AngleConstraint<3>, EdgeLengthConstraint<3>, ClosenessConstraint<3>,
//       PointToRefSurfaceConstraint (shared TriMeshAABB built from an OpenMesh TriMesh),
//       ReferenceSurfceConstraint (Constraint.h:194-414)
//     add_laplacian / add_relative_laplacian / add_closeness (ALMGeometrySolver.h:296-318)
//     setup_ADMM(n, penalty, LDLT) (:81-161), solve_ADMM(x0, eps, iters, m) (:163-283)
//   -> AAGEOMR1 result: function_values_, elapsed_time_, get_solution(), timings.
// Built with -DREF_PLAIN (oracle/_ref/ref_geom_plain) the same scene drives the reference's
// GeometrySolver<3> instead (Geometry/GeometrySolver.h:85-263: project_and_combine for the
// soft constraints, Anderson on (u, x) with `replace` on a residual increase).
#ifdef REF_PLAIN
#include "GeometrySolver.h"
typedef GeometrySolver<3> RefSolver;
#else
#include "ALMGeometrySolver.h"
typedef ALMGeometrySolver<3> RefSolver;
#endif
#include "Constraint.h"
#include "MeshTypes.h"
#include "TriMeshAABB.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

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

enum { PLANE = 0, ANGLE = 1, EDGE = 2, CLOSENESS = 3, POINT_TO_REF = 4, REF_SURFACE = 5 };

struct Surface {
    std::vector<double> V;
    std::vector<int> F;
    std::shared_ptr<TriMeshAABB> aabb;
    int faces_added = 0;
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: %s scene.bin out.bin\n", argv[0]); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("scene"); return 2; }
    Reader r{f};
    char magic[8];
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "AAGEOM01", 8) != 0) { fprintf(stderr, "bad magic\n"); return 2; }
    const int n = r.get<int>();
    std::vector<double> x0, refp;
    r.arr(x0, 3 * (size_t)n);
    r.arr(refp, 3 * (size_t)n);
    const int n_surf = r.get<int>();
    std::vector<Surface> surf(n_surf);
    int faces_added = 0;
    for (auto& s : surf) {
        const int nv = r.get<int>(), nf = r.get<int>();
        r.arr(s.V, 3 * (size_t)nv);
        r.arr(s.F, 3 * (size_t)nf);
        TriMesh tm;
        std::vector<TriMesh::VertexHandle> vh(nv);
        for (int i = 0; i < nv; ++i) vh[i] = tm.add_vertex(TriMesh::Point(s.V[3 * i], s.V[3 * i + 1], s.V[3 * i + 2]));
        for (int i = 0; i < nf; ++i)
            if (tm.add_face(vh[s.F[3 * i]], vh[s.F[3 * i + 1]], vh[s.F[3 * i + 2]]).is_valid()) ++s.faces_added;
        faces_added += s.faces_added;
        s.aabb = std::make_shared<TriMeshAABB>(tm);
    }
    Eigen::Map<const Matrix3X> X0(x0.data(), 3, n), REF(refp.data(), 3, n);

    RefSolver solver;
    const int n_groups = r.get<int>();
    for (int gi = 0; gi < n_groups; ++gi) {
        const int hard = r.get<int>(), type = r.get<int>(), k = r.get<int>(), count = r.get<int>();
        const double weight = r.get<double>();
        const int npar = r.get<int>();
        std::vector<int> idx;
        std::vector<double> prm;
        r.arr(idx, (size_t)count * k);
        r.arr(prm, (size_t)count * npar);
        auto add = [&](Constraint<3>* c) { if (hard) solver.add_hard_constraint(c); else solver.add_soft_constraint(c); };
        if (type == REF_SURFACE) {   // one constraint over all points (WireMeshOpt.cpp:255-259)
            const Surface& s = surf[(int)prm[0]];
            Eigen::Map<const Matrix3X> V(s.V.data(), 3, s.V.size() / 3);
            Eigen::Map<const Eigen::Matrix3Xi> F(s.F.data(), 3, s.F.size() / 3);
            add(new ReferenceSurfceConstraint(count, weight, V, F));
            continue;
        }
        for (int c = 0; c < count; ++c) {
            const int* id = &idx[(size_t)c * k];
            const double* p = &prm[(size_t)c * npar];
            switch (type) {
                case PLANE: add(new PlaneConstraint(std::vector<int>(id, id + k), weight)); break;
                case ANGLE: add(new AngleConstraint<3>(id[0], id[1], id[2], weight, p[0], p[1])); break;
                case EDGE: add(new EdgeLengthConstraint<3>(id[0], id[1], weight, p[0])); break;
                case CLOSENESS: add(new ClosenessConstraint<3>(id[0], weight, Vector3(p[0], p[1], p[2]))); break;
                case POINT_TO_REF: add(new PointToRefSurfaceConstraint(id[0], weight, surf[(int)p[0]].aabb)); break;
                default: fprintf(stderr, "unknown constraint type %d\n", type); return 2;
            }
        }
    }
    const int n_reg = r.get<int>();
    for (int i = 0; i < n_reg; ++i) {
        const int kind = r.get<int>(), k = r.get<int>();
        const double w = r.get<double>();
        std::vector<int> idx;
        std::vector<double> coef, tgt;
        r.arr(idx, k);
        r.arr(coef, k);
        r.arr(tgt, 3);
        if (kind == 0) solver.add_laplacian(idx, coef, w);
        else if (kind == 1) solver.add_relative_laplacian(idx, coef, w, Matrix3X(REF));
        else solver.add_closeness(idx[0], w, Vector3(tgt[0], tgt[1], tgt[2]));
    }
    const double penalty = r.get<double>();
    const int iters = r.get<int>(), m = r.get<int>();
    fclose(f);

    auto t0 = std::chrono::steady_clock::now();
    if (!solver.setup_ADMM(n, penalty)) { fprintf(stderr, "setup_ADMM failed\n"); return 3; }
    auto t1 = std::chrono::steady_clock::now();
    solver.solve_ADMM(Matrix3X(X0), 1e-8, iters, m);   // eps is unused by the reference loop
    auto t2 = std::chrono::steady_clock::now();
    const double setup_s = std::chrono::duration<double>(t1 - t0).count();
    const double loop_s = std::chrono::duration<double>(t2 - t1).count();

    FILE* o = fopen(argv[2], "wb");
    if (!o) { perror("out"); return 2; }
    fwrite("AAGEOMR1", 1, 8, o);
    const int nrec = (int)solver.function_values_.size();
    fwrite(&nrec, 4, 1, o);
    fwrite(solver.function_values_.data(), 8, nrec, o);
    fwrite(solver.elapsed_time_.data(), 8, nrec, o);
    const Matrix3X& xs = solver.get_solution();
    fwrite(xs.data(), 8, 3 * (size_t)n, o);
    fwrite(&setup_s, 8, 1, o);
    fwrite(&loop_s, 8, 1, o);
    fwrite(&faces_added, 4, 1, o);
    fclose(o);
    return 0;
}
