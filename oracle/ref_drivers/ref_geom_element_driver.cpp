// Element-level driver for the REFERENCE Geometry constraints (test infrastructure only):
// feeds seeded transformed points to the public Constraint<3>::project
// (Geometry/Constraint.h:96-116) of each constraint type and writes the projections.
//   op 0: PlaneConstraint (Constraint.h:396-414)            in: 3 x k mean-centred points
//   op 1: AngleConstraint<3> (:220-296)  prm min, max rad   in: 3 x 2 (v1, v2)
//   op 2: EdgeLengthConstraint<3> (:194-218) prm length      in: 3 x 1
//   op 3: PointToRefSurfaceConstraint (:328-349) via TriMeshAABB (TriMeshAABB.h:57-69)
// input : op, count, [op 3: nv, nf, V[3nv], F[3nf]], per case: int k, double prm[3], double in[3*cols]
// output: per case double out[3*cols]
#include "Constraint.h"
#include "MeshTypes.h"
#include "TriMeshAABB.h"

#include <cstdio>
#include <memory>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    FILE* o = fopen(argv[2], "wb");
    if (!f || !o) return 2;
    int op, count;
    if (fread(&op, 4, 1, f) != 1 || fread(&count, 4, 1, f) != 1) return 2;
    std::shared_ptr<TriMeshAABB> aabb;
    if (op == 3) {
        int nv, nf;
        if (fread(&nv, 4, 1, f) != 1 || fread(&nf, 4, 1, f) != 1) return 2;
        std::vector<double> V(3 * (size_t)nv);
        std::vector<int> F(3 * (size_t)nf);
        if (fread(V.data(), 8, V.size(), f) != V.size() || fread(F.data(), 4, F.size(), f) != F.size()) return 2;
        TriMesh tm;
        std::vector<TriMesh::VertexHandle> vh(nv);
        for (int i = 0; i < nv; ++i) vh[i] = tm.add_vertex(TriMesh::Point(V[3 * i], V[3 * i + 1], V[3 * i + 2]));
        for (int i = 0; i < nf; ++i) tm.add_face(vh[F[3 * i]], vh[F[3 * i + 1]], vh[F[3 * i + 2]]);
        aabb = std::make_shared<TriMeshAABB>(tm);
    }
    for (int c = 0; c < count; ++c) {
        int k;
        double prm[3];
        if (fread(&k, 4, 1, f) != 1 || fread(prm, 8, 3, f) != 3) return 2;
        Constraint<3>* con = nullptr;
        std::vector<int> ids(k);
        for (int i = 0; i < k; ++i) ids[i] = i;
        switch (op) {
            case 0: con = new PlaneConstraint(ids, 1.0); break;
            case 1: con = new AngleConstraint<3>(0, 1, 2, 1.0, prm[0], prm[1]); break;
            case 2: con = new EdgeLengthConstraint<3>(0, 1, 1.0, prm[0]); break;
            default: con = new PointToRefSurfaceConstraint(0, 1.0, aabb); break;
        }
        const int cols = con->num_transformed_points();
        Matrix3X in(3, cols), out(3, cols);
        if (fread(in.data(), 8, 3 * (size_t)cols, f) != 3 * (size_t)cols) return 2;
        // register the constraint at column 0 (sets idO_), then project
        std::vector<Triplet> trip;
        int idO = 0;
        con->add_constraint(false, trip, idO);
        con->project(in, out);
        fwrite(out.data(), 8, 3 * (size_t)cols, o);
        delete con;
    }
    fclose(o);
    fclose(f);
    return 0;
}
