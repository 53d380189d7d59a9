// Driver for the REFERENCE WireMeshOpt pre-processing (test infrastructure only): reads a
// polygon mesh with the reference's OpenMesh OBJ reader exactly as WireMeshOpt's main does
// (Geometry/WireMeshOpt.cpp:349-353), runs subdivide_and_smooth_mesh (Geometry/MeshTypes.h:
// 214-342: one subdivision step -- edge midpoints, face centroids, one quad per face corner --
// then the interior and boundary uniform Laplacian smoothing solve with the original vertices
// fixed) and average_edge_length, and writes the result.
// output: int nv, int nf, double edge_length, double V[3 nv], per face int k, int idx[k]
#include "MeshTypes.h"

#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    PolyMesh mesh;
    if (!OpenMesh::IO::read_mesh(mesh, argv[1])) return 3;
    const Scalar edge_length = average_edge_length(mesh);
    PolyMesh sub = subdivide_and_smooth_mesh(mesh);
    FILE* o = fopen(argv[2], "wb");
    if (!o) return 2;
    const int nv = (int)sub.n_vertices(), nf = (int)sub.n_faces();
    const double el = edge_length;
    fwrite(&nv, 4, 1, o);
    fwrite(&nf, 4, 1, o);
    fwrite(&el, 8, 1, o);
    for (auto v : sub.vertices()) {
        const PolyMesh::Point& p = sub.point(v);
        const double q[3] = {p[0], p[1], p[2]};
        fwrite(q, 8, 3, o);
    }
    for (auto f : sub.faces()) {
        std::vector<int> idx;
        for (auto fv = sub.cfv_iter(f); fv.is_valid(); ++fv) idx.push_back(fv->idx());
        const int k = (int)idx.size();
        fwrite(&k, 4, 1, o);
        fwrite(idx.data(), 4, k, o);
    }
    fclose(o);
    return 0;
}
