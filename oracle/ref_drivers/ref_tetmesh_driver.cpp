// Tet-mesh binding driver for the REFERENCE (test infrastructure only): mcl's own loader and mesh
// operations, as the plinko samples use them (samples/Asia2019/plinkohit.cpp:41-53,
// samples/utils/AddMeshes.hpp:97-120):
//   mcl::meshio::load_elenode (deps/mclscene/include/MCL/MeshIO.hpp:180-290)
//   TetMesh::apply_xform(make_trans(t) * make_scale(s))   (TetMesh.hpp:134-138, XForm.hpp:43-61)
//   TetMesh::weighted_masses(m, 1522)                      (TetMesh.hpp:297-315)
// usage: ref_tetmesh <path without .ele/.node> sx sy sz tx ty tz out.bin
// out: int32 n_verts, int32 n_tets, float32 verts[n][3], int32 tets[t][4], float32 masses[n]
#include "MCL/MeshIO.hpp"
#include "MCL/TetMesh.hpp"
#include "MCL/XForm.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 9) { fprintf(stderr, "usage: %s mesh sx sy sz tx ty tz out.bin\n", argv[0]); return 2; }
    mcl::TetMesh::Ptr mesh = mcl::TetMesh::create();
    if (!mcl::meshio::load_elenode(mesh.get(), argv[1])) return 1;
    const float s[3] = {(float)atof(argv[2]), (float)atof(argv[3]), (float)atof(argv[4])};
    const float t[3] = {(float)atof(argv[5]), (float)atof(argv[6]), (float)atof(argv[7])};
    mcl::XForm<float> xf = mcl::xform::make_trans(t[0], t[1], t[2]) * mcl::xform::make_scale(s[0], s[1], s[2]);
    mesh->apply_xform(xf);
    std::vector<float> masses;
    mesh->weighted_masses(masses, 1522.f);
    FILE* o = fopen(argv[8], "wb");
    if (!o) return 2;
    const int nv = (int)mesh->vertices.size(), nt = (int)mesh->tets.size();
    fwrite(&nv, 4, 1, o);
    fwrite(&nt, 4, 1, o);
    for (int i = 0; i < nv; ++i) fwrite(&mesh->vertices[i][0], 4, 3, o);
    for (int i = 0; i < nt; ++i) fwrite(&mesh->tets[i][0], 4, 4, o);
    fwrite(masses.data(), 4, nv, o);
    fclose(o);
    return 0;
}
