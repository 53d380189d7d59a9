// Element-level driver for the REFERENCE (test infrastructure only): feeds seeded inputs to
// the reference's public per-element operators and writes their outputs, for golden tables.
//   op 0: TetEnergyTerm::prox            (admm_anderson_hard_zxu/src/TetEnergyTerm.cpp:74-96)
//   op 1: NeoHookeanTet prox (L-BFGS)   (TetEnergyTerm.cpp:151-162, 206-251)
//   op 2: StVKTet prox (L-BFGS)         (TetEnergyTerm.cpp:151-162, 256-307)
//   op 3: TriEnergyTerm::prox  H        (admm_anderson_hard_zxu/src/TriEnergyTerm.cpp:74-105)
//   op 4: Eigen COD solve of a k x k normal-equation matrix (AndersonAcceleration.h:193-196)
// input : int32 op, int32 count, then per case: double params[4], double in[K] (K = 9 tet, 6 tri,
//         1+k*k+k for COD with k stored as params[0])
// output: per case double out[9] (or k for COD)
#include "TetEnergyTerm.hpp"
#include "TriEnergyTerm.hpp"
#include <Eigen/Dense>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    FILE* o = fopen(argv[2], "wb");
    if (!f || !o) return 2;
    int op, count;
    if (fread(&op, 4, 1, f) != 1 || fread(&count, 4, 1, f) != 1) return 2;
    for (int c = 0; c < count; ++c) {
        double prm[4];
        if (fread(prm, 8, 4, f) != 4) return 2;
        if (op <= 2) {
            double in[9];
            if (fread(in, 8, 9, f) != 9) return 2;
            // unit right tet scaled by prm[2] so that vol = prm[2]^3/6
            std::vector<Eigen::Vector3d> v = {Eigen::Vector3d(0, 0, 0), Eigen::Vector3d(prm[2], 0, 0),
                                              Eigen::Vector3d(0, prm[2], 0), Eigen::Vector3d(0, 0, prm[2])};
            admm::Lame lame(prm[0], prm[1]);
            Eigen::Matrix<int, 4, 1> tet(0, 1, 2, 3);
            Eigen::VectorXd zi = Eigen::Map<Eigen::VectorXd>(in, 9);
            Eigen::VectorXd vi = zi;
            Eigen::MatrixXd W = Eigen::MatrixXd::Identity(9, 9);
            if (op == 0) { admm::TetEnergyTerm t(tet, v, lame); t.prox(W, zi, vi); }
            else if (op == 1) { admm::NeoHookeanTet t(tet, v, lame); t.prox(W, zi, vi); }
            else { admm::StVKTet t(tet, v, lame); t.prox(W, zi, vi); }
            fwrite(zi.data(), 8, 9, o);
        } else if (op == 3) {
            double in[6];
            if (fread(in, 8, 6, f) != 6) return 2;
            std::vector<Eigen::Vector3d> v = {Eigen::Vector3d(0, 0, 0), Eigen::Vector3d(1, 0, 0), Eigen::Vector3d(0, 1, 0)};
            admm::Lame lame(prm[0], prm[1]);
            lame.limit_min = prm[2];
            lame.limit_max = prm[3];
            Eigen::Matrix<int, 3, 1> tri(0, 1, 2);
            admm::TriEnergyTerm t(tri, v, lame);
            Eigen::VectorXd zi = Eigen::Map<Eigen::VectorXd>(in, 6);
            Eigen::VectorXd vi = zi;
            Eigen::MatrixXd W = Eigen::MatrixXd::Identity(6, 6);
            t.prox(W, zi, vi);
            fwrite(zi.data(), 8, 6, o);
        } else {
            const int k = (int)prm[0];
            std::vector<double> M(k * k), b(k);
            if (fread(M.data(), 8, k * k, f) != (size_t)(k * k) || fread(b.data(), 8, k, f) != (size_t)k) return 2;
            Eigen::MatrixXd A = Eigen::Map<Eigen::MatrixXd>(M.data(), k, k);
            Eigen::VectorXd bb = Eigen::Map<Eigen::VectorXd>(b.data(), k);
            Eigen::CompleteOrthogonalDecomposition<Eigen::MatrixXd> cod;
            cod.compute(A);
            Eigen::VectorXd th = cod.solve(bb);
            fwrite(th.data(), 8, k, o);
        }
    }
    fclose(f);
    fclose(o);
    return 0;
}
