// GPU supernodal triangular solves against the host multifrontal factor (spd_direct.hpp).
//
// Replaces the reference's per-iteration LDLTSolver::solve (LinearSolver.hpp:87-90): one
// forward and one backward sweep over the supernode tree, level by level (all supernodes of
// equal height are independent). Per level and sweep two fully parallel kernels:
//   forward   t_i = b_i - sum_{j in descendants} L(i,j) y_j        (sparse row pulls, CSR)
//             y_P = Linv_PP t_P                                     (dense GEMV, inverted block)
//   backward  t_j = y_j - sum_{i in ancestors} L(i,j) x_i           (dense GEMV over the boundary)
//             x_P = Linv_PP^T t_P
// Every sum is computed by one wavefront in a fixed order: results are deterministic and
// there are no atomics. Three right-hand sides (x, y, z) are processed together.
#pragma once
#include <vector>

#include "common.hpp"
#include "elastic_kernels.hpp"
#include "spd_direct.hpp"

namespace aa {

struct SolveItem { int node, r0, r1, pad; };

class DirectSolver {
public:
    void build(const SupernodalFactor& F, hipStream_t s);
    // x (n x 3, stride 3 doubles) = A^-1 b ; b is destroyed. gate: skip when ctrl->done (or !reject).
    void solve(double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s);
    int n() const { return n_; }
    int levels() const { return n_levels_; }
    size_t nnz_L() const { return nnz_L_; }
    // algorithmic bytes of one full solve (forward + backward, 3 RHS)
    double bytes_per_solve() const { return bytes_; }
    int kernels_per_solve() const { return 4 * n_levels_; }

private:
    int n_ = 0, nn_ = 0, n_levels_ = 0;
    size_t nnz_L_ = 0;
    double bytes_ = 0;
    DevBuf<int> beg_, p_, nb_, bnd_off_, bnd_, fptr_, fcol_;
    DevBuf<long long> linv_off_, lbp_off_;
    DevBuf<double> linv_, linvT_, lbpt_, fval_, Y_;
    DevBuf<SolveItem> items_;
    std::vector<int> level_off_;  // host: item range per level (height order)
};

}  // namespace aa
