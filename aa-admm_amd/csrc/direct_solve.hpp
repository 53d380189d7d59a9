// GPU supernodal triangular solves against the host multifrontal factor (spd_direct.hpp).
//
// Replaces the reference's per-iteration LDLTSolver::solve (LinearSolver.hpp:87-90) with a
// multifrontal solve over the nested-dissection supernode tree, one kernel per tree height
// and sweep (all supernodes of equal height are independent), one workgroup per supernode:
//   forward   f = [b_P ; 0] + extend_add(children's update vectors)
//             y_P = Linv_PP f_P                 (dense, inverted diagonal block)
//             u   = f_B - L_BP y_P              (dense; this node's update vector for its parent)
//   backward  t   = y_P - L_BP^T x_B            (x_B gathered from the ancestors' solution)
//             x_P = Linv_PP^T t
// Every dense product is thread-per-row over a column-major (coalesced) copy of the block,
// with the vector operand broadcast from LDS: no cross-lane reductions, no atomics,
// deterministic. The three coordinates (x, y, z right-hand sides) are processed together.
#pragma once
#include <vector>

#include "common.hpp"
#include "elastic_kernels.hpp"
#include "spd_direct.hpp"

namespace aa {

class DirectSolver {
public:
    static constexpr int kMaxFront = 3200;   // p + |bnd| of a supernode kept in LDS (3 RHS fp64)
    static constexpr int kBigP = 512;        // larger supernodes use the multi-workgroup path
    static constexpr int kTopRows = 2048;    // upper tree levels amalgamated into one dense root

    void build(const SupernodalFactor& F, hipStream_t s);
    // x (n x 3, stride 3 doubles) = A^-1 b ; b is read only. gate: skip when ctrl->done (or !reject).
    void solve(double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s);
    int n() const { return n_; }
    size_t nnz_L() const { return nnz_L_; }
    double bytes_per_solve() const { return bytes_; }
    int kernels_per_solve() const { return kernels_; }

private:
    struct Level { int first, count, block, lds_fwd, lds_bwd; std::vector<int> big; };
    struct Big { int node, b0, p, nb, bnd_off, pptr_off; long long loff, boff, uoff, foff, toff; };
    int n_ = 0, nn_ = 0, kernels_ = 0;
    size_t nnz_L_ = 0;
    double bytes_ = 0;
    DevBuf<int> beg_, p_, nb_, bnd_off_, bnd_, kid_ptr_, kids_, map_off_, map_, lvl_nodes_;
    DevBuf<long long> loff_, boff_, uoff_;
    DevBuf<double> linv_rm_, linv_cm_, lbp_rm_, lbp_cm_, Y_, U_, Fg_, Tg_;
    DevBuf<int> big_pptr_;
    DevBuf<long long> big_psrc_;
    std::vector<Level> levels_;
    std::vector<Big> bigs_;
};

}  // namespace aa
