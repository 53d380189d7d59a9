// Host-side setup of the global SPD solve (the reference's LDLTSolver::update_system,
// admm_anderson_hard_zxu/src/LinearSolver.hpp:79-84, and Geometry/SPDSolver.h:37-95).
//
// The reference factors A once with Eigen SimplicialLDLT (AMD ordering) and does serial
// forward/back substitution every ADMM iteration. MI355X design: order the free nodes by
// geometric nested dissection (recursive coordinate bisection with vertex separators), do a
// multifrontal Cholesky of the scalar matrix A_s (A = A_s (x) I3) once on the host, and
// hand the GPU a level schedule of supernodes whose diagonal blocks are stored INVERTED,
// so that each triangular solve is a short sequence of fully parallel kernels
// (sparse row pulls + dense GEMVs) instead of a column-serial substitution.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

namespace aa {

struct CsrMatrix {  // scalar CSR, full symmetric pattern
    int n = 0;
    std::vector<int> ptr, col;
    std::vector<double> val;
};

// Geometric nested dissection over the adjacency graph of `n` vertices with coordinates
// xyz[3*i]. Returns perm (new -> old) and the supernode tree in postorder.
struct NdTree {
    std::vector<int> perm;          // new index -> old index
    std::vector<int> beg, end;      // pivot range of node s in new indexing
    std::vector<int> parent;        // -1 for roots
    std::vector<std::vector<int>> children;
    std::vector<int> part;          // partition of node s (part_levels > 0), -1 = top separator
    int n_parts = 1;
    // partitioned ordering: part q owns pivots [part_beg[q], part_end[q]) (contiguous, in
    // part order), the shared top separators are [top_beg, n)
    std::vector<int> part_beg, part_end;
    int top_beg = 0;
};
// top_rows > 0: the upper levels of the tree (up to top_rows pivots) are amalgamated into
// one dense root supernode. part_levels = L > 0: the first L bisections are forced and give
// 2^L parts (one per GPU of the partitioned solver); their separators form the "top" of the
// tree (part -1) and no amalgamation is done.
NdTree nested_dissection(int n, const double* xyz, const std::vector<int>& adj_ptr, const std::vector<int>& adj,
                         int leaf_size, int top_rows = 0, int part_levels = 0);

struct SupernodalFactor {
    int n = 0;
    int n_nodes = 0;
    std::vector<int> beg, end, parent, height;
    std::vector<std::vector<int>> bnd;      // row structure below the diagonal block (new indices, ascending)
    std::vector<std::vector<double>> Linv;  // p x p row-major, inverse of the (lower) diagonal block L_PP
    std::vector<std::vector<double>> LBP;   // b x p row-major, L(bnd, P)
    int max_height = 0;
    double flops = 0;
    size_t nnz_L = 0;                       // scalar nnz(L) incl. diagonal blocks (lower)
};

// Factor the matrix A (given in NEW ordering as a full-pattern CSR) along the tree.
// Throws std::runtime_error if A is not positive definite.
SupernodalFactor multifrontal_cholesky(const CsrMatrix& A, const NdTree& tree);

// Host reference solve with the factor (used by self-checks): x = A^-1 b, b is n x 3.
void factor_solve_host(const SupernodalFactor& F, std::vector<double>& b3);

// Host reference of ONE rank's share of the partitioned solve (tests/cpp/part_solve.cpp):
// forward over the supernodes of `part` and of the top with b3 holding this rank's PARTIAL
// right-hand side (its own rows complete, top rows partial), `reduce_top` sums the top rows
// [top_beg, n) x 3 over the ranks, then backward over the same supernodes. On return the rows
// of the part and of the top hold x; other rows are untouched.
void factor_solve_host_part(const SupernodalFactor& F, const NdTree* T, int part, std::vector<double>& b3,
                            const std::function<void(double*, size_t)>& reduce_top);

}  // namespace aa
