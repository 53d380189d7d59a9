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
#include <algorithm>
#include <cstdlib>
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
// Dissection leaf size (AA_ND_LEAF overrides): below ~150k unknowns the triangular solves are
// bound by their per-level latency chains, and leaves of 128 cut levels (C2 cloth 25k nodes
// 5 940 -> 6 610 it/s, C3 101k points 1 082 -> 1 126); above, leaves of 32 keep the fronts small
// (C4 211k nodes: 364 it/s at 32, 343 at 64, 336 at 128; C5 501k points: 160 at 32 and 64, 158 at
// 128). Measured on one MI355X, DESIGN.md §3.2.
inline int default_nd_leaf(long long n_unknowns) {
    if (const char* e = std::getenv("AA_ND_LEAF")) return std::max(1, std::atoi(e));
    return n_unknowns <= 150000 ? 128 : 32;
}

// top_rows > 0: the upper levels of the tree (up to top_rows pivots) are amalgamated into
// one dense root supernode. n_parts = P > 1: the top bisections are forced until there are P
// parts (one per GPU of the partitioned solver; any P, uneven counts split by vertex count);
// their separators form the "top" of the tree (part -1): with merge_top one dense root
// supernode, else one supernode per separator. No top_rows amalgamation when partitioned;
// part_top_rows > 0 (with merge_top) amalgamates each part's own top levels instead.
NdTree nested_dissection(int n, const double* xyz, const std::vector<int>& adj_ptr, const std::vector<int>& adj,
                         int leaf_size, int top_rows = 0, int n_parts = 0, bool merge_top = true,
                         int part_top_rows = 0);

struct SupernodalFactor {
    int n = 0;
    int n_nodes = 0;
    std::vector<int> beg, end, parent, height;
    std::vector<std::vector<int>> bnd;      // row structure below the diagonal block (new indices, ascending)
    std::vector<std::vector<double>> Linv;  // p x p row-major, inverse of the (lower) diagonal block L_PP
    std::vector<std::vector<double>> LBP;   // b x p row-major, L(bnd, P)
    std::vector<std::vector<double>> M;     // b x p row-major, L(bnd, P) Linv -- when the dense
                                            // backend computed it (empty: the solver forms it)
    int max_height = 0;
    double flops = 0;
    size_t nnz_L = 0;                       // scalar nnz(L) incl. diagonal blocks (lower)
};

// Dense assembly + partial factorization of one front on an accelerator (dense_gpu.hip: rocSOLVER
// / rocBLAS on the solver's GPU). The front (order f = p + nb, column-major, lower triangle) is
// assembled from A's pivot columns (COO in front-local indices, row >= column) and then the
// children's update matrices in child order -- the host loop's order, so the same sums -- after
// which its first p columns are factored (L11 = chol, L21 = F21 L11^-T, F22 -= L21 L21^T).
// Outputs: Linv = L11^-1 (row-major p x p, zero above the diagonal), LBP = L21 (row-major
// nb x p), M = L21 Linv (row-major nb x p), and the update matrix F22: kept by the backend
// (keep_update: the parent is factored there too) or returned in *U (row-major nb x nb, lower).
// Throws std::runtime_error when the block is not positive definite.
struct DenseFrontBackend {
    struct Child {
        int id;                          // supernode
        const int* map;                  // front-local row of each of its m boundary rows
        int m;
        const std::vector<double>* U;    // host update matrix (row-major lower); null: held
    };
    virtual ~DenseFrontBackend() = default;
    virtual void factor(int s, int f, int p, const std::vector<int>& ai, const std::vector<int>& aj,
                        const std::vector<double>& av, const std::vector<Child>& kids, bool keep_update,
                        std::vector<double>& Linv, std::vector<double>& LBP, std::vector<double>& M,
                        std::vector<double>* U) = 0;
    virtual bool holds(int s) const = 0;   // s's update matrix is held by the backend
    virtual void drop(int s) = 0;          // free s's held update matrix (a parent that skips it)
    int min_front = 1024;                  // fronts of at least this order go to the backend
    // set for the partitioned top fronts (PartFactor): called on the assembled device front
    // (f x f doubles) before it is factored -- the sum of the ranks' partial fronts
    std::function<void(double*, size_t)> reduce_front;
};

// Partitioned factorization, one rank of P: only the supernodes of
// part `my_part` and of the shared top (part -1) are factored here. A top front is assembled from
// this rank's share only -- A's entries and the update matrices of top children on the `first`
// rank, the own part's children on every rank -- and summed over the ranks (reduce_host on a
// host front, reduce_dev on a backend front) before its partial Cholesky, so every rank factors
// the same top and no rank factors another rank's part. The top fronts are factored after the
// part, one at a time in postorder (the same collective sequence on every rank).
struct PartFactor {
    int my_part = -1;
    bool first = false;
    std::function<void(double*, size_t)> reduce_host;
    std::function<void(double*, size_t)> reduce_dev;
};

// Factor the matrix A (given in NEW ordering as a full-pattern CSR) along the tree.
// Throws std::runtime_error if A is not positive definite.
// dense == nullptr: everything on the host, supernodes in postorder. Otherwise independent
// subtrees are factored in parallel (OpenMP tasks) and the large fronts by `dense`.
SupernodalFactor multifrontal_cholesky(const CsrMatrix& A, const NdTree& tree, DenseFrontBackend* dense = nullptr,
                                       const PartFactor* part = nullptr);

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
