// Host-side nested dissection + multifrontal Cholesky (see spd_direct.hpp).
#include "spd_direct.hpp"

#include <algorithm>
#include <cmath>
#include <exception>
#include <functional>
#include <omp.h>
#include <numeric>
#include <stdexcept>
#include <string>

namespace aa {

// ------------------------------------------------------------------ nested dissection
namespace {
struct NdBuilder {
    int n;
    const double* xyz;
    const std::vector<int>& ap;
    const std::vector<int>& aj;
    int leaf;
    std::vector<int> mark, side;
    int stamp = 0;
    // output tree under construction (nodes appended in postorder)
    std::vector<std::vector<int>> piv;       // pivots (old ids) per node
    std::vector<std::vector<int>> kids;

    NdBuilder(int n_, const double* x_, const std::vector<int>& p_, const std::vector<int>& j_, int l_)
        : n(n_), xyz(x_), ap(p_), aj(j_), leaf(l_), mark(n_, 0), side(n_, 0) {}

    // one bisection step: median split (or, for an uneven part count, a split at the fraction
    // num/den of the vertices) along the longest bounding-box axis, then the vertices of the lower
    // side adjacent to the upper side form the (one-sided) vertex separator
    void split(std::vector<int>& verts, std::vector<int>& left, std::vector<int>& right, std::vector<int>& sep,
               int num = 1, int den = 2) {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int v : verts)
            for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], xyz[3 * v + d]); hi[d] = std::max(hi[d], xyz[3 * v + d]); }
        int ax = 0;
        for (int d = 1; d < 3; ++d) if (hi[d] - lo[d] > hi[ax] - lo[ax]) ax = d;
        auto key = [&](int v) { return xyz[3 * v + ax]; };
        const size_t half = den == 2 * num ? verts.size() / 2 : (size_t)((long long)verts.size() * num / den);
        std::nth_element(verts.begin(), verts.begin() + half, verts.end(), [&](int a, int b) {
            double ka = key(a), kb = key(b);
            return ka < kb || (ka == kb && a < b);
        });
        const int st = ++stamp;
        for (size_t i = 0; i < verts.size(); ++i) { mark[verts[i]] = st; side[verts[i]] = i < half ? 0 : 1; }
        for (size_t i = 0; i < verts.size(); ++i) {
            int v = verts[i];
            if (i >= half) { right.push_back(v); continue; }
            bool touches = false;
            for (int k = ap[v]; k < ap[v + 1] && !touches; ++k) {
                int u = aj[k];
                touches = mark[u] == st && side[u] == 1;
            }
            (touches ? sep : left).push_back(v);
        }
    }

    int add_node(std::vector<int> p, std::vector<int> k) {
        std::sort(p.begin(), p.end());
        piv.push_back(std::move(p));
        kids.push_back(std::move(k));
        return (int)piv.size() - 1;
    }

    // returns the list of root node ids of the forest built over `verts`
    std::vector<int> build(std::vector<int> verts) {
        if (verts.empty()) return {};
        if ((int)verts.size() <= leaf) return {add_node(std::move(verts), {})};
        std::vector<int> left, right, sep;
        split(verts, left, right, sep);
        if (left.empty() && right.empty()) return {add_node(std::move(sep), {})};  // degenerate
        std::vector<int> roots = build(std::move(left));
        std::vector<int> r2 = build(std::move(right));
        roots.insert(roots.end(), r2.begin(), r2.end());
        if (sep.empty()) return roots;
        return {add_node(std::move(sep), roots)};
    }

    // the top bisections are forced until there are `parts` parts (one per leaf of the top, in
    // left-to-right order; an odd count is split floor(parts/2) : ceil(parts/2) by vertex count);
    // each part is then dissected by build(). part_of[node] = part id, -1 = top separator
    std::vector<int> part_of;
    std::vector<int> build_parts(std::vector<int> verts, int parts, int& next_part) {
        if (parts <= 1) {
            const int id = next_part++;
            const size_t first = piv.size();
            std::vector<int> r = build(std::move(verts));
            part_of.resize(piv.size(), -1);
            for (size_t k = first; k < piv.size(); ++k) part_of[k] = id;
            return r;
        }
        std::vector<int> left, right, sep;
        const int pl = parts / 2, pr = parts - pl;
        if (!verts.empty()) split(verts, left, right, sep, pl, parts);
        if (left.empty() && right.empty() && !sep.empty()) std::swap(left, sep);   // tiny: keep it in a part
        std::vector<int> roots = build_parts(std::move(left), pl, next_part);
        std::vector<int> r2 = build_parts(std::move(right), pr, next_part);
        roots.insert(roots.end(), r2.begin(), r2.end());
        if (sep.empty()) return roots;
        const int s = add_node(std::move(sep), roots);
        part_of.resize(piv.size(), -1);
        return {s};
    }
};
}  // namespace

NdTree nested_dissection(int n, const double* xyz, const std::vector<int>& adj_ptr, const std::vector<int>& adj,
                         int leaf_size, int top_rows, int n_parts, bool merge_top, int part_top_rows) {
    NdBuilder b(n, xyz, adj_ptr, adj, std::max(1, leaf_size));
    std::vector<int> all(n);
    std::iota(all.begin(), all.end(), 0);
    int nparts = 0;
    const int part_levels = n_parts > 1 ? 1 : 0;   // (flag) partitioned ordering
    std::vector<int> roots = part_levels > 0 ? b.build_parts(all, n_parts, nparts) : b.build(all);
    std::vector<std::vector<int>> piv = std::move(b.piv), kids = std::move(b.kids);
    std::vector<int> part_of = std::move(b.part_of);
    part_of.resize(piv.size(), part_levels > 0 ? -1 : 0);
    if (part_levels > 0) top_rows = 0;   // the partition roots must stay separate supernodes
    // ---- amalgamate the top levels of the subtree under `root` into one dense supernode (up to
    // `budget` pivots, whole levels, only while every node of the level is an inner node): upper
    // levels have few, mid-sized supernodes whose level-by-level solve is pure latency; as one
    // dense block they are a single wide GEMV per sweep. Returns the new root (or `root`).
    auto amalgamate = [&](int root, long long budget) -> int {
        std::vector<std::vector<int>> depth_nodes(1, {root});
        long long rows = (long long)piv[root].size();
        int K = 1;
        for (;;) {
            std::vector<int> next;
            for (int s : depth_nodes.back()) next.insert(next.end(), kids[s].begin(), kids[s].end());
            long long add = 0;
            for (int s : next) add += (long long)piv[s].size();
            bool all_inner = !next.empty();
            for (int s : next) all_inner = all_inner && !kids[s].empty();
            if (!all_inner || rows + add > budget) break;
            rows += add;
            depth_nodes.push_back(next);
            ++K;
        }
        if (K <= 1) return root;
        std::vector<char> top(piv.size(), 0);
        for (auto& d : depth_nodes) for (int s : d) top[s] = 1;
        std::vector<int> merged, below;
        std::function<void(int)> post = [&](int s) {   // postorder over the merged nodes only
            for (int c : kids[s]) {
                if (top[c]) post(c);
                else below.push_back(c);
            }
            merged.insert(merged.end(), piv[s].begin(), piv[s].end());
        };
        post(root);
        const int pr = part_of[root];
        piv.push_back(merged);
        kids.push_back(below);
        part_of.push_back(pr);
        for (int s = 0; s < (int)top.size(); ++s) if (top[s]) { piv[s].clear(); kids[s].clear(); }
        return (int)piv.size() - 1;
    };
    if (top_rows > 0 && roots.size() == 1) roots = {amalgamate(roots[0], top_rows)};
    // ---- partitioned, merge_top: all shared top separators become ONE dense root supernode
    // (children = the parts' roots). Its two sweeps are then dense GEMVs the GPUs split by rows
    // (DirectSolver::build) instead of a replicated level-by-level solve. Each
    // part's own top levels are amalgamated too (part_top_rows): a part is a small tree whose
    // upper levels would otherwise each cost a latency-bound launch per sweep.
    if (part_levels > 0 && merge_top && roots.size() == 1 && part_of[roots[0]] < 0) {
        std::vector<int> merged, below;
        std::function<void(int)> post = [&](int s) {   // postorder over the top separators
            for (int c : kids[s]) {
                if (part_of[c] < 0) post(c);
                else below.push_back(c);
            }
            merged.insert(merged.end(), piv[s].begin(), piv[s].end());
            piv[s].clear();
            kids[s].clear();
        };
        post(roots[0]);
        if (part_top_rows > 0)
            for (int& c : below)
                if (!kids[c].empty()) c = amalgamate(c, part_top_rows);
        piv.push_back(merged);
        kids.push_back(below);
        part_of.push_back(-1);
        roots = {(int)piv.size() - 1};
    }
    // ---- postorder numbering from the roots (children first). Partitioned: the subtrees of
    // part 0, 1, ... first (each a contiguous pivot range), then the top separators in
    // postorder -- every GPU's own rows and the shared separator rows are then contiguous.
    NdTree t;
    std::vector<int> order;
    std::function<void(int)> dfs = [&](int s) {
        for (int c : kids[s]) dfs(c);
        order.push_back(s);
    };
    if (part_levels > 0) {
        std::vector<std::vector<int>> part_roots(nparts);
        std::function<void(int)> find = [&](int s) {
            if (part_of[s] >= 0) { part_roots[part_of[s]].push_back(s); return; }
            for (int c : kids[s]) find(c);
        };
        for (int r : roots) find(r);
        for (auto& pr : part_roots) for (int r : pr) dfs(r);
        std::function<void(int)> dfs_top = [&](int s) {
            for (int c : kids[s]) if (part_of[c] < 0) dfs_top(c);
            order.push_back(s);
        };
        for (int r : roots) if (part_of[r] < 0) dfs_top(r);
    } else {
        for (int r : roots) dfs(r);
    }
    const int nn = (int)order.size();
    std::vector<int> newid(piv.size(), -1);
    for (int i = 0; i < nn; ++i) newid[order[i]] = i;
    t.beg.resize(nn); t.end.resize(nn); t.parent.assign(nn, -1); t.children.resize(nn);
    t.part.assign(nn, 0);
    t.n_parts = part_levels > 0 ? nparts : 1;
    int c = 0;
    for (int i = 0; i < nn; ++i) {
        const int s = order[i];
        t.beg[i] = c;
        for (int v : piv[s]) t.perm.push_back(v);
        c += (int)piv[s].size();
        t.end[i] = c;
        t.part[i] = s < (int)part_of.size() ? part_of[s] : (part_levels > 0 ? -1 : 0);
        for (int k : kids[s]) { t.children[i].push_back(newid[k]); t.parent[newid[k]] = i; }
    }
    if (c != n) throw std::runtime_error("nested_dissection: lost vertices");
    // pivot ranges of the parts and of the shared top (partitioned ordering only)
    t.part_beg.assign(t.n_parts, 0);
    t.part_end.assign(t.n_parts, 0);
    t.top_beg = part_levels > 0 ? n : 0;
    if (part_levels > 0) {
        int cur = 0;
        for (int pp = 0; pp < t.n_parts; ++pp) {
            t.part_beg[pp] = cur;
            for (int i = 0; i < nn; ++i) if (t.part[i] == pp) cur = std::max(cur, t.end[i]);
            t.part_end[pp] = cur;
        }
        t.top_beg = cur;
        for (int i = 0; i < nn; ++i)
            if ((t.part[i] < 0) != (t.beg[i] >= t.top_beg) && t.end[i] > t.beg[i])
                throw std::runtime_error("nested_dissection: partitioned ordering is not contiguous");
    } else {
        t.part_end[0] = n;
    }
    return t;
}

// ------------------------------------------------------------------ multifrontal Cholesky
namespace {

// symbolic: boundary rows of every supernode (postorder: from A's columns and the children's)
void symbolic(const CsrMatrix& A, const NdTree& tree, SupernodalFactor& F) {
    const int nn = (int)tree.beg.size();
    for (int s = 0; s < nn; ++s) {
        const int b0 = tree.beg[s], e0 = tree.end[s];
        std::vector<int> bnd;
        for (int j = b0; j < e0; ++j)
            for (int k = A.ptr[j]; k < A.ptr[j + 1]; ++k) if (A.col[k] >= e0) bnd.push_back(A.col[k]);
        for (int c : tree.children[s]) {
            for (int i : F.bnd[c]) if (i >= e0) bnd.push_back(i);
            F.height[s] = std::max(F.height[s], F.height[c] + 1);
        }
        std::sort(bnd.begin(), bnd.end());
        bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
        F.bnd[s] = std::move(bnd);
    }
}

struct FrontCtx {
    const CsrMatrix& A;
    const NdTree& tree;
    SupernodalFactor& F;
    std::vector<std::vector<double>>& U;   // host update matrices, freed when consumed
    std::vector<double>& flops;
    DenseFrontBackend* dense;
    const PartFactor* part;   // partitioned: this rank's share of a top front, summed (see PartFactor)
};

int front_order(const SupernodalFactor& F, int s) { return F.end[s] - F.beg[s] + (int)F.bnd[s].size(); }

// numeric work of supernode s: assemble the front (A's pivot columns, then the children's update
// matrices in child order), partial Cholesky of its first p columns, outputs. pos: n-sized scratch
// (every entry read is written first). Fronts of order >= dense->min_front go to the backend.
void factor_front(FrontCtx& C, int s, std::vector<int>& pos, bool inner_parallel) {
    const CsrMatrix& A = C.A;
    const NdTree& tree = C.tree;
    SupernodalFactor& F = C.F;
    const int b0 = tree.beg[s], e0 = tree.end[s], p = e0 - b0;
    const std::vector<int>& bnd = F.bnd[s];
    const int nb = (int)bnd.size(), f = p + nb;
    for (int j = b0; j < e0; ++j) pos[j] = j - b0;
    for (int k = 0; k < nb; ++k) pos[bnd[k]] = p + k;
    double fl = 0;
    for (int k = 0; k < p; ++k) fl += (double)(f - k) * (f - k);
    C.flops[s] = fl;
    // partitioned top front: this rank's terms only (A and top children on the first rank, the
    // own part's children everywhere), summed over the ranks after assembly
    const PartFactor* P = (C.part && tree.part[s] == -1) ? C.part : nullptr;
    const bool add_a = !P || P->first;
    auto take_child = [&](int c) {
        if (!C.part) return true;
        if (tree.part[c] == -1) return P == nullptr || P->first;
        return tree.part[c] == C.part->my_part;
    };
    if (C.dense && f >= C.dense->min_front) {
        std::vector<int> ai, aj;
        std::vector<double> av;
        if (add_a)
            for (int j = b0; j < e0; ++j)
                for (int k = A.ptr[j]; k < A.ptr[j + 1]; ++k) {
                    const int i = A.col[k];
                    if (i < j) continue;
                    ai.push_back(pos[i]); aj.push_back(pos[j]); av.push_back(A.val[k]);
                }
        std::vector<DenseFrontBackend::Child> kids;
        std::vector<std::vector<int>> maps(tree.children[s].size());
        for (size_t q = 0; q < tree.children[s].size(); ++q) {
            const int c = tree.children[s][q];
            if (!take_child(c)) {   // another rank's share: free what this rank holds of it now
                if (C.dense->holds(c)) C.dense->drop(c);
                else std::vector<double>().swap(C.U[c]);
                continue;
            }
            for (int i : F.bnd[c]) maps[q].push_back(pos[i]);
            kids.push_back({c, maps[q].data(), (int)maps[q].size(), C.dense->holds(c) ? nullptr : &C.U[c]});
        }
        const int par = tree.parent[s];
        const bool keep = par >= 0 && front_order(F, par) >= C.dense->min_front;
        std::vector<double> Us;
        if (P) C.dense->reduce_front = P->reduce_dev;
        try {
            C.dense->factor(s, f, p, ai, aj, av, kids, keep, F.Linv[s], F.LBP[s], F.M[s], keep ? nullptr : &Us);
        } catch (...) {
            C.dense->reduce_front = nullptr;
            throw;
        }
        C.dense->reduce_front = nullptr;
        for (int c : tree.children[s]) std::vector<double>().swap(C.U[c]);
        if (nb > 0 && !keep) C.U[s] = std::move(Us);
        return;
    }
    // ---- assemble front (lower triangle, column-major f x f: Fc(i,j) at j*f + i)
    std::vector<double> Fc((size_t)f * f, 0.0);
    auto FC = [&](int i, int j) -> double& { return Fc[(size_t)j * f + i]; };
    if (add_a)
        for (int j = b0; j < e0; ++j)
            for (int k = A.ptr[j]; k < A.ptr[j + 1]; ++k) {
                int i = A.col[k];
                if (i < j) continue;
                FC(pos[i], pos[j]) += A.val[k];
            }
    for (int c : tree.children[s]) {
        if (!take_child(c)) { std::vector<double>().swap(C.U[c]); continue; }
        const std::vector<int>& cb = F.bnd[c];
        const int m = (int)cb.size();
        if (C.dense && C.dense->holds(c)) throw std::runtime_error("multifrontal_cholesky: update matrix held by the backend");
        const std::vector<double>& Uc = C.U[c];
        for (int a = 0; a < m; ++a)
            for (int bb = 0; bb <= a; ++bb) {
                int ra = pos[cb[a]], rb = pos[cb[bb]];
                if (ra < rb) std::swap(ra, rb);
                FC(ra, rb) += Uc[(size_t)a * m + bb];
            }
        std::vector<double>().swap(C.U[c]);
    }
    if (P) P->reduce_host(Fc.data(), Fc.size());
    // ---- partial dense Cholesky (right-looking, column-major) of the first p columns
    for (int k = 0; k < p; ++k) {
        double* ck = &Fc[(size_t)k * f];
        const double d = ck[k];
        if (!(d > 0.0))
            throw std::runtime_error("multifrontal_cholesky: matrix not positive definite (host front " + std::to_string(s) +
                                     ", order " + std::to_string(f) + ", pivot " + std::to_string(k) + " of " +
                                     std::to_string(p) + ", d = " + std::to_string(d) + ")");
        const double dk = std::sqrt(d);
        ck[k] = dk;
        const double inv = 1.0 / dk;
        for (int i = k + 1; i < f; ++i) ck[i] *= inv;
        const long long work = (long long)(f - k) * (f - k);
        (void)work;   // (only read by the OpenMP if-clause)
#pragma omp parallel for schedule(dynamic, 16) if (inner_parallel && work > 200000)
        for (int j = k + 1; j < f; ++j) {
            const double ljk = ck[j];
            if (ljk == 0.0) continue;
            double* cj = &Fc[(size_t)j * f];
            for (int i = j; i < f; ++i) cj[i] -= ck[i] * ljk;
        }
    }
    // ---- outputs: Linv (p x p lower, row-major), LBP (nb x p, row-major), update matrix (nb x nb)
    std::vector<double> Li((size_t)p * p, 0.0);
#pragma omp parallel for schedule(dynamic, 8) if (inner_parallel && p > 256)
    for (int j = 0; j < p; ++j) {  // column j of L^-1: column-oriented forward substitution
        std::vector<double> r((size_t)p, 0.0);
        r[j] = 1.0;
        for (int k = j; k < p; ++k) {
            const double xk = r[k] / FC(k, k);
            Li[(size_t)k * p + j] = xk;
            if (xk == 0.0) continue;
            const double* ck = &Fc[(size_t)k * f];
            for (int i = k + 1; i < p; ++i) r[i] -= ck[i] * xk;
        }
    }
    F.Linv[s] = std::move(Li);
    std::vector<double> LBP((size_t)nb * p);
    for (int a = 0; a < nb; ++a)
        for (int j = 0; j < p; ++j) LBP[(size_t)a * p + j] = FC(p + a, j);
    F.LBP[s] = std::move(LBP);
    if (nb > 0) {
        std::vector<double> Us((size_t)nb * nb);
        for (int a = 0; a < nb; ++a)
            for (int bb = 0; bb <= a; ++bb) Us[(size_t)a * nb + bb] = FC(p + a, p + bb);
        C.U[s] = std::move(Us);
    }
}

}  // namespace

SupernodalFactor multifrontal_cholesky(const CsrMatrix& A, const NdTree& tree, DenseFrontBackend* dense,
                                       const PartFactor* part) {
    SupernodalFactor F;
    const int n = A.n, nn = (int)tree.beg.size();
    F.n = n; F.n_nodes = nn;
    F.beg = tree.beg; F.end = tree.end; F.parent = tree.parent;
    F.bnd.resize(nn); F.Linv.resize(nn); F.LBP.resize(nn); F.M.resize(nn); F.height.assign(nn, 0);
    symbolic(A, tree, F);
    std::vector<std::vector<double>> U(nn);
    std::vector<double> flops(nn, 0.0);
    FrontCtx C{A, tree, F, U, flops, dense, part};
    if (part && (int)tree.part.size() != nn) throw std::runtime_error("multifrontal_cholesky: partitioned factor needs a partitioned tree");
    auto mine = [&](int s) { return !part || tree.part[s] == part->my_part; };
    // partitioned: a rank whose own part fails (not positive definite) must not leave the others
    // waiting in the first top front's sum -- every rank reports its own-part outcome first and
    // all of them throw together (the top fronts are summed, so they fail or pass on all ranks)
    // the failure keeps its own type (aa::Error codes, std::bad_alloc) on the rank it happened on;
    // only the other ranks throw the synthesized "another rank's part" error
    auto agree = [&](const std::exception_ptr& err, const char* where = "part") {
        if (!part) {
            if (err) std::rethrow_exception(err);
            return;
        }
        double bad = err ? 1.0 : 0.0;
        part->reduce_host(&bad, 1);
        if (err) std::rethrow_exception(err);
        if (bad > 0)
            throw std::runtime_error(std::string("multifrontal_cholesky: matrix not positive definite (on another rank's ") +
                                     where + ")");
    };
    // the shared top fronts, one at a time in postorder: every rank factors the same summed front,
    // so an outcome that differs between ranks is a defect -- each front's outcome is agreed, so
    // all ranks stop together and the others name it instead of failing in a later collective
    auto factor_top = [&](std::vector<int>& pos) {
        for (int s = 0; s < nn; ++s) {
            if (tree.part[s] != -1) continue;
            std::exception_ptr err;
            try {
                factor_front(C, s, pos, true);
            } catch (...) {
                err = std::current_exception();
            }
            agree(err, "copy of a top front");
        }
    };
    if (!dense) {   // host only: postorder, parallel inside the large fronts
        std::vector<int> pos(n, -1);
        std::exception_ptr err;
        try {
            for (int s = 0; s < nn; ++s)
                if (part ? mine(s) : true) factor_front(C, s, pos, true);
        } catch (...) {
            err = std::current_exception();
        }
        agree(err);
        if (part) factor_top(pos);
    } else {
        // tree-parallel: independent subtrees are OpenMP tasks (a front waits for its children),
        // each host front is factored by one thread; the large fronts near the root go to the
        // dense backend, one at a time (it serialises its calls)
        std::vector<long long> sub(nn, 0);   // pivots in the subtree
        for (int s = 0; s < nn; ++s) {
            sub[s] += tree.end[s] - tree.beg[s];
            if (tree.parent[s] >= 0) sub[tree.parent[s]] += sub[s];
        }
        const long long grain = std::max<long long>(256, n / 1024);
        std::exception_ptr err;
        std::function<void(int)> rec = [&](int s) {
            for (int c : tree.children[s]) {
                if (sub[c] > grain) {
#pragma omp task firstprivate(c) shared(rec)
                    rec(c);
                } else {
                    rec(c);
                }
            }
#pragma omp taskwait
            static thread_local std::vector<int> pos;
            if ((int)pos.size() < n) pos.assign(n, -1);
            bool failed;
#pragma omp critical(aa_factor_err)
            failed = (bool)err;
            if (failed) return;
            try {
                factor_front(C, s, pos, false);
            } catch (...) {
#pragma omp critical(aa_factor_err)
                if (!err) err = std::current_exception();
            }
        };
        // partitioned: the own part's subtrees (roots: own supernodes whose parent is not own)
        // in parallel, then the top fronts one at a time in postorder (collectives)
        auto is_root = [&](int s) {
            if (!part) return tree.parent[s] < 0;
            return mine(s) && (tree.parent[s] < 0 || !mine(tree.parent[s]));
        };
#pragma omp parallel
#pragma omp single
        {
            for (int s = 0; s < nn; ++s)
                if (is_root(s)) {
#pragma omp task firstprivate(s) shared(rec)
                    rec(s);
                }
#pragma omp taskwait
        }
        agree(err);
        if (part) {
            std::vector<int> pos(n, -1);
            factor_top(pos);
        }
    }
    for (int s = 0; s < nn; ++s) {
        const int p = tree.end[s] - tree.beg[s], nb = (int)F.bnd[s].size();
        F.flops += flops[s];
        F.nnz_L += (size_t)p * (p + 1) / 2 + (size_t)p * nb;
        F.max_height = std::max(F.max_height, F.height[s]);
    }
    return F;
}

void factor_solve_host(const SupernodalFactor& F, std::vector<double>& b) {
    factor_solve_host_part(F, nullptr, -1, b, nullptr);
}

void factor_solve_host_part(const SupernodalFactor& F, const NdTree* T, int part, std::vector<double>& b,
                            const std::function<void(double*, size_t)>& reduce_top) {
    const int nn = F.n_nodes;
    auto skip = [&](int s) { return T && T->part[s] != part && T->part[s] != -1; };
    std::vector<double> t;
    for (int s = 0; s < nn; ++s) {  // forward (postorder)
        if (skip(s)) continue;
        const int b0 = F.beg[s], p = F.end[s] - b0, nb = (int)F.bnd[s].size();
        t.assign((size_t)p * 3, 0.0);
        for (int i = 0; i < p; ++i)
            for (int k = 0; k <= i; ++k)
                for (int c = 0; c < 3; ++c) t[3 * i + c] += F.Linv[s][(size_t)i * p + k] * b[3 * (size_t)(b0 + k) + c];
        for (int i = 0; i < p; ++i) for (int c = 0; c < 3; ++c) b[3 * (size_t)(b0 + i) + c] = t[3 * i + c];
        for (int a = 0; a < nb; ++a)
            for (int j = 0; j < p; ++j)
                for (int c = 0; c < 3; ++c) b[3 * (size_t)F.bnd[s][a] + c] -= F.LBP[s][(size_t)a * p + j] * t[3 * j + c];
    }
    // partitioned: the top rows now hold this rank's share of the forward result (linear in
    // the right-hand side and in the children's update vectors) -- their sum is the full one
    if (T && reduce_top && T->top_beg < F.n) reduce_top(b.data() + 3 * (size_t)T->top_beg, 3 * (size_t)(F.n - T->top_beg));
    for (int s = nn - 1; s >= 0; --s) {  // backward
        if (skip(s)) continue;
        const int b0 = F.beg[s], p = F.end[s] - b0, nb = (int)F.bnd[s].size();
        t.assign((size_t)p * 3, 0.0);
        for (int j = 0; j < p; ++j)
            for (int c = 0; c < 3; ++c) {
                double v = b[3 * (size_t)(b0 + j) + c];
                for (int a = 0; a < nb; ++a) v -= F.LBP[s][(size_t)a * p + j] * b[3 * (size_t)F.bnd[s][a] + c];
                t[3 * j + c] = v;
            }
        for (int j = 0; j < p; ++j)
            for (int c = 0; c < 3; ++c) {
                double v = 0;
                for (int i = j; i < p; ++i) v += F.Linv[s][(size_t)i * p + j] * t[3 * i + c];
                b[3 * (size_t)(b0 + j) + c] = v;
            }
    }
}

}  // namespace aa
