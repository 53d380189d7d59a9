// CPU test of the fused-subtree cut height (aa-admm_amd/csrc/solve_plan.hpp):
// the launch sizes its LDS from the widest level vector of ANY subtree plus the node records of
// the LARGEST subtree, so the cut must be checked on those aggregates. Two unbalanced subtrees:
// A has one wide leaf (a large LDS vector, few records), B is a long chain (narrow vectors, many
// records). Each passes a per-subtree check at the top cut; together they do not.
//
//   g++ -O2 -std=c++17 -I aa-admm_amd/csrc tests/cpp/cut_height.cpp -o cut_height && ./cut_height
#include <cstdio>
#include <vector>

#include "solve_plan.hpp"

int main() {
    using namespace aa;
    // supernodes: 0 = A's wide leaf, 1 = A's root; 2..(2+L-1) = B's chain (leaf first), then the
    // global root R above both subtrees
    const int L = 700;
    const int nn = 2 + L + 1;
    const int R = nn - 1;
    std::vector<int> parent(nn), height(nn), p(nn, 1), nb(nn, 0);
    std::vector<char> inc(nn, 1);
    parent[0] = 1; height[0] = 0; p[0] = 100;   // backward: 24 * 3 * (100 + 164 segment slots) = 19 KB at level 0
    parent[1] = R; height[1] = L - 1;
    for (int k = 0; k < L; ++k) { parent[2 + k] = (k + 1 < L) ? 2 + k + 1 : R; height[2 + k] = k; }
    height[R] = L; parent[R] = -1;
    CutPlanIn a;
    a.parent = &parent; a.height = &height; a.inc = &inc; a.p = &p; a.nb = &nb;
    a.max_height = L; a.ks = 3; a.min_sub = 2; a.seg_rows = 64; a.node_bytes = 56;
    // limits scaled down so the example stays small: A's backward vectors 19.0 KB (ks 3), B's
    // records 700 * 2 * 56 = 78.4 KB; per subtree each fits 90 KiB, together 97.4 KB do not
    a.lds_fwd_level = 1 << 20; a.lds_bwd_level = 1 << 20; a.lds_max = 90 * 1024;
    const int H = choose_cut_height(a);
    int fails = 0;
    // at H = L - 1 the two subtrees are A (0, 1) and the whole chain: the aggregate does not fit;
    // lower cuts keep A's wide leaf as one subtree and shorten the chain's top subtree until its
    // records fit beside that leaf's vectors (H = 652 here)
    auto bwd = [&](int pp) {   // backward LDS vector of one supernode (nb = 0), ks 3
        long long slots = 0;
        for (int sg = 0; sg < (pp + 63) / 64; ++sg) slots += std::min(pp, (sg + 1) * 64);
        return 24LL * 3 * (pp + slots);
    };
    const long long max_f = bwd(100);
    auto rec = [&](int nodes) { return 2LL * nodes * 56; };
    // per-subtree check (the old rule) would accept the top cut:
    const bool old_a = sub_lds_fits(max_f, rec(2), a.lds_max);
    const bool old_b = sub_lds_fits(bwd(1), rec(L), a.lds_max);
    const bool agg = sub_lds_fits(max_f, rec(L), a.lds_max);
    if (!(old_a && old_b && !agg)) { std::printf("FAIL: example does not separate the rules\n"); ++fails; }
    if (H == L - 1) { std::printf("FAIL: cut at the top although the aggregate exceeds the budget\n"); ++fails; }
    if (H != 652) { std::printf("FAIL: cut %d, want 652\n", H); ++fails; }
    // whatever cut is returned, the launch's aggregate must fit
    if (H >= 0) {
        // recompute the aggregate at H: roots at height <= H whose parent is above H
        long long mf = 0, mr = 0;
        std::vector<std::vector<int>> kids(nn);
        for (int s = 0; s < nn; ++s) if (parent[s] >= 0) kids[parent[s]].push_back(s);
        for (int s = 0; s < nn; ++s) {
            if (!(height[s] <= H && (parent[s] < 0 || height[parent[s]] > H))) continue;
            std::vector<int> st{s}, all;
            while (!st.empty()) { int v = st.back(); st.pop_back(); all.push_back(v); for (int c : kids[v]) st.push_back(c); }
            mr = std::max(mr, rec((int)all.size()));
            std::vector<long long> lf(H + 1, 0);
            for (int v : all) lf[height[v]] += bwd(p[v]);
            for (long long x : lf) mf = std::max(mf, x);
        }
        if (!sub_lds_fits(mf, mr, a.lds_max)) { std::printf("FAIL: chosen cut %d exceeds the budget\n", H); ++fails; }
    }
    // a balanced tree (no aggregate conflict) still cuts at the top
    {
        // leaves 0, 1 -> parents 2, 3 -> root 4: two subtrees at the cut height 1
        std::vector<int> par2 = {2, 3, 4, 4, -1}, h2 = {0, 0, 1, 1, 2}, p2 = {10, 10, 10, 10, 10}, nb2 = {5, 5, 5, 5, 0};
        std::vector<char> inc2(5, 1);
        CutPlanIn b = a;
        b.parent = &par2; b.height = &h2; b.inc = &inc2; b.p = &p2; b.nb = &nb2; b.max_height = 2; b.min_sub = 2;
        const int H2 = choose_cut_height(b);
        if (H2 != 1) { std::printf("FAIL: balanced tree cut %d, want 1\n", H2); ++fails; }
    }
    std::printf("cut height %d (L = %d): %s\n", H, L, fails ? "FAIL" : "ok");
    return fails ? 1 : 0;
}
