// Host-only planning of the fused bottom subtrees of DirectSolver (no HIP dependency, so the
// CPU test tests/cpp/cut_height.cpp compiles it with g++).
//
// The fused kernels (k_fwd_sub / k_bwd_sub) take their dynamic LDS from maxima over ALL
// subtrees: the widest level vectors of any subtree (16-B aligned) plus the node records of the
// largest subtree (DirectSolver::sub_lds_bytes). Those two maxima may come from different
// subtrees, so the cut height is chosen against the same aggregates (a per-subtree
// check let subtree A's wide level and subtree B's many records exceed 160 KiB together).
#pragma once
#include <algorithm>
#include <vector>

namespace aa {

struct CutPlanIn {
    const std::vector<int>* parent;   // supernode -> parent (-1 = root)
    const std::vector<int>* height;   // 0 at the leaves
    const std::vector<char>* inc;     // supernodes this solver holds
    const std::vector<int>* p;        // pivots per supernode
    const std::vector<int>* nb;       // boundary rows per supernode
    int max_height = 0;
    int ks = 1;                       // right-hand-side sets (the LDS figures scale with it)
    int min_sub = 256;                // fused subtrees wanted (workgroups)
    int seg_rows = 64;                // backward segment rows (kSubSegRows)
    long long node_bytes = 56;        // sizeof(SubNode)
    long long lds_fwd_level = 64 * 1024, lds_bwd_level = 144 * 1024, lds_max = 160 * 1024;
    int max_item_row = 0xffff;
};

inline bool sub_lds_fits(long long vec_bytes, long long rec_bytes, long long lds_max) {
    return (vec_bytes + 15) / 16 * 16 + rec_bytes <= lds_max;
}

// the largest cut height H (< max_height) such that at least min_sub subtrees root at height
// <= H and the fused launch's aggregate LDS fits; -1 if none
inline int choose_cut_height(const CutPlanIn& a) {
    const auto& parent = *a.parent;
    const auto& height = *a.height;
    const auto& inc = *a.inc;
    const auto& p = *a.p;
    const auto& nb = *a.nb;
    const int nn = (int)parent.size();
    std::vector<std::vector<int>> kids(nn);
    for (int sn = 0; sn < nn; ++sn) if (parent[sn] >= 0 && inc[sn]) kids[parent[sn]].push_back(sn);
    for (int H = a.max_height - 1; H >= 1; --H) {
        std::vector<int> roots;
        for (int sn = 0; sn < nn; ++sn)
            if (inc[sn] && height[sn] <= H && (parent[sn] < 0 || height[parent[sn]] > H)) roots.push_back(sn);
        if ((int)roots.size() < a.min_sub) continue;
        bool ok = true;
        long long max_f = 0, max_b = 0, max_rec = 0;
        for (int rt : roots) {
            std::vector<long long> lf(H + 1, 0), lb(H + 1, 0), nodes_at(H + 1, 0);
            std::vector<int> all, st{rt};
            while (!st.empty()) { int v = st.back(); st.pop_back(); all.push_back(v); for (int c : kids[v]) st.push_back(c); }
            // two records per supernode (forward and backward LDS offsets)
            max_rec = std::max(max_rec, 2LL * (long long)all.size() * a.node_bytes);
            for (int v : all) {
                lf[height[v]] += 24LL * a.ks * p[v];
                long long slots = 0;
                for (int sg = 0; sg < (p[v] + nb[v] + a.seg_rows - 1) / a.seg_rows; ++sg)
                    slots += std::min(p[v], (sg + 1) * a.seg_rows);
                lb[height[v]] += 24LL * a.ks * (p[v] + nb[v] + slots);
                nodes_at[height[v]] += 1;
                if (p[v] + nb[v] > a.max_item_row) ok = false;
            }
            for (int h = 0; h <= H; ++h) {
                if (lf[h] > a.lds_fwd_level || lb[h] > a.lds_bwd_level || nodes_at[h] > a.max_item_row) ok = false;
                max_f = std::max(max_f, lf[h]);
                max_b = std::max(max_b, lb[h]);
            }
            if (!ok) break;
        }
        if (ok && sub_lds_fits(max_f, max_rec, a.lds_max) && sub_lds_fits(max_b, max_rec, a.lds_max)) return H;
    }
    return -1;
}

// LDS slots (in rows) for the update vectors a fused subtree keeps on chip (kSubU). `all` is the
// subtree's supernodes, root first; the root's update vector leaves the subtree (slot -1). The
// forward kernel runs a level in two phases -- (1) the front gathers of the level's supernodes,
// (2) their rows, whose boundary rows gather their own front values again and then write the
// supernode's update vector -- so a child's slot is live from its own level until its parent's
// level has finished both phases: slots of level h are taken first-fit, and the children of
// level h are released after them. Returns the peak row count (the LDS region's size).
inline int plan_update_slots(const std::vector<int>& all, const std::vector<std::vector<int>>& kids,
                             const std::vector<int>& height, const std::vector<int>& nb, std::vector<int>& slot) {
    if (all.empty()) return 0;
    const int root = all[0];
    int H = 0;
    for (int v : all) H = std::max(H, height[v]);
    std::vector<std::vector<int>> at(H + 1);
    for (int v : all) at[height[v]].push_back(v);
    std::vector<std::pair<int, int>> used;   // (first row, rows), sorted by first row
    int peak = 0;
    for (int h = 0; h <= H; ++h) {
        std::sort(at[h].begin(), at[h].end());
        for (int v : at[h]) {
            slot[v] = -1;
            if (v == root || nb[v] == 0) continue;
            int pos = 0;
            size_t i = 0;
            for (; i < used.size(); ++i) {
                if (used[i].first - pos >= nb[v]) break;
                pos = used[i].first + used[i].second;
            }
            used.insert(used.begin() + (long)i, {pos, nb[v]});
            slot[v] = pos;
            peak = std::max(peak, pos + nb[v]);
        }
        for (int v : at[h])
            for (int c : kids[v]) {
                if (slot[c] < 0) continue;
                for (size_t i = 0; i < used.size(); ++i)
                    if (used[i].first == slot[c]) { used.erase(used.begin() + (long)i); break; }
            }
    }
    return peak;
}

}  // namespace aa
