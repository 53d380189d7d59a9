// CPU test of the LDS slot plan for the fused subtrees' update vectors
// (aa-admm_amd/csrc/solve_plan.hpp plan_update_slots, DirectSolver kSubU). Random trees (heights
// = longest path to a leaf, as the factor's), random boundary sizes; the forward kernel's
// schedule is replayed level by level: phase 1 reads the children's slots, phase 2 reads them
// again (boundary rows' own fronts) and writes the level's slots. Checked: no slot written in a
// level overlaps a slot still to be read in that level or later, the root has none, every other
// supernode with a boundary has one, and the peak is what the slots span.
//
//   g++ -O2 -std=c++17 -I aa-admm_amd/csrc tests/cpp/update_slots.cpp -o update_slots && ./update_slots
#include <cstdio>
#include <random>
#include <vector>

#include "solve_plan.hpp"

static int fail(const char* what, int t) {
    std::printf("FAIL %s (tree %d)\n", what, t);
    return 1;
}

int main() {
    std::mt19937 rng(12345);
    for (int t = 0; t < 300; ++t) {
        const int nn = 1 + (int)(rng() % 400);
        // node 0 is the root; a node's parent has a smaller index
        std::vector<int> parent(nn, -1), nb(nn), height(nn, 0);
        for (int v = 1; v < nn; ++v) parent[v] = (int)(rng() % (unsigned)v);
        for (int v = 0; v < nn; ++v) nb[v] = (rng() % 5 == 0) ? 0 : 1 + (int)(rng() % 90);
        for (int v = nn - 1; v >= 1; --v) height[parent[v]] = std::max(height[parent[v]], height[v] + 1);
        std::vector<std::vector<int>> kids(nn);
        for (int v = 1; v < nn; ++v) kids[parent[v]].push_back(v);
        std::vector<int> all;
        for (int v = 0; v < nn; ++v) all.push_back(v);   // root first
        std::vector<int> slot(nn, -7);
        const int peak = aa::plan_update_slots(all, kids, height, nb, slot);
        int span = 0;
        for (int v = 0; v < nn; ++v) {
            if (v == 0 && slot[v] != -1) return fail("root has a slot", t);
            if (v != 0 && nb[v] > 0 && slot[v] < 0) return fail("missing slot", t);
            if (v != 0 && nb[v] == 0 && slot[v] != -1) return fail("slot without a boundary", t);
            if (slot[v] >= 0) span = std::max(span, slot[v] + nb[v]);
        }
        if (span != peak) return fail("peak", t);
        // replay: at level h the live set is every slotted node written at a level < h whose
        // parent is at level >= h, plus the nodes written at h; written ones must not overlap them
        const int H = height[0];
        for (int h = 0; h <= H; ++h) {
            std::vector<int> live;
            for (int v = 1; v < nn; ++v)
                if (slot[v] >= 0 && height[v] <= h && height[parent[v]] >= h) live.push_back(v);
            for (size_t i = 0; i < live.size(); ++i)
                for (size_t j = i + 1; j < live.size(); ++j) {
                    const int a = live[i], b = live[j];
                    if (slot[a] < slot[b] + nb[b] && slot[b] < slot[a] + nb[a]) return fail("live slots overlap", t);
                }
        }
    }
    std::printf("ok\n");
    return 0;
}
