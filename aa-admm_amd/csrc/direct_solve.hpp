// GPU supernodal triangular solves against the host multifrontal factor (spd_direct.hpp).
//
// Replaces the reference's per-iteration LDLTSolver::solve (LinearSolver.hpp:87-90) and
// SPDSolver::solve (Geometry/SPDSolver.h:60-63) with a level-scheduled solve over the
// nested-dissection supernode tree. Per supernode s (pivots P, boundary rows B, |P| = p,
// |B| = nb) the host pre-multiplies the factor into one dense (p + nb) x p matrix
//        G_s = [ Linv_PP ; M ],   M = L_BP Linv_PP,
// so that both sweeps of a supernode are single matrix-vector products with no dependency
// inside the supernode:
//   forward   f = [b_P ; 0] + extend_add(children's update vectors)
//             y_P = Linv_PP f_P ,   u = f_B - M f_P        (rows of G_s . f_P)
//   backward  x_P = Linv_PP^T y_P - M^T x_B                (columns of G_s . [y_P ; -x_B])
// All supernodes of one tree height are independent, so a level is one launch whose work is
// cut into row tasks: small supernodes get a workgroup (thread per row, front vector in LDS),
// large ones are spread over many workgroups (wave per row, lanes across the row). Every
// product reads a coalesced copy of G_s (row-major for lane-across-row, column-major for
// thread-per-row); sums are in a fixed order (no atomics): deterministic. Three right-hand
// sides (x, y, z coordinates) are processed together -- or six: solve2() runs two independent
// solves in one pass over the factor (bit-identical to two solve() calls).
#pragma once
#include <cstdlib>
#include <vector>

#include "comm.hpp"
#include "common.hpp"
#include "elastic_kernels.hpp"
#include "spd_direct.hpp"

namespace aa {

class DirectSolver {
public:
    static constexpr int kTopRows = 2048;    // upper tree levels amalgamated into one dense root
    // the amalgamation budget in pivots for an n-unknown system (AA_TOP_ROWS overrides): 4096 below
    // 300 k unknowns, kTopRows above. Measured (same-box sweeps 2048 / 4096 / 6500 / 10000): C2
    // (25 k) 6 740 -> 8 173 it/s at 4096 (solve 91 -> 66 us: the top levels of a small tree are
    // latency, not bytes), C3 (101 k) 1 238 -> 1 300, C4 (211 k) flat, C5 (501 k) 167.9 -> 164.9
    // (the larger dense top costs more bytes than its levels cost latency)
    static int top_rows(int n) {
        const char* e = std::getenv("AA_TOP_ROWS");
        return e ? std::atoi(e) : (n < 300000 ? 4096 : kTopRows);
    }
    static constexpr int kPartTopRows = 4096;   // partitioned: a part's upper levels amalgamated (rows)
    static constexpr int kWaveP = 192;       // forward rows longer than this: wave per row
    static constexpr int kWaveR = 384;       // backward columns longer than this: wave per column

    // Partitioned (comm with size > 1): node_part[s] is the part of supernode s
    // (-1 = shared top separator, rows [top_beg, n)); only the supernodes of `my_part` and of
    // the top are stored and solved here, and the top rows of the forward result are summed
    // over the GPUs between the two sweeps.
    // max_sets = 2 sizes the workspaces and the fused subtrees' LDS budget for solve2().
    // wide: plan the layout (subtree cut, 256-wide split-K tiles) for two sets even when
    // max_sets = 1, so both solvers sum in the same order.
    // wave_p / wave_r: supernodes with p above wave_p (forward) / R above wave_r (backward) are
    // split-K tiled, the rest run as row tasks (defaults kWaveP / kWaveR; AA_SOLVE_WAVEP / _WAVER)
    void build(const SupernodalFactor& F, hipStream_t s, const std::vector<int>* node_part = nullptr, int my_part = -1,
               int top_beg = -1, Comm* comm = nullptr, int max_sets = 1, bool wide = false, int wave_p = kWaveP,
               int wave_r = kWaveR);
    // x (n x 3, stride 3 doubles) = A^-1 b ; b is read only. gate: skip when ctrl->done (or !reject).
    void solve(const double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s);
    // x0 = A^-1 b0 and x1 = A^-1 b1 in one pass (needs build(..., max_sets = 2))
    void solve2(const double* b0, double* x0, const double* b1, double* x1, const Ctrl* ctrl, int gate_reject,
                hipStream_t s);
    int n() const { return n_; }
    size_t nnz_L() const { return nnz_L_; }
    double bytes_per_solve() const { return bytes_; }
    double bytes_per_solve2() const { return bytes2_; }
    int kernels_per_solve() const { return kernels_; }

    // One workgroup's share of a level: rows [r0, r0 + nr) of supernode `node` (forward) or
    // its columns (backward), a thread per row. The supernode's metadata rides along so a
    // workgroup needs one (scalar) load before its first product.
    struct Task {
        int node, r0, nr, pad0;
        int p, nb, beg, bnd_off;
        int ell_w, ldr, pad1, pad2;   // ldr: row stride of the row-major G (p padded to even)
        long long goff, uoff, ell_off, pad3;
    };

    // Bottom subtrees (all supernodes up to a cut height) are solved whole by one workgroup
    // each: their levels are separated by workgroup barriers instead of kernel boundaries.
    struct SubNode {   // a supernode inside a fused subtree; lds = its vector's offset in LDS,
        int p, nb, beg, bnd_off, ell_w, lds, slot, ldr;   // slot = its backward segment partials
        long long goff, uoff, ell_off;
        int xo, pad;   // backward copy, kSubX: LDS offset of its x rows (-1: no boundary names them)
    };
    struct SubLevel { int n0, fa0, nfa, fr0, nfr, bv0, nbv, bc0, nbc, bs0, nbs, pad; };   // item ranges
    // nodes [node0, node0 + nnode) staged in LDS. flags: kSubU = the children's update vectors
    // stay in LDS (the forward records' slot = the LDS offset of their own, -1 = global U; the
    // ELL pull lists of the subtree's supernodes hold LDS offsets); kSubX = the x rows a boundary
    // inside the subtree can name stay in LDS -- the columns of its inner supernodes (backward
    // record's xo) and the root's boundary (entry a at xst + 3a, staged from x[xg[xg_off + a]]);
    // the subtree's boundary lists hold those LDS offsets.
    // Offsets are in doubles of a 3-column solve (scaled by NR / 3 on the device, like U's).
    static constexpr int kSubU = 1, kSubX = 2;
    struct SubTree { int lvl0, nlvl, node0, nnode, flags, xst, nxg, xg_off; };
    // split-K backward of large supernodes: a tile (64 columns from c0, nr rows from r0) and the
    // per-column-block reduction of its nt tile partials (64 x 3 doubles each, from poff)
    // toff: the tile's block in the packed tile stream Gt_ (see build: every tile's factor entries
    // stored contiguously in the order its waves consume them)
    // streamed levels (see stream_*): dep = the counter a tile waits on (its parent's, -1 = none)
    // until it reaches need; a reduction adds 1 to counter sig (its own supernode's) when done;
    // xso = the supernode's first row in the padded in-launch copy Xs_ of x
    struct BTile { int beg, p, nb, bnd_off, c0, r0, nr, rid, ldr, dep; long long goff, poff, toff; int need, pad; };
    struct BRed { int beg, c0, nc, nt; long long poff; int sig, xso; };
    // split-K forward of large supernodes: tile (64 rows from r0, nc columns from c0) and the
    // per-row-block reduction of its nt partials
    // streamed levels: dep / need as for BTile (dep = the tile's own supernode: its children's
    // update vectors), sig = the parent's counter a reduction writing update rows adds to
    struct FTile { int beg, p, R, c0, r0, nc, rid, ell_w; long long goff, ell_off, poff, toff; int dep, need, pad0, pad1; };
    struct FRed { int beg, p, r0, nr, nt, ell_w; long long uoff, ell_off, poff; int sig, pad; };

    // Branches (AA_SOLVE_BRANCHES=B, default kBranches; single GPU, not with AA_SOLVE_STREAM): the
    // tree below its top supernodes split into B disjoint groups of subtrees, each swept on its own
    // stream (fork/join by events, so a captured step records them as parallel graph branches)
    static constexpr int kMaxBranches = 8;
    int default_branches = 1;   // set by the caller before build(); AA_SOLVE_BRANCHES overrides
    struct BrRange { int fwd_first = 0, fwd_count = 0, ft_first = 0, ft_count = 0, bwd_first = 0, bwd_count = 0,
                     bt_first = 0, bt_count = 0; };

private:
    struct SideStream {   // branch b's stream (b >= 1; branch 0 runs on the caller's) and its events
        hipStream_t st = nullptr;
        hipEvent_t fork_f = nullptr, join_f = nullptr, fork_b = nullptr, join_b = nullptr;
        void create(int dev) {
            if (st) return;
            AA_HIP(hipSetDevice(dev));
            AA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            for (hipEvent_t* e : {&fork_f, &join_f, &fork_b, &join_b}) AA_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
        }
        ~SideStream() {
            for (hipEvent_t e : {fork_f, join_f, fork_b, join_b}) if (e) (void)hipEventDestroy(e);
            if (st) (void)hipStreamDestroy(st);
        }
    };
    int nbr_ = 1;
    bool branch_reject_ = false;                  // AA_SOLVE_BRANCHES_REJECT: the gated reject solve branched too
    std::vector<int> brn_;                        // branch of every supernode (nbr_ = top)
    std::vector<BrRange> lbr_;                    // [level][nbr_ + 1]
    std::vector<std::pair<int, int>> sub_rng_;    // fused subtrees per branch: (first, count)
    SideStream side_[kMaxBranches];
    void plan_branches(const SupernodalFactor& F, const std::vector<char>& inc, const std::vector<char>& fused,
                       const std::vector<std::vector<int>>& kids, const std::vector<int>& p, const std::vector<int>& nb,
                       bool stats);
    struct Level {
        int fwd_first = 0, fwd_count = 0, bwd_first = 0, bwd_count = 0;
        int bt_first = 0, bt_count = 0, br_first = 0, br_count = 0;   // split-K backward tiles
        int ft_first = 0, ft_count = 0, fr_first = 0, frd_count = 0;  // split-K forward tiles
        int fblock = 256, bblock = 256, lds_fwd = 0, lds_bwd = 0;
        int ftw = 256, btw = 256;   // split-K tile widths (forward columns / backward rows)
    };
    int n_ = 0, nn_ = 0, kernels_ = 0, top_beg_ = 0;
    Comm* comm_ = nullptr;
    size_t nnz_L_ = 0;
    double bytes_ = 0, bytes2_ = 0;
    int max_sets_ = 1;
    template <int NR>
    void launch_ftiles(int w, int count, int first, const double* b0, const double* b1, int ext_off, const Ctrl* ctrl,
                       int gate_reject, hipStream_t s);
    template <int NR>
    void launch_btiles(int w, int count, int first, double* x0, double* x1, int ext_off, const Ctrl* ctrl,
                       int gate_reject, hipStream_t s);
    struct Stream;
    template <int NR>
    void launch_fstream(const Stream& S, const double* b0, const double* b1, const Ctrl* ctrl, int gate_reject,
                        hipStream_t s);
    template <int NR>
    void launch_bstream(const Stream& S, double* x0, double* x1, const Ctrl* ctrl, int gate_reject, hipStream_t s);
    template <int NR>
    void solve_nr(const double* b0, double* x0, const double* b1, double* x1, const Ctrl* ctrl, int gate_reject,
                  hipStream_t s);
    DevBuf<int> bnd_;
    DevBuf<long long> ell_;   // per front row, ell_w pull offsets into U (-1 = none)
    DevBuf<double> Gr_, Gc_, Y_, U_;
    // packed split-K tiles (AA_SOLVE_PACKED, default on): per tile one contiguous block, per wave
    // a sequential stream of 1-KB rows (64 lanes x 16 B): forward [wave][column pair][row][2],
    // backward [wave][row][column pair][2]; zero-padded to whole tiles
    DevBuf<double> Gt_;
    bool packed_ = true;
    // non-temporal factor loads (AA_FACTOR_NT=0/1 forces): on when both sweeps' factor bytes
    // exceed kNtBytes, i.e. the factor streams past the 256 MB Infinity Cache every solve
    static constexpr double kNtBytes = 192e6, kNtRowsMaxBytes = 512e6;
    bool nt_ = true, nt_rows_ = true;

    DevBuf<Task> tasks_;
    DevBuf<BTile> btiles_;
    DevBuf<BRed> breds_;
    DevBuf<FTile> ftiles_;
    DevBuf<FRed> freds_;
    DevBuf<int> fcnt_, bcnt_;   // tiles finished per reduction task (reset by the last tile)
    DevBuf<double> bpart_;
    std::vector<Level> levels_;
    // Streamed tile levels (AA_SOLVE_STREAM=1; measured slower than one launch per level on C4): a run of consecutive levels that have
    // split-K tiles only is ONE launch. Its workgroups take tiles in level order from a queue
    // (ticket = atomic add), issue their factor loads, and only then wait for the tile's inputs:
    // the children's update vectors (forward) or the parent's x rows (backward), published
    // in-launch by the reductions (write-through stores, drained, then a counter add; the waiting
    // workgroup polls, takes one agent acquire, then reads -- MI355X_MICROARCH.md "Valid
    // forms"). A level's factor stream thus overlaps the previous level's tail and reductions
    // instead of waiting for its kernel boundary. Same tiles, partials and sums: bit-identical.
    struct Stream { int l0, l1, first, count, head; };   // levels [l0, l1), queue order_[first, +count)
    std::vector<Stream> fstreams_, bstreams_;
    bool stream_ = false;        // every solve streams its tile runs (AA_SOLVE_STREAM=1)
    bool stream_gated_ = false;  // the reject path's gated solves do (AA_SOLVE_STREAM_GATED, default on)
    bool stream_plan_ = false;   // the runs are planned (either of the above)
    DevBuf<int> forder_, border_, bndx_;   // tile queues; per boundary entry its Xs_ row (-1: read x)
    DevBuf<int> sync_;   // [queue heads | forward counters (nn_) | backward counters (nn_)], zeroed per solve
    int n_heads_ = 0;
    DevBuf<double> Xs_;   // backward: x rows of streamed supernodes, each supernode 128-B aligned
    // partitioned with a dense shared top (nested_dissection merge_top): the top root supernode
    // top_sn_ is solved outside the levels -- its front assembled locally and summed over the
    // GPUs, then each GPU runs the forward rows [top_r0_, top_r1_) and the backward products of
    // those rows (a partial x_top), and one more sum gives every GPU the whole x_top.
    static constexpr int kTopBlk = 64;   // row granularity of the split (the forward tiles' rows)
    int top_sn_ = -1, top_p_ = 0, top_r0_ = 0, top_r1_ = 0;
    int top_ft_first_ = 0, top_ft_count_ = 0, top_bt_first_ = 0, top_bt_count_ = 0, top_ftw_ = 256, top_btw_ = 256;
    Task top_task_{};
    DevBuf<Task> top_task_d_;
    DevBuf<double> top_f_, top_x_;   // [set][3 * top_p_]: summed front, partial then summed x_top
    // fused bottom subtrees
    int n_sub_ = 0, sub_lds_f_ = 0, sub_lds_b_ = 0, cut_height_ = -1, sub_block_ = 256, sub_nodes_max_ = 0;
    int sub_lds_u_ = 0, sub_lds_x_ = 0;   // LDS-resident update vectors / x rows (bytes per 3 columns)
    DevBuf<int> sub_xg_;                  // per kSubX subtree: its root's boundary (global x rows)
    size_t sub_lds_bytes(int K, bool fwd) const;
    // kSubU / kSubX per subtree where the extra LDS fits beside the level vectors and records;
    // rewrites those subtrees' ELL pull lists and boundary lists to LDS offsets (build only)
    void plan_sub_lds(const SupernodalFactor& F, const std::vector<std::vector<int>>& kids, const std::vector<int>& p,
                      const std::vector<int>& nb, const std::vector<int>& beg, const std::vector<long long>& uoff,
                      const std::vector<int>& bnd_off, const std::vector<int>& ell_w,
                      const std::vector<long long>& ell_off, std::vector<long long>& ell, std::vector<int>& bnd,
                      const std::vector<int>& fidx, const std::vector<int>& bidx,
                      const std::vector<std::vector<int>>& sub_all,
                      std::vector<SubTree>& strees, std::vector<SubNode>& snodes, int KS, bool stats, hipStream_t s);
    int wave_p_ = kWaveP, wave_r_ = kWaveR;   // row-task / split-K thresholds (AA_SOLVE_WAVEP / _WAVER)
    DevBuf<SubNode> sub_nodes_;
    DevBuf<SubLevel> sub_levels_;
    DevBuf<SubTree> sub_trees_;
    DevBuf<int> sub_items_;   // (local node << 16 | row) per item
    DevBuf<long long> sub_items2_;   // backward segment items (local node << 40 | segment << 20 | column)
    int sub_timing_ = 0;              // AA_SUB_TIMING: solves left to time phase by phase
    DevBuf<long long> sub_clk_;       // [2][n_sub_][64] s_memrealtime stamps
};

}  // namespace aa
