// Host orchestration of the Geometry (ALM) hot path on one MI355X: the reference's
// ALMGeometrySolver<3> (Geometry/ALMGeometrySolver.h) with its Constraint<3> plugins
// (Geometry/Constraint.h), LinearRegularization (Geometry/LinearRegularization.h) and the
// AndersonAcceleration on (u, x) (Geometry/AndersonAcceleration.h).
#pragma once
#include <map>
#include <string>
#include <tuple>
#include <cstdlib>
#include <vector>

#include "../../include/aa_admm.h"
#include "common.hpp"
#include "direct_solve.hpp"
#include "elastic.hpp"
#include "geom_kernels.hpp"

namespace aa {

class GeomSolver {
public:
    // plain = false: ALMGeometrySolver<3>; true: GeometrySolver<3> (Geometry/GeometrySolver.h)
    explicit GeomSolver(Context* ctx, bool plain = false) : ctx_(ctx), plain_(plain) {}
    ~GeomSolver();

    int add_ref_surface(const double* V3, int nv, const int* F3, int nf);
    void add_constraints(int hard, int type, const int* idx, int k, int count, double weight, const double* params);
    void add_laplacian(const int* idx, const double* coefs, int k, double weight, const double* ref_points3);
    void add_closeness(int idx, double weight, const double* target3);
    void setup(int n_points, double penalty, int spd_solver_type);
    void solve(const double* init_x3, double rel_residual_eps, int max_iter, int anderson_m);
    // run-to-epsilon (not in the reference's loop, whose test is commented out at
    // ALMGeometrySolver.h:258-260): at_eps stops after the accepted iteration whose combined
    // residual falls below rel_residual_eps^2 * hard_cols^2 * 2 (ALMGeometrySolver.h:172);
    // eps_rel > 0 also stops once comb <= eps_rel * comb of the first accepted iteration
    void set_stop(int at_eps, double eps_rel);
    void get_solution(double* x3) const;
    int history(double* comb, double* time_s, int cap) const;
    aa_geom_runtime runtime() const { return rt_; }
    void closest_points(int surface, const double* p3, int n, double* out3);
    // multi-GPU: partition the points over comm's ranks at the first solve;
    // every rank passes the same problem. Not owned; must outlive the solver.
    void set_comm(Comm* c);

    double bench_iterations(int iters);
    bool kernel_stats(const std::string& name, double* avg_ms, double* bytes, int* launches) const;

private:
    struct HostGroup {
        int hard, type, K, surf;
        double weight;
        std::vector<int> idx;      // [count][K] user point ids
        std::vector<double> prm;   // [count][P]
        int count() const { return (int)(idx.size() / K); }
    };
    struct DevGroup {
        DevBuf<int> idx, warm;
        DevBuf<double> prm;
        GeoGroupDev d{};
    };
    void enqueue_chunk(int chunk, int m);
    struct Surface {
        std::vector<BvhNode> nodes;
        std::vector<BvhTri> tris;
        DevBuf<BvhNode> dnodes;
        std::vector<BvhNode> wide;   // collapsed tree of the group traversal (wide_g children)
        DevBuf<BvhNode> dwide;
        int wide_g = 0;
        DevBuf<BvhTri> dtris;
        SurfDev dev() const {
            return SurfDev{dnodes.p, dtris.p, (int)nodes.size(), (int)tris.size(), wide_g ? dwide.p : nullptr, wide_g};
        }
    };
    struct Reg { std::vector<int> idx; std::vector<double> coef; double tgt[3]; };
    // reference-surface constraints processed in the points' nested-dissection order
    // (AA_SURF_ND_ORDER=0: the caller's order)
    bool nd_sort_surf_ = !(std::getenv("AA_SURF_ND_ORDER") && std::getenv("AA_SURF_ND_ORDER")[0] == '0');

    Context* ctx_;
    bool plain_ = false;
    bool has_u(const HostGroup& g) const { return plain_ || g.hard; }   // z / u columns on device
    hipStream_t s() const { return ctx_->stream; }

    // host model
    std::vector<HostGroup> hgroups_;
    std::map<std::tuple<int, int, int, double, int>, int> group_of_;
    std::vector<Surface> surfs_;
    std::vector<Reg> regs_;
    int n_ = 0;
    double rho_ = 1.0;
    bool setup_done_ = false, factored_ = false;

    // internal numbering: points in nested-dissection order (fixed at the first solve, which
    // is the first time point positions are known: ALMGeometrySolver::solve_ADMM(init_x, ...))
    std::vector<int> user2int_, int2user_;
    std::vector<std::vector<std::pair<int, double>>> arows_;   // assembled global matrix (user ids)
    std::vector<double> rhs_fixed_user_;
    long long Zh_ = 0, slots_ = 0;
    bool stop_eps_ = false;
    double stop_rel_ = 0.0;
    long long hard_cols() const;
    int red_blocks_ = 0;

    // device
    std::vector<DevGroup> groups_;
    DirectSolver solver_;
    DevBuf<int> slot_ptr_, slot_idx_;
    DevBuf<double> rhs_fixed_, b_, y_;
    DevBuf<double> cur_x_, new_x_, def_x_, cur_u_, new_u_, def_u_, z_;
    DevBuf<double> aa_cur_, aa_dF_, aa_dG_, aa_red_, red_;
    // partition: own points [own_beg_, own_end_), shared top [top_beg_, n_); all-rank sums of
    // the residual / Anderson partials (aliases of the local ones on one GPU)
    Comm* comm_ = nullptr;
    int rank_ = 0, own_beg_ = 0, own_end_ = 0, top_beg_ = 0, nbg_ = 0;
    long long zh_max_ = 0;
    DevBuf<double> red_g_, aa_red_g_;
    double* redg_ = nullptr;
    double* aag_ = nullptr;
    AAMask aamask_;
    DevBuf<Ctrl> ctrl_;
    DevBuf<double> hist_comb_;
    DevBuf<unsigned long long> hist_clock_, clock0_;
    int aa_blocks_ = 0, cur_m_ = -1, hist_cap_ = 0;
    bool have_solution_ = false;
    std::vector<double> last_init_;
    std::vector<double> h_comb_, h_time_;
    aa_geom_runtime rt_{};
    double clock_khz_ = 0;

    // captured loop passes, one graph per chunk size kChunks[i] (captured on first use)
    static constexpr int kNChunks = 4;
    static constexpr int kChunks[kNChunks] = {64, 16, 4, 1};
    hipGraph_t graph_[kNChunks] = {};
    hipGraphExec_t gexec_[kNChunks] = {};
    int graph_m_ = -1;
    void drop_graph();

    DevBuf<int> mk_log_;   // (aa_mk, aa_skip) per instrumented Anderson launch
    int n_mk_log_ = 0;
    bool instrument_ = false;
    struct KStat { std::vector<hipEvent_t> ev; double bytes = 0; double total_ms = 0; int launches = 0; };
    std::map<std::string, KStat> kstats_;
    void ev_mark(const char* name);

    void factor_and_upload(const double* init_x3);
    void prepare_m(int m);
    void prologue(const double* init_x3, int max_iter, int m, int cap, double eps_abs = 0.0, double eps_rel = 0.0);
    void enqueue_iteration(int m);
    void enqueue_iteration_plain(int m);
    void enqueue_u_update(double* red, hipStream_t st);
    // Constraint groups on parallel graph branches (opt-in, AA_GEOM_CONCURRENT=1; measured slower,
    // DESIGN.md §3.4 -- off by default, one stream): each
    // group's z / u kernels write only its own z, u, rhs slots and residual partials, so the
    // groups other than the heaviest run on side_ beside it (joined before the next consumer)
    bool conc_ = false;
    int heavy_ = 0;   // the group kept on the main stream (the closest-point group, else the largest)
    hipStream_t side_ = nullptr;
    hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
    void fork();
    void join();
    void fetch_results();
    double* solution_buf() { return plain_ ? cur_x_.p : new_x_.p; }
};

}  // namespace aa
