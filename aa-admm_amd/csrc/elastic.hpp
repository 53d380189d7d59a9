// Host orchestration of the admm-elastic hot path on one MI355X (the reference's
// admm::Solver, admm_anderson_hard_zxu/src/Solver.{hpp,cpp} and admm_anderson_xzu/src/...).
#pragma once
#include <array>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/aa_admm.h"
#include "comm.hpp"
#include "common.hpp"
#include "direct_solve.hpp"
#include "elastic_kernels.hpp"

namespace aa {

struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
};

class ElasticSolver {
public:
    explicit ElasticSolver(Context* ctx) : ctx_(ctx) {}
    ~ElasticSolver();

    int add_nodes(const double* x3, const double* m3, int n);
    void add_elements(int kind, int material, const double* verts3, const int* idx, int count, const aa_lame& lame,
                      int vertex_offset);
    void set_pins(const int* inds, const double* pts3, int n);
    // energy-based collisions of the (u,x) variant (admm_anderson_hard_zxu Solver.cpp:318-348)
    void add_obstacle(int type, const double* params);
    void set_collisions(const int* inds, int n);
    // WindForce (ExplicitForce.hpp:39-47) on the given triangles; returns its id
    int add_wind(const int* tris3, int ntris, const double* dir3);
    void set_wind(int id, const double* dir3);
    // multi-GPU: partition the mesh over comm's ranks at initialize(); every
    // rank passes the same scene. Not owned; must outlive the solver.
    void set_comm(Comm* c);
    void initialize(const aa_settings& s);
    void step();

    int num_nodes() const { return (int)x_.size() / 3; }
    void get_x(double* out);
    void get_v(double* out);
    void set_v(const double* v3);
    void set_x(const double* x3);
    int history(double* prim, double* comb, int* rej, int cap) const;
    int times(double* time_ms, int cap) const;
    void set_iterations(int admm_iters, double eps_rel);
    aa_runtime runtime() const { return rt_; }

    // benchmarking: run `iters` iterations of the ADMM loop body of a fresh time step;
    // returns device-synchronised wall ms. Per-kernel-class event timings are collected.
    double bench_iterations(int iters);
    bool kernel_stats(const std::string& name, double* avg_ms, double* bytes, int* launches) const;
    // the local-step work queue's diagnostics (kLqStats counters; 0 when not enabled); reset after
    int local_stats(long long* out, int cap, bool reset);
    const std::vector<std::pair<std::string, double>>& setup_phases() const { return setup_phases_; }

private:
    struct HostGroup {
        int kind, material, nv, ncol;
        aa_lame lame;
        std::vector<int> idx;       // [count][nv] global node ids
        std::vector<double> G;      // [count][ncol][nv]
        std::vector<double> vol, w;
    };
    struct DevGroup {
        DevBuf<int> idx, spos;
        DevBuf<double> G, w, vol;
        GroupDev d{};
    };
    Context* ctx_;
    hipStream_t s() const { return ctx_->stream; }

    // host model
    std::vector<double> x_, v_, m3_;
    std::vector<HostGroup> hgroups_;
    std::map<int, std::array<double, 3>> pins_;
    std::vector<std::array<double, kObsStride>> obstacles_;
    std::vector<int> coll_nodes_;   // collision-checked nodes (sorted, as the reference's map)
    struct Wind {
        std::vector<int> tris;      // user node ids
        double dir[3];
        DevBuf<int> dtris, dord, dlvl;
        int nlvl = 0;
    };
    std::vector<std::unique_ptr<Wind>> winds_;
    DevBuf<double> obs_dev_;
    void upload_obstacles();
    void build_wind(Wind& w);
    std::vector<int> pin_order_;
    aa_settings st_{};
    bool initialized_ = false;

    // internal numbering: free nodes in nested-dissection order, then pinned (sorted)
    int n_ = 0, nf_ = 0, np_ = 0;
    long long Z_ = 0, Yslots_ = 0;
    std::vector<int> node2int_, int2node_;
    double pdt2_ = 0;

    // device
    std::vector<DevGroup> groups_;
    DirectSolver solver_;
    DevBuf<int> dt_ptr_;
    DevBuf<double> xs_, vs_, mass_, xfull_, xlast_, xbar_, Mxbar_, b_, b2_, cxfull_;
    DevBuf<double> z_, u_, y_, du_, dz_, dx_, lastz_, cz_;
    DevBuf<double> aa_cur_, aa_dF_, aa_dG_, aa_red_, aa_red_g_;
    // residual block partials: this rank's [a | b] (pa_, pb_) and their sums over the ranks
    // (ga_, gb_; aliases of pa_, pb_ on one GPU); nbg_ = the largest rank's block count
    DevBuf<double> red_ab_, red_gab_;
    double *pa_ = nullptr, *pb_ = nullptr, *ga_ = nullptr, *gb_ = nullptr, *aag_ = nullptr;
    int nbg_ = 0;
    DevBuf<Ctrl> ctrl_;
    DevBuf<int> lzq_;          // work-queue counter of the hyperelastic local step
    DevBuf<unsigned long long> lq_stats_;   // its diagnostics (AA_LQ_STATS=1)
    LocalQueue lq_;
    bool use_queue_ = true;
    DevBuf<double> hist_prim_, hist_comb_;
    DevBuf<int> hist_rej_;
    DevBuf<long long> hist_clock_;
    double clock_khz_ = 100000.0;
    std::vector<double> h_time_;
    int red_blocks_ = 0, aa_blocks_ = 0, hist_cap_ = 0;
    // partition: own free nodes [own_beg_, own_end_), shared top [top_beg_, nf_)
    Comm* comm_ = nullptr;
    int rank_ = 0, own_beg_ = 0, own_end_ = 0, top_beg_ = 0;
    void reduce_partials();
    void reduce_aa();
    void gather_state(DevBuf<double>& v);
    std::vector<double> h_prim_, h_comb_;
    std::vector<int> h_rej_;
    int nrec_ = 0;
    aa_runtime rt_{};
    std::vector<std::pair<std::string, double>> setup_phases_;   // last initialize(): (phase, ms)
    bool pins_dirty_ = true;

    // the whole ADMM loop of a time step, captured once into a hipGraph and replayed per step
    hipGraph_t graph_ = nullptr;
    hipGraphExec_t gexec_ = nullptr;
    bool use_graph_ = true;
    bool pipe_z_ = false;   // Z variant + Anderson: comb solve batched with the next solve
    void drop_graph();
    // Concurrent combined-residual pass (pipelined Z variant, one GPU; AA_CONCURRENT=0 turns it
    // off): iteration k-1's pass runs on side_ beside iteration k, with its own control block,
    // partials and work-queue counter; default_{u,z,x} alternate between two buffers by
    // iteration parity so the pass reads k-1's while iteration k writes its own.
    bool conc_ = false;
    int conc_fork_ = 1;   // where the side pass forks: after the local step (0), AA reduce (1), mix (2)
    bool join_wait_ = false;
    double* join_dx_ = nullptr;
    void join_side();
    hipStream_t side_ = nullptr;
    hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
    DevBuf<Ctrl> ctrl_c_;
    DevBuf<int> lzq2_;
    LocalQueue lq2_;
    DevBuf<double> red_c_, du2_, dz2_, dx2_;
    double* du_at(int it) { return conc_ && (it & 1) ? du2_.p : du_.p; }
    double* dz_at(int it) { return conc_ && (it & 1) ? dz2_.p : dz_.p; }
    double* dx_at(int it) { return conc_ && (it & 1) ? dx2_.p : dx_.p; }

    // kernel-class event timing (bench only)
    bool instrument_ = false;
    struct KStat { std::vector<hipEvent_t> ev; double bytes = 0; double total_ms = 0; int launches = 0; };
    std::map<std::string, KStat> kstats_;
    void ev_begin(const char* name);
    void ev_end(const char* name);

    void upload_pins();
    void prologue();
    void enqueue_iteration_ux(bool accel);
    void enqueue_iteration_z(bool accel, int it);
    void comb_finish_z(int op, hipStream_t st, Ctrl* c, double* pa, double* pb, const LocalQueue* q,
                       const double* du, const double* dz);
    void enqueue_comb_tail_z(int iters);
    void enqueue_iterations(int iters, bool accel);
    void epilogue_enqueue(bool accel);
    void fetch_results();
    int nb_elems() const { return red_blocks_; }
    void local_z_all(const double* xfull, const double* u, double* z, double* y, int mode, bool red);
    void local_z_on(const double* xfull, const double* u, double* z, int mode, hipStream_t st, Ctrl* c,
                    const LocalQueue* q);
};

}  // namespace aa
