// Device data structures and kernel launchers of the admm-elastic hot path.
#pragma once
#include <hip/hip_runtime.h>

namespace aa {

constexpr int kMaxM = 32;          // largest Anderson window supported on device
constexpr double kCombEps = 1e-20; // Solver.cpp:93 eps

// One homogeneous block of energy terms (same kind / material / Lame), SoA on device.
struct GroupDev {
    int kind;            // 0 tet, 1 tri, 2 collision point (CollisionEnergyTerm.hpp:41-117)
    int mat;             // 0 linear, 1 NeoHookean, 2 StVK
    int count;           // elements
    int nv, ncol, dim;   // 4/3/9 for tets, 3/2/6 for tris
    int pinned;          // some element of the group has a pinned node (C_fix terms exist)
    long long zoff;      // z/u offset: component c of element e at zoff + c*count + e
    long long yrow;      // first vertex slot of this group in the slot array y (slot e*nv + a, 3 doubles)
    const int* idx;      // [nv][count] internal node ids
    const int* spos;     // [nv][count] position of the vertex's rhs slot (node order), -1 = pinned
    const double* G;     // [(c*nv + a)][count]  F[:,c] = sum_a G[c][a] x_a
    const double* w;     // [count] ADMM weights sqrt(k*vol)
    const double* vol;   // [count]
    double mu, lambda, k, lmin, lmax;
    const double* obs;   // collision points: the obstacle table (obs[0] = count, then kObsStride per obstacle)
};
// passive obstacles of the collision terms (PassiveObject.hpp:32-136): type, then up to 7 parameters
enum ObsType { OBS_FLOOR = 0, OBS_SLIDE_FLOOR = 1, OBS_SPHERE = 2, OBS_PLANE_HALF_SPHERE = 3, OBS_CYLINDER = 4 };
constexpr int kObsStride = 8, kMaxObstacles = 256;
__host__ __device__ constexpr int ncol_of(int nv) { return nv > 1 ? nv - 1 : 1; }   // 1 vertex: identity reduction

// Device-side control block: residual bookkeeping, reject/done flags, Anderson state.
struct Ctrl {
    double prim, prev_prim, comb, prim2, dual2;
    int reject, done, nrec, nrej;
    int cap, fail, iters_run, aa_skip;   // aa_skip: ALM reject -> no Anderson step this iteration
    // Anderson acceleration (AndersonAcceleration.h state)
    int aa_m, aa_iter, aa_col, aa_mk;
    int aa_j, aa_jn, aa_first, aa_active;
    double aa_s;
    double scale[kMaxM], coef[kMaxM];
    double M[kMaxM * kMaxM];      // normal-equation matrix, column-major m x m
    // Geometry ALM loop (ALMGeometrySolver.h:186-263): `reset` flag and accepted-iteration cap
    int alm_reset, max_iter;
    // time-to-epsilon: device clock (wall_clock64) of every recorded iteration and
    // of the step's start; optional stop once comb <= eps_rel * comb of the first recorded
    // iteration (eps_rel = 0: the reference's loop, only the comb < 1e-20 break).
    long long* hist_clock;
    long long clock0;
    double eps_rel, eps_abs;
    int eps_hit, pad_;
};
// device stamp of the step's start (ctrl->clock0)
void launch_stamp(Ctrl* ctrl, hipStream_t s);

// A vector seen as two concatenated segments (e.g. (u, x) of the UX variant).
struct Seg2 {
    double* a; long long na;
    double* b; long long nb;
};

// Entries of the second segment that enter the Anderson dot products (partitioned solvers: the
// x entries this rank owns -- its part and, on rank 0, the shared separators); the first
// segment always counts. Default: everything.
struct AAMask {
    long long lo1 = 0, hi1 = 0x7fffffffffffffffLL, lo2 = 0, hi2 = 0;
};

struct ElasticLaunch;  // fwd

// ---- launchers (elastic_kernels.hip) ---------------------------------------------------
enum LocalMode { LZ_NORMAL = 0, LZ_REDO = 1, LZ_INIT = 2 };

// Work queue of the hyperelastic local step: a device counter, the resident grid on the solver's
// device and the refill threshold (computed once per solver, make_local_queue)
struct LocalQueue {
    int* counter = nullptr;
    int resident = 0, refill = 60, margin = 0;
    bool ahead = false;  // AA_LQ_AHEAD=1: k_local_z_hqa (one-element lookahead per lane)
    bool split = false;  // AA_LQ_SPLIT=1: k_local_z_hq2 (each element's L-BFGS over a lane pair)
    bool fused = false;  // AA_LQ_FUSED=1: k_local_z_hqf (the refill's loads regrouped; groups without pins)
    bool chunk = false;  // AA_LQ_CHUNK=1: k_local_z_hq<4, REGS, 1> (64-element chunks claimed one ahead)
    int hist = 0;        // LqHistory: where the L-BFGS history lives (AA_LQ_LDS=1: y half in LDS)
    size_t lds_bytes = 0;
    // optional diagnostics (AA_LQ_STATS=1): [0..100] elements by L-BFGS iterations (0 = the start
    // point passed the gradient test), [101] trips, [102] refills, [103] waves; summed over launches
    unsigned long long* stats = nullptr;
};
constexpr int kLqStats = 104;
constexpr size_t kLqLdsBytes = sizeof(double) * 6 * 10 * kBlock;   // HyperLbfgsLds ring, one block
enum LqHistory { LQ_HIST_REGS = 0, LQ_HIST_YLDS = 1 };
LocalQueue make_local_queue(int device, int* counter);
// z = prox(P x + u/w); prim partials; optional y = w(w z + c - u). gate: !done (and reject for REDO)
// queue given: hyperelastic groups without partials run as a persistent work queue
void launch_local_z(const GroupDev& g, const double* xfull, const double* u, double* z, double* y, int nf,
                    int variant, int mode, Ctrl* ctrl, double* red, int red_off, hipStream_t s,
                    const LocalQueue* queue = nullptr);
// r = w(P x - z); prim2/dual2 partials; u += r (UX variant update_u fused with the residual)
void launch_resid_update_u(const GroupDev& g, const double* xfull, const double* xlast, const double* z, double* u,
                           int nf, Ctrl* ctrl, double* red_a, double* red_b, int red_off, hipStream_t s);
// Z variant: u += w(Px - z) [mode 0] or u = grad E(z)/w [mode 1]; then y = w(w z + c - u). gate !done (+reject if redo)
void launch_u_and_y(const GroupDev& g, const double* xfull, const double* z, double* u, double* y, int nf, int mode,
                    int redo, Ctrl* ctrl, hipStream_t s);
// prim2 partials of |w(Px - z)|^2 and optionally dual2 partials of |w(z - zref)|^2. gate !done (+reject if redo)
void launch_prim_z(const GroupDev& g, const double* xfull, const double* z, const double* zref, int nf, int redo,
                   Ctrl* ctrl, double* red_a, double* red_b, int red_off, hipStream_t s);
// b = Mxbar + pdt2 * (D^T rows) . y ; optionally xlast = xsrc (free part) in the same pass
// red_final: UX "prim final" fused in block 0 (prim recomputed after a reject; prev_prim = prim)
void launch_rhs(int nf, const int* ptr, const int* row, const double* val, const double* y, const double* Mxbar,
                double pdt2, double* b, Ctrl* ctrl, int gate_reject, hipStream_t s,
                const double* xsrc = nullptr, double* xlast = nullptr, const double* red_final = nullptr,
                int nb_final = 0);
// UX reject test + restore fused (replaces CTL_PRIM_CHECK + launch_restore_ux)
// Z variant: k_control's CTL_PRIM_CHECK_Z and the reject branch's three restores in one launch
void launch_check_restore_z(Ctrl* ctrl, const double* red, int nb, int accel, double* u, double* x, double* z,
                            const double* du, const double* dx, const double* dz, long long nz, long long nx,
                            hipStream_t s);
void launch_check_restore_ux(Ctrl* ctrl, const double* red, int nb, int accel, double* u, double* x, double* cur,
                             const double* du, const double* dx, long long nz, long long nx, hipStream_t s);
// UX reject: u = du, x = dx, cur = (du, dx) (gate: reject)
void launch_restore_ux(double* u, double* x, double* cur, const double* du, const double* dx, long long nz,
                       long long nx, const Ctrl* ctrl, hipStream_t s);
// control steps
enum CtlOp { CTL_PRIM_CHECK = 0, CTL_PRIM_FINAL = 1, CTL_COMB_UX = 2, CTL_PRIM_CHECK_Z = 3, CTL_PRIM_FINAL_Z = 4,
             CTL_COMB_Z = 5, CTL_COMB_ZP = 6 };
void launch_control(int op, Ctrl* ctrl, const double* red_a, const double* red_b, int nblocks, int accel,
                    double* hist_prim, double* hist_comb, int* hist_rej, hipStream_t s);
// concurrent combined-residual pass: side = *ctrl (fork); records merged back, a break taken
// as done = 2 with x = dx and the later iterations' reject count / failure flag restored, once (join)
void launch_ctrl_fork(const Ctrl* ctrl, Ctrl* side, hipStream_t s);
void launch_ctrl_join(Ctrl* ctrl, const Ctrl* side, double* x, const double* dx, long long n, hipStream_t s);
// dst = src (gate: !done, and reject if gate_reject)
void launch_copy(double* dst, const double* src, long long n, const Ctrl* ctrl, int gate_reject, hipStream_t s);
// GB/s of a 16-B/lane streaming read of `bytes` (the measured HBM read ceiling; bench.py)
double bench_stream_read(long long bytes, int reps, hipStream_t s);
// predictor: v_y += dt g (free); xbar = x + dt v; Mxbar = m xbar; xfull = xbar (free) / xpin (pinned)
void launch_predict(int n, int nf, double* xstate, double* vstate, const double* mass, double dt, double gravity,
                    double* xbar, double* Mxbar, double* xfull, hipStream_t s);
// z = P xbar (initial z = W^-1 (D xbar - C))
void launch_init_z(const GroupDev& g, const double* xfull, double* z, hipStream_t s);
// new state: x = xsrc (free) / xfull (pinned); v = (x_new - x_old)/dt
void launch_finalize(int n, int nf, const double* xsrc, const double* xfull, double* xstate, double* vstate, double dt,
                     hipStream_t s);
// WindForce::project (ExplicitForce.cpp:47-104) on the step's start state: v += dt 0.33 f_n per
// triangle vertex, triangles in the given order. lvl_ptr[l]..lvl_ptr[l+1] index tri_ord: a level's
// triangles share no vertex with each other, and every earlier triangle sharing a vertex with one
// of them sits in an earlier level -- so one workgroup sweeping the levels reproduces the
// sequential loop (the reference's single-thread order) exactly.
void launch_wind(const int* tris3, const int* tri_ord, const int* lvl_ptr, int nlvl, const double* x, double* v,
                 double dir0, double dir1, double dir2, double dt, hipStream_t s);

// ---- Anderson acceleration (device-side AndersonAcceleration::compute_impl) -----------
// G: the fixed-point map output (2 segments); cur: the stored current iterate (current_u_);
// dF/dG: history (column-major, eff x m / dim x m); copy_to: optional copy of G (the
// "default" iterate kept for the reject test); out: where the accelerated iterate goes.
// m: window (selects the register-resident accumulator bucket 8/12/16/32, aa_window_bucket;
// the block partials hold 2 + 2 aa_window_bucket(m) values).
int aa_window_bucket(int m);
int aa_reduce_blocks(long long dim);
// comb_a/comb_b given: the UX combined residual, break test and record are fused in front
void launch_aa_reduce(Seg2 G, const double* cur, long long eff, double* dF, double* dG, Ctrl* ctrl, double* red,
                      int nblocks, Seg2 copy_to, int m, hipStream_t s, const double* comb_a = nullptr,
                      const double* comb_b = nullptr, int comb_nb = 0, double* hist_prim = nullptr,
                      double* hist_comb = nullptr, int* hist_rej = nullptr, AAMask mask = AAMask());
void launch_aa_solve(Ctrl* ctrl, const double* red, int nblocks, int m, hipStream_t s);
void launch_aa_mix(Seg2 G, double* cur, long long eff, double* dF, double* dG, Ctrl* ctrl, Seg2 out, int m,
                   hipStream_t s);

// ---- element-level test hooks (aa_test_* in the C ABI; tests only)
void launch_test_prox(int op, const double* prm4, const double* in, int n, double* out, int* iters, hipStream_t s);
void launch_test_cod(int n, const double* M, const double* b, double* x, hipStream_t s);

}  // namespace aa
