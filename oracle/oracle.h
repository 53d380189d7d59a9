/* ORACLE -- test infrastructure only.
 *
 * CPU restatement (plain C++, no Eigen) of the reference's admm-elastic hot path, used as
 * the checker for the HIP product path (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg). Nothing in aa-admm_amd/ links, loads or calls this library.
 *
 * Parity is pinned against outputs of the REFERENCE itself, compiled here from its own
 * sources (oracle/_ref, see oracle/Makefile) -- golden vectors under tests/golden/.
 */
#ifndef AA_ADMM_ORACLE_H
#define AA_ADMM_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int variant;     /* 0 = admm_anderson_xzu (z-AA), 1 = admm_anderson_hard_zxu ((u,x)-AA) */
    double dt, gravity, penalty;
    int iters, accel, aa_m;
} oracle_settings;

/* Runs n_steps time steps of Solver::step on the scene; returns 0 on success.
 * x3: initial node positions; rest3: rest positions of the elements (NULL = x3).
 * groups: kind (0 tet / 1 tri), material (0 linear / 1 NH / 2 StVK), E, nu, limit_min/max,
 * count and offset into idx (int32, 4 per tet / 3 per tri).
 * Per-step records are written to rec_* at [step*cap + i]; nrec[step] = count. */
int oracle_elastic_run(int n_nodes, const double* x3, const double* rest3, const double* masses,
                       int n_groups, const int* g_kind, const int* g_mat, const double* g_E, const double* g_nu,
                       const double* g_lmin, const double* g_lmax, const int* g_count, const int* g_off,
                       const int* idx, int n_pins, const int* pin_idx, const double* pin_pts,
                       const double* pin_vel, const oracle_settings* st, int n_steps, int cap,
                       int* nrec, double* rec_prim, double* rec_comb, int* rec_rej,
                       double* out_x3, double* out_v3, double* step_ms, char* err, int err_cap);

/* element-level kernels (column-major F as in Eigen::Map) */
void oracle_svd3(const double* F9, double* U9, double* S3, double* V9);
void oracle_tri_prox_h(const double* z6, double limit_min, double limit_max, double* out6);
void oracle_tri_prox_x(const double* z6, double limit_min, double limit_max, double* out6);
void oracle_tet_prox_linear(const double* z9, double* out9);
int  oracle_tet_prox_hyper(int material, double mu, double lambda, double k, double vol, const double* v9,
                           double* out9);
void oracle_cod_solve(int n, const double* M_colmajor, const double* b, double* theta);

/* Geometry ALM path (ALMGeometrySolver<3>::setup_ADMM + solve_ADMM): reads an AAGEOM01 scene
 * file, writes an AAGEOMR1 result file (formats: aa-admm_amd/geom_scenes.py). 0 on success. */
int  oracle_geom_run_file(const char* scene_path, const char* out_path, char* err, int err_cap);
/* mode 1: GeometrySolver<3> (Geometry/GeometrySolver.h) instead of ALMGeometrySolver<3> */
int  oracle_geom_run_file_mode(const char* scene_path, const char* out_path, int mode, char* err, int err_cap);
/* closest points on a triangle mesh (igl AABB::squared_distance semantics) */
void oracle_closest_point(const double* V, int nv, const int* F, int nf, const double* P, int np, double* out);
/* Constraint<3>::project_impl of one constraint on transformed points (3 x cols, column-major) */
void oracle_geom_project(int type, int k, const double* params, const double* in, double* out);

#ifdef __cplusplus
}
#endif
#endif
