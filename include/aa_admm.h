/* aa_admm.h -- C ABI of the MI355X-native Anderson-accelerated ADMM hot path.
 *
 * This is the drop-in boundary for the reference's admm-elastic plugin API
 * (bldeng/AA-ADMM, admm_anderson_{xzu,hard_zxu}/src). Plain pointers and sizes only; no
 * torch or HIP types. Every call returns AA_OK (0) or a negative status; the message of the
 * last failure on the calling thread is available from aa_last_error(). The reference
 * throws std::runtime_error / returns bool at the same points -- the C++ facade in
 * include/aa_admm.hpp re-raises these codes as std::runtime_error.
 *
 * Arrays are fp64 (the reference computes in double throughout, Types.h) and int32 indices
 * (Eigen's default StorageIndex). Node arrays are xyz-interleaved ("scaled x3" as in
 * Solver::m_x / m_masses, admm_anderson_hard_zxu/src/Solver.hpp:84-87).
 */
#ifndef AA_ADMM_H
#define AA_ADMM_H
#ifdef __cplusplus
extern "C" {
#endif

#define AA_OK 0
#define AA_ERR_ARG -1       /* bad input (reference: "Bad input" runtime_error)            */
#define AA_ERR_STATE -2     /* call order violated (e.g. step before initialize)           */
#define AA_ERR_DEVICE -3    /* HIP runtime failure                                         */
#define AA_ERR_NUMERIC -4   /* inverted element, weight <= 0, matrix not SPD              */

typedef struct aa_ctx_s* aa_ctx;          /* one GPU + one HIP stream                    */
typedef struct aa_elastic_s* aa_elastic;  /* one admm::Solver instance                   */

/* Element materials (binding::MeshFlags, samples/utils/AddMeshes.hpp:45-50). */
#define AA_LINEAR 0      /* TetEnergyTerm (corotated-linear via 3x3 SVD) / TriEnergyTerm */
#define AA_NEOHOOKEAN 1  /* NeoHookeanTet (9-D L-BFGS prox)                              */
#define AA_STVK 2        /* StVKTet       (9-D L-BFGS prox)                              */

/* Solver variants: the two reference solver copies. */
#define AA_VARIANT_Z 0   /* admm_anderson_xzu: Anderson on z (Solver.cpp:34-263)            */
#define AA_VARIANT_UX 1  /* admm_anderson_hard_zxu: Anderson on (u,x) (Solver.cpp:34-234)    */

/* Lame (EnergyTerm.hpp:35-61): mu, lambda and strain limits (tris only). */
typedef struct {
    double mu, lambda;
    double limit_min, limit_max;   /* defaults -100 / 100 = no limiting */
} aa_lame;

/* Solver::Settings (Solver.hpp:45-67) + variant selection. */
typedef struct {
    double timestep_s;      /* -dt   default 1/30                                  */
    int verbose;            /* -v                                                  */
    int admm_iters;         /* -it   default 500                                   */
    double gravity;         /* -g    default -9.8 (applied to y of free nodes)     */
    double constraint_w;    /* -ck   (unused by the LDLT path, kept for parity)    */
    int anderson_m;         /* -am   window (>0 with acceleration)                 */
    double penalty;         /* -ap   (UX variant; the Z variant uses 1)            */
    int acceleration_type;  /* 0 = NOACC, 1 = ANDERSON  (-a)                       */
    int variant;            /* AA_VARIANT_Z / AA_VARIANT_UX                        */
    double eps_rel;         /* run-to-epsilon (new, not in the reference): > 0 ends a
                               step once comb <= eps_rel * comb of its first iteration;
                               0 = the reference's loop (admm_iters, comb < 1e-20 break) */
} aa_settings;

/* RuntimeData (Solver.hpp:69-80) plus device-side counters. */
typedef struct {
    double global_ms, local_ms, acceleration_ms, initialization_ms;  /* host wall, per step */
    double step_ms;          /* wall time of the last step() (device-synchronised)  */
    double setup_ms;         /* initialize(): assembly + ordering + factorisation   */
    int iterations;          /* ADMM iterations executed in the last step (incl. a  
                                breaking one; history() holds the recorded rows)     */
    int rejects;             /* Anderson rejections in the last step                */
    long long nnz_factor;    /* scalar nnz(L) of the global factor                  */
    int n_free, n_pinned, n_elements, z_dim;
} aa_runtime;

const char* aa_last_error(void);
const char* aa_version(void);

/* ---- context --------------------------------------------------------------------- */
int aa_ctx_create(int device_id, aa_ctx* out);
int aa_ctx_destroy(aa_ctx ctx);
int aa_ctx_synchronize(aa_ctx ctx);
/* Measurement hook (no reference counterpart): GB/s of a 16-B-per-lane streaming read of `bytes`
 * on the context's stream -- the measured HBM read ceiling bench.py reports beside the spec. */
int aa_ctx_bench_read(aa_ctx ctx, long long bytes, double* gbps);
/* One-time library load, made explicit (no reference counterpart): the first rocBLAS / rocSOLVER
 * calls of a process load their code objects (seconds on a fresh box with a cold page cache),
 * which would otherwise land inside the first aa_elastic_initialize / aa_geom_setup that factors
 * a front on the GPU (SolverCommon / Solver.cpp:414-482 factor step). Runs the dense-front
 * backend once on a synthetic front of the smallest GPU order; *ms = its wall time (0 when
 * already warm or AA_DENSE_GPU=0). */
int aa_ctx_warm_dense(aa_ctx ctx, double* ms);

/* ---- admm::Solver ------------------------------------------------------------------ */
int aa_lame_from_young(double youngs, double poisson, aa_lame* out);    /* Lame(k, v)        */
int aa_settings_default(aa_settings* out);                               /* Settings()        */

int aa_elastic_create(aa_ctx ctx, aa_elastic* out);                      /* Solver()          */
int aa_elastic_destroy(aa_elastic h);
/* Solver::add_nodes(x, m, n): x and m are "scaled x3"; returns the node count in *total. */
int aa_elastic_add_nodes(aa_elastic h, const double* x3, const double* m3, int n_verts, int* total);
/* create_tets_from_mesh<IN_SCALAR,TYPE>(energyterms, verts, inds, n, lame, vertex_offset)
 * (TetEnergyTerm.hpp:36-51): rest shape from verts3[inds], node ids inds + vertex_offset. */
int aa_elastic_add_tets(aa_elastic h, const double* verts3, const int* tets4, int n_tets, int material,
                        const aa_lame* lame, int vertex_offset);
/* create_tris_from_mesh<IN_SCALAR,TriEnergyTerm> (TriEnergyTerm.hpp:33-47). */
int aa_elastic_add_tris(aa_elastic h, const double* verts3, const int* tris3, int n_tris, const aa_lame* lame,
                        int vertex_offset);
/* Solver::set_pins(inds, points): points3 == NULL pins in place (Solver.cpp:280-315). */
int aa_elastic_set_pins(aa_elastic h, const int* inds, const double* points3, int n_pins);

/* Passive obstacles (admm_anderson_hard_zxu/src/PassiveObject.hpp:32-136), Solver::add_obstacle
 * (Solver.cpp:346-348). params: FLOOR {y}; SLIDE_FLOOR {cx,cy,cz, nx,ny,nz} (the normal is
 * normalised, as the SlideFloor constructor does); SPHERE / PLANE_HALF_SPHERE / CYLINDER
 * {cx,cy,cz, r} (the cylinder's axis is z). The collision terms test every obstacle in insertion
 * order each iteration; obstacles may be added after initialize. The z-AA variant rejects
 * obstacles at initialize (admm_anderson_xzu/src/Solver.cpp:485-489). The BVH mesh obstacle
 * (PassiveMesh) is not provided. */
#define AA_OBS_FLOOR 0
#define AA_OBS_SLIDE_FLOOR 1
#define AA_OBS_SPHERE 2
#define AA_OBS_PLANE_HALF_SPHERE 3
#define AA_OBS_CYLINDER 4
int aa_elastic_add_obstacle(aa_elastic h, int type, const double* params);
/* Solver::set_collisions(inds, points) (admm_anderson_hard_zxu/src/Solver.cpp:318-344): one
 * Collision energy term (CollisionEnergyTerm.hpp:41-117: identity reduction, weight
 * sqrt(2 k(soft rubber)), prox = closest obstacle surface point when inside one) per listed node,
 * created at initialize after the other terms in node order. The reference's points are never read
 * by the prox and are not taken here. (u,x) variant only; after initialize it changes nothing. */
int aa_elastic_set_collisions(aa_elastic h, const int* inds, int n);
/* WindForce (ExplicitForce.hpp:39-47, ExplicitForce.cpp:47-104) pushed to Solver::ext_forces:
 * every step, before gravity, v += 0.33 dt f_n on the vertices of each listed triangle (the
 * Wejchert-Haumann normal force of the relative velocity v - dir), triangles in the given order
 * (the reference's loop run on one thread). *id names it for aa_elastic_set_wind. */
int aa_elastic_add_wind(aa_elastic h, const int* tris3, int n_tris, const double dir3[3], int* id);
int aa_elastic_set_wind(aa_elastic h, int id, const double dir3[3]);   /* WindForce::direction */
int aa_elastic_initialize(aa_elastic h, const aa_settings* settings);    /* Solver::initialize */
int aa_elastic_step(aa_elastic h);                                       /* Solver::step       */
int aa_elastic_num_nodes(aa_elastic h, int* n);
int aa_elastic_get_x(aa_elastic h, double* x3);                          /* Solver::m_x        */
int aa_elastic_get_v(aa_elastic h, double* v3);                          /* Solver::m_v        */
int aa_elastic_set_v(aa_elastic h, const double* v3);
int aa_elastic_set_x(aa_elastic h, const double* x3);                    /* Solver::m_x = x   */
/* Per-iteration (prim, comb, reject) of the last step -- the rows Solver::save() writes
 * (Solver.hpp:130-155). Returns the count in *n (<= cap copied). */
int aa_elastic_get_history(aa_elastic h, double* prim, double* comb, int* reject, int cap, int* n);
/* Change Settings::admm_iters / eps_rel of later steps without re-initialising (no refactor). */
int aa_elastic_set_iterations(aa_elastic h, int admm_iters, double eps_rel);
/* Device-clock time (ms) from the start of the last step() to the end of each recorded
 * iteration (the reference's per-iteration elapsed times; time-to-epsilon). */
int aa_elastic_get_times(aa_elastic h, double* time_ms, int cap, int* n);
int aa_elastic_runtime(aa_elastic h, aa_runtime* out);                   /* runtime_data()    */

/* ---- multi-GPU: mesh partitioned over the GPUs of one node -----------
 * The reference is one OpenMP process (no MPI/NCCL); this is new surface. One process per GPU;
 * every rank builds the SAME scene through the calls above, attaches a communicator, then
 * initialize() partitions the free nodes by nested dissection into `size` parts (any count
 * >= 1: an odd count is split floor/ceil by vertex count at each forced bisection) plus the
 * shared separator rows, and each rank keeps the elements of its part. step()
 * runs the identical reference iteration on all ranks (all-reduced residuals, Anderson dot
 * products and separator rows of the global solve); afterwards every rank holds the full
 * x and v. */
typedef struct aa_comm_s* aa_comm;
/* Host transport callback: in-place SUM of n doubles over all ranks; return 0 on success. */
typedef int (*aa_host_allreduce_fn)(double* buf, long long n, void* user);
/* Which ROCm runtime this process is bound to (no reference counterpart): "name=path\n" for the
 * objects defining hipMalloc, hsa_init, rocblas_create_handle, rocsolver_dpotrf and ncclAllReduce
 * (librccl is loaded from the HIP runtime's directory first). Needs no GPU. A process that loaded
 * another ROCm build's libamdhip64 before this library (e.g. a framework's bundled runtime) shows
 * it here; the multi-rank launchers check it. Copies at most cap-1 bytes; *len = full length. */
int aa_runtime_libraries(char* buf, long long cap, long long* len);
/* ncclGetUniqueId: called on rank 0, the 128 bytes are broadcast by the caller. */
int aa_comm_unique_id(unsigned char id[128]);
/* RCCL communicator over xGMI on ctx's GPU (ncclCommInitRank; collective over all ranks). */
int aa_comm_create_rccl(aa_ctx ctx, const unsigned char id[128], int rank, int size, aa_comm* out);
/* Host-staged transport through a caller callback (e.g. torch.distributed/gloo); lets several
 * ranks share one GPU (tests). Never captured into a hipGraph. */
int aa_comm_create_host(aa_host_allreduce_fn fn, void* user, int rank, int size, aa_comm* out);
/* Timing rehearsal (no reference counterpart): rank `rank` of a `size`-way partition alone on
 * its GPU -- device all-reduces keep the local values, host all-reduces multiply by size. The
 * results are NOT a solution; it times one rank's share of a multi-GPU step (bench.py --rehearse). */
int aa_comm_create_solo(int rank, int size, aa_comm* out);
int aa_comm_destroy(aa_comm c);
int aa_comm_info(aa_comm c, int* rank, int* size);
/* In-place SUM of a host array over the ranks (blocking; setup-time agreements, tests). */
int aa_comm_allreduce_host(aa_comm c, double* buf, long long n);
/* Attach before aa_elastic_initialize; the communicator must outlive the solver. */
int aa_elastic_set_comm(aa_elastic h, aa_comm c);

/* ---- benchmarking hooks (device-resident inputs, no host traffic) ------------------ */
/* Enqueue `iters` iterations of the ADMM loop of the current time step without the
 * per-step prologue/epilogue; used by bench.py to time the hot loop alone. */
int aa_elastic_bench_iterations(aa_elastic h, int iters, double* ms);
/* Average device time (ms) per launch of the named kernel class over the last bench call,
 * measured with HIP events on the solver's stream; and its algorithmic bytes per launch. */
int aa_elastic_kernel_stats(aa_elastic h, const char* name, double* avg_ms, double* bytes, int* launches);
/* Diagnostics of the hyperelastic local step's work queue, summed over its launches since the
 * last reset (enabled by AA_LQ_STATS=1 in the environment at aa_elastic_initialize; zeros
 * otherwise): out[0..100] elements by L-BFGS iteration count (mcloptlib LBFGS.hpp:205-305 outer
 * iterations; 0 = the start point passed the gradient test), out[101] trips (one L-BFGS
 * iteration for every busy lane of a wave), out[102] queue refills, out[103] waves. Writes
 * min(cap, 104) counters into *count. */
int aa_elastic_local_stats(aa_elastic h, long long* out, int cap, int reset, int* count);
/* Wall-clock phases of the last aa_elastic_initialize (Solver::initialize, Solver.cpp:373-498):
 * names '\n'-separated into names[0..names_cap) (NUL-terminated), milliseconds into
 * ms[0..cap); *count = number of phases. */
int aa_elastic_setup_phases(aa_elastic h, char* names, int names_cap, double* ms, int cap, int* count);

/* ==== Geometry: ALMGeometrySolver<3> + Constraint<3> (bldeng/AA-ADMM Geometry/) ============= */
typedef struct aa_geom_s* aa_geom;        /* one ALMGeometrySolver<3> instance             */

/* Constraint types (Geometry/Constraint.h). Index count k per constraint and the per-constraint
 * parameters each type takes (params is [count][P], row-major):
 *   AA_CON_PLANE        PlaneConstraint(idI, w)                     k >= 3    P = 0  (:396-414)
 *   AA_CON_ANGLE        AngleConstraint<3>(tip, s1, s2, w, min, max) k = 3     P = 2  (:220-296)
 *   AA_CON_EDGE         EdgeLengthConstraint<3>(i1, i2, w, length)   k = 2     P = 1  (:194-218)
 *   AA_CON_CLOSENESS    ClosenessConstraint<3>(i, w, target)         k = 1     P = 3  (:299-326;
 *                       its projection is the identity in the reference, kept as such)
 *   AA_CON_POINT_TO_REF PointToRefSurfaceConstraint(i, w, aabb)      k = 1     P = 1 = surface id (:328-349)
 *   AA_CON_REF_SURFACE  ReferenceSurfceConstraint(n, w, V, F): one   k = 1     P = 1 = surface id (:351-394)
 *                       constraint over points 0..count-1 (idx may be NULL)                    */
#define AA_CON_PLANE 0
#define AA_CON_ANGLE 1
#define AA_CON_EDGE 2
#define AA_CON_CLOSENESS 3
#define AA_CON_POINT_TO_REF 4
#define AA_CON_REF_SURFACE 5

/* SPDSolverType (Geometry/SolverCommon.h:34-38); both factorisations are a Cholesky here. */
#define AA_SPD_LDLT 0
#define AA_SPD_LLT 1

typedef struct {
    double setup_ms;         /* setup_ADMM: assembly of the global matrix and rhs_fixed       */
    double factor_ms;        /* nested-dissection ordering + factorisation (first solve)     */
    double solve_ms;         /* wall time of the last solve_ADMM (device-synchronised)       */
    int iterations;          /* x-updates of the last solve (accepted + rejected)            */
    int accepted;            /* accepted iterations (= function_values_.size())              */
    int rejects;             /* Anderson rejections                                          */
    int n_points;
    long long nnz_factor;    /* scalar nnz(L) of the global factor                           */
    long long hard_cols, soft_cols, n_constraints;
} aa_geom_runtime;

int aa_geom_create(aa_ctx ctx, aa_geom* out);                                  /* ALMGeometrySolver() */
/* Solver kinds: AA_GEOM_ALM = ALMGeometrySolver<3> (Geometry/ALMGeometrySolver.h);
 * AA_GEOM_PLAIN = GeometrySolver<3> (Geometry/GeometrySolver.h:85-263): every constraint row
 * unweighted and scaled by the penalty, u on every column, soft constraints projected with
 * Constraint::project_and_combine (Constraint.h:118-130), residual |Dx - z|, Anderson on (u, x)
 * with u the effective part and `replace` (no history reset) when the residual increases;
 * get_solution() = current_x_. Same calls otherwise.                                         */
#define AA_GEOM_ALM 0
#define AA_GEOM_PLAIN 1
int aa_geom_create_kind(aa_ctx ctx, int kind, aa_geom* out);
int aa_geom_destroy(aa_geom h);                                                /* ~ALMGeometrySolver  */
/* Reference surface (TriMeshAABB / igl::AABB over V (nv x 3), F (nf x 3)); returns its id. */
int aa_geom_add_ref_surface(aa_geom h, const double* V3, int nv, const int* F3, int nf, int* id);
/* add_hard_constraint (hard = 1) / add_soft_constraint (hard = 0) of `count` constraints of one
 * type: idx is [count][k] point ids, weight the constructor weight, params [count][P]. */
int aa_geom_add_constraints(aa_geom h, int hard, int type, const int* idx, int k, int count, double weight,
                            const double* params);
/* add_laplacian / add_uniform_laplacian (coefs as given; ref_points3 == NULL) and
 * add_relative_laplacian / add_relative_uniform_laplacian (ref_points3 = 3 x n points). */
int aa_geom_add_laplacian(aa_geom h, const int* idx, const double* coefs, int k, double weight,
                          const double* ref_points3);
int aa_geom_add_closeness(aa_geom h, int idx, double weight, const double* target3);   /* add_closeness */
/* Batched forms for bindings whose per-call overhead dominates (one call per point is ~10 us from
 * Python): the same rows in the same order as n_rows aa_geom_add_laplacian calls (row r: indices
 * idx[row_ptr[r] .. row_ptr[r+1]), coefficients coefs[same range], weight weights[r]; relative[r]
 * != 0 -- relative may be NULL -- passes ref_points3 as add_relative_laplacian does), and as n
 * aa_geom_add_closeness calls (targets3: n x 3). Reference: the per-point loops of
 * Geometry/PlanarityOpt.cpp / WireMeshOpt.cpp over LinearRegularization.h:91-117. */
int aa_geom_add_laplacians(aa_geom h, int n_rows, const int* row_ptr, const int* idx, const double* coefs,
                           const double* weights, const int* relative, const double* ref_points3);
int aa_geom_add_closenesses(aa_geom h, int n, const int* idx, const double* weights, const double* targets3);
int aa_geom_setup(aa_geom h, int n_points, double penalty, int spd_solver_type);       /* setup_ADMM    */
/* solve_ADMM(init_x (3 x n), rel_residual_eps, max_iter, Anderson_m): max_iter accepted
 * iterations; Anderson_m = 0 runs plain ADMM. */
int aa_geom_solve(aa_geom h, const double* init_x3, double rel_residual_eps, int max_iter, int anderson_m);
int aa_geom_get_solution(aa_geom h, double* x3);                               /* get_solution()      */
/* Run-to-epsilon for later solves (new surface; the reference computes residual_eps at
 * ALMGeometrySolver.h:172 but its stopping test is commented out at :258-260). stop_at_eps = 1
 * ends the loop after the first accepted iteration whose combined residual is below
 * rel_residual_eps^2 * hard_cols^2 * 2; eps_rel > 0 also ends it once comb <= eps_rel * comb of
 * the first accepted iteration. (0, 0) = the reference loop (max_iter accepted iterations).
 * ALMGeometrySolver only. */
int aa_geom_set_stop(aa_geom h, int stop_at_eps, double eps_rel);
/* function_values_ (combined residual per accepted iteration) and elapsed_time_ (s since the
 * loop started, device clock). Returns the count in *n (<= cap copied). */
int aa_geom_get_history(aa_geom h, double* comb, double* time_s, int cap, int* n);
int aa_geom_runtime_info(aa_geom h, aa_geom_runtime* out);
/* closest points on a reference surface (PointToRefSurfaceConstraint's projection) */
int aa_geom_closest_points(aa_geom h, int surface, const double* p3, int n, double* out3);
int aa_geom_bench_iterations(aa_geom h, int iters, double* ms);
int aa_geom_kernel_stats(aa_geom h, const char* name, double* avg_ms, double* bytes, int* launches);
/* Multi-GPU (see aa_comm above): attach before the first aa_geom_solve; every rank adds the same
 * constraints; the first solve partitions the points (nested dissection of the global matrix on
 * the initial positions) and each rank projects the constraints of its part. */
int aa_geom_set_comm(aa_geom h, aa_comm c);

/* ---- element-level test hooks (parity tests only; not part of the reference API) ----------
 * The device functions of the local step / Anderson solve / projections applied to host arrays
 * (uploaded, one device thread per element), so tests can pin them to the reference's element
 * tables (tests/golden/elements.npz, geom_elements.npz) directly:
 *   aa_test_prox: op 0 TetEnergyTerm::prox (in/out 9 per tet, TetEnergyTerm.cpp:74-96),
 *     1 NeoHookeanTet / 2 StVKTet prox (L-BFGS, TetEnergyTerm.cpp:151-162; prm4 = E, nu, h with
 *     vol = h^3/6; iters = L-BFGS iterations, -1 on a line-search failure), 3 / 4 TriEnergyTerm
 *     prox of the H / X solver copy (6 per tri; prm4[2..3] = limit_min, limit_max)
 *   aa_test_cod_solve: the Anderson normal-equation solve (Eigen CompleteOrthogonalDecomposition,
 *     AndersonAcceleration.h:186-188) of a k x k column-major M
 *   aa_test_geom_project: Constraint::project_impl of plane (k 3..8) / angle (k 3) / edge (k 2)
 *     on n transformed point sets (3 x cols each, column-major); prm2 = angle min, max / edge length */
int aa_test_prox(aa_ctx ctx, int op, const double* prm4, const double* in, int n, double* out, int* iters);
int aa_test_cod_solve(aa_ctx ctx, int k, const double* M, const double* b, double* theta);
int aa_test_geom_project(aa_ctx ctx, int type, int k, const double* prm2, const double* in, int n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* AA_ADMM_H */
