// extern "C" boundary (include/aa_admm.h). Every entry point catches and maps exceptions to
// status codes; the message is kept per thread for aa_last_error().
#include <algorithm>
#include <cstring>
#include <exception>
#include <memory>
#include <string>

#include "../../include/aa_admm.h"
#include "comm.hpp"
#include "dense_gpu.hpp"
#include "elastic.hpp"
#include "geom.hpp"

struct aa_ctx_s { aa::Context c; };
struct aa_elastic_s { aa::ElasticSolver* s; aa_ctx_s* ctx; };
struct aa_geom_s { aa::GeomSolver* s; aa_ctx_s* ctx; };
struct aa_comm_s { std::unique_ptr<aa::Comm> c; };

namespace {
thread_local std::string g_err;

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return AA_OK;
    } catch (const aa::Error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return AA_ERR_DEVICE;
    } catch (const std::exception& e) {
        g_err = e.what();
        return AA_ERR_ARG;
    }
}

#define NEED(p, what) do { if (!(p)) throw aa::Error(AA_ERR_ARG, what); } while (0)
}  // namespace

extern "C" {

const char* aa_last_error(void) { return g_err.c_str(); }
const char* aa_version(void) { return "aa_admm 0.1 (gfx950)"; }

int aa_ctx_create(int device_id, aa_ctx* out) {
    return guarded([&] {
        NEED(out, "aa_ctx_create: null out");
        int n = 0;
        AA_HIP(hipGetDeviceCount(&n));
        if (device_id < 0 || device_id >= n) throw aa::Error(AA_ERR_ARG, "aa_ctx_create: no such device");
        AA_HIP(hipSetDevice(device_id));
        auto* c = new aa_ctx_s;
        c->c.device = device_id;
        AA_HIP(hipStreamCreateWithFlags(&c->c.stream, hipStreamNonBlocking));
        *out = c;
    });
}

int aa_ctx_destroy(aa_ctx ctx) {
    return guarded([&] {
        if (!ctx) return;
        (void)hipStreamSynchronize(ctx->c.stream);
        (void)hipStreamDestroy(ctx->c.stream);
        delete ctx;
    });
}

int aa_ctx_synchronize(aa_ctx ctx) {
    return guarded([&] { NEED(ctx, "null ctx"); AA_HIP(hipStreamSynchronize(ctx->c.stream)); });
}

int aa_ctx_bench_read(aa_ctx ctx, long long bytes, double* gbps) {
    return guarded([&] {
        NEED(ctx && gbps && bytes >= 16, "aa_ctx_bench_read: bad argument");
        AA_HIP(hipSetDevice(ctx->c.device));
        *gbps = aa::bench_stream_read(bytes, 10, ctx->c.stream);
    });
}

int aa_ctx_warm_dense(aa_ctx ctx, double* ms) {
    return guarded([&] {
        NEED(ctx && ms, "aa_ctx_warm_dense: bad argument");
        AA_HIP(hipSetDevice(ctx->c.device));
        *ms = aa::warm_gpu_front_backend(ctx->c.stream);
    });
}

int aa_lame_from_young(double k, double v, aa_lame* out) {
    return guarded([&] {
        NEED(out, "null out");
        out->mu = k / (2.0 * (1.0 + v));
        out->lambda = k * v / ((1.0 + v) * (1.0 - 2.0 * v));
        out->limit_min = -100.0;
        out->limit_max = 100.0;
    });
}

int aa_settings_default(aa_settings* s) {
    return guarded([&] {
        NEED(s, "null out");
        s->timestep_s = 1.0 / 30.0;
        s->verbose = 1;
        s->admm_iters = 500;
        s->gravity = -9.8;
        s->constraint_w = -1;
        s->anderson_m = 2;
        s->penalty = 1.0;
        s->acceleration_type = 0;
        s->variant = AA_VARIANT_UX;
        s->eps_rel = 0.0;
    });
}

int aa_elastic_create(aa_ctx ctx, aa_elastic* out) {
    return guarded([&] {
        NEED(ctx && out, "aa_elastic_create: null argument");
        AA_HIP(hipSetDevice(ctx->c.device));
        auto* h = new aa_elastic_s;
        h->ctx = ctx;
        h->s = new aa::ElasticSolver(&ctx->c);
        *out = h;
    });
}

int aa_elastic_destroy(aa_elastic h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->ctx->c.device);
        delete h->s;
        delete h;
    });
}

int aa_elastic_add_nodes(aa_elastic h, const double* x3, const double* m3, int n, int* total) {
    return guarded([&] {
        NEED(h, "null handle");
        int t = h->s->add_nodes(x3, m3, n);
        if (total) *total = t;
    });
}

int aa_elastic_add_tets(aa_elastic h, const double* verts3, const int* tets4, int n, int material, const aa_lame* lame,
                        int vertex_offset) {
    return guarded([&] {
        NEED(h && lame, "null argument");
        h->s->add_elements(0, material, verts3, tets4, n, *lame, vertex_offset);
    });
}

int aa_elastic_add_tris(aa_elastic h, const double* verts3, const int* tris3, int n, const aa_lame* lame,
                        int vertex_offset) {
    return guarded([&] {
        NEED(h && lame, "null argument");
        h->s->add_elements(1, AA_LINEAR, verts3, tris3, n, *lame, vertex_offset);
    });
}

int aa_elastic_set_pins(aa_elastic h, const int* inds, const double* pts3, int n) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_pins(inds, pts3, n); });
}

int aa_elastic_add_obstacle(aa_elastic h, int type, const double* params) {
    return guarded([&] {
        NEED(h, "null handle");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        h->s->add_obstacle(type, params);
    });
}

int aa_elastic_set_collisions(aa_elastic h, const int* inds, int n) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_collisions(inds, n); });
}

int aa_elastic_add_wind(aa_elastic h, const int* tris3, int n_tris, const double dir3[3], int* id) {
    return guarded([&] {
        NEED(h, "null handle");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        const int k = h->s->add_wind(tris3, n_tris, dir3);
        if (id) *id = k;
    });
}

int aa_elastic_set_wind(aa_elastic h, int id, const double dir3[3]) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_wind(id, dir3); });
}

int aa_elastic_initialize(aa_elastic h, const aa_settings* s) {
    return guarded([&] {
        NEED(h && s, "null argument");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        h->s->initialize(*s);
    });
}

int aa_elastic_step(aa_elastic h) {
    return guarded([&] {
        NEED(h, "null handle");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        h->s->step();
    });
}

int aa_elastic_num_nodes(aa_elastic h, int* n) {
    return guarded([&] { NEED(h && n, "null argument"); *n = h->s->num_nodes(); });
}

int aa_elastic_get_x(aa_elastic h, double* x3) {
    return guarded([&] { NEED(h && x3, "null argument"); h->s->get_x(x3); });
}

int aa_elastic_get_v(aa_elastic h, double* v3) {
    return guarded([&] { NEED(h && v3, "null argument"); h->s->get_v(v3); });
}

int aa_elastic_set_v(aa_elastic h, const double* v3) {
    return guarded([&] { NEED(h && v3, "null argument"); h->s->set_v(v3); });
}

int aa_elastic_set_x(aa_elastic h, const double* x3) {
    return guarded([&] { NEED(h && x3, "null argument"); h->s->set_x(x3); });
}

int aa_elastic_get_history(aa_elastic h, double* prim, double* comb, int* reject, int cap, int* n) {
    return guarded([&] {
        NEED(h, "null handle");
        int k = h->s->history(prim, comb, reject, cap);
        if (n) *n = k;
    });
}

int aa_elastic_set_iterations(aa_elastic h, int admm_iters, double eps_rel) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_iterations(admm_iters, eps_rel); });
}

int aa_elastic_get_times(aa_elastic h, double* time_ms, int cap, int* n) {
    return guarded([&] {
        NEED(h, "null handle");
        int k = h->s->times(time_ms, cap);
        if (n) *n = k;
    });
}

int aa_elastic_runtime(aa_elastic h, aa_runtime* out) {
    return guarded([&] { NEED(h && out, "null argument"); *out = h->s->runtime(); });
}

int aa_runtime_libraries(char* buf, long long cap, long long* len) {
    return guarded([&] {
        std::string s = aa::runtime_libraries();
        if (len) *len = (long long)s.size();
        if (buf && cap > 0) {
            size_t k = std::min((size_t)(cap - 1), s.size());
            std::memcpy(buf, s.data(), k);
            buf[k] = 0;
        }
    });
}

int aa_comm_unique_id(unsigned char id[128]) {
    return guarded([&] { NEED(id, "null argument"); aa::rccl_unique_id(id); });
}

int aa_comm_create_rccl(aa_ctx ctx, const unsigned char id[128], int rank, int size, aa_comm* out) {
    return guarded([&] {
        NEED(ctx && id && out, "null argument");
        NEED(size >= 1 && rank >= 0 && rank < size, "aa_comm_create_rccl: bad rank/size");
        AA_HIP(hipSetDevice(ctx->c.device));
        auto* c = new aa_comm_s;
        try { c->c = aa::make_rccl_comm(id, rank, size); } catch (...) { delete c; throw; }
        *out = c;
    });
}

int aa_comm_create_host(aa_host_allreduce_fn fn, void* user, int rank, int size, aa_comm* out) {
    return guarded([&] {
        NEED(fn && out, "null argument");
        NEED(size >= 1 && rank >= 0 && rank < size, "aa_comm_create_host: bad rank/size");
        auto* c = new aa_comm_s;
        c->c = aa::make_host_comm(fn, user, rank, size);
        *out = c;
    });
}

int aa_comm_create_solo(int rank, int size, aa_comm* out) {
    return guarded([&] {
        NEED(out, "aa_comm_create_solo: null out");
        NEED(size >= 1 && rank >= 0 && rank < size, "aa_comm_create_solo: bad rank/size");
        auto* c = new aa_comm_s;
        c->c = aa::make_solo_comm(rank, size);
        *out = c;
    });
}

int aa_comm_destroy(aa_comm c) {
    return guarded([&] { delete c; });
}

int aa_comm_info(aa_comm c, int* rank, int* size) {
    return guarded([&] {
        NEED(c, "null handle");
        if (rank) *rank = c->c->rank();
        if (size) *size = c->c->size();
    });
}

int aa_comm_allreduce_host(aa_comm c, double* buf, long long n) {
    return guarded([&] {
        NEED(c && (n == 0 || buf) && n >= 0, "bad argument");
        c->c->allreduce_sum_host(buf, (size_t)n);
    });
}

int aa_elastic_set_comm(aa_elastic h, aa_comm c) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_comm(c ? c->c.get() : nullptr); });
}

int aa_geom_set_comm(aa_geom h, aa_comm c) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_comm(c ? c->c.get() : nullptr); });
}

int aa_elastic_bench_iterations(aa_elastic h, int iters, double* ms) {
    return guarded([&] {
        NEED(h && iters >= 0, "bad argument");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        double t = h->s->bench_iterations(iters);
        if (ms) *ms = t;
    });
}

int aa_elastic_kernel_stats(aa_elastic h, const char* name, double* avg_ms, double* bytes, int* launches) {
    return guarded([&] {
        NEED(h && name, "null argument");
        if (!h->s->kernel_stats(name, avg_ms, bytes, launches)) throw aa::Error(AA_ERR_ARG, std::string("no kernel class ") + name);
    });
}

int aa_elastic_local_stats(aa_elastic h, long long* out, int cap, int reset, int* count) {
    return guarded([&] {
        NEED(h && out && cap >= 0, "bad argument");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        const int n = h->s->local_stats(out, cap, reset != 0);
        if (count) *count = n;
    });
}

int aa_elastic_setup_phases(aa_elastic h, char* names, int names_cap, double* ms, int cap, int* count) {
    return guarded([&] {
        NEED(h && cap >= 0 && names_cap >= 0, "bad argument");
        const auto& ph = h->s->setup_phases();
        std::string all;
        for (size_t i = 0; i < ph.size(); ++i) {
            if (i) all += '\n';
            all += ph[i].first;
            if ((int)i < cap && ms) ms[i] = ph[i].second;
        }
        if (names && names_cap > 0) {
            const size_t k = std::min(all.size(), (size_t)names_cap - 1);
            std::memcpy(names, all.data(), k);
            names[k] = 0;
        }
        if (count) *count = (int)ph.size();
    });
}

// ---- Geometry (ALMGeometrySolver<3>) -------------------------------------------------------
int aa_geom_create(aa_ctx ctx, aa_geom* out) { return aa_geom_create_kind(ctx, AA_GEOM_ALM, out); }

int aa_geom_create_kind(aa_ctx ctx, int kind, aa_geom* out) {
    return guarded([&] {
        NEED(ctx && out, "aa_geom_create: null argument");
        NEED(kind == AA_GEOM_ALM || kind == AA_GEOM_PLAIN, "aa_geom_create_kind: unknown solver kind");
        AA_HIP(hipSetDevice(ctx->c.device));
        auto* h = new aa_geom_s;
        h->ctx = ctx;
        h->s = new aa::GeomSolver(&ctx->c, kind == AA_GEOM_PLAIN);
        *out = h;
    });
}

int aa_geom_destroy(aa_geom h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->ctx->c.device);
        delete h->s;
        delete h;
    });
}

int aa_geom_add_ref_surface(aa_geom h, const double* V3, int nv, const int* F3, int nf, int* id) {
    return guarded([&] {
        NEED(h, "null handle");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        const int i = h->s->add_ref_surface(V3, nv, F3, nf);
        if (id) *id = i;
    });
}

int aa_geom_add_constraints(aa_geom h, int hard, int type, const int* idx, int k, int count, double weight,
                            const double* params) {
    return guarded([&] { NEED(h, "null handle"); h->s->add_constraints(hard, type, idx, k, count, weight, params); });
}

int aa_geom_add_laplacian(aa_geom h, const int* idx, const double* coefs, int k, double weight, const double* ref3) {
    return guarded([&] { NEED(h, "null handle"); h->s->add_laplacian(idx, coefs, k, weight, ref3); });
}

int aa_geom_add_closeness(aa_geom h, int idx, double weight, const double* target3) {
    return guarded([&] { NEED(h, "null handle"); h->s->add_closeness(idx, weight, target3); });
}

int aa_geom_add_laplacians(aa_geom h, int n_rows, const int* row_ptr, const int* idx, const double* coefs,
                           const double* weights, const int* relative, const double* ref_points3) {
    return guarded([&] {
        NEED(h, "null handle");
        NEED(n_rows >= 0 && (n_rows == 0 || (row_ptr && idx && coefs && weights)), "bad laplacian rows");
        for (int r = 0; r < n_rows; ++r) {
            const int a = row_ptr[r], k = row_ptr[r + 1] - a;
            NEED(k > 0, "empty laplacian row");
            const bool rel = relative && relative[r];
            NEED(!rel || ref_points3, "relative laplacian row without reference points");
            h->s->add_laplacian(idx + a, coefs + a, k, weights[r], rel ? ref_points3 : nullptr);
        }
    });
}

int aa_geom_add_closenesses(aa_geom h, int n, const int* idx, const double* weights, const double* targets3) {
    return guarded([&] {
        NEED(h, "null handle");
        NEED(n >= 0 && (n == 0 || (idx && weights && targets3)), "bad closeness rows");
        for (int r = 0; r < n; ++r) h->s->add_closeness(idx[r], weights[r], targets3 + 3 * (size_t)r);
    });
}

int aa_geom_setup(aa_geom h, int n_points, double penalty, int spd_solver_type) {
    return guarded([&] { NEED(h, "null handle"); h->s->setup(n_points, penalty, spd_solver_type); });
}

int aa_geom_solve(aa_geom h, const double* init_x3, double rel_eps, int max_iter, int m) {
    return guarded([&] {
        NEED(h, "null handle");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        h->s->solve(init_x3, rel_eps, max_iter, m);
    });
}

int aa_geom_set_stop(aa_geom h, int stop_at_eps, double eps_rel) {
    return guarded([&] { NEED(h, "null handle"); h->s->set_stop(stop_at_eps, eps_rel); });
}

int aa_geom_get_solution(aa_geom h, double* x3) {
    return guarded([&] { NEED(h && x3, "null argument"); h->s->get_solution(x3); });
}

int aa_geom_get_history(aa_geom h, double* comb, double* time_s, int cap, int* n) {
    return guarded([&] {
        NEED(h, "null handle");
        const int k = h->s->history(comb, time_s, cap);
        if (n) *n = k;
    });
}

int aa_geom_runtime_info(aa_geom h, aa_geom_runtime* out) {
    return guarded([&] { NEED(h && out, "null argument"); *out = h->s->runtime(); });
}

int aa_geom_closest_points(aa_geom h, int surface, const double* p3, int n, double* out3) {
    return guarded([&] {
        NEED(h && (n == 0 || (p3 && out3)), "null argument");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        h->s->closest_points(surface, p3, n, out3);
    });
}

int aa_geom_bench_iterations(aa_geom h, int iters, double* ms) {
    return guarded([&] {
        NEED(h && iters >= 0, "bad argument");
        AA_HIP(hipSetDevice(h->ctx->c.device));
        const double t = h->s->bench_iterations(iters);
        if (ms) *ms = t;
    });
}

int aa_geom_kernel_stats(aa_geom h, const char* name, double* avg_ms, double* bytes, int* launches) {
    return guarded([&] {
        NEED(h && name, "null argument");
        if (!h->s->kernel_stats(name, avg_ms, bytes, launches)) throw aa::Error(AA_ERR_ARG, std::string("no kernel class ") + name);
    });
}

}  // extern "C"

// ---- element-level test hooks (tests only): device prox / COD / projections on host arrays ----
namespace {
template <class F>
int with_device_arrays(aa_ctx ctx, F&& f) {
    return guarded([&] {
        NEED(ctx, "null context");
        AA_HIP(hipSetDevice(ctx->c.device));
        f(ctx->c.stream);
        AA_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
}  // namespace

extern "C" int aa_test_prox(aa_ctx ctx, int op, const double* prm4, const double* in, int n, double* out, int* iters) {
    return with_device_arrays(ctx, [&](hipStream_t s) {
        NEED(prm4 && in && out && n >= 0 && op >= 0 && op <= 4, "aa_test_prox: bad argument");
        const int D = op >= 3 ? 6 : 9;
        aa::DevBuf<double> di, dout((size_t)D * std::max(n, 1));
        aa::DevBuf<int> dit(std::max(n, 1));
        di.upload(in, (size_t)D * n, s);
        aa::launch_test_prox(op, prm4, di.p, n, dout.p, dit.p, s);
        AA_HIP(hipMemcpyAsync(out, dout.p, sizeof(double) * D * n, hipMemcpyDeviceToHost, s));
        if (iters) AA_HIP(hipMemcpyAsync(iters, dit.p, sizeof(int) * n, hipMemcpyDeviceToHost, s));
        AA_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int aa_test_cod_solve(aa_ctx ctx, int k, const double* M, const double* b, double* theta) {
    return with_device_arrays(ctx, [&](hipStream_t s) {
        NEED(M && b && theta && k >= 1 && k <= aa::kMaxM, "aa_test_cod_solve: bad argument");
        aa::DevBuf<double> dM, db, dx(k);
        dM.upload(M, (size_t)k * k, s);
        db.upload(b, k, s);
        aa::launch_test_cod(k, dM.p, db.p, dx.p, s);
        AA_HIP(hipMemcpyAsync(theta, dx.p, sizeof(double) * k, hipMemcpyDeviceToHost, s));
        AA_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int aa_test_geom_project(aa_ctx ctx, int type, int k, const double* prm2, const double* in, int n,
                                    double* out) {
    return with_device_arrays(ctx, [&](hipStream_t s) {
        NEED(prm2 && in && out && n >= 0 && k >= 2, "aa_test_geom_project: bad argument");
        const int C = (type == aa::GEO_ANGLE || type == aa::GEO_EDGE) ? k - 1 : k;
        aa::DevBuf<double> di, dout((size_t)3 * C * std::max(n, 1));
        di.upload(in, (size_t)3 * C * n, s);
        aa::launch_test_geo_project(type, k, prm2, di.p, n, dout.p, s);
        AA_HIP(hipMemcpyAsync(out, dout.p, sizeof(double) * 3 * C * n, hipMemcpyDeviceToHost, s));
        AA_HIP(hipStreamSynchronize(s));
    });
}

