// Dense front assembly + partial factorization on the GPU (see spd_direct.hpp DenseFrontBackend):
// the large fronts near the root of the nested-dissection tree, which hold most of the factor's
// flops (C4: ~240 of 247 GFLOP in fronts of order >= 1024), are assembled and factored with
// rocSOLVER / rocBLAS on the solver's stream instead of the host's right-looking loop.
//   assembly   scatter-add of A's pivot columns, then of each child's update matrix (child order,
//              one launch each: every front entry receives its terms in the host loop's order)
//   factor     L11 by a blocked Cholesky (k_potf2 diagonal blocks + dtrsm / dsyrk; not rocsolver_dpotrf,
//              see potrf()), dtrsm (L21 = F21 L11^-T), dsyrk (F22 -= L21 L21^T)
//   outputs    dtrtri (Linv = L11^-1), dtrmm (M = L21 Linv), transposed to the host's row-major
//              layouts on the device; F22 stays on the device when the parent is factored here
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>

#include "common.hpp"
#include "dense_gpu.hpp"

namespace aa {

namespace {

void rb_check(rocblas_status st, const char* what) {
    if (st != rocblas_status_success) throw Error(ERR_DEVICE, std::string(what) + ": " + rocblas_status_to_string(st));
}

// F(i, j) += v for the COO entries (distinct entries: no conflicts)
__global__ void k_scatter_coo(double* __restrict__ F, int f, const int* __restrict__ ri, const int* __restrict__ cj,
                              const double* __restrict__ v, int n) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) F[(size_t)cj[k] * f + ri[k]] += v[k];
}

// extend-add of one child's update matrix (lower triangle, m x m; row-major a*m+b or column-major
// b*m+a) into the front: entry (a, b), b <= a, lands on F(max(ra, rb), min(ra, rb)). Distinct
// (a, b) land on distinct entries (map is injective), so one launch per child has no conflicts.
__global__ void k_extend_add(double* __restrict__ F, int f, const double* __restrict__ U, int m, int rowmajor,
                             const int* __restrict__ map) {
    const int a = blockIdx.y * blockDim.y + threadIdx.y;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= m || b > a) return;
    int ra = map[a], rb = map[b];
    if (ra < rb) { const int t = ra; ra = rb; rb = t; }
    F[(size_t)rb * f + ra] += rowmajor ? U[(size_t)a * m + b] : U[(size_t)b * m + a];
}

// dst (rows x cols, row-major) = src (column-major, leading dimension ld); lower = true keeps
// only entries with column <= row (zero elsewhere). 32 x 32 tiles through LDS.
__global__ void k_to_rowmajor(double* __restrict__ dst, const double* __restrict__ src, int ld, int rows, int cols,
                              int lower) {
    __shared__ double t[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    for (int q = threadIdx.y; q < 32; q += blockDim.y) {   // read: consecutive threads, consecutive rows
        const int c = c0 + q, r = r0 + threadIdx.x;
        if (r < rows && c < cols) t[q][threadIdx.x] = src[(size_t)c * ld + r];
    }
    __syncthreads();
    for (int q = threadIdx.y; q < 32; q += blockDim.y) {   // write: consecutive threads, consecutive columns
        const int r = r0 + q, c = c0 + threadIdx.x;
        if (r < rows && c < cols) dst[(size_t)r * cols + c] = (lower && c > r) ? 0.0 : t[threadIdx.x][q];
    }
}

// number of non-finite entries of the column-major rows x cols block at a (leading dimension ld),
// added into *out (one atomic per workgroup)
__global__ void k_count_nonfinite(const double* __restrict__ a, int ld, int rows, int cols, int* out) {
    __shared__ int sc[kBlock / 64];
    int c = 0;
    const long long n = (long long)rows * cols;
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
        c += !isfinite(a[(k / rows) * ld + k % rows]);
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sc[w];
        if (t) atomicAdd(out, t);
    }
}

// Unblocked Cholesky of one kb x kb diagonal block (kb <= kPotfBlock) of the column-major matrix
// at A (leading dimension lda), lower triangle, in LDS: column j scaled by 1 / sqrt(a_jj), then the
// trailing triangle updated, one workgroup of 256 threads = a thread per row x four column groups
// (measured on C4 setup, 394 blocks: 128-column blocks with k / m, k % m per trailing entry 390 us
// per block, with two column groups 216 us, with a wave-uniform predicated loop 268 us).
// A pivot that is not > 0 (or NaN) stops the block and stores its global index + 1 in *info (the
// first failing pivot, as rocsolver's info). Every entry is updated by j ascending.
constexpr int kPotfBlock = 64, kPotfGroups = 256 / kPotfBlock;
__global__ __launch_bounds__(256) void k_potf2(double* __restrict__ A, int lda, int kb, int k0, int* info) {
    __shared__ double a[kPotfBlock * (kPotfBlock + 1)];   // column-major, padded leading dimension
    constexpr int LD = kPotfBlock + 1, NG = kPotfGroups;
    if (*info != 0) return;   // an earlier block failed
    const int r = threadIdx.x % kPotfBlock, cg = threadIdx.x / kPotfBlock;   // row, column group
    if (r < kb)
        for (int c = cg; c < kb; c += NG) a[c * LD + r] = r >= c ? A[(size_t)c * lda + r] : 0.0;
    __syncthreads();
    for (int j = 0; j < kb; ++j) {
        const double d = a[j * LD + j];
        if (!(d > 0.0)) {   // uniform: every thread read the same value
            if (threadIdx.x == 0) *info = k0 + j + 1;
            return;
        }
        const double ljj = sqrt(d), inv = 1.0 / ljj;
        __syncthreads();   // d read by all before column j is rewritten
        if (cg == 0 && r >= j && r < kb) a[j * LD + r] = r == j ? ljj : a[j * LD + r] * inv;
        __syncthreads();
        if (r > j && r < kb) {
            const double lrj = a[j * LD + r];
            for (int c = j + 1 + cg; c <= r; c += NG) a[c * LD + r] -= lrj * a[j * LD + c];
        }
        __syncthreads();
    }
    if (r < kb)
        for (int c = cg; c <= r && c < kb; c += NG) A[(size_t)c * lda + r] = a[c * LD + r];
}

template <class T>
struct Grow {   // device buffer that only grows
    DevBuf<T> b;
    T* get(size_t n) {
        if (b.n < n) b.alloc(n);
        return b.p;
    }
};

class RocFrontBackend final : public DenseFrontBackend {
public:
    // dev_: the stream's device. factor() runs on OpenMP worker threads whose HIP current device
    // is 0 unless set, so every entry point selects dev_ first: buffers, the handle and the
    // stream must all live on the solver's GPU (ranks 1..P-1 of a partitioned run).
    explicit RocFrontBackend(hipStream_t s, bool test_hooks = true) : s_(s) {
        if (!test_hooks) poison_ = 0;
        AA_HIP(hipStreamGetDevice(s_, &dev_));
        AA_HIP(hipSetDevice(dev_));

        info_.alloc(3);   // potrf info, trtri info, non-finite output count
    }
    ~RocFrontBackend() override {
        for (auto& kv : handles_) (void)rocblas_destroy_handle(kv.second);
    }
    bool holds(int s) const override {
        std::lock_guard<std::mutex> g(mu_);
        return held_.count(s) > 0;
    }
    void drop(int s) override {
        std::lock_guard<std::mutex> g(mu_);
        AA_HIP(hipSetDevice(dev_));
        held_.erase(s);
    }
    void factor(int s, int f, int p, const std::vector<int>& ai, const std::vector<int>& aj, const std::vector<double>& av,
                const std::vector<Child>& kids, bool keep_update, std::vector<double>& Linv, std::vector<double>& LBP,
                std::vector<double>& M, std::vector<double>* U) override {
        std::lock_guard<std::mutex> g(mu_);
        AA_HIP(hipSetDevice(dev_));
        // one rocBLAS handle per calling thread (rocBLAS handles are per-thread objects; the
        // OpenMP workers of the tree-parallel factorization take turns here); everything below is
        // ordered on s_
        rocblas_handle h_ = handle();
        const auto t0 = std::chrono::steady_clock::now();
        struct Tally {   // time inside the backend (AA_SETUP_TIMES)
            RocFrontBackend* b;
            std::chrono::steady_clock::time_point t0;
            ~Tally() { b->busy_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); ++b->fronts; }
        } tally{this, t0};
        const int nb = f - p;
        double* F = F_.get((size_t)f * f);
        AA_HIP(hipMemsetAsync(F, 0, (size_t)f * f * sizeof(double), s_));
        // ---- assembly
        const int na = (int)ai.size();
        if (na > 0) {
            int* di = ii_.get(2 * (size_t)na);
            double* dv = dv_.get(na);
            // host data through pinned staging (common.hpp PinnedBuf): stream-ordered DMA
            int* hi = hint_.get(2 * (size_t)na);
            double* hv = hdbl_.get(na);
            std::memcpy(hi, ai.data(), na * sizeof(int));
            std::memcpy(hi + na, aj.data(), na * sizeof(int));
            std::memcpy(hv, av.data(), na * sizeof(double));
            AA_HIP(hipMemcpyAsync(di, hi, 2 * (size_t)na * sizeof(int), hipMemcpyHostToDevice, s_));
            AA_HIP(hipMemcpyAsync(dv, hv, na * sizeof(double), hipMemcpyHostToDevice, s_));
            hipLaunchKernelGGL(k_scatter_coo, dim3(blocks_for(na)), dim3(kBlock), 0, s_, F, f, di, di + na, dv, na);
            AA_CHECK_LAUNCH();
            AA_HIP(hipStreamSynchronize(s_));   // the host vectors are the caller's
        }
        for (const Child& c : kids) {
            if (c.m == 0) continue;
            int* dmap = map_.get(c.m);
            int* hm = hint_.get(c.m);
            std::memcpy(hm, c.map, c.m * sizeof(int));
            AA_HIP(hipMemcpyAsync(dmap, hm, c.m * sizeof(int), hipMemcpyHostToDevice, s_));
            const double* Usrc;
            int rowmajor;
            std::unique_ptr<DevBuf<double>> own;
            if (c.U) {
                double* du = up_.get((size_t)c.m * c.m);
                double* hu = hdbl_.get((size_t)c.m * c.m);
                std::memcpy(hu, c.U->data(), (size_t)c.m * c.m * sizeof(double));
                AA_HIP(hipMemcpyAsync(du, hu, (size_t)c.m * c.m * sizeof(double), hipMemcpyHostToDevice, s_));
                Usrc = du;
                rowmajor = 1;
            } else {
                auto it = held_.find(c.id);
                if (it == held_.end()) throw Error(ERR_STATE, "dense front backend: missing update matrix");
                own = std::move(it->second);
                held_.erase(it);
                Usrc = own->p;
                rowmajor = 0;
            }
            const dim3 blk(32, 8), grd((c.m + 31) / 32, (c.m + 7) / 8);
            hipLaunchKernelGGL(k_extend_add, grd, blk, 0, s_, F, f, Usrc, c.m, rowmajor, dmap);
            AA_CHECK_LAUNCH();
            AA_HIP(hipStreamSynchronize(s_));   // before the staging buffers / held matrix are reused
        }
        if (reduce_front) reduce_front(F, (size_t)f * f);   // partitioned top: the ranks' partial fronts summed
        double* Fk = nullptr;   // the kept copy (below)
        if (check_) {
            Fk = K_.get((size_t)f * f);
            AA_HIP(hipMemcpyAsync(Fk, F, (size_t)f * f * sizeof(double), hipMemcpyDeviceToDevice, s_));
        }
        // ---- partial factorization: potrf, trsm, syrk, trtri, trmm; returns the potrf / trtri infos
        // and (check_) the number of non-finite entries in F (L11, L21, Schur complement), L11^-1 and M
        const double one = 1.0, mone = -1.0;
        double* L = L_.get((size_t)p * p);
        double* Md = nb > 0 ? M_.get((size_t)nb * p) : nullptr;
        auto attempt = [&](int* out) {
            AA_HIP(hipMemsetAsync(info_.p, 0, 3 * sizeof(int), s_));
            if (own_potrf_) potrf(h_, F, f, p);
            else rb_check(rocsolver_dpotrf(h_, rocblas_fill_lower, p, F, f, info_.p), "rocsolver_dpotrf");
            if (nb > 0) {
                rb_check(rocblas_dtrsm(h_, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                                       rocblas_diagonal_non_unit, nb, p, &one, F, f, F + p, f), "rocblas_dtrsm");
                rb_check(rocblas_dsyrk(h_, rocblas_fill_lower, rocblas_operation_none, nb, p, &mone, F + p, f, &one,
                                       F + (size_t)p * f + p, f), "rocblas_dsyrk");
            }
            AA_HIP(hipMemcpy2DAsync(L, p * sizeof(double), F, f * sizeof(double), p * sizeof(double), p,
                                    hipMemcpyDeviceToDevice, s_));
            rb_check(rocsolver_dtrtri(h_, rocblas_fill_lower, rocblas_diagonal_non_unit, p, L, p, info_.p + 1),
                     "rocsolver_dtrtri");
            if (nb > 0)
                rb_check(rocblas_dtrmm(h_, rocblas_side_right, rocblas_fill_lower, rocblas_operation_none,
                                       rocblas_diagonal_non_unit, nb, p, &one, L, p, F + p, f, Md, nb), "rocblas_dtrmm");
            if (check_) {
                const auto cnt = [&](const double* a, int ld, int rows, int cols) {
                    if ((long long)rows * cols == 0) return;
                    const long long n = (long long)rows * cols;
                    hipLaunchKernelGGL(k_count_nonfinite, dim3((unsigned)std::min<long long>((n + kBlock - 1) / kBlock, 1024)),
                                       dim3(kBlock), 0, s_, a, ld, rows, cols, info_.p + 2);
                    AA_CHECK_LAUNCH();
                };
                cnt(F, f, f, f);
                cnt(L, p, p, p);
                if (nb > 0) cnt(Md, nb, nb, p);
            }
            AA_HIP(hipMemcpyAsync(out, info_.p, 3 * sizeof(int), hipMemcpyDeviceToHost, s_));
            AA_HIP(hipStreamSynchronize(s_));
        };
        if (check_ && poison_ > 0 && --poison_ == 0) {   // test hook: this front's first attempt starts from a NaN
            AA_HIP(hipMemsetAsync(F, 0xff, sizeof(double), s_));
        }
        // Product check (check_): with a fixed pseudo-random r, the factored front must reproduce the
        // kept copy -- Fk r = [L11 0; L21 I] [I 0; 0 S] [L11 0; L21 I]^T r (S the Schur complement) --
        // and L11^-1 (L11 r1) = r1, M r1 = L21 (L11^-1 r1); O(f^2) matrix-vector products against the
        // O(f^3) factorization. Returns the largest relative deviation (a transient that leaves wrong
        // but finite numbers shows up as O(1); rounding as < 1e-10).
        auto verify = [&]() -> double {
            if (!check_) return 0.0;
            double* v = V_.get(6 * (size_t)f);
            double *r = v, *y = v + f, *t = v + 2 * (size_t)f, *y2 = v + 3 * (size_t)f, *a = v + 4 * (size_t)f, *b = v + 5 * (size_t)f;
            double* hr = hdbl_.get(8 * (size_t)f);
            unsigned long long z = 0x9e3779b97f4a7c15ull;
            for (int i = 0; i < f; ++i) { z = z * 6364136223846793005ull + 1442695040888963407ull; hr[i] = (double)(z >> 11) * 0x1.0p-53 - 0.5; }
            AA_HIP(hipMemcpyAsync(r, hr, (size_t)f * sizeof(double), hipMemcpyHostToDevice, s_));
            const double zero = 0.0;
            rb_check(rocblas_dsymv(h_, rocblas_fill_lower, f, &one, Fk, f, r, 1, &zero, y, 1), "rocblas_dsymv");
            // t = L11^T r1 + L21^T r2
            AA_HIP(hipMemcpyAsync(t, r, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s_));
            rb_check(rocblas_dtrmv(h_, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit, p, F, f, t, 1), "rocblas_dtrmv");
            if (nb > 0) rb_check(rocblas_dgemv(h_, rocblas_operation_transpose, nb, p, &one, F + p, f, r + p, 1, &one, t, 1), "rocblas_dgemv");
            // y2 = [L11 t; L21 t + S r2]
            AA_HIP(hipMemcpyAsync(y2, t, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s_));
            rb_check(rocblas_dtrmv(h_, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, p, F, f, y2, 1), "rocblas_dtrmv");
            if (nb > 0) {
                rb_check(rocblas_dsymv(h_, rocblas_fill_lower, nb, &one, F + (size_t)p * f + p, f, r + p, 1, &zero, y2 + p, 1), "rocblas_dsymv");
                rb_check(rocblas_dgemv(h_, rocblas_operation_none, nb, p, &one, F + p, f, t, 1, &one, y2 + p, 1), "rocblas_dgemv");
            }
            // a = L11^-1 (L11 r1); b = L11^-1 r1, then M r1 vs L21 b (in t[.. nb], y2 reused below)
            AA_HIP(hipMemcpyAsync(a, r, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s_));
            rb_check(rocblas_dtrmv(h_, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, p, F, f, a, 1), "rocblas_dtrmv");
            rb_check(rocblas_dtrmv(h_, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, p, L, p, a, 1), "rocblas_dtrmv");
            AA_HIP(hipMemcpyAsync(b, r, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s_));
            rb_check(rocblas_dtrmv(h_, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit, p, L, p, b, 1), "rocblas_dtrmv");
            double* hm = hr + f;   // host copies: y, y2, a; then the M check
            AA_HIP(hipMemcpyAsync(hm, y, 2 * (size_t)f * sizeof(double), hipMemcpyDeviceToHost, s_));   // y (and t: unused)
            AA_HIP(hipMemcpyAsync(hm + 2 * (size_t)f, y2, (size_t)f * sizeof(double), hipMemcpyDeviceToHost, s_));
            AA_HIP(hipMemcpyAsync(hm + 3 * (size_t)f, a, (size_t)p * sizeof(double), hipMemcpyDeviceToHost, s_));
            double dev = 0;
            auto rel = [](const double* u, const double* w, int n) {
                double d = 0, m = 0;
                for (int i = 0; i < n; ++i) { d = std::max(d, std::fabs(u[i] - w[i])); m = std::max(m, std::fabs(u[i])); }
                return m > 0 ? d / m : d;
            };
            if (nb > 0) {   // M r1 (into y) and L21 b (into y2 + p)
                rb_check(rocblas_dgemv(h_, rocblas_operation_none, nb, p, &one, Md, nb, r, 1, &zero, y, 1), "rocblas_dgemv");
                rb_check(rocblas_dgemv(h_, rocblas_operation_none, nb, p, &one, F + p, f, b, 1, &zero, t, 1), "rocblas_dgemv");
            }
            AA_HIP(hipStreamSynchronize(s_));
            const double* hy = hm;
            const double* hy2 = hm + 2 * (size_t)f;
            const double* ha = hm + 3 * (size_t)f;
            dev = std::max(dev, rel(hy, hy2, f));
            dev = std::max(dev, rel(hr, ha, p));
            if (nb > 0) {
                double* hq = hm + 4 * (size_t)f;   // (hdbl_ holds 8 f >= 5 f + 2 nb)
                AA_HIP(hipMemcpyAsync(hq, y, (size_t)nb * sizeof(double), hipMemcpyDeviceToHost, s_));
                AA_HIP(hipMemcpyAsync(hq + nb, t, (size_t)nb * sizeof(double), hipMemcpyDeviceToHost, s_));
                AA_HIP(hipStreamSynchronize(s_));
                dev = std::max(dev, rel(hq + nb, hq, nb));
            }
            return std::isfinite(dev) ? dev : 1e300;
        };
        int* hinfo = hint_.get(3);
        attempt(hinfo);
        double dev1 = (hinfo[0] == 0 && hinfo[2] == 0) ? verify() : 0.0;
        if (dev1 < 1e300) max_dev = std::max(max_dev, dev1);
        // Front check (default on; AA_FRONT_CHECK=0 off): the assembled front is kept (one device
        // copy) and every output is checked -- potrf info, non-finite entries, the product check.
        // An SPD front fails none of them, so a failure is an ERROR: the kept copy's diagnostics
        // (and, with AA_FRONT_DUMP=<dir>, the kept copy and the first attempt's outputs, for a replay)
        // and, if the kept copy factors cleanly, the statement that the first attempt was at fault.
        // AA_FRONT_RETRY=1 (opt-in, and the poison test) goes on with the second factorization
        // instead, reported on stderr. History: the wrong factorizations of round 5 came
        // from rank processes bound to another ROCm build's HIP / rocBLAS / rocSOLVER.
        if (check_ && (hinfo[0] != 0 || hinfo[2] != 0 || dev1 > kVerifyTol)) {
            const int first = hinfo[0], bad = hinfo[2];
            if (const char* d = std::getenv("AA_FRONT_DUMP")) dump(d, s, f, p, nb, Fk, F, L, Md);
            double* hf = hdbl_.get((size_t)f * f);
            AA_HIP(hipMemcpyAsync(hf, Fk, (size_t)f * f * sizeof(double), hipMemcpyDeviceToHost, s_));
            AA_HIP(hipStreamSynchronize(s_));
            size_t nonfinite = 0;
            double dmin = 1e300, dmax = 0;
            for (size_t q = 0; q < (size_t)f * f; ++q) nonfinite += !std::isfinite(hf[q]);
            for (int q = 0; q < f; ++q) { dmin = std::min(dmin, hf[(size_t)q * f + q]); dmax = std::max(dmax, hf[(size_t)q * f + q]); }
            AA_HIP(hipMemcpyAsync(F, Fk, (size_t)f * f * sizeof(double), hipMemcpyDeviceToDevice, s_));
            attempt(hinfo);
            const double dev2 = (hinfo[0] == 0 && hinfo[2] == 0) ? verify() : 0.0;
            char msg[480];
            std::snprintf(msg, sizeof msg, "[front-check] front %d order %d p %d: potrf info %d, %d non-finite outputs, "
                          "product deviation %.2e; kept copy: %zu non-finite, diag [%.3e, %.3e]; again on the copy: potrf "
                          "info %d, %d non-finite outputs, product deviation %.2e",
                          s, f, p, first, bad, dev1, nonfinite, dmin, dmax, hinfo[0], hinfo[2], dev2);
            std::fprintf(stderr, "%s\n", msg);
            ++retries;
            if (hinfo[0] != 0) throw Error(ERR_NUMERIC, std::string("multifrontal_cholesky: matrix not positive definite ") + msg);
            if (hinfo[2] != 0) throw Error(ERR_NUMERIC, std::string("multifrontal_cholesky: non-finite factor ") + msg);
            if (dev2 > kVerifyTol) throw Error(ERR_NUMERIC, std::string("multifrontal_cholesky: factor fails the product check ") + msg);
            if (!retry_)
                throw Error(ERR_NUMERIC, std::string("multifrontal_cholesky: GPU front factored wrongly on the first attempt "
                                                     "(the kept copy factors cleanly; AA_FRONT_RETRY=1 continues with it) ") + msg);
        }
        const int info[2] = {hinfo[0], hinfo[1]};
        if (info[0] != 0)
            throw std::runtime_error("multifrontal_cholesky: matrix not positive definite (GPU front " + std::to_string(s) +
                                     ", order " + std::to_string(f) + ", pivot " + std::to_string(info[0]) + " of " +
                                     std::to_string(p) + ", " + std::to_string(kids.size()) + " children)");
        if (info[1] != 0) throw std::runtime_error("multifrontal_cholesky: singular diagonal block");
        // ---- outputs in the host layouts
        auto fetch = [&](std::vector<double>& out, const double* src, int ld, int rows, int cols, int lower) {
            out.resize((size_t)rows * cols);
            if (out.empty()) return;
            double* t = T_.get(out.size());
            const dim3 blk(32, 8), grd((cols + 31) / 32, (rows + 31) / 32);
            hipLaunchKernelGGL(k_to_rowmajor, grd, blk, 0, s_, t, src, ld, rows, cols, lower);
            AA_CHECK_LAUNCH();
            double* h = hdbl_.get(out.size());
            AA_HIP(hipMemcpyAsync(h, t, out.size() * sizeof(double), hipMemcpyDeviceToHost, s_));
            AA_HIP(hipStreamSynchronize(s_));
            std::memcpy(out.data(), h, out.size() * sizeof(double));
        };
        fetch(Linv, L, p, p, p, 1);
        fetch(LBP, F + p, f, nb, p, 0);
        if (nb > 0) fetch(M, Md, nb, nb, p, 0);
        else M.clear();
        if (nb > 0) {
            if (keep_update) {   // column-major nb x nb, for the parent's extend-add
                auto u = std::make_unique<DevBuf<double>>((size_t)nb * nb);
                AA_HIP(hipMemcpy2DAsync(u->p, nb * sizeof(double), F + (size_t)p * f + p, f * sizeof(double),
                                        nb * sizeof(double), nb, hipMemcpyDeviceToDevice, s_));
                AA_HIP(hipStreamSynchronize(s_));
                held_[s] = std::move(u);
            } else {
                fetch(*U, F + (size_t)p * f + p, f, nb, nb, 1);
            }
        }
    }

    double busy_ms = 0;
    int fronts = 0;
    int retries = 0;      // fronts whose first attempt failed a check (an error unless AA_FRONT_RETRY=1)
    double max_dev = 0;   // largest first-attempt product deviation (AA_SETUP_TIMES)

private:
    // Cholesky of the p x p leading block of the column-major front F (lower), blocked right-looking:
    // per 64-column block k_potf2 on the diagonal block, then rocblas_dtrsm for the block's rows
    // below it and rocblas_dsyrk for the trailing p x p triangle. Replaces rocsolver_dpotrf, which
    // returns wrong factors (info 0) when several processes run it on one GPU at the same time
    // (tools/front_stress.hip); rocBLAS trsm / syrk / gemm are unaffected. info_.p[0]:
    // the first failing pivot + 1.
    void potrf(rocblas_handle h, double* F, int f, int p) {
        const double one = 1.0, mone = -1.0;
        for (int k0 = 0; k0 < p; k0 += kPotfBlock) {
            const int kb = std::min(kPotfBlock, p - k0), rest = p - k0 - kb;
            double* Akk = F + (size_t)k0 * f + k0;
            hipLaunchKernelGGL(k_potf2, dim3(1), dim3(256), 0, s_, Akk, f, kb, k0, info_.p);
            AA_CHECK_LAUNCH();
            if (rest > 0) {   // (after a failed pivot the rest runs on garbage; info already says so)
                rb_check(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                                       rocblas_diagonal_non_unit, rest, kb, &one, Akk, f, Akk + kb, f), "rocblas_dtrsm");
                rb_check(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, rest, kb, &mone, Akk + kb, f, &one,
                                       Akk + (size_t)kb * f + kb, f), "rocblas_dsyrk");
            }
        }
    }
    // AA_FRONT_POTRF=rocsolver: rocsolver_dpotrf instead of potrf() above (single-process A/B)
    bool own_potrf_ = !(std::getenv("AA_FRONT_POTRF") && std::strcmp(std::getenv("AA_FRONT_POTRF"), "rocsolver") == 0);
    // AA_FRONT_DUMP: the kept front and the first attempt's outputs of front s, column-major
    // doubles, for a replay in one process (tools/front_replay.py)
    void dump(const char* dir, int s, int f, int p, int nb, const double* Fk, const double* F, const double* L,
              const double* Md) {
        auto put = [&](const char* what, const double* src, size_t n) {
            std::vector<double> h(n);
            AA_HIP(hipMemcpyAsync(h.data(), src, n * sizeof(double), hipMemcpyDeviceToHost, s_));
            AA_HIP(hipStreamSynchronize(s_));
            const std::string path = std::string(dir) + "/front" + std::to_string(s) + "_f" + std::to_string(f) + "_p" +
                                     std::to_string(p) + "_" + what + ".bin";
            if (FILE* fo = std::fopen(path.c_str(), "wb")) {
                std::fwrite(h.data(), sizeof(double), n, fo);
                std::fclose(fo);
            }
        };
        put("kept", Fk, (size_t)f * f);
        put("first_F", F, (size_t)f * f);
        put("first_Linv", L, (size_t)p * p);
        if (nb > 0) put("first_M", Md, (size_t)nb * p);
    }

    hipStream_t s_;
    int dev_ = 0;
    std::map<std::thread::id, rocblas_handle> handles_;
    rocblas_handle handle() {   // (under mu_)
        auto it = handles_.find(std::this_thread::get_id());
        if (it != handles_.end()) return it->second;
        rocblas_handle h = nullptr;
        rb_check(rocblas_create_handle(&h), "rocblas_create_handle");
        rb_check(rocblas_set_stream(h, s_), "rocblas_set_stream");
        // deterministic rocBLAS kernels: every rank must factor the shared top bit-identically
        rb_check(rocblas_set_atomics_mode(h, rocblas_atomics_not_allowed), "rocblas_set_atomics_mode");
        handles_[std::this_thread::get_id()] = h;
        return h;
    }
    mutable std::mutex mu_;
    std::map<int, std::unique_ptr<DevBuf<double>>> held_;
    DevBuf<int> info_;
    Grow<double> F_, L_, M_, T_, dv_, up_;
    Grow<int> ii_, map_;
    PinnedBuf<double> hdbl_;   // host staging (pinned) for the copies above
    PinnedBuf<int> hint_;
    Grow<double> K_;           // AA_FRONT_CHECK: the assembled front, kept
    Grow<double> V_;           // AA_FRONT_CHECK: the product check's vectors
    // a deviation above this is a wrong factorization, not rounding (the check's products of an
    // SPD front deviate by ~1e-15 .. 1e-12 relative)
    static constexpr double kVerifyTol = 1e-8;
    bool retry_ = std::getenv("AA_FRONT_RETRY") && std::getenv("AA_FRONT_RETRY")[0] == '1';
    bool check_ = !(std::getenv("AA_FRONT_CHECK") && std::getenv("AA_FRONT_CHECK")[0] == '0');
    // AA_FRONT_CHECK_POISON=k (tests): the k-th front this backend factors gets a NaN in its first
    // attempt (after the copy is kept) -- the retry must give the unpoisoned run's bits
    int poison_ = std::getenv("AA_FRONT_CHECK_POISON") ? std::atoi(std::getenv("AA_FRONT_CHECK_POISON")) : 0;
};

}  // namespace

std::unique_ptr<DenseFrontBackend> make_gpu_front_backend(hipStream_t s) {
    auto b = std::unique_ptr<DenseFrontBackend>(new RocFrontBackend(s));
    if (const char* e = std::getenv("AA_DENSE_MIN_FRONT")) b->min_front = std::max(1, std::atoi(e));
    return b;
}

double warm_gpu_front_backend(hipStream_t s) {
    const char* e = std::getenv("AA_DENSE_GPU");
    if (e && e[0] == '0') return 0.0;
    int dev = 0;
    AA_HIP(hipStreamGetDevice(s, &dev));
    static std::mutex mu;
    static std::set<int> warm;
    std::lock_guard<std::mutex> g(mu);
    if (warm.count(dev)) return 0.0;
    const auto t0 = std::chrono::steady_clock::now();
    {   // a diagonally dominant front of the smallest GPU order with a boundary block: potrf, trsm,
        // syrk, trtri, trmm and the assembly / layout kernels, as every GPU front of a factor runs
        RocFrontBackend b(s, false);
        const int p = b.min_front, f = p + 64;
        std::vector<int> ai, aj;
        std::vector<double> av;
        for (int j = 0; j < p; ++j)
            for (int i = j; i < f && i < j + 2; ++i) { ai.push_back(i); aj.push_back(j); av.push_back(i == j ? 4.0 : -1.0); }
        std::vector<double> Linv, LBP, M, U;
        b.factor(0, f, p, ai, aj, av, {}, false, Linv, LBP, M, &U);
    }
    warm.insert(dev);
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

std::unique_ptr<PartFactor> make_part_factor(Comm* comm, int rank, hipStream_t s) {
    const char* e = std::getenv("AA_PART_FACTOR");
    if (!comm || comm->size() < 2 || comm->rehearsal() || (e && e[0] == '0')) return nullptr;
    auto pf = std::make_unique<PartFactor>();
    pf->my_part = rank;
    pf->first = rank == 0;
    pf->reduce_host = [comm](double* p, size_t n) { comm->allreduce_sum_host(p, n); };
    pf->reduce_dev = [comm, s](double* p, size_t n) { comm->allreduce_sum(p, p, n, s); };
    return pf;
}

SupernodalFactor factor_on_device(const CsrMatrix& A, const NdTree& tree, hipStream_t s, const PartFactor* part) {
    const char* e = std::getenv("AA_DENSE_GPU");
    if (e && e[0] == '0') return multifrontal_cholesky(A, tree, nullptr, part);
    auto b = make_gpu_front_backend(s);
    const auto t0 = std::chrono::steady_clock::now();
    SupernodalFactor F = multifrontal_cholesky(A, tree, b.get(), part);
    if (const char* t = std::getenv("AA_SETUP_TIMES"); t && t[0] == '1') {
        const auto* rb = static_cast<const RocFrontBackend*>(b.get());
        std::fprintf(stderr, "[setup]   factor %.1f ms: %d fronts on the GPU (%.1f ms inside the backend, product check "
                     "deviation <= %.1e, %d retried), %.1f GFLOP\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), rb->fronts,
                     rb->busy_ms, rb->max_dev, rb->retries, F.flops * 1e-9);
    }
    return F;
}

}  // namespace aa
