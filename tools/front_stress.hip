// Stand-alone repro for the GPU front backend's sequence (aa-admm_amd/csrc/dense_gpu.hip) without
// the solver: a random SPD front of order f with p pivots is factored twice from the same input
// -- rocsolver_dpotrf, rocblas_dtrsm / dsyrk, rocsolver_dtrtri, rocblas_dtrmm on one stream,
// rocBLAS atomics off, exactly the backend's calls -- and the two results compared bit for bit
// on the device. Deterministic kernels give identical bits; any difference is a wrong result.
// Run one process, then several processes on the same GPU at once, to separate "multi-process
// GPU sharing" from everything else the partitioned solver does.
//
//   hipcc --offload-arch=gfx950 -O2 tools/front_stress.hip -lrocsolver -lrocblas -o /tmp/front_stress
//   /tmp/front_stress <rounds> <f> <p> [seed] [mode]    -> "front_stress: rounds R mismatching M ..."
// mode: full (the backend's sequence, default) | potrf (rocsolver_dpotrf alone) | gemm (rocblas_dgemm
// alone, f x p times p x f) | trsm | syrk | trtri | blocked (the product's own blocked Cholesky:
// k_potf2 diagonal blocks + rocBLAS trsm / syrk, dense_gpu.hip) | noise (no library call: a streaming copy kernel for `rounds` x 20 ms,
// the aggressor beside another process's checks)
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(2); } } while (0)
#define RB(x) do { rocblas_status s_ = (x); if (s_ != rocblas_status_success) { std::fprintf(stderr, "%s: %d\n", #x, (int)s_); std::exit(2); } } while (0)

// lower triangle of a diagonally dominant SPD matrix (column-major), values from a hash of (i, j, seed)
__global__ void k_fill(double* F, int f, unsigned seed) {
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k >= (long long)f * f) return;
    const int i = (int)(k % f), j = (int)(k / f);
    if (i < j) { F[k] = 0.0; return; }
    unsigned h = (unsigned)i * 2654435761u ^ (unsigned)j * 40503u ^ seed * 2246822519u;
    h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const double r = (double)(h & 0xffffff) / 16777216.0 - 0.5;
    F[k] = i == j ? (double)f + r : r;
}

__global__ void k_cmp(const double* a, const double* b, long long n, unsigned long long* bad) {
    const long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    if (k < n && __double_as_longlong(a[k]) != __double_as_longlong(b[k])) atomicAdd(bad, 1ull);
}

__global__ void k_copy(double* __restrict__ d, const double* __restrict__ s, long long n) {
    for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x) d[k] = s[k] + 1.0;
}

static double max_rel_diff(const double* da, const double* db, size_t n) {
    std::vector<double> a(n), b(n);
    CK(hipMemcpy(a.data(), da, n * sizeof(double), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), db, n * sizeof(double), hipMemcpyDeviceToHost));
    double d = 0, m = 0;
    for (size_t k = 0; k < n; ++k) { d = std::max(d, std::fabs(a[k] - b[k])); m = std::max(m, std::fabs(b[k])); }
    return m > 0 ? d / m : d;
}

// the product's replacement (aa-admm_amd/csrc/dense_gpu.hip RocFrontBackend::potrf), same code
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

static void potrf_blocked(rocblas_handle h, hipStream_t s, double* F, int f, int p, int* info) {
    const double one = 1.0, mone = -1.0;
    for (int k0 = 0; k0 < p; k0 += kPotfBlock) {
        const int kb = std::min(kPotfBlock, p - k0), rest = p - k0 - kb;
        double* Akk = F + (size_t)k0 * f + k0;
        k_potf2<<<1, 256, 0, s>>>(Akk, f, kb, k0, info);
        if (rest > 0) {
            RB(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                             rocblas_diagonal_non_unit, rest, kb, &one, Akk, f, Akk + kb, f));
            RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, rest, kb, &mone, Akk + kb, f, &one,
                             Akk + (size_t)kb * f + kb, f));
        }
    }
}

struct Out { double *F, *L, *M; };

static void factor(rocblas_handle h, hipStream_t s, const double* Fk, Out o, int f, int p, int* info) {
    const int nb = f - p;
    const double one = 1.0, mone = -1.0;
    CK(hipMemcpyAsync(o.F, Fk, (size_t)f * f * sizeof(double), hipMemcpyDeviceToDevice, s));
    RB(rocsolver_dpotrf(h, rocblas_fill_lower, p, o.F, f, info));
    if (nb > 0) {
        RB(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_non_unit,
                         nb, p, &one, o.F, f, o.F + p, f));
        RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, nb, p, &mone, o.F + p, f, &one,
                         o.F + (size_t)p * f + p, f));
    }
    CK(hipMemcpy2DAsync(o.L, p * sizeof(double), o.F, f * sizeof(double), p * sizeof(double), p, hipMemcpyDeviceToDevice, s));
    RB(rocsolver_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_non_unit, p, o.L, p, info + 1));
    if (nb > 0)
        RB(rocblas_dtrmm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_non_unit,
                         nb, p, &one, o.L, p, o.F + p, f, o.M, nb));
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 20;
    const int f = argc > 2 ? std::atoi(argv[2]) : 2844;
    const int p = argc > 3 ? std::atoi(argv[3]) : 1422;
    const unsigned seed0 = argc > 4 ? (unsigned)std::atoi(argv[4]) : 1u;
    const char* mode = argc > 5 ? argv[5] : "full";
    const int nb = f - p;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    rocblas_handle h;
    RB(rocblas_create_handle(&h));
    RB(rocblas_set_stream(h, s));
    RB(rocblas_set_atomics_mode(h, rocblas_atomics_not_allowed));
    double *Fk, *buf;
    const size_t nF = (size_t)f * f, nL = (size_t)p * p, nM = (size_t)(nb > 0 ? nb : 1) * p;
    CK(hipMalloc(&Fk, nF * sizeof(double)));
    CK(hipMalloc(&buf, 2 * (nF + nL + nM) * sizeof(double)));
    Out a{buf, buf + nF, buf + nF + nL}, b{buf + nF + nL + nM, buf + 2 * nF + nL + nM, buf + 2 * nF + 2 * nL + nM};
    int* info;
    unsigned long long* bad;
    CK(hipMalloc(&info, 4 * sizeof(int)));
    CK(hipMalloc(&bad, 3 * sizeof(unsigned long long)));
    long long mism = 0, infos = 0;
    if (!std::strcmp(mode, "noise")) {   // aggressor: streaming copies, no library call
        const auto t0 = std::chrono::steady_clock::now();
        long long launches = 0;
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.02 * rounds) {
            k_copy<<<2048, 256, 0, s>>>(buf, Fk, (long long)nF);
            ++launches;
            if (launches % 64 == 0) CK(hipStreamSynchronize(s));
        }
        CK(hipStreamSynchronize(s));
        std::printf("front_stress: noise %lld launches\n", launches);
        return 0;
    }
    if (!std::strcmp(mode, "gemm") || !std::strcmp(mode, "potrf") || !std::strcmp(mode, "trsm") ||
        !std::strcmp(mode, "syrk") || !std::strcmp(mode, "trtri") || !std::strcmp(mode, "blocked")) {
        const bool gm = mode[0] == 'g';
        const double one = 1.0, zero = 0.0, mone = -1.0;
        double worst = 0;
        for (int r = 0; r < rounds; ++r) {
            k_fill<<<(unsigned)((nF + 255) / 256), 256, 0, s>>>(Fk, f, seed0 * 7919u + r);
            for (Out* o : {&a, &b}) {
                CK(hipMemcpyAsync(o->F, Fk, nF * sizeof(double), hipMemcpyDeviceToDevice, s));
                // trsm / syrk / trtri on the diagonally dominant lower triangle of Fk as L (well conditioned)
                if (gm) RB(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, f, f, p, &one, Fk, f, Fk, f,
                                         &zero, o->F, f));
                else if (mode[1] == 'o') RB(rocsolver_dpotrf(h, rocblas_fill_lower, f, o->F, f, info));
                else if (mode[0] == 'b') {
                    CK(hipMemsetAsync(info, 0, sizeof(int), s));
                    potrf_blocked(h, s, o->F, f, f, info);
                }
                else if (mode[1] == 'r' && mode[2] == 's')
                    RB(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                                     rocblas_diagonal_non_unit, f - p, p, &one, Fk, f, o->F + p, f));
                else if (mode[1] == 'y')
                    RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, f - p, p, &mone, Fk + p, f, &one,
                                     o->F + (size_t)p * f + p, f));
                else RB(rocsolver_dtrtri(h, rocblas_fill_lower, rocblas_diagonal_non_unit, f, o->F, f, info));
            }
            CK(hipMemsetAsync(bad, 0, sizeof(unsigned long long), s));
            k_cmp<<<(unsigned)((nF + 255) / 256), 256, 0, s>>>(a.F, b.F, (long long)nF, bad);
            unsigned long long hb = 0;
            CK(hipMemcpyAsync(&hb, bad, sizeof hb, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            if (hb) {
                ++mism;
                const double d = max_rel_diff(a.F, b.F, nF);
                worst = std::max(worst, d);
                std::printf("front_stress: %s round %d: %llu entries differ, max relative difference %.3e\n", mode, r, hb, d);
            }
        }
        std::printf("front_stress: %s f %d p %d rounds %d mismatching %lld worst %.3e\n", mode, f, p, rounds, mism, worst);
        return mism ? 1 : 0;
    }
    for (int r = 0; r < rounds; ++r) {
        k_fill<<<(unsigned)((nF + 255) / 256), 256, 0, s>>>(Fk, f, seed0 * 7919u + r);
        CK(hipMemsetAsync(info, 0, 4 * sizeof(int), s));
        factor(h, s, Fk, a, f, p, info);
        factor(h, s, Fk, b, f, p, info + 2);
        CK(hipMemsetAsync(bad, 0, 3 * sizeof(unsigned long long), s));
        k_cmp<<<(unsigned)((nF + 255) / 256), 256, 0, s>>>(a.F, b.F, (long long)nF, bad);
        k_cmp<<<(unsigned)((nL + 255) / 256), 256, 0, s>>>(a.L, b.L, (long long)nL, bad + 1);
        if (nb > 0) k_cmp<<<(unsigned)((nM + 255) / 256), 256, 0, s>>>(a.M, b.M, (long long)nb * p, bad + 2);
        unsigned long long hb[3];
        int hi[4];
        CK(hipMemcpyAsync(hb, bad, sizeof hb, hipMemcpyDeviceToHost, s));
        CK(hipMemcpyAsync(hi, info, sizeof hi, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        if (hb[0] || hb[1] || hb[2]) {
            ++mism;
            std::printf("front_stress: round %d: F %llu, Linv %llu, M %llu entries differ between two factorizations "
                        "(max relative difference F %.3e)\n", r, hb[0], hb[1], hb[2], max_rel_diff(a.F, b.F, nF));
        }
        if (hi[0] || hi[1] || hi[2] || hi[3]) {
            ++infos;
            std::printf("front_stress: round %d: infos %d %d %d %d\n", r, hi[0], hi[1], hi[2], hi[3]);
        }
    }
    std::printf("front_stress: f %d p %d rounds %d mismatching %lld nonzero-info %lld\n", f, p, rounds, mism, infos);
    return mism || infos ? 1 : 0;
}
