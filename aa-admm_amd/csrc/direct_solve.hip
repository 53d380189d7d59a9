// GPU supernodal triangular solves (see direct_solve.hpp).
#include "direct_solve.hpp"

#include <omp.h>

#include <algorithm>
#include <string>

namespace aa {

namespace {

__device__ __forceinline__ bool solve_gated(const Ctrl* c, int gate_reject) {
    if (!c) return false;
    if (c->done) return true;
    return gate_reject && !c->reject;
}

struct Plan {  // kernel arguments shared by the solve kernels
    const int* beg; const int* p; const int* nb; const int* bnd_off; const int* bnd;
    const int* pull_off; const int* pptr; const long long* psrc;
    const long long* goff; const long long* uoff; const long long* foff;
    const double* Gr; const double* Gc;
};
using Task = DirectSolver::Task;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// front row q of supernode s: [b_P ; 0]_q + the children's update entries landing on it
__device__ __forceinline__ void front_row(const Plan& P, int s, int q, const double* __restrict__ B,
                                          const double* __restrict__ U, double& a0, double& a1, double& a2) {
    a0 = a1 = a2 = 0;
    if (q < P.p[s]) { const size_t o = 3 * (size_t)(P.beg[s] + q); a0 = B[o]; a1 = B[o + 1]; a2 = B[o + 2]; }
    const int r = P.pull_off[s] + q;
    for (int e = P.pptr[r]; e < P.pptr[r + 1]; ++e) {
        const double* u = U + P.psrc[e];
        a0 += u[0]; a1 += u[1]; a2 += u[2];
    }
}

// assembly of the front vectors of wave-mode supernodes into Fg
__global__ __launch_bounds__(256) void k_asm(Plan P, const Task* __restrict__ tasks, int first,
                                             const double* __restrict__ B, const double* __restrict__ U,
                                             double* __restrict__ Fg, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const Task t = tasks[first + blockIdx.x];
    if ((int)threadIdx.x >= t.nr) return;
    const int q = t.r0 + threadIdx.x;
    double a0, a1, a2;
    front_row(P, t.node, q, B, U, a0, a1, a2);
    double* f = Fg + P.foff[t.node] + 3 * (size_t)q;
    f[0] = a0; f[1] = a1; f[2] = a2;
}

// forward sweep of one tree level: y_P = Linv f_P (rows r < p), u = f_B - M f_P (rows r >= p)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_fwd(Plan P, const Task* __restrict__ tasks, int first,
                                               const double* __restrict__ B, double* __restrict__ Y,
                                               double* __restrict__ U, const double* __restrict__ Fg,
                                               const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Task t = tasks[first + blockIdx.x];
    const int s = t.node, p = P.p[s], R = p + P.nb[s], b0 = P.beg[s];
    const int tid = threadIdx.x;
    if (t.mode == 0) {   // thread per row, f_P in LDS, column-major G (lanes read consecutive rows)
        double* f = lds;
        for (int c = tid; c < p; c += BLOCK) front_row(P, s, c, B, U, f[3 * c], f[3 * c + 1], f[3 * c + 2]);
        __syncthreads();
        if (tid >= t.nr) return;
        const int r = t.r0 + tid;
        const double* G = P.Gc + P.goff[s] + r;
        const int cmax = r < p ? r + 1 : p;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int c = 0; c < cmax; ++c) {
            const double v = G[(size_t)c * R];
            a0 += v * f[3 * c]; a1 += v * f[3 * c + 1]; a2 += v * f[3 * c + 2];
        }
        if (r < p) {
            const size_t o = 3 * (size_t)(b0 + r);
            Y[o] = a0; Y[o + 1] = a1; Y[o + 2] = a2;
        } else {
            double f0, f1, f2;
            front_row(P, s, r, B, U, f0, f1, f2);
            double* u = U + P.uoff[s] + 3 * (size_t)(r - p);
            u[0] = f0 - a0; u[1] = f1 - a1; u[2] = f2 - a2;
        }
    } else {             // wave per row, lanes across the row of the row-major G, f from Fg
        const int lane = tid & 63, w = tid >> 6;
        const double* F = Fg + P.foff[s];
        for (int rr = w; rr < t.nr; rr += BLOCK / 64) {
            const int r = t.r0 + rr;
            const double* row = P.Gr + P.goff[s] + (size_t)r * p;
            const int cmax = r < p ? r + 1 : p;
            double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 4
            for (int c = lane; c < cmax; c += 64) {
                const double v = row[c];
                a0 += v * F[3 * c]; a1 += v * F[3 * c + 1]; a2 += v * F[3 * c + 2];
            }
            a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
            if (lane == 0) {
                if (r < p) {
                    const size_t o = 3 * (size_t)(b0 + r);
                    Y[o] = a0; Y[o + 1] = a1; Y[o + 2] = a2;
                } else {
                    double* u = U + P.uoff[s] + 3 * (size_t)(r - p);
                    u[0] = F[3 * r] - a0; u[1] = F[3 * r + 1] - a1; u[2] = F[3 * r + 2] - a2;
                }
            }
        }
    }
}

// backward sweep of one tree level: x_P = Linv^T y_P - M^T x_B (columns j of G)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_bwd(Plan P, const Task* __restrict__ tasks, int first,
                                               const double* __restrict__ Y, double* __restrict__ X,
                                               const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Task t = tasks[first + blockIdx.x];
    const int s = t.node, p = P.p[s], nb = P.nb[s], R = p + nb, b0 = P.beg[s];
    const int* bi = P.bnd + P.bnd_off[s];
    const int tid = threadIdx.x;
    if (t.mode == 0) {   // thread per column, [y_P ; x_B] in LDS, row-major G (lanes read consecutive columns)
        double* v = lds;
        for (int r = tid; r < R; r += BLOCK) {
            const size_t o = r < p ? 3 * (size_t)(b0 + r) : 3 * (size_t)bi[r - p];
            const double sg = r < p ? 1.0 : -1.0;
            const double* src = r < p ? Y : X;
            v[3 * r] = sg * src[o]; v[3 * r + 1] = sg * src[o + 1]; v[3 * r + 2] = sg * src[o + 2];
        }
        __syncthreads();
        if (tid >= t.nr) return;
        const int j = t.r0 + tid;
        const double* G = P.Gr + P.goff[s] + j;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int r = j; r < R; ++r) {
            const double g = G[(size_t)r * p];
            a0 += g * v[3 * r]; a1 += g * v[3 * r + 1]; a2 += g * v[3 * r + 2];
        }
        const size_t o = 3 * (size_t)(b0 + j);
        X[o] = a0; X[o + 1] = a1; X[o + 2] = a2;
    } else {             // wave per column, lanes down the column of the column-major G
        const int lane = tid & 63, w = tid >> 6;
        for (int jj = w; jj < t.nr; jj += BLOCK / 64) {
            const int j = t.r0 + jj;
            const double* col = P.Gc + P.goff[s] + (size_t)j * R;
            double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 4
            for (int r = j + lane; r < R; r += 64) {
                const double g = col[r];
                if (r < p) {
                    const size_t o = 3 * (size_t)(b0 + r);
                    a0 += g * Y[o]; a1 += g * Y[o + 1]; a2 += g * Y[o + 2];
                } else {
                    const size_t o = 3 * (size_t)bi[r - p];
                    a0 -= g * X[o]; a1 -= g * X[o + 1]; a2 -= g * X[o + 2];
                }
            }
            a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
            if (lane == 0) {
                const size_t o = 3 * (size_t)(b0 + j);
                X[o] = a0; X[o + 1] = a1; X[o + 2] = a2;
            }
        }
    }
}

constexpr int kWaveRowsPerTask = 8;   // wave-mode rows per 256-thread task (2 per wave)
constexpr int kMaxLdsMode0 = 96 * 1024;

}  // namespace

void DirectSolver::build(const SupernodalFactor& F, hipStream_t s) {
    n_ = F.n;
    nn_ = F.n_nodes;
    nnz_L_ = F.nnz_L;
    std::vector<int> beg(nn_), p(nn_), nb(nn_), bnd_off(nn_), bnd, pull_off(nn_);
    std::vector<long long> goff(nn_), uoff(nn_), foff(nn_, -1);
    long long go = 0, uo = 0, fo = 0;
    double dense = 0, offd = 0, bsum = 0;
    int rows_total = 0;
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = F.end[sn] - F.beg[sn], nbs = (int)F.bnd[sn].size();
        beg[sn] = F.beg[sn]; p[sn] = ps; nb[sn] = nbs;
        goff[sn] = go; uoff[sn] = uo;
        bnd_off[sn] = (int)bnd.size();
        bnd.insert(bnd.end(), F.bnd[sn].begin(), F.bnd[sn].end());
        pull_off[sn] = rows_total;
        rows_total += ps + nbs;
        go += (long long)(ps + nbs) * ps;
        uo += 3LL * nbs;
        dense += 0.5 * ps * (ps + 1.0);
        offd += (double)ps * nbs;
        bsum += nbs;
    }
    // G_s = [Linv ; M], M = L_BP Linv (row-major copy Gr and column-major copy Gc)
    std::vector<double> Gr(go), Gc(go);
#pragma omp parallel for schedule(dynamic, 1)
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = p[sn], nbs = nb[sn], R = ps + nbs;
        double* gr = Gr.data() + goff[sn];
        const std::vector<double>& Li = F.Linv[sn];
        const std::vector<double>& LB = F.LBP[sn];
        for (int r = 0; r < ps; ++r)
            for (int c = 0; c < ps; ++c) gr[(size_t)r * ps + c] = c <= r ? Li[(size_t)r * ps + c] : 0.0;
        for (int a = 0; a < nbs; ++a) {
            double* m = gr + (size_t)(ps + a) * ps;
            for (int c = 0; c < ps; ++c) m[c] = 0.0;
            for (int k = 0; k < ps; ++k) {
                const double l = LB[(size_t)a * ps + k];
                if (l == 0.0) continue;
                const double* lr = Li.data() + (size_t)k * ps;
                for (int c = 0; c <= k; ++c) m[c] += l * lr[c];
            }
        }
        double* gc = Gc.data() + goff[sn];
        for (int r = 0; r < R; ++r)
            for (int c = 0; c < ps; ++c) gc[(size_t)c * R + r] = gr[(size_t)r * ps + c];
    }
    // children lists and pull lists (front row q of a parent <- child update entries, fixed order)
    std::vector<std::vector<int>> kl(nn_);
    for (int sn = 0; sn < nn_; ++sn) if (F.parent[sn] >= 0) kl[F.parent[sn]].push_back(sn);
    std::vector<std::vector<long long>> pull(rows_total);
    for (int par = 0; par < nn_; ++par) {
        const std::vector<int>& pb = F.bnd[par];
        for (int c : kl[par]) {
            for (int a = 0; a < nb[c]; ++a) {
                const int i = F.bnd[c][a];
                int q;
                if (i >= F.beg[par] && i < F.end[par]) q = i - F.beg[par];
                else {
                    auto it = std::lower_bound(pb.begin(), pb.end(), i);
                    if (it == pb.end() || *it != i) throw Error(ERR_NUMERIC, "DirectSolver: inconsistent supernode structure");
                    q = p[par] + (int)(it - pb.begin());
                }
                pull[pull_off[par] + q].push_back(uoff[c] + 3LL * a);
            }
        }
    }
    std::vector<int> pptr(rows_total + 1, 0);
    std::vector<long long> psrc;
    for (int r = 0; r < rows_total; ++r) {
        psrc.insert(psrc.end(), pull[r].begin(), pull[r].end());
        pptr[r + 1] = (int)psrc.size();
    }
    // levels by height and their row tasks
    std::vector<std::vector<int>> hl(F.max_height + 1);
    for (int sn = 0; sn < nn_; ++sn) hl[F.height[sn]].push_back(sn);
    std::vector<Task> tasks;
    levels_.clear();
    kernels_ = 0;
    int max_lds = 0;
    for (auto& l : hl) {
        if (l.empty()) continue;
        Level L;
        int max_rows0 = 0;
        bool any_wave = false;
        std::vector<int> wave;
        for (int sn : l) {
            const bool m0 = p[sn] <= kWaveP && 24 * (p[sn] + nb[sn]) <= kMaxLdsMode0;
            if (m0) max_rows0 = std::max(max_rows0, std::max(p[sn] + nb[sn], p[sn]));
            else { any_wave = true; wave.push_back(sn); }
        }
        L.block = (any_wave || max_rows0 > 128) ? 256 : (max_rows0 > 64 ? 128 : 64);
        // assembly tasks of wave-mode supernodes
        L.asm_first = (int)tasks.size();
        for (int sn : wave) {
            foff[sn] = fo;
            fo += 3LL * (p[sn] + nb[sn]);
            for (int r0 = 0; r0 < p[sn] + nb[sn]; r0 += 256) tasks.push_back({sn, r0, std::min(256, p[sn] + nb[sn] - r0), 1});
        }
        L.asm_count = (int)tasks.size() - L.asm_first;
        L.fwd_first = (int)tasks.size();
        for (int sn : l) {
            const int R = p[sn] + nb[sn];
            if (foff[sn] < 0) {
                for (int r0 = 0; r0 < R; r0 += L.block) tasks.push_back({sn, r0, std::min(L.block, R - r0), 0});
                L.lds_fwd = std::max(L.lds_fwd, 24 * p[sn]);
            } else {
                for (int r0 = 0; r0 < R; r0 += kWaveRowsPerTask) tasks.push_back({sn, r0, std::min(kWaveRowsPerTask, R - r0), 1});
            }
        }
        L.fwd_count = (int)tasks.size() - L.fwd_first;
        L.bwd_first = (int)tasks.size();
        for (int sn : l) {
            if (foff[sn] < 0) {
                for (int j0 = 0; j0 < p[sn]; j0 += L.block) tasks.push_back({sn, j0, std::min(L.block, p[sn] - j0), 0});
                L.lds_bwd = std::max(L.lds_bwd, 24 * (p[sn] + nb[sn]));
            } else {
                for (int j0 = 0; j0 < p[sn]; j0 += kWaveRowsPerTask) tasks.push_back({sn, j0, std::min(kWaveRowsPerTask, p[sn] - j0), 1});
            }
        }
        L.bwd_count = (int)tasks.size() - L.bwd_first;
        max_lds = std::max(max_lds, std::max(L.lds_fwd, L.lds_bwd));
        kernels_ += 2 + (L.asm_count ? 1 : 0);
        levels_.push_back(L);
    }
    beg_.upload(beg, s); p_.upload(p, s); nb_.upload(nb, s);
    bnd_off_.upload(bnd_off, s); bnd_.upload(bnd, s); pull_off_.upload(pull_off, s); pptr_.upload(pptr, s);
    goff_.upload(goff, s); uoff_.upload(uoff, s); foff_.upload(foff, s); psrc_.upload(psrc, s);
    Gr_.upload(Gr, s); Gc_.upload(Gc, s);
    tasks_.upload(tasks, s);
    Y_.alloc(3 * (size_t)n_);
    U_.alloc(std::max<long long>(uo, 3));
    Fg_.alloc(std::max<long long>(fo, 3));
    if (max_lds > 64 * 1024) {   // large fronts: opt in to more than the default 64 KiB of LDS
        for (const void* k : {(const void*)k_fwd<64>, (const void*)k_fwd<128>, (const void*)k_fwd<256>,
                              (const void*)k_bwd<64>, (const void*)k_bwd<128>, (const void*)k_bwd<256>})
            AA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    // algorithmic bytes of one solve: the factor once per sweep (dense triangles + boundary
    // blocks, fp64), b/y/x (24 B per node each way) and the update vectors (write + read)
    bytes_ = 2.0 * 8.0 * (dense + offd) + 4.0 * 24.0 * n_ + 3.0 * 24.0 * bsum;
    AA_HIP(hipStreamSynchronize(s));
}

void DirectSolver::solve(double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    Plan P{beg_.p, p_.p, nb_.p, bnd_off_.p, bnd_.p, pull_off_.p, pptr_.p, psrc_.p,
           goff_.p, uoff_.p, foff_.p, Gr_.p, Gc_.p};
    const Task* T = tasks_.p;
    for (auto& L : levels_) {
        if (L.asm_count)
            hipLaunchKernelGGL(k_asm, dim3(L.asm_count), dim3(256), 0, s, P, T, L.asm_first, b, U_.p, Fg_.p, ctrl, gate_reject);
        switch (L.block) {
            case 64: hipLaunchKernelGGL(k_fwd<64>, dim3(L.fwd_count), dim3(64), L.lds_fwd, s, P, T, L.fwd_first, b, Y_.p, U_.p, Fg_.p, ctrl, gate_reject); break;
            case 128: hipLaunchKernelGGL(k_fwd<128>, dim3(L.fwd_count), dim3(128), L.lds_fwd, s, P, T, L.fwd_first, b, Y_.p, U_.p, Fg_.p, ctrl, gate_reject); break;
            default: hipLaunchKernelGGL(k_fwd<256>, dim3(L.fwd_count), dim3(256), L.lds_fwd, s, P, T, L.fwd_first, b, Y_.p, U_.p, Fg_.p, ctrl, gate_reject); break;
        }
    }
    for (auto it = levels_.rbegin(); it != levels_.rend(); ++it) {
        const Level& L = *it;
        switch (L.block) {
            case 64: hipLaunchKernelGGL(k_bwd<64>, dim3(L.bwd_count), dim3(64), L.lds_bwd, s, P, T, L.bwd_first, Y_.p, x, ctrl, gate_reject); break;
            case 128: hipLaunchKernelGGL(k_bwd<128>, dim3(L.bwd_count), dim3(128), L.lds_bwd, s, P, T, L.bwd_first, Y_.p, x, ctrl, gate_reject); break;
            default: hipLaunchKernelGGL(k_bwd<256>, dim3(L.bwd_count), dim3(256), L.lds_bwd, s, P, T, L.bwd_first, Y_.p, x, ctrl, gate_reject); break;
        }
    }
    AA_CHECK_LAUNCH();
}

}  // namespace aa
