// GPU supernodal triangular solves (see direct_solve.hpp).
#include "direct_solve.hpp"

#include <algorithm>

namespace aa {

namespace {

constexpr int kRowsPerItem = 16;   // 4 waves x 4 rows

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

__device__ __forceinline__ bool solve_gated(const Ctrl* c, int gate_reject) {
    if (!c) return false;
    if (c->done) return true;
    return gate_reject && !c->reject;
}

// forward, sparse part: B[i] -= sum_k fval[k] * Y[fcol[k]]
__global__ __launch_bounds__(256) void k_fwd_sparse(const SolveItem* __restrict__ items, int item0,
                                                    const int* __restrict__ beg, const int* __restrict__ fptr,
                                                    const int* __restrict__ fcol, const double* __restrict__ fval,
                                                    double* __restrict__ B, const double* __restrict__ Y,
                                                    const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const SolveItem it = items[item0 + blockIdx.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b0 = beg[it.node];
    for (int r = it.r0 + wid; r < it.r1; r += 4) {
        const int i = b0 + r;
        double a0 = 0, a1 = 0, a2 = 0;
        for (int k = fptr[i] + lane; k < fptr[i + 1]; k += 64) {
            const double v = fval[k];
            const size_t j = 3 * (size_t)fcol[k];
            a0 += v * Y[j]; a1 += v * Y[j + 1]; a2 += v * Y[j + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) { B[3 * (size_t)i] -= a0; B[3 * (size_t)i + 1] -= a1; B[3 * (size_t)i + 2] -= a2; }
    }
}

// forward, dense part: Y[P] = Linv * B[P]
__global__ __launch_bounds__(256) void k_fwd_dense(const SolveItem* __restrict__ items, int item0,
                                                   const int* __restrict__ beg, const int* __restrict__ pp,
                                                   const long long* __restrict__ loff, const double* __restrict__ linv,
                                                   const double* __restrict__ B, double* __restrict__ Y,
                                                   const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const SolveItem it = items[item0 + blockIdx.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b0 = beg[it.node], p = pp[it.node];
    const double* L = linv + loff[it.node];
    for (int r = it.r0 + wid; r < it.r1; r += 4) {
        double a0 = 0, a1 = 0, a2 = 0;
        for (int k = lane; k <= r; k += 64) {
            const double v = L[(size_t)r * p + k];
            const size_t j = 3 * (size_t)(b0 + k);
            a0 += v * B[j]; a1 += v * B[j + 1]; a2 += v * B[j + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) { const size_t o = 3 * (size_t)(b0 + r); Y[o] = a0; Y[o + 1] = a1; Y[o + 2] = a2; }
    }
}

// backward, boundary part: T[j] = Y[j] - sum_a LBP(a,j) X[bnd[a]]   (T stored in B)
__global__ __launch_bounds__(256) void k_bwd_sparse(const SolveItem* __restrict__ items, int item0,
                                                    const int* __restrict__ beg, const int* __restrict__ nbv,
                                                    const long long* __restrict__ boff, const double* __restrict__ lbpt,
                                                    const int* __restrict__ bnd_off, const int* __restrict__ bnd,
                                                    const double* __restrict__ Y, const double* __restrict__ X,
                                                    double* __restrict__ T, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const SolveItem it = items[item0 + blockIdx.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b0 = beg[it.node], nb = nbv[it.node];
    const double* L = lbpt + boff[it.node];
    const int* bi = bnd + bnd_off[it.node];
    for (int r = it.r0 + wid; r < it.r1; r += 4) {
        double a0 = 0, a1 = 0, a2 = 0;
        for (int k = lane; k < nb; k += 64) {
            const double v = L[(size_t)r * nb + k];
            const size_t j = 3 * (size_t)bi[k];
            a0 += v * X[j]; a1 += v * X[j + 1]; a2 += v * X[j + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) {
            const size_t o = 3 * (size_t)(b0 + r);
            T[o] = Y[o] - a0; T[o + 1] = Y[o + 1] - a1; T[o + 2] = Y[o + 2] - a2;
        }
    }
}

// backward, dense part: X[P] = Linv^T T[P]
__global__ __launch_bounds__(256) void k_bwd_dense(const SolveItem* __restrict__ items, int item0,
                                                   const int* __restrict__ beg, const int* __restrict__ pp,
                                                   const long long* __restrict__ loff, const double* __restrict__ linvT,
                                                   const double* __restrict__ T, double* __restrict__ X,
                                                   const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const SolveItem it = items[item0 + blockIdx.x];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int b0 = beg[it.node], p = pp[it.node];
    const double* L = linvT + loff[it.node];
    for (int r = it.r0 + wid; r < it.r1; r += 4) {
        double a0 = 0, a1 = 0, a2 = 0;
        for (int k = r + lane; k < p; k += 64) {
            const double v = L[(size_t)r * p + k];
            const size_t j = 3 * (size_t)(b0 + k);
            a0 += v * T[j]; a1 += v * T[j + 1]; a2 += v * T[j + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) { const size_t o = 3 * (size_t)(b0 + r); X[o] = a0; X[o + 1] = a1; X[o + 2] = a2; }
    }
}

}  // namespace

void DirectSolver::build(const SupernodalFactor& F, hipStream_t s) {
    n_ = F.n;
    nn_ = F.n_nodes;
    nnz_L_ = F.nnz_L;
    std::vector<int> beg(nn_), p(nn_), nb(nn_), bnd_off(nn_), bnd;
    std::vector<long long> loff(nn_), boff(nn_);
    std::vector<double> linv, linvT, lbpt;
    long long lo = 0, bo = 0;
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = F.end[sn] - F.beg[sn], nbs = (int)F.bnd[sn].size();
        beg[sn] = F.beg[sn]; p[sn] = ps; nb[sn] = nbs;
        loff[sn] = lo; boff[sn] = bo;
        bnd_off[sn] = (int)bnd.size();
        bnd.insert(bnd.end(), F.bnd[sn].begin(), F.bnd[sn].end());
        linv.insert(linv.end(), F.Linv[sn].begin(), F.Linv[sn].end());
        for (int r = 0; r < ps; ++r)
            for (int c = 0; c < ps; ++c) linvT.push_back(F.Linv[sn][(size_t)c * ps + r]);
        for (int j = 0; j < ps; ++j)
            for (int a = 0; a < nbs; ++a) lbpt.push_back(F.LBP[sn][(size_t)a * ps + j]);
        lo += (long long)ps * ps;
        bo += (long long)ps * nbs;
    }
    // forward CSR of the off-diagonal-block entries, by row
    std::vector<int> cnt(n_ + 1, 0);
    for (int sn = 0; sn < nn_; ++sn)
        for (int i : F.bnd[sn]) cnt[i + 1] += F.end[sn] - F.beg[sn];
    for (int i = 0; i < n_; ++i) cnt[i + 1] += cnt[i];
    std::vector<int> fcol(cnt[n_]), fill(cnt.begin(), cnt.end() - 1);
    std::vector<double> fval(cnt[n_]);
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = F.end[sn] - F.beg[sn];
        for (size_t a = 0; a < F.bnd[sn].size(); ++a) {
            const int i = F.bnd[sn][a];
            for (int j = 0; j < ps; ++j) {
                fcol[fill[i]] = F.beg[sn] + j;
                fval[fill[i]++] = F.LBP[sn][a * ps + j];
            }
        }
    }
    // level schedule by height
    n_levels_ = F.max_height + 1;
    std::vector<std::vector<SolveItem>> lv(n_levels_);
    for (int sn = 0; sn < nn_; ++sn)
        for (int r = 0; r < p[sn]; r += kRowsPerItem)
            lv[F.height[sn]].push_back(SolveItem{sn, r, std::min(p[sn], r + kRowsPerItem), 0});
    std::vector<SolveItem> items;
    level_off_.assign(1, 0);
    for (auto& l : lv) { items.insert(items.end(), l.begin(), l.end()); level_off_.push_back((int)items.size()); }

    beg_.upload(beg, s); p_.upload(p, s); nb_.upload(nb, s); bnd_off_.upload(bnd_off, s); bnd_.upload(bnd, s);
    linv_off_.upload(loff, s); lbp_off_.upload(boff, s);
    linv_.upload(linv, s); linvT_.upload(linvT, s); lbpt_.upload(lbpt, s);
    fptr_.upload(cnt, s); fcol_.upload(fcol, s); fval_.upload(fval, s);
    items_.upload(items, s);
    Y_.alloc(3 * (size_t)n_);
    // algorithmic bytes: every factor entry read once per sweep (12 B: value + index for the sparse
    // parts; 8 B for dense blocks, which are read as lower/upper triangles), plus the 3-RHS vectors.
    double dense = 0;
    for (int sn = 0; sn < nn_; ++sn) dense += 0.5 * p[sn] * (p[sn] + 1.0);
    const double offd = (double)fcol.size();
    bytes_ = 2.0 * (8.0 * dense + 12.0 * offd) + 2.0 * 4.0 * 24.0 * n_;
    AA_HIP(hipStreamSynchronize(s));
}

void DirectSolver::solve(double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    for (int l = 0; l < n_levels_; ++l) {
        const int i0 = level_off_[l], ni = level_off_[l + 1] - i0;
        if (!ni) continue;
        hipLaunchKernelGGL(k_fwd_sparse, dim3(ni), dim3(256), 0, s, items_.p, i0, beg_.p, fptr_.p, fcol_.p, fval_.p, b, Y_.p, ctrl, gate_reject);
        hipLaunchKernelGGL(k_fwd_dense, dim3(ni), dim3(256), 0, s, items_.p, i0, beg_.p, p_.p, linv_off_.p, linv_.p, b, Y_.p, ctrl, gate_reject);
    }
    for (int l = n_levels_ - 1; l >= 0; --l) {
        const int i0 = level_off_[l], ni = level_off_[l + 1] - i0;
        if (!ni) continue;
        hipLaunchKernelGGL(k_bwd_sparse, dim3(ni), dim3(256), 0, s, items_.p, i0, beg_.p, nb_.p, lbp_off_.p, lbpt_.p, bnd_off_.p, bnd_.p, Y_.p, x, b, ctrl, gate_reject);
        hipLaunchKernelGGL(k_bwd_dense, dim3(ni), dim3(256), 0, s, items_.p, i0, beg_.p, p_.p, linv_off_.p, linvT_.p, b, x, ctrl, gate_reject);
    }
    AA_CHECK_LAUNCH();
}

}  // namespace aa
