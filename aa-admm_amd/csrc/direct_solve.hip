// GPU multifrontal triangular solves (see direct_solve.hpp).
#include "direct_solve.hpp"

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
    const int* kid_ptr; const int* kids; const int* map_off; const int* map;
    const long long* loff; const long long* boff; const long long* uoff;
    const double* linv_rm; const double* linv_cm; const double* lbp_rm; const double* lbp_cm;
};

// forward: f = [b_P; 0] + sum_children extend_add(u_c);  y_P = Linv f_P;  u = f_B - L_BP y_P
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_fwd_level(Plan P, const int* __restrict__ nodes, int first,
                                                     const double* __restrict__ B, double* __restrict__ Y,
                                                     double* __restrict__ U, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int sn = nodes[first + blockIdx.x];
    const int b0 = P.beg[sn], p = P.p[sn], nb = P.nb[sn];
    double* f = lds;
    double* yl = lds + 3 * (p + nb);
    const int tid = threadIdx.x;
    for (int t = tid; t < 3 * p; t += BLOCK) f[t] = B[3 * (size_t)b0 + t];
    for (int t = tid; t < 3 * nb; t += BLOCK) f[3 * p + t] = 0.0;
    __syncthreads();
    for (int k = P.kid_ptr[sn]; k < P.kid_ptr[sn + 1]; ++k) {   // children in a fixed order
        const int c = P.kids[k], nbc = P.nb[c];
        const int* mp = P.map + P.map_off[c];
        const double* uc = U + P.uoff[c];
        for (int a = tid; a < nbc; a += BLOCK) {
            const int q = 3 * mp[a];
            f[q] += uc[3 * a]; f[q + 1] += uc[3 * a + 1]; f[q + 2] += uc[3 * a + 2];
        }
        __syncthreads();
    }
    const double* Lc = P.linv_cm + P.loff[sn];
    for (int r = tid; r < p; r += BLOCK) {
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int c = 0; c <= r; ++c) {
            const double v = Lc[(size_t)c * p + r];
            a0 += v * f[3 * c]; a1 += v * f[3 * c + 1]; a2 += v * f[3 * c + 2];
        }
        yl[3 * r] = a0; yl[3 * r + 1] = a1; yl[3 * r + 2] = a2;
        const size_t o = 3 * (size_t)(b0 + r);
        Y[o] = a0; Y[o + 1] = a1; Y[o + 2] = a2;
    }
    if (nb == 0) return;
    __syncthreads();
    const double* Bc = P.lbp_cm + P.boff[sn];
    double* us = U + P.uoff[sn];
    for (int a = tid; a < nb; a += BLOCK) {
        double s0 = f[3 * (p + a)], s1 = f[3 * (p + a) + 1], s2 = f[3 * (p + a) + 2];
#pragma unroll 8
        for (int j = 0; j < p; ++j) {
            const double v = Bc[(size_t)j * nb + a];
            s0 -= v * yl[3 * j]; s1 -= v * yl[3 * j + 1]; s2 -= v * yl[3 * j + 2];
        }
        us[3 * a] = s0; us[3 * a + 1] = s1; us[3 * a + 2] = s2;
    }
}

// backward: t = y_P - L_BP^T x_B ;  x_P = Linv^T t
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_bwd_level(Plan P, const int* __restrict__ nodes, int first,
                                                     const double* __restrict__ Y, double* __restrict__ X,
                                                     const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int sn = nodes[first + blockIdx.x];
    const int b0 = P.beg[sn], p = P.p[sn], nb = P.nb[sn];
    double* xb = lds;
    double* t = lds + 3 * nb;
    const int tid = threadIdx.x;
    const int* bi = P.bnd + P.bnd_off[sn];
    for (int a = tid; a < nb; a += BLOCK) {
        const size_t q = 3 * (size_t)bi[a];
        xb[3 * a] = X[q]; xb[3 * a + 1] = X[q + 1]; xb[3 * a + 2] = X[q + 2];
    }
    __syncthreads();
    const double* Br = P.lbp_rm + P.boff[sn];
    for (int j = tid; j < p; j += BLOCK) {
        const size_t o = 3 * (size_t)(b0 + j);
        double s0 = Y[o], s1 = Y[o + 1], s2 = Y[o + 2];
#pragma unroll 8
        for (int a = 0; a < nb; ++a) {
            const double v = Br[(size_t)a * p + j];
            s0 -= v * xb[3 * a]; s1 -= v * xb[3 * a + 1]; s2 -= v * xb[3 * a + 2];
        }
        t[3 * j] = s0; t[3 * j + 1] = s1; t[3 * j + 2] = s2;
    }
    __syncthreads();
    const double* Lr = P.linv_rm + P.loff[sn];
    for (int j = tid; j < p; j += BLOCK) {
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int k = j; k < p; ++k) {
            const double v = Lr[(size_t)k * p + j];
            a0 += v * t[3 * k]; a1 += v * t[3 * k + 1]; a2 += v * t[3 * k + 2];
        }
        const size_t o = 3 * (size_t)(b0 + j);
        X[o] = a0; X[o + 1] = a1; X[o + 2] = a2;
    }
}

// ------------------------------------------------------------------ big supernodes (multi-WG)
constexpr int kBigRowsPerWG = 4;   // one row per wave: more waves, more loads in flight

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// f_q = [b_P; 0]_q + sum of the children's update-vector entries that land on front row q
__global__ __launch_bounds__(256) void k_big_gather(int b0, int p, int nf, const int* __restrict__ pptr,
                                                    const long long* __restrict__ psrc, const double* __restrict__ B,
                                                    const double* __restrict__ U, double* __restrict__ Fg,
                                                    const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nf) return;
    double a0 = 0, a1 = 0, a2 = 0;
    if (q < p) { const size_t o = 3 * (size_t)(b0 + q); a0 = B[o]; a1 = B[o + 1]; a2 = B[o + 2]; }
    for (int e = pptr[q]; e < pptr[q + 1]; ++e) {
        const double* u = U + psrc[e];
        a0 += u[0]; a1 += u[1]; a2 += u[2];
    }
    Fg[3 * q] = a0; Fg[3 * q + 1] = a1; Fg[3 * q + 2] = a2;
}

// y_r = sum_{c<=r} Linv(r,c) f_c     (row-major Linv: lanes read a contiguous row)
__global__ __launch_bounds__(256) void k_big_y(int b0, int p, const double* __restrict__ L, const double* __restrict__ Fg,
                                               double* __restrict__ Y, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int r = blockIdx.x * kBigRowsPerWG + wid; r < min(p, (int)(blockIdx.x + 1) * kBigRowsPerWG); r += 4) {
        const double* row = L + (size_t)r * p;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int c = lane; c <= r; c += 64) {
            const double v = row[c];
            a0 += v * Fg[3 * c]; a1 += v * Fg[3 * c + 1]; a2 += v * Fg[3 * c + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) { const size_t o = 3 * (size_t)(b0 + r); Y[o] = a0; Y[o + 1] = a1; Y[o + 2] = a2; }
    }
}

// u_a = f_{p+a} - sum_j LBP(a,j) y_j   (row-major LBP)
__global__ __launch_bounds__(256) void k_big_u(int b0, int p, int nb, const double* __restrict__ LB,
                                               const double* __restrict__ Fg, const double* __restrict__ Y,
                                               double* __restrict__ Uo, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int a = blockIdx.x * kBigRowsPerWG + wid; a < min(nb, (int)(blockIdx.x + 1) * kBigRowsPerWG); a += 4) {
        const double* row = LB + (size_t)a * p;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int j = lane; j < p; j += 64) {
            const double v = row[j];
            const size_t o = 3 * (size_t)(b0 + j);
            a0 += v * Y[o]; a1 += v * Y[o + 1]; a2 += v * Y[o + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) {
            const int q = 3 * (p + a);
            Uo[3 * a] = Fg[q] - a0; Uo[3 * a + 1] = Fg[q + 1] - a1; Uo[3 * a + 2] = Fg[q + 2] - a2;
        }
    }
}

// t_j = y_j - sum_a LBP(a,j) x_{bnd a}   (LBP^T row-major = the column-major copy)
__global__ __launch_bounds__(256) void k_big_t(int b0, int p, int nb, const double* __restrict__ LBt,
                                               const int* __restrict__ bi, const double* __restrict__ Y,
                                               const double* __restrict__ X, double* __restrict__ Tg,
                                               const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int j = blockIdx.x * kBigRowsPerWG + wid; j < min(p, (int)(blockIdx.x + 1) * kBigRowsPerWG); j += 4) {
        const double* row = LBt + (size_t)j * nb;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int a = lane; a < nb; a += 64) {
            const double v = row[a];
            const size_t q = 3 * (size_t)bi[a];
            a0 += v * X[q]; a1 += v * X[q + 1]; a2 += v * X[q + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) {
            const size_t o = 3 * (size_t)(b0 + j);
            Tg[3 * j] = Y[o] - a0; Tg[3 * j + 1] = Y[o + 1] - a1; Tg[3 * j + 2] = Y[o + 2] - a2;
        }
    }
}

// x_j = sum_{k>=j} Linv(k,j) t_k   (Linv^T row-major = the column-major copy)
__global__ __launch_bounds__(256) void k_big_x(int b0, int p, const double* __restrict__ Lt, const double* __restrict__ Tg,
                                               double* __restrict__ X, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int j = blockIdx.x * kBigRowsPerWG + wid; j < min(p, (int)(blockIdx.x + 1) * kBigRowsPerWG); j += 4) {
        const double* row = Lt + (size_t)j * p;
        double a0 = 0, a1 = 0, a2 = 0;
#pragma unroll 8
        for (int k = j + lane; k < p; k += 64) {
            const double v = row[k];
            a0 += v * Tg[3 * k]; a1 += v * Tg[3 * k + 1]; a2 += v * Tg[3 * k + 2];
        }
        a0 = wsum(a0); a1 = wsum(a1); a2 = wsum(a2);
        if (lane == 0) { const size_t o = 3 * (size_t)(b0 + j); X[o] = a0; X[o + 1] = a1; X[o + 2] = a2; }
    }
}

}  // namespace

void DirectSolver::build(const SupernodalFactor& F, hipStream_t s) {
    n_ = F.n;
    nn_ = F.n_nodes;
    nnz_L_ = F.nnz_L;
    std::vector<int> beg(nn_), p(nn_), nb(nn_), bnd_off(nn_), bnd;
    std::vector<long long> loff(nn_), boff(nn_), uoff(nn_);
    std::vector<double> linv_rm, linv_cm, lbp_rm, lbp_cm;
    long long lo = 0, bo = 0, uo = 0;
    double dense = 0, offd = 0, bsum = 0;
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = F.end[sn] - F.beg[sn], nbs = (int)F.bnd[sn].size();
        beg[sn] = F.beg[sn]; p[sn] = ps; nb[sn] = nbs;
        loff[sn] = lo; boff[sn] = bo; uoff[sn] = uo;
        bnd_off[sn] = (int)bnd.size();
        bnd.insert(bnd.end(), F.bnd[sn].begin(), F.bnd[sn].end());
        linv_rm.insert(linv_rm.end(), F.Linv[sn].begin(), F.Linv[sn].end());
        for (int c = 0; c < ps; ++c)
            for (int r = 0; r < ps; ++r) linv_cm.push_back(F.Linv[sn][(size_t)r * ps + c]);
        lbp_rm.insert(lbp_rm.end(), F.LBP[sn].begin(), F.LBP[sn].end());
        for (int j = 0; j < ps; ++j)
            for (int a = 0; a < nbs; ++a) lbp_cm.push_back(F.LBP[sn][(size_t)a * ps + j]);
        lo += (long long)ps * ps;
        bo += (long long)ps * nbs;
        uo += 3LL * nbs;
        dense += 0.5 * ps * (ps + 1.0);
        offd += (double)ps * nbs;
        bsum += nbs;
    }
    // children lists and extend-add maps (child boundary -> parent front positions)
    std::vector<std::vector<int>> kl(nn_);
    for (int sn = 0; sn < nn_; ++sn) if (F.parent[sn] >= 0) kl[F.parent[sn]].push_back(sn);
    std::vector<int> kid_ptr(nn_ + 1, 0), kids, map_off(nn_, 0), map;
    for (int sn = 0; sn < nn_; ++sn) {
        kids.insert(kids.end(), kl[sn].begin(), kl[sn].end());
        kid_ptr[sn + 1] = (int)kids.size();
    }
    for (int c = 0; c < nn_; ++c) {
        map_off[c] = (int)map.size();
        const int par = F.parent[c];
        if (par < 0) continue;
        const std::vector<int>& pb = F.bnd[par];
        for (int i : F.bnd[c]) {
            if (i >= F.beg[par] && i < F.end[par]) map.push_back(i - F.beg[par]);
            else {
                auto it = std::lower_bound(pb.begin(), pb.end(), i);
                if (it == pb.end() || *it != i) throw Error(ERR_NUMERIC, "DirectSolver: inconsistent supernode structure");
                map.push_back(p[par] + (int)(it - pb.begin()));
            }
        }
    }
    // levels by height; small supernodes -> one kernel per level, big ones -> multi-WG path
    std::vector<std::vector<int>> hl(F.max_height + 1);
    for (int sn = 0; sn < nn_; ++sn) hl[F.height[sn]].push_back(sn);
    std::vector<int> lvl_nodes, big_pptr;
    std::vector<long long> big_psrc;
    long long foff = 0, toff = 0;
    levels_.clear();
    bigs_.clear();
    kernels_ = 0;
    for (auto& l : hl) {
        if (l.empty()) continue;
        int rows = 0, lf = 0, lb = 0;
        Level L{};
        L.first = (int)lvl_nodes.size();
        for (int sn : l) {
            if (p[sn] > kBigP || p[sn] + nb[sn] > kMaxFront) {
                Big B{sn, beg[sn], p[sn], nb[sn], bnd_off[sn], (int)big_pptr.size(), loff[sn], boff[sn], uoff[sn], foff, toff};
                // pull lists: for every front row q, the children's update entries landing on it
                std::vector<std::vector<long long>> pull(p[sn] + nb[sn]);
                for (int c : kl[sn]) {
                    const int* mp = &map[map_off[c]];
                    for (int a2 = 0; a2 < nb[c]; ++a2) pull[mp[a2]].push_back(uoff[c] + 3LL * a2);
                }
                for (auto& q : pull) { big_pptr.push_back((int)big_psrc.size()); big_psrc.insert(big_psrc.end(), q.begin(), q.end()); }
                big_pptr.push_back((int)big_psrc.size());
                foff += 3LL * (p[sn] + nb[sn]);
                toff += 3LL * p[sn];
                L.big.push_back((int)bigs_.size());
                bigs_.push_back(B);
                kernels_ += 5;
                continue;
            }
            lvl_nodes.push_back(sn);
            rows = std::max(rows, std::max(p[sn], nb[sn]));
            lf = std::max(lf, 24 * (2 * p[sn] + nb[sn]));
            lb = std::max(lb, 24 * (p[sn] + nb[sn]));
        }
        L.count = (int)lvl_nodes.size() - L.first;
        L.block = rows <= 64 ? 64 : (rows <= 128 ? 128 : 256);
        L.lds_fwd = lf;
        L.lds_bwd = lb;
        if (L.count) kernels_ += 2;
        levels_.push_back(L);
    }
    big_pptr_.upload(big_pptr, s);
    big_psrc_.upload(big_psrc, s);
    Fg_.alloc(std::max<long long>(foff, 3));
    Tg_.alloc(std::max<long long>(toff, 3));
    beg_.upload(beg, s); p_.upload(p, s); nb_.upload(nb, s); bnd_off_.upload(bnd_off, s); bnd_.upload(bnd, s);
    kid_ptr_.upload(kid_ptr, s); kids_.upload(kids, s); map_off_.upload(map_off, s); map_.upload(map, s);
    lvl_nodes_.upload(lvl_nodes, s);
    loff_.upload(loff, s); boff_.upload(boff, s); uoff_.upload(uoff, s);
    linv_rm_.upload(linv_rm, s); linv_cm_.upload(linv_cm, s); lbp_rm_.upload(lbp_rm, s); lbp_cm_.upload(lbp_cm, s);
    Y_.alloc(3 * (size_t)n_);
    U_.alloc(std::max<long long>(uo, 3));
    int max_lds = 0;
    for (auto& L : levels_) max_lds = std::max(max_lds, std::max(L.lds_fwd, L.lds_bwd));
    if (max_lds > 64 * 1024) {   // large fronts: opt in to the full 160 KiB LDS of a CU
        AA_HIP(hipFuncSetAttribute((const void*)k_fwd_level<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        AA_HIP(hipFuncSetAttribute((const void*)k_bwd_level<256>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    // algorithmic bytes of one solve: the factor once per sweep (dense triangles + boundary
    // blocks, fp64), b/y/x (24 B per node each way) and the update vectors (write + read)
    bytes_ = 2.0 * 8.0 * (dense + offd) + 4.0 * 24.0 * n_ + 3.0 * 24.0 * bsum;
    AA_HIP(hipStreamSynchronize(s));
}

void DirectSolver::solve(double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    Plan P{beg_.p, p_.p, nb_.p, bnd_off_.p, bnd_.p, kid_ptr_.p, kids_.p, map_off_.p, map_.p,
           loff_.p, boff_.p, uoff_.p, linv_rm_.p, linv_cm_.p, lbp_rm_.p, lbp_cm_.p};
    auto nblk = [](int rows) { return dim3((rows + kBigRowsPerWG - 1) / kBigRowsPerWG); };
    for (auto& L : levels_) {
        if (L.count) {
            switch (L.block) {
                case 64: hipLaunchKernelGGL(k_fwd_level<64>, dim3(L.count), dim3(64), L.lds_fwd, s, P, lvl_nodes_.p, L.first, b, Y_.p, U_.p, ctrl, gate_reject); break;
                case 128: hipLaunchKernelGGL(k_fwd_level<128>, dim3(L.count), dim3(128), L.lds_fwd, s, P, lvl_nodes_.p, L.first, b, Y_.p, U_.p, ctrl, gate_reject); break;
                default: hipLaunchKernelGGL(k_fwd_level<256>, dim3(L.count), dim3(256), L.lds_fwd, s, P, lvl_nodes_.p, L.first, b, Y_.p, U_.p, ctrl, gate_reject); break;
            }
        }
        for (int bi : L.big) {
            const Big& B = bigs_[bi];
            double* Fg = Fg_.p + B.foff;
            const int nf = B.p + B.nb;
            hipLaunchKernelGGL(k_big_gather, dim3((nf + 255) / 256), dim3(256), 0, s, B.b0, B.p, nf, big_pptr_.p + B.pptr_off,
                               big_psrc_.p, b, U_.p, Fg, ctrl, gate_reject);
            hipLaunchKernelGGL(k_big_y, nblk(B.p), dim3(256), 0, s, B.b0, B.p, linv_rm_.p + B.loff, Fg, Y_.p, ctrl, gate_reject);
            if (B.nb)
                hipLaunchKernelGGL(k_big_u, nblk(B.nb), dim3(256), 0, s, B.b0, B.p, B.nb, lbp_rm_.p + B.boff, Fg, Y_.p,
                                   U_.p + B.uoff, ctrl, gate_reject);
        }
    }
    for (auto it = levels_.rbegin(); it != levels_.rend(); ++it) {
        const Level& L = *it;
        for (int bi : L.big) {
            const Big& B = bigs_[bi];
            double* Tg = Tg_.p + B.toff;
            hipLaunchKernelGGL(k_big_t, nblk(B.p), dim3(256), 0, s, B.b0, B.p, B.nb, lbp_cm_.p + B.boff, bnd_.p + B.bnd_off,
                               Y_.p, x, Tg, ctrl, gate_reject);
            hipLaunchKernelGGL(k_big_x, nblk(B.p), dim3(256), 0, s, B.b0, B.p, linv_cm_.p + B.loff, Tg, x, ctrl, gate_reject);
        }
        if (L.count) {
            switch (L.block) {
                case 64: hipLaunchKernelGGL(k_bwd_level<64>, dim3(L.count), dim3(64), L.lds_bwd, s, P, lvl_nodes_.p, L.first, Y_.p, x, ctrl, gate_reject); break;
                case 128: hipLaunchKernelGGL(k_bwd_level<128>, dim3(L.count), dim3(128), L.lds_bwd, s, P, lvl_nodes_.p, L.first, Y_.p, x, ctrl, gate_reject); break;
                default: hipLaunchKernelGGL(k_bwd_level<256>, dim3(L.count), dim3(256), L.lds_bwd, s, P, lvl_nodes_.p, L.first, Y_.p, x, ctrl, gate_reject); break;
            }
        }
    }
    AA_CHECK_LAUNCH();
}

}  // namespace aa
