// GPU supernodal triangular solves (see direct_solve.hpp).
#include "direct_solve.hpp"
#include "solve_plan.hpp"

#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>

namespace aa {

namespace {

__device__ __forceinline__ bool solve_gated(const Ctrl* c, int gate_reject) {
    if (!c) return false;
    if (c->done) return true;
    return gate_reject && !c->reject;
}

using Task = DirectSolver::Task;

// Split-K hand-off inside one launch (MI355X_MICROARCH.md "Valid forms"; the publish recipe of
// cdna_hip_programming.md Guideline 16): partials are stored write-through (sc1: relaxed
// agent-scope 8-B atomic stores, so no release / L2 write-back), the storing wave drains
// (s_waitcnt vmcnt(0)), then one lane adds to the block's counter; the workgroup whose add
// returns nt-1 takes ONE agent acquire and reads the partials with plain (pipelined) loads.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// storing wave: drain its sc1 stores, then lane 0 adds; returns true (wave-uniform) in the
// workgroup whose add completes the count
__device__ __forceinline__ bool arrive_last(int* cnt, int nt, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0, 64);
    return (int)prev == nt - 1;
}

// Factor loads (NT = DirectSolver::nt_): a factor streamed past the Infinity Cache (both sweeps'
// copies > kNtBytes: C3, C4, C5) is read with non-temporal loads -- each entry is read once per
// sweep by exactly one workgroup (MI355X_MICROARCH.md, nt-weights): C4 two-set solve 753 -> 741 us,
// C3 1 138 -> 1 207 it/s. A factor that stays resident (C2, ~120 MB working set) keeps plain
// loads: nt there costs its MALL hits (6 774 -> 5 801 it/s).
typedef double dbl2v __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double ld_f(const double* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ double2 ld_f2(const double2* p) {
    if constexpr (NT) {
        const dbl2v v = __builtin_nontemporal_load(reinterpret_cast<const dbl2v*>(p));
        return make_double2(v.x, v.y);
    } else {
        return *p;
    }
}

// Thread-per-row / thread-per-column factor products:
// a[k] += sum_{i0 <= i < i1} G[i * stride] * V[NR * i + k], i ascending (one fused multiply-add
// chain per k, the order of a plain loop). dot_rows: `#pragma unroll 8` -- a remainder loop of up to
// 7 serial load -> use steps follows the unrolled bodies. dot_rows_chunk: chunks of CH whose loads
// are issued together (indices clamped to i1 - 1, the extra terms adding 0), so a row costs
// ceil(n / CH) round trips and no serial remainder. Measured per call site (A/B builds, phase
// clocks): the fused subtrees' one-set forward rows -12 us per sweep with chunks of 8 (C3 solve
// 240 -> 236 us); the two-set (6 RHS) forward rows, the fused backward segments and the row-task
// kernels are slower chunked (C4 two-set solve 738 -> 763 us with the fused forward chunked,
// 734 -> 769 with every loop chunked), so they keep the unrolled loop.
template <int NR, bool NT>
__device__ __forceinline__ void dot_rows(const double* __restrict__ G, size_t stride, int i0, int i1,
                                         const double* __restrict__ V, double* a) {
#pragma unroll 8
    for (int i = i0; i < i1; ++i) {
        const double g = ld_f<NT>(G + (size_t)i * stride);
#pragma unroll
        for (int k = 0; k < NR; ++k) a[k] += g * V[NR * i + k];
    }
}
#ifndef AA_ROW_CHUNK
#define AA_ROW_CHUNK 8
#endif
template <int NR, bool NT, int CH = AA_ROW_CHUNK>
__device__ __forceinline__ void dot_rows_chunk(const double* __restrict__ G, size_t stride, int i0, int i1,
                                               const double* __restrict__ V, double* a) {
    for (int c0 = i0; c0 < i1; c0 += CH) {
        double g[CH];
#pragma unroll
        for (int q = 0; q < CH; ++q) g[q] = ld_f<NT>(G + (size_t)min(c0 + q, i1 - 1) * stride);
        __builtin_amdgcn_sched_barrier(0);   // every load of the chunk issued before the first use
        // no branch per term (the compiler would sink a skipped term's load into it, after the
        // other terms' wait): a term past i1 adds 0 * V[i1 - 1] (finite), which leaves a unchanged
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const bool in = c0 + q < i1;
            const double gq = in ? g[q] : 0.0;
            const int iv = in ? c0 + q : i1 - 1;
#pragma unroll
            for (int k = 0; k < NR; ++k) a[k] += gq * V[NR * iv + k];
        }
    }
}

// chunked gathers without serial remainder loops (front rows, split-K reductions); 0 = the plain
// loops (A/B)
#ifndef AA_FRONT_CHUNK
#define AA_FRONT_CHUNK 1
#endif
// a split-K block's partial sums: b[m] += q[k * STRIDE + m] over its nt tiles, in tile order, in
// chunks of CH tiles whose loads are issued together (tile index clamped, the extra terms adding 0)
// -- no serial remainder loop
template <int W, int STRIDE, int CH = (W >= 12 ? 2 : (W >= 6 ? 4 : 8))>
__device__ __forceinline__ void red_tiles(const double* __restrict__ q, int nt, double* b) {
#if AA_FRONT_CHUNK
    for (int k0 = 0; k0 < nt; k0 += CH) {
        double t[CH][W];
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int m = 0; m < W; ++m) t[c][m] = q[(size_t)min(k0 + c, nt - 1) * STRIDE + m];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int m = 0; m < W; ++m) b[m] += k0 + c < nt ? t[c][m] : 0.0;
    }
#else
#pragma unroll 4
    for (int k = 0; k < nt; ++k, q += STRIDE)
#pragma unroll
        for (int m = 0; m < W; ++m) b[m] += q[m];
#endif
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// Right-hand-side sets. NR = 3: one solve (the x, y, z columns of A_s X = B). NR = 6: two
// independent solves batched into one pass, so the factor is streamed from HBM once for both
// (the Z variant's main solve and the previous iteration's combined-residual solve). The
// caller's vectors b and x stay 3-interleaved per node, one array per set (P0, P1); the
// solver's own vectors (Y, U, split-K partials, LDS) are NR-interleaved, and every offset the
// host built for 3 columns is scaled by NR / 3 on the device. Each column's sums run in the
// same order for NR = 3 and 6, so a batched solve is bit-identical to two single ones.
template <int NR>
__device__ __forceinline__ void ld_ext(const double* __restrict__ P0, const double* __restrict__ P1, size_t node,
                                       double* a) {
    const size_t o = 3 * node;
    a[0] = P0[o]; a[1] = P0[o + 1]; a[2] = P0[o + 2];
    if constexpr (NR == 6) { a[3] = P1[o]; a[4] = P1[o + 1]; a[5] = P1[o + 2]; }
}
template <int NR>
__device__ __forceinline__ void st_ext(double* P0, double* P1, size_t node, const double* a) {
    const size_t o = 3 * node;
    P0[o] = a[0]; P0[o + 1] = a[1]; P0[o + 2] = a[2];
    if constexpr (NR == 6) { P1[o] = a[3]; P1[o + 1] = a[4]; P1[o + 2] = a[5]; }
}
template <int NR>
__device__ __forceinline__ void zero(double* a) {
#pragma unroll
    for (int k = 0; k < NR; ++k) a[k] = 0;
}

// front row q of a supernode (any record with beg, p, ell_w, ell_off): [b_P ; 0]_q + the
// children's update entries landing on it (ELL pull list: ell_w offsets into U per row, -1 =
// none; fixed order -> deterministic)
// (ext_off: B0 / B1 hold rows from ext_off on -- the partitioned top's summed front)
// CHUNK (the default): the pulls in issued-together chunks, for gathers followed by a barrier (the
// LDS front slices); false: the plain loop, for a boundary row's own front value gathered ahead of
// its factor stream (chunked, its waits would come before the stream's first loads)
template <int NR, bool CHUNK = true, class N>
__device__ __forceinline__ void front_row(const N& t, int q, const long long* __restrict__ ell,
                                          const double* __restrict__ B0, const double* __restrict__ B1,
                                          const double* __restrict__ U, double* a, int ext_off = 0) {
    zero<NR>(a);
    if (q < t.p) ld_ext<NR>(B0, B1, (size_t)(t.beg + q - ext_off), a);
    const long long* e = ell + t.ell_off + (size_t)q * t.ell_w;
#if AA_FRONT_CHUNK
    if constexpr (CHUNK) {
    // the row's pull offsets, then its update entries, each group issued together (chunks of FC,
    // offsets clamped to the row's last, absent ones reading U[0] and adding 0): two round trips
    // per chunk instead of two per pull; the same sums in the same order
    constexpr int FC = NR == 6 ? 2 : 4;   // 6 RHS: fewer rows in flight (registers beside the tile's factor chunks)
    for (int k0 = 0; k0 < t.ell_w; k0 += FC) {
        long long o[FC];
#pragma unroll
        for (int m = 0; m < FC; ++m) o[m] = e[min(k0 + m, t.ell_w - 1)];
        __builtin_amdgcn_sched_barrier(0);
        double u[FC][NR];
#pragma unroll
        for (int m = 0; m < FC; ++m) {
            const bool in = k0 + m < t.ell_w && o[m] >= 0;
            o[m] = in ? o[m] : -1;
            const double* up = U + (NR / 3) * (in ? o[m] : 0);
#pragma unroll
            for (int j = 0; j < NR; ++j) u[m][j] = up[j];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < FC; ++m)
#pragma unroll
            for (int j = 0; j < NR; ++j) a[j] += o[m] >= 0 ? u[m][j] : 0.0;
    }
    return;
    }
#endif
    for (int k = 0; k < t.ell_w; ++k) {
        const long long o = e[k];
        if (o >= 0) {
            const double* u = U + (NR / 3) * o;
#pragma unroll
            for (int j = 0; j < NR; ++j) a[j] += u[j];
        }
    }
}

// forward sweep of one tree level: y_P = Linv f_P (rows r < p), u = f_B - M f_P (rows r >= p);
// thread per row, f_P in LDS, column-major G (lanes read consecutive rows)
template <int BLOCK, int NR, bool NT>
__global__ __launch_bounds__(BLOCK) void k_fwd(const Task* __restrict__ tasks, int first, const double* __restrict__ Gc,
                                               const long long* __restrict__ ell, const double* __restrict__ B0,
                                               const double* __restrict__ B1, double* __restrict__ Y,
                                               double* __restrict__ U, const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Task t = tasks[first + blockIdx.x];
    const int p = t.p, R = p + t.nb;
    const int tid = threadIdx.x;
    double* f = lds;
    for (int c = tid; c < p; c += BLOCK) front_row<NR>(t, c, ell, B0, B1, U, f + NR * c);
    __syncthreads();
    if (tid >= t.nr) return;
    const int r = t.r0 + tid;
    const double* G = Gc + t.goff + r;
    const int cmax = r < p ? r + 1 : p;
    // a boundary row's own front value is gathered first: its two dependent loads overlap the
    // factor stream instead of following it
    double fr[NR];
    if (r >= p) front_row<NR, false>(t, r, ell, B0, B1, U, fr);
    double a[NR];
    zero<NR>(a);
    dot_rows<NR, NT>(G, (size_t)R, 0, cmax, f, a);
    if (r < p) {
        double* y = Y + NR * (size_t)(t.beg + r);
#pragma unroll
        for (int k = 0; k < NR; ++k) y[k] = a[k];
    } else {
        double* u = U + (NR / 3) * t.uoff + NR * (size_t)(r - p);
#pragma unroll
        for (int k = 0; k < NR; ++k) u[k] = fr[k] - a[k];
    }
}

// [y_P ; -x_B]_r of a supernode (backward input vector)
template <int NR, class N>
__device__ __forceinline__ void bwd_row(const N& t, int r, const int* __restrict__ bnd, const double* __restrict__ Y,
                                        const double* __restrict__ X0, const double* __restrict__ X1, double* v) {
    if (r < t.p) {
        const double* y = Y + NR * (size_t)(t.beg + r);
#pragma unroll
        for (int k = 0; k < NR; ++k) v[k] = y[k];
    } else {
        ld_ext<NR>(X0, X1, (size_t)bnd[t.bnd_off + r - t.p], v);
#pragma unroll
        for (int k = 0; k < NR; ++k) v[k] = -v[k];
    }
}

// backward sweep of one tree level: x_P = Linv^T y_P - M^T x_B (columns j of G); thread per
// column, [y_P ; -x_B] in LDS, row-major G (lanes read consecutive columns)
template <int BLOCK, int NR, bool NT>
__global__ __launch_bounds__(BLOCK) void k_bwd(const Task* __restrict__ tasks, int first, const double* __restrict__ Gr,
                                               const int* __restrict__ bnd, const double* __restrict__ Y,
                                               double* __restrict__ X0, double* __restrict__ X1, const Ctrl* ctrl,
                                               int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const Task t = tasks[first + blockIdx.x];
    const int R = t.p + t.nb;
    const int tid = threadIdx.x;
    double* v = lds;
    for (int r = tid; r < R; r += BLOCK) bwd_row<NR>(t, r, bnd, Y, X0, X1, v + NR * r);
    __syncthreads();
    if (tid >= t.nr) return;
    const int j = t.r0 + tid;
    const double* G = Gr + t.goff + j;
    const int ld = t.ldr;
    double a[NR];
    zero<NR>(a);
    dot_rows<NR, NT>(G, (size_t)ld, j, R, v, a);
    st_ext<NR>(X0, X1, (size_t)(t.beg + j), a);
}

// Backward sweep of the large supernodes (R > kWaveR) as a split-K GEMV: tile = 128 columns
// (2 per lane, one 16-B load each: rows of G are padded to an even length) x kBwdTileRows rows
// (4 waves x kBwdTileRows/4 rows; kBwdTileRows = DirectSolver::tile_w_, 128 or 256) of the
// row-major G, the tile's slice of [y_P ; -x_B] staged in LDS, one
// 128 x NR partial per tile; the last tile of a column block to finish sums the block's partials
// in tile order (deterministic; hand-off protocol above). Gives (columns/128) x (rows/kBwdTileRows)
// workgroups per supernode instead of one wave per column with a serial loop over all R rows.
// minimum waves per SIMD the split-K tiles' register budget is set for, and the load chunks of
// their software pipelines (build-time A/B knobs)
#ifndef AA_TILE_MINW
#define AA_TILE_MINW 1
#endif
#ifndef AA_FWD_CH
#define AA_FWD_CH 16
#endif
#ifndef AA_BWD_CH
#define AA_BWD_CH 8
#endif
// chunks of a packed tile's factor stream in flight per wave (build-time; 3 and 4 measured
// slower on C4: 2 waves fewer per SIMD, or no gain at 128 VGPRs -- DESIGN.md §3.2)
#ifndef AA_TILE_DEPTH
#define AA_TILE_DEPTH 2
#endif
using BTile = DirectSolver::BTile;
using BRed = DirectSolver::BRed;
template <int NR, int CH, int kBwdTileRows>
__global__ __launch_bounds__(256, AA_TILE_MINW) void k_bwd_tile(const BTile* __restrict__ tiles, int first, const double* __restrict__ Gr,
                                                  const int* __restrict__ bnd, const double* __restrict__ Y,
                                                  double* __restrict__ X0, double* __restrict__ X1,
                                                  double* __restrict__ part, const BRed* __restrict__ reds,
                                                  int* __restrict__ cnt, const Ctrl* ctrl, int gate_reject,
                                                  int ext_off) {
    if (solve_gated(ctrl, gate_reject)) return;
    constexpr int W = 2 * NR;   // accumulators per lane: columns c and c + 1
    __shared__ double v[NR * kBwdTileRows];
    __shared__ double red[3][W * 64];
    const BTile t = tiles[first + blockIdx.x];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int c = t.c0 + 2 * lane;   // columns c, c+1 (c+1 may be the zero pad column)
    constexpr int per = kBwdTileRows / 4;
    constexpr int C = CH < per ? CH : per;
    constexpr int NC = per / C;
    const int i0 = w * per;
    const int nloc = min(per, t.nr - i0);   // rows of this wave's slice (<= 0: none)
    const bool live = c < t.p && nloc > 0;
    // software pipeline over chunks of C rows, two chunks in flight: the first two are issued
    // before the vector slice is staged (their latency overlaps the gathers and the barrier),
    // chunk k + 2 right after chunk k is consumed. Loads are unconditional (row index clamped to
    // the slice; the extra rows count zero), so no load waits behind a branch.
    const double2* G = reinterpret_cast<const double2*>(Gr + t.goff + (size_t)(t.r0 + i0) * t.ldr + (live ? c : 0));
    const int ld2 = t.ldr / 2;
    double2 ga[C], gb[C];
    auto ld = [&](double2* g, int k) {
#pragma unroll
        for (int q = 0; q < C; ++q) g[q] = G[(size_t)min(k * C + q, nloc - 1) * ld2];
    };
    if (live) {
        ld(ga, 0);
        if (NC > 1) ld(gb, 1);
    }
    for (int i = tid; i < kBwdTileRows; i += 256) {
        if (i < t.nr) bwd_row<NR>(t, t.r0 + i, bnd, Y, X0, X1, v + NR * i);
        else zero<NR>(v + NR * i);   // rows past the tile: finite zeros (their G entries are zeroed too)
    }
    __syncthreads();
    double a[W];
    zero<W>(a);
    if (live) {
        auto use = [&](const double2* g, int k) {
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const int i = k * C + q;
                const double2 gq = i < nloc ? g[q] : make_double2(0.0, 0.0);
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    const double vk = v[NR * (i0 + i) + m];
                    a[m] += gq.x * vk;
                    a[NR + m] += gq.y * vk;
                }
            }
        };
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (k & 1) { use(gb, k); if (k + 2 < NC) ld(gb, k + 2); }
            else       { use(ga, k); if (k + 2 < NC) ld(ga, k + 2); }
        }
    }
    if (w > 0)
#pragma unroll
        for (int k = 0; k < W; ++k) red[w - 1][W * lane + k] = a[k];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < W; ++k) a[k] += red[q][W * lane + k];
    double* o = part + (NR / 3) * t.poff + W * lane;
#pragma unroll
    for (int k = 0; k < W; ++k) st_sc1(o + k, a[k]);
    const BRed rd = reds[t.rid];
    if (!arrive_last(cnt + t.rid, rd.nt, lane)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // last tile of the column block: sum its partials in tile order (deterministic)
    if (2 * lane < rd.nc) {
        double b[W];
        zero<W>(b);
        const double* q = part + (NR / 3) * rd.poff + W * lane;
        red_tiles<W, W * 64>(q, rd.nt, b);
        const size_t xo = (size_t)(rd.beg + rd.c0 + 2 * lane - ext_off);
        st_ext<NR>(X0, X1, xo, b);
        if (2 * lane + 1 < rd.nc) st_ext<NR>(X0, X1, xo + 1, b + NR);
    }
    if (lane == 0) __hip_atomic_store((gu32*)(cnt + t.rid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Forward sweep of the large supernodes (p > kWaveP) as a split-K GEMV on the column-major G:
// tile = 64 rows (lanes) x kFwdTileCols columns (4 waves; 128 or 256), the tile's slice of the
// assembled front f_P staged in LDS, one 64 x NR partial per tile; the last tile of a row block
// to finish sums its partials in tile order and writes y_P (rows < p) or the update vector
// u = f_B - M f_P.
using FTile = DirectSolver::FTile;
using FRed = DirectSolver::FRed;
template <int NR, int CH, int kFwdTileCols>
__global__ __launch_bounds__(256, AA_TILE_MINW) void k_fwd_tile(const FTile* __restrict__ tiles, int first, const double* __restrict__ Gc,
                                                  const long long* __restrict__ ell, const double* __restrict__ B0,
                                                  const double* __restrict__ B1, double* __restrict__ part,
                                                  const FRed* __restrict__ reds, int* __restrict__ cnt,
                                                  double* __restrict__ Y, double* __restrict__ U, const Ctrl* ctrl,
                                                  int gate_reject, int ext_off) {
    if (solve_gated(ctrl, gate_reject)) return;
    __shared__ double f[NR * kFwdTileCols];
    __shared__ double red[3][NR * 64];
    const FTile t = tiles[first + blockIdx.x];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int r = t.r0 + lane;
    constexpr int per = kFwdTileCols / 4;
    constexpr int C = CH < per ? CH : per;
    constexpr int NC = per / C;
    const int i0 = w * per;
    int nloc = min(per, t.nc - i0);   // columns of this wave's slice (<= 0: none)
    // a row block inside L_PP^-1 (all 64 rows < p): its columns past the block's last row are the
    // zero upper triangle -- not loaded (the skipped terms are exact zeros: same sums)
    if (t.r0 + 64 <= t.p) nloc = min(nloc, t.r0 + 64 - (t.c0 + i0));
    const bool live = r < t.R && nloc > 0;
    // software pipeline over chunks of C columns, two chunks in flight (see k_bwd_tile); the
    // first two overlap the extend-add gathers that assemble the front slice
    const double* G = Gc + t.goff + (size_t)(t.c0 + i0) * t.R + (live ? r : 0);
    double ga[C], gb[C];
    auto ld = [&](double* g, int k) {
#pragma unroll
        for (int q = 0; q < C; ++q) g[q] = G[(size_t)min(k * C + q, nloc - 1) * t.R];
    };
    if (live) {
        ld(ga, 0);
        if (NC > 1) ld(gb, 1);
    }
    // this tile's slice of the front f_P = b_P + extend-add of the children's update vectors
    for (int i = tid; i < kFwdTileCols; i += 256) {
        if (i < t.nc) front_row<NR>(t, t.c0 + i, ell, B0, B1, U, f + NR * i, ext_off);
        else zero<NR>(f + NR * i);   // columns past the tile: finite zeros
    }
    __syncthreads();
    double a[NR];
    zero<NR>(a);
    if (live) {
        auto use = [&](const double* g, int k) {
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const int i = k * C + q;
                const double gq = i < nloc ? g[q] : 0.0;
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] += gq * f[NR * (i0 + i) + m];
            }
        };
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            if (k & 1) { use(gb, k); if (k + 2 < NC) ld(gb, k + 2); }
            else       { use(ga, k); if (k + 2 < NC) ld(ga, k + 2); }
        }
    }
    if (w > 0)
#pragma unroll
        for (int k = 0; k < NR; ++k) red[w - 1][NR * lane + k] = a[k];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < NR; ++k) a[k] += red[q][NR * lane + k];
    double* o = part + (NR / 3) * t.poff + NR * lane;
#pragma unroll
    for (int k = 0; k < NR; ++k) st_sc1(o + k, a[k]);
    const FRed rd = reds[t.rid];
    if (!arrive_last(cnt + t.rid, rd.nt, lane)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // last tile of the row block: sum its partials in tile order (deterministic)
    if (lane < rd.nr) {
        const int rr = rd.r0 + lane;
        double fr[NR];   // a boundary row's front value: gathered before the partials are summed
        if (rr >= rd.p) front_row<NR, false>(rd, rr, ell, B0, B1, U, fr, ext_off);
        double b[NR];
        zero<NR>(b);
        const double* q = part + (NR / 3) * rd.poff + NR * lane;
        red_tiles<NR, NR * 64>(q, rd.nt, b);
        if (rr < rd.p) {
            double* y = Y + NR * (size_t)(rd.beg + rr);
#pragma unroll
            for (int k = 0; k < NR; ++k) y[k] = b[k];
        } else {
            double* u = U + (NR / 3) * rd.uoff + NR * (size_t)(rr - rd.p);
#pragma unroll
            for (int k = 0; k < NR; ++k) u[k] = fr[k] - b[k];
        }
    }
    if (lane == 0) __hip_atomic_store((gu32*)(cnt + t.rid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Packed split-K tiles (the default): the same tiles, partials and reductions as k_fwd_tile /
// k_bwd_tile -- so the same sums in the same order, bit-identical -- but the factor entries of a
// tile come from its own contiguous block of Gt (DirectSolver::build packs them), laid out in the
// order the tile's waves consume them: each wave streams a sequential run of 1-KB rows (64 lanes
// x 16 B, two columns or two rows' entries per lane). The column-major / row-major copies put a
// tile's 64 x 256 entries in 256 pieces of 512 B (or 1 KB) at strides of the supernode's height,
// spread over several MB: a DRAM-page and TLB pattern a contiguous stream avoids.
// Streamed levels (DirectSolver::Stream): the workgroup's tile is the next ticket of the launch's
// queue (level order), not blockIdx -- so every tile a workgroup waits for was taken earlier by a
// workgroup that is running or done, whatever the dispatch order (no deadlock).
__device__ __forceinline__ int stream_ticket(const int* __restrict__ order, int first, int* sync, int head) {
    __shared__ int s_t;
    if (threadIdx.x == 0)
        s_t = order[first + (int)__hip_atomic_fetch_add((gu32*)(sync + head), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)];
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_t);
}
// wait until counter sync[dep] reaches need (one lane polls; write-through producers, so a relaxed
// agent load sees the adds). No agent acquire follows (AA_STREAM_ACQ=1 builds it in): it exists to
// drop stale copies of the published lines from this CU's L1, and there are none -- every line a
// tile waits for (update vectors, Xs rows: each producer's rows on 128-B lines of their own) is
// written once per launch and read by nobody before its producer has signalled, and a launch
// starts with clean caches. The acquire cost ~1.7 us per workgroup (x4 at 4 workgroups per CU,
// MI355X_MICROARCH.md price table) and waits for the wave's factor loads in flight.
#ifndef AA_STREAM_ACQ
#define AA_STREAM_ACQ 0
#endif
__device__ __forceinline__ void stream_wait(int* sync, int dep, int need, int w, int lane) {
    if (need <= 0) return;
    if (w == 0) {
        if (lane == 0) {
            const gu32* d = (const gu32*)(sync + dep);
            while ((int)__hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) __builtin_amdgcn_s_sleep(2);
        }
#if AA_STREAM_ACQ
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    }
    __syncthreads();
}
// publish: the calling wave's write-through stores drained, then one counter add
__device__ __forceinline__ void stream_signal(int* sync, int sig, int lane) {
    if (sig < 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add((gu32*)(sync + sig), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifndef AA_FWD_TRI
#define AA_FWD_TRI 0   // 1: k_fwd_ptile padding rows load nothing, zero upper triangle skipped per lane (measured: no gain)
#endif
template <int NR, int CH, int kFwdTileCols, int DEPTH, bool STREAM, bool NT>
__global__ __launch_bounds__(256, AA_TILE_MINW) void k_fwd_ptile(const FTile* __restrict__ tiles, int first,
                                                   const double* __restrict__ Gt, const long long* __restrict__ ell,
                                                   const double* __restrict__ B0, const double* __restrict__ B1,
                                                   double* __restrict__ part, const FRed* __restrict__ reds,
                                                   int* __restrict__ cnt, double* __restrict__ Y, double* __restrict__ U,
                                                   const Ctrl* ctrl, int gate_reject, int ext_off,
                                                   const int* __restrict__ order, int* sync, int head) {
    if (solve_gated(ctrl, gate_reject)) return;
    __shared__ double f[NR * kFwdTileCols];
    __shared__ double red[3][NR * 64];
    const FTile t = tiles[STREAM ? stream_ticket(order, first, sync, head) : first + blockIdx.x];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    constexpr int per = kFwdTileCols / 4;   // columns of a wave's slice (even)
    constexpr int C = CH < per ? CH : per;   // columns per chunk (even)
    constexpr int NC = per / C;
    constexpr int C2 = C / 2;                // 16-B loads per chunk: column pairs
    const int i0 = w * per;
    int nloc = min(per, t.nc - i0);
    if (t.r0 + 64 <= t.p) nloc = min(nloc, t.r0 + 64 - (t.c0 + i0));   // zero upper triangle: not loaded
    const bool live = nloc > 0;   // wave-uniform: rows past R read the block's zero padding
    const int qmax = (nloc - 1) >> 1;   // last pair with a live column (later indices re-read it: cache hits)
#if AA_FWD_TRI
    // per lane (= row r0 + lane): rows past R are zero padding (load nothing), and a row of the
    // diagonal block needs columns <= its own only (the upper triangle of L_PP^-1 is zero): its
    // later pairs re-read its last needed pair (cache hits) and their terms are masked
    const int row = t.r0 + lane;
    const bool lane_live = row < t.R;
    const int hi = row < t.p ? row - (t.c0 + i0) : per;   // last needed wave-local column
    const int qlane = hi < 0 ? 0 : min(qmax, hi >> 1);
#else
    constexpr bool lane_live = true;
    const int hi = per, qlane = qmax;
#endif
    const double2* G = reinterpret_cast<const double2*>(Gt + t.toff) + (size_t)w * (per / 2) * 64 + lane;
    constexpr int DP = DEPTH < NC ? DEPTH : NC;   // chunks in flight
    double2 gbuf[DP][C2];
    auto ld = [&](double2* g, int k) {
#pragma unroll
        for (int q = 0; q < C2; ++q) g[q] = ld_f2<NT>(G + (size_t)min(k * C2 + q, qlane) * 64);
    };
    if (live && lane_live) {
#pragma unroll
        for (int d = 0; d < DP; ++d) ld(gbuf[d], d);
    }
    if constexpr (STREAM) stream_wait(sync, t.dep, t.need, w, lane);   // the children's update vectors
    for (int i = tid; i < kFwdTileCols; i += 256) {
        if (i < t.nc) front_row<NR>(t, t.c0 + i, ell, B0, B1, U, f + NR * i, ext_off);
        else zero<NR>(f + NR * i);
    }
    __syncthreads();
    double a[NR];
    zero<NR>(a);
    if (live && lane_live) {
        auto use = [&](const double2* g, int k) {
#pragma unroll
            for (int q = 0; q < C2; ++q) {
                const int i = k * C + 2 * q;
                const double g0 = i < nloc && i <= hi ? g[q].x : 0.0;
                const double g1 = i + 1 < nloc && i + 1 <= hi ? g[q].y : 0.0;
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] += g0 * f[NR * (i0 + i) + m];
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] += g1 * f[NR * (i0 + i + 1) + m];
            }
        };
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            use(gbuf[k % DP], k);
            if (k + DP < NC) ld(gbuf[k % DP], k + DP);
        }
    }
    if (w > 0)
#pragma unroll
        for (int k = 0; k < NR; ++k) red[w - 1][NR * lane + k] = a[k];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < NR; ++k) a[k] += red[q][NR * lane + k];
    double* o = part + (NR / 3) * t.poff + NR * lane;
#pragma unroll
    for (int k = 0; k < NR; ++k) st_sc1(o + k, a[k]);
    const FRed rd = reds[t.rid];
    if (!arrive_last(cnt + t.rid, rd.nt, lane)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane < rd.nr) {
        const int rr = rd.r0 + lane;
        double fr[NR];
        if (rr >= rd.p) front_row<NR, false>(rd, rr, ell, B0, B1, U, fr, ext_off);
        double b[NR];
        zero<NR>(b);
        const double* q = part + (NR / 3) * rd.poff + NR * lane;
        red_tiles<NR, NR * 64>(q, rd.nt, b);
        if (rr < rd.p) {
            double* y = Y + NR * (size_t)(rd.beg + rr);
#pragma unroll
            for (int k = 0; k < NR; ++k) y[k] = b[k];
        } else {
            double* u = U + (NR / 3) * rd.uoff + NR * (size_t)(rr - rd.p);
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                if constexpr (STREAM) st_sc1(u + k, fr[k] - b[k]);   // read by the parent in this launch
                else u[k] = fr[k] - b[k];
            }
        }
    }
    if constexpr (STREAM) stream_signal(sync, rd.sig, lane);
    if (lane == 0) __hip_atomic_store((gu32*)(cnt + t.rid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// [y_P ; -x_B]_r of a streamed supernode: x_B rows of supernodes solved in this launch come
// from the padded copy Xs (bndx >= 0: its row; each supernode's rows on lines of their own, so no
// line is read before every row on it is final), the others from x
template <int NR, class N>
__device__ __forceinline__ void bwd_row_s(const N& t, int r, const int* __restrict__ bnd, const int* __restrict__ bndx,
                                          const double* __restrict__ Y, const double* __restrict__ X0,
                                          const double* __restrict__ X1, const double* __restrict__ Xs, double* v) {
    if (r < t.p) {
        const double* y = Y + NR * (size_t)(t.beg + r);
#pragma unroll
        for (int k = 0; k < NR; ++k) v[k] = y[k];
        return;
    }
    const int xi = bndx[t.bnd_off + r - t.p];
    if (xi >= 0) {
        const double* xs = Xs + NR * (size_t)xi;
#pragma unroll
        for (int k = 0; k < NR; ++k) v[k] = -xs[k];
    } else {
        ld_ext<NR>(X0, X1, (size_t)bnd[t.bnd_off + r - t.p], v);
#pragma unroll
        for (int k = 0; k < NR; ++k) v[k] = -v[k];
    }
}

#ifndef AA_BWD_TRI
#define AA_BWD_TRI 0   // 1: k_bwd_ptile skips the zero upper triangle of L_PP^-1 per lane (measured slower)
#endif
template <int NR, int CH, int kBwdTileRows, int DEPTH, bool STREAM, bool NT>
__global__ __launch_bounds__(256, AA_TILE_MINW) void k_bwd_ptile(const BTile* __restrict__ tiles, int first,
                                                   const double* __restrict__ Gt, const int* __restrict__ bnd,
                                                   const double* __restrict__ Y, double* __restrict__ X0,
                                                   double* __restrict__ X1, double* __restrict__ part,
                                                   const BRed* __restrict__ reds, int* __restrict__ cnt, const Ctrl* ctrl,
                                                   int gate_reject, int ext_off, const int* __restrict__ order,
                                                   int* sync, int head, const int* __restrict__ bndx,
                                                   double* __restrict__ Xs) {
    if (solve_gated(ctrl, gate_reject)) return;
    constexpr int W = 2 * NR;
    __shared__ double v[NR * kBwdTileRows];
    __shared__ double red[3][W * 64];
    const BTile t = tiles[STREAM ? stream_ticket(order, first, sync, head) : first + blockIdx.x];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    constexpr int per = kBwdTileRows / 4;
    constexpr int C = CH < per ? CH : per;
    constexpr int NC = per / C;
    const int i0 = w * per;
    const int nloc = min(per, t.nr - i0);
    const bool live = nloc > 0;   // wave-uniform: columns past p read the block's zero padding
    // narrow block (<= 64 columns, block-uniform): lane l holds column c0 + l, and its 16-B load
    // covers two consecutive rows of it (k_pack_btiles) -- half the bytes of a 128-column block,
    // whose upper half would be zero padding. Each column still sums its rows in ascending order.
    const bool nar = t.p - t.c0 <= 64;
    const int nld = nar ? (nloc + 1) >> 1 : nloc;   // 16-B rows of this wave
    const double2* G = reinterpret_cast<const double2*>(Gt + t.toff) + (size_t)w * (nar ? per / 2 : per) * 64 + lane;
    constexpr int DP = DEPTH < NC ? DEPTH : NC;   // chunks in flight
    constexpr int NCN = (per / 2 + C - 1) / C;     // chunks of a narrow wave (per / 2 row pairs)
    // lanes whose columns all lie past p hold zero padding: they load nothing (no lines fetched)
    const bool lane_live = (nar ? lane : 2 * lane) < t.p - t.c0;
    // rows above the diagonal of L_PP^-1 (row < the lane's first column) are zeros: the lane's
    // loads for them re-read its first needed 16-B row (cache hits) and their terms are masked
    // (the stored zeros added nothing, so the sums are unchanged)
#if AA_BWD_TRI
    const int lo_row = t.c0 + (nar ? lane : 2 * lane) - (t.r0 + i0);
    const int lo = lo_row <= 0 ? 0 : min(nar ? lo_row >> 1 : lo_row, nld - 1);
#else
    constexpr int lo = 0;
#endif
    double2 gbuf[DP][C];
    auto ld = [&](double2* g, int k) {
#pragma unroll
        for (int q = 0; q < C; ++q)
            g[q] = ld_f2<NT>(G + (size_t)min(max(k * C + q, lo), nld - 1) * 64);
    };
    if (live && lane_live) {
#pragma unroll
        for (int d = 0; d < DP; ++d)
            if (!nar || d < NCN) ld(gbuf[d], d);
    }
    if constexpr (STREAM) stream_wait(sync, t.dep, t.need, w, lane);   // the parent's x rows
    for (int i = tid; i < kBwdTileRows; i += 256) {
        if (i < t.nr) {
            if constexpr (STREAM) bwd_row_s<NR>(t, t.r0 + i, bnd, bndx, Y, X0, X1, Xs, v + NR * i);
            else bwd_row<NR>(t, t.r0 + i, bnd, Y, X0, X1, v + NR * i);
        } else {
            zero<NR>(v + NR * i);
        }
    }
    __syncthreads();
    double a[W];
    zero<W>(a);
    if (live && lane_live && !nar) {
        auto use = [&](const double2* g, int k) {
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const int i = k * C + q;
                const double2 gq = i < nloc && i >= lo ? g[q] : make_double2(0.0, 0.0);
#pragma unroll
                for (int m = 0; m < NR; ++m) {
                    const double vk = v[NR * (i0 + i) + m];
                    a[m] += gq.x * vk;
                    a[NR + m] += gq.y * vk;
                }
            }
        };
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            use(gbuf[k % DP], k);
            if (k + DP < NC) ld(gbuf[k % DP], k + DP);
        }
    } else if (live && lane_live) {   // narrow: rows 2i, 2i+1 of column c0 + lane (the odd tail row is zero)
        auto use = [&](const double2* g, int k) {
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const int i = k * C + q;
                const double2 gq = i < nld && i >= lo ? g[q] : make_double2(0.0, 0.0);
                const double* v0 = v + NR * (i0 + 2 * min(i, nld - 1));   // masked terms: finite
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] += gq.x * v0[m];
#pragma unroll
                for (int m = 0; m < NR; ++m) a[m] += gq.y * v0[NR + m];
            }
        };
#pragma unroll
        for (int k = 0; k < NCN; ++k) {
            use(gbuf[k % DP], k);
            if (k + DP < NCN) ld(gbuf[k % DP], k + DP);
        }
    }
    if (w > 0)
#pragma unroll
        for (int k = 0; k < W; ++k) red[w - 1][W * lane + k] = a[k];
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
        for (int k = 0; k < W; ++k) a[k] += red[q][W * lane + k];
    double* o = part + (NR / 3) * t.poff + W * lane;
#pragma unroll
    for (int k = 0; k < W; ++k) st_sc1(o + k, a[k]);
    const BRed rd = reds[t.rid];
    if (!arrive_last(cnt + t.rid, rd.nt, lane)) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int cl = nar ? lane : 2 * lane;   // this lane's first column in the block
    if (cl < rd.nc) {
        double b[W];
        zero<W>(b);
        const double* q = part + (NR / 3) * rd.poff + W * lane;
        red_tiles<W, W * 64>(q, rd.nt, b);
        const bool two = !nar && cl + 1 < rd.nc;
        const size_t xo = (size_t)(rd.beg + rd.c0 + cl - ext_off);
        st_ext<NR>(X0, X1, xo, b);
        if (two) st_ext<NR>(X0, X1, xo + 1, b + NR);
        if constexpr (STREAM) {
            if (rd.sig >= 0) {   // the children of this supernode read these rows in this launch
                double* xs = Xs + NR * (size_t)(rd.xso + rd.c0 + cl);
#pragma unroll
                for (int m = 0; m < NR; ++m) st_sc1(xs + m, b[m]);
                if (two)
#pragma unroll
                    for (int m = 0; m < NR; ++m) st_sc1(xs + NR + m, b[NR + m]);
            }
        }
    }
    if constexpr (STREAM) stream_signal(sync, rd.sig, lane);
    if (lane == 0) __hip_atomic_store((gu32*)(cnt + t.rid), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// packing (setup): one workgroup per tile, every entry of its block written (zeros outside the
// supernode), read from the row-major copy Gr (row stride ldr = p rounded up to even)
__global__ void k_pack_ftiles(const FTile* __restrict__ tiles, const int* __restrict__ width,
                              const double* __restrict__ Gr, double* __restrict__ Gt) {
    const FTile t = tiles[blockIdx.x];
    const int W = width[blockIdx.x], per2 = W / 8, ldr = t.p + (t.p & 1);
    const long long n = 64LL * W;
    for (long long idx = threadIdx.x; idx < n; idx += blockDim.x) {
        const int j = (int)(idx & 1), r = (int)((idx >> 1) & 63);
        const long long rest = idx >> 7;
        const int w = (int)(rest / per2), cp = (int)(rest % per2);
        const int c = t.c0 + w * (W / 4) + 2 * cp + j, row = t.r0 + r;
        Gt[t.toff + idx] = (c < t.c0 + t.nc && row < t.R) ? Gr[t.goff + (size_t)row * ldr + c] : 0.0;
    }
}
__global__ void k_pack_btiles(const BTile* __restrict__ tiles, const int* __restrict__ width,
                              const double* __restrict__ Gr, double* __restrict__ Gt) {
    const BTile t = tiles[blockIdx.x];
    const int W = width[blockIdx.x], R = t.p + t.nb;
    const bool nar = t.p - t.c0 <= 64;   // narrow block: lane = column, a 16-B pair = two rows
    const long long n = (nar ? 64LL : 128LL) * W;
    for (long long idx = threadIdx.x; idx < n; idx += blockDim.x) {
        const int j = (int)(idx & 1), lane = (int)((idx >> 1) & 63), q0 = (int)(idx >> 7);
        const int q = nar ? 2 * q0 + j : q0;
        const int row = t.r0 + q, col = nar ? t.c0 + lane : t.c0 + 2 * lane + j;
        Gt[t.toff + idx] = (q < t.nr && row < R && col < t.p) ? Gr[t.goff + (size_t)row * t.ldr + col] : 0.0;
    }
}

// partitioned dense top: this GPU's share of the top front f_T = b_T + its own children's
// update vectors (thread per row), written set-major [set][3 * p] for the all-reduce
template <int NR>
__global__ __launch_bounds__(256) void k_top_front(const Task* __restrict__ top, const long long* __restrict__ ell,
                                                   const double* __restrict__ B0, const double* __restrict__ B1,
                                                   const double* __restrict__ U, double* __restrict__ F,
                                                   const Ctrl* ctrl, int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const Task t = *top;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= t.p) return;
    double a[NR];
    front_row<NR>(t, q, ell, B0, B1, U, a);
#pragma unroll
    for (int k = 0; k < NR; ++k) F[(size_t)(k / 3) * 3 * t.p + 3 * (size_t)q + k % 3] = a[k];
}
// ... and the summed x_top (set-major) back into the caller's x rows
template <int NR>
__global__ __launch_bounds__(256) void k_top_scatter(const Task* __restrict__ top, const double* __restrict__ X,
                                                     double* __restrict__ X0, double* __restrict__ X1, const Ctrl* ctrl,
                                                     int gate_reject) {
    if (solve_gated(ctrl, gate_reject)) return;
    const Task t = *top;
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= t.p) return;
    double a[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) a[k] = X[(size_t)(k / 3) * 3 * t.p + 3 * (size_t)q + k % 3];
    st_ext<NR>(X0, X1, (size_t)(t.beg + q), a);
}

using SubNode = DirectSolver::SubNode;
using SubLevel = DirectSolver::SubLevel;
using SubTree = DirectSolver::SubTree;

// forward sweep of a whole bottom subtree (one workgroup), its levels bottom-up
template <int BLOCK, int NR, bool NT>
__global__ __launch_bounds__(BLOCK) void k_fwd_sub(const SubTree* __restrict__ trees, const SubLevel* __restrict__ lvls,
                                                 const SubNode* __restrict__ nodes, const int* __restrict__ items,
                                                 const double* __restrict__ Gc, const long long* __restrict__ ell,
                                                 const double* __restrict__ B0, const double* __restrict__ B1,
                                                 double* __restrict__ Y, double* __restrict__ U, const Ctrl* ctrl,
                                                 int gate_reject, long long* clk, int clk_stride, int node_off, int tree0) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int K = NR / 3;
    const SubTree T = trees[tree0 + blockIdx.x];
    const int tid = threadIdx.x;
    // the subtree's supernode records, staged in LDS once: a row item then needs one (coalesced)
    // load, its item, before its factor stream, instead of the item and then its record
    SubNode* sn = reinterpret_cast<SubNode*>(reinterpret_cast<char*>(lds) + node_off);
    {
        const long long* src = reinterpret_cast<const long long*>(nodes + T.node0);
        long long* dst = reinterpret_cast<long long*>(sn);
        constexpr int W8 = sizeof(SubNode) / 8;
        for (int i = tid; i < T.nnode * W8; i += BLOCK) dst[i] = src[i];
    }
    __syncthreads();
    // optional phase clock (AA_SUB_TIMING): kernel start, then after every barrier
    long long* ck = clk ? clk + (size_t)(tree0 + blockIdx.x) * clk_stride : nullptr;
    if (ck && tid == 0) ck[0] = (long long)__builtin_amdgcn_s_memrealtime();
    // kSubU: every update vector consumed inside the subtree lives in LDS (its slot planned by the
    // host over the levels' lifetimes), so a front pull is one LDS read after its ELL offset and
    // only the root's update vector goes to HBM. Same sums in the same order: bit-identical.
    const bool ul = (T.flags & DirectSolver::kSubU) != 0;
    for (int l = 0; l < T.nlvl; ++l) {
        const SubLevel L = lvls[T.lvl0 + l];
        const SubNode* ln = sn + (L.n0 - T.node0);
        for (int i = tid; i < L.nfa; i += BLOCK) {          // front vectors f_P of the level's supernodes
            const int it = items[L.fa0 + i];
            const SubNode nd = ln[it >> 16];
            const int c = it & 0xffff;
            if (ul) front_row<NR>(nd, c, ell, B0, B1, lds, lds + K * nd.lds + NR * c);
            else front_row<NR>(nd, c, ell, B0, B1, U, lds + K * nd.lds + NR * c);
        }
        __syncthreads();
        if (ck && tid == 0) ck[1 + 2 * l] = (long long)__builtin_amdgcn_s_memrealtime();
        for (int i = tid; i < L.nfr; i += BLOCK) {          // rows of G . f_P
            const int it = items[L.fr0 + i];
            const SubNode nd = ln[it >> 16];
            const int r = it & 0xffff, p = nd.p, R = p + nd.nb;
            const double* f = lds + K * nd.lds;
            const double* G = Gc + nd.goff + r;
            const int cmax = r < p ? r + 1 : p;
            double fr[NR];   // a boundary row's own front value, gathered before the factor stream
            if (r >= p) {
                if (ul) front_row<NR, false>(nd, r, ell, B0, B1, lds, fr);
                else front_row<NR, false>(nd, r, ell, B0, B1, U, fr);
            }
            double a[NR];
            zero<NR>(a);
            if constexpr (NR == 3) dot_rows_chunk<NR, NT>(G, (size_t)R, 0, cmax, f, a);
            else dot_rows<NR, NT>(G, (size_t)R, 0, cmax, f, a);
            if (r < p) {
                double* y = Y + NR * (size_t)(nd.beg + r);
#pragma unroll
                for (int k = 0; k < NR; ++k) y[k] = a[k];
            } else if (nd.slot >= 0) {   // consumed by the parent, inside this subtree (kSubU)
                double* u = lds + K * nd.slot + NR * (r - p);
#pragma unroll
                for (int k = 0; k < NR; ++k) u[k] = fr[k] - a[k];
            } else {
                double* u = U + K * nd.uoff + NR * (size_t)(r - p);
#pragma unroll
                for (int k = 0; k < NR; ++k) u[k] = fr[k] - a[k];
            }
        }
        __syncthreads();
        if (ck && tid == 0) ck[2 + 2 * l] = (long long)__builtin_amdgcn_s_memrealtime();
    }
}

// backward sweep of a whole bottom subtree (one workgroup), its levels top-down
// The column products are split over row segments of kSubSegRows rows (items (node, segment,
// column), consecutive threads on consecutive columns of one row -> coalesced), partials in
// LDS, then one item per column sums its segments in order: short loops instead of one thread
// walking all R rows of a column.
#ifndef AA_SUB_SEG
#define AA_SUB_SEG 64
#endif
constexpr int kSubSegRows = AA_SUB_SEG;
__device__ __forceinline__ int sub_seg_off(int seg, int p) {   // partial slots before segment seg
    int o = 0;
    for (int q = 0; q < seg; ++q) o += min(p, (q + 1) * kSubSegRows);
    return o;
}

template <int BLOCK, int NR, bool NT>
__global__ __launch_bounds__(BLOCK) void k_bwd_sub(const SubTree* __restrict__ trees, const SubLevel* __restrict__ lvls,
                                                 const SubNode* __restrict__ nodes, const int* __restrict__ items,
                                                 const long long* __restrict__ items2,
                                                 const double* __restrict__ Gr, const int* __restrict__ bnd,
                                                 const double* __restrict__ Y, double* __restrict__ X0,
                                                 double* __restrict__ X1, const int* __restrict__ xg,
                                                 const Ctrl* ctrl, int gate_reject,
                                                 long long* clk, int clk_stride, int node_off, int tree0) {
    if (solve_gated(ctrl, gate_reject)) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int K = NR / 3;
    const SubTree T = trees[tree0 + blockIdx.x];
    const int tid = threadIdx.x;
    SubNode* sn = reinterpret_cast<SubNode*>(reinterpret_cast<char*>(lds) + node_off);   // as k_fwd_sub
    {
        const long long* src = reinterpret_cast<const long long*>(nodes + T.node0);
        long long* dst = reinterpret_cast<long long*>(sn);
        constexpr int W8 = sizeof(SubNode) / 8;
        for (int i = tid; i < T.nnode * W8; i += BLOCK) dst[i] = src[i];
    }
    // kSubX: the x rows a boundary can name -- the subtree's own columns (written below, level by
    // level, top-down) and the root's boundary (solved above the cut, staged here once) -- in LDS,
    // so [y_P ; -x_B] needs one LDS read after its boundary offset instead of a second HBM trip
    const bool xl = (T.flags & DirectSolver::kSubX) != 0;
    if (xl)
        for (int a = tid; a < T.nxg; a += BLOCK) {
            double v[NR];
            ld_ext<NR>(X0, X1, (size_t)xg[T.xg_off + a], v);
            double* d = lds + K * (T.xst + 3 * a);
#pragma unroll
            for (int k = 0; k < NR; ++k) d[k] = v[k];
        }
    __syncthreads();
    long long* ck = clk ? clk + (size_t)(tree0 + blockIdx.x) * clk_stride : nullptr;
    if (ck && tid == 0) ck[0] = (long long)__builtin_amdgcn_s_memrealtime();
    int ph = 1;
    for (int l = T.nlvl - 1; l >= 0; --l) {
        const SubLevel L = lvls[T.lvl0 + l];
        const SubNode* ln = sn + (L.n0 - T.node0);
        for (int i = tid; i < L.nbv; i += BLOCK) {          // [y_P ; -x_B] of the level's supernodes
            const int it = items[L.bv0 + i];
            const SubNode nd = ln[it >> 16];
            const int r = it & 0xffff;
            if (xl) {
                double* v = lds + K * nd.lds + NR * r;
                if (r < nd.p) {
                    const double* y = Y + NR * (size_t)(nd.beg + r);
#pragma unroll
                    for (int k = 0; k < NR; ++k) v[k] = y[k];
                } else {
                    const double* xs = lds + K * bnd[nd.bnd_off + r - nd.p];
#pragma unroll
                    for (int k = 0; k < NR; ++k) v[k] = -xs[k];
                }
            } else {
                bwd_row<NR>(nd, r, bnd, Y, X0, X1, lds + K * nd.lds + NR * r);
            }
        }
        __syncthreads();
        if (ck && tid == 0) ck[ph++] = (long long)__builtin_amdgcn_s_memrealtime();
        for (int i = tid; i < L.nbs; i += BLOCK) {          // segment partials of G^T . v
            const long long it = items2[L.bs0 + i];
            const SubNode nd = ln[(int)(it >> 40)];
            const int seg = (int)((it >> 20) & 0xfffff), j = (int)(it & 0xfffff), p = nd.p, R = p + nd.nb;
            const double* v = lds + K * nd.lds;
            const double* G = Gr + nd.goff + j;
            const int ld = nd.ldr;
            const int r1 = min(R, (seg + 1) * kSubSegRows);
            double a[NR];
            zero<NR>(a);
            dot_rows<NR, NT>(G, (size_t)ld, max(j, seg * kSubSegRows), r1, v, a);
            double* q = lds + K * nd.slot + NR * (sub_seg_off(seg, p) + j);
#pragma unroll
            for (int k = 0; k < NR; ++k) q[k] = a[k];
        }
        __syncthreads();
        if (ck && tid == 0) ck[ph++] = (long long)__builtin_amdgcn_s_memrealtime();
        for (int i = tid; i < L.nbc; i += BLOCK) {          // columns: sum of their segments
            const int it = items[L.bc0 + i];
            const SubNode nd = ln[it >> 16];
            const int j = it & 0xffff, p = nd.p, R = p + nd.nb;
            const int nseg = (R + kSubSegRows - 1) / kSubSegRows, s0 = j / kSubSegRows;
            int off = sub_seg_off(s0, p);
            double a[NR];
            zero<NR>(a);
            for (int seg = s0; seg < nseg; ++seg) {
                const double* q = lds + K * nd.slot + NR * (off + j);
#pragma unroll
                for (int k = 0; k < NR; ++k) a[k] += q[k];
                off += min(p, (seg + 1) * kSubSegRows);
            }
            st_ext<NR>(X0, X1, (size_t)(nd.beg + j), a);
            if (xl && nd.xo >= 0) {
                double* xs = lds + K * (nd.xo + 3 * j);
#pragma unroll
                for (int k = 0; k < NR; ++k) xs[k] = a[k];
            }
        }
        __syncthreads();
        if (ck && tid == 0) ck[ph++] = (long long)__builtin_amdgcn_s_memrealtime();
    }
}

// column-major copy of the factor blocks: Gc[goff + c*R + r] = Gr[goff + r*ld + c] (32 x 32 tile
// per workgroup through LDS: coalesced reads along the row, coalesced writes along the column)
struct TrTile { long long goff; int R, ld, p, r0, c0; };
__global__ void k_gr_to_gc(const TrTile* __restrict__ tiles, const double* __restrict__ Gr, double* __restrict__ Gc) {
    __shared__ double t[32][33];
    const TrTile T = tiles[blockIdx.x];
    for (int q = threadIdx.y; q < 32; q += blockDim.y) {
        const int r = T.r0 + q, c = T.c0 + threadIdx.x;
        if (r < T.R && c < T.p) t[q][threadIdx.x] = Gr[T.goff + (size_t)r * T.ld + c];
    }
    __syncthreads();
    for (int q = threadIdx.y; q < 32; q += blockDim.y) {
        const int c = T.c0 + q, r = T.r0 + threadIdx.x;
        if (r < T.R && c < T.p) Gc[T.goff + (size_t)c * T.R + r] = t[threadIdx.x][q];
    }
}

}  // namespace

void DirectSolver::build(const SupernodalFactor& F, hipStream_t s, const std::vector<int>* node_part, int my_part,
                         int top_beg, Comm* comm, int max_sets, bool wide, int wave_p, int wave_r) {
    n_ = F.n;
    max_sets_ = max_sets >= 2 ? 2 : 1;
    // LDS scale the layout (fused-subtree cut, tile width) is planned for: the two-set budget
    // whenever `wide`, so a one-set solver built wide sums every column in the same order as a
    // two-set one (bit-identical AA_Z_PIPELINE=0 / 1)
    const int KS = (wide || max_sets_ >= 2) ? 2 : 1;
    nn_ = F.n_nodes;
    comm_ = (node_part && comm && comm->size() > 1) ? comm : nullptr;
    top_beg_ = comm_ ? top_beg : n_;
    // partitioned: this GPU holds the supernodes of its own part and the shared top only
    std::vector<char> inc(nn_, 1);
    if (comm_)
        for (int sn = 0; sn < nn_; ++sn) inc[sn] = (*node_part)[sn] == my_part || (*node_part)[sn] == -1;
    std::vector<int> beg(nn_), p(nn_), nb(nn_), bnd_off(nn_), bnd, pull_off(nn_);
    std::vector<long long> goff(nn_), uoff(nn_);
    std::vector<int> ldr(nn_, 0);
    long long go = 0, uo = 0;
    double dense = 0, offd = 0, bsum = 0, piv = 0;
    int rows_total = 0;
    nnz_L_ = 0;
    for (int sn = 0; sn < nn_; ++sn) {
        const int ps = F.end[sn] - F.beg[sn], nbs = (int)F.bnd[sn].size();
        beg[sn] = F.beg[sn]; p[sn] = ps; nb[sn] = nbs;
        goff[sn] = go; uoff[sn] = uo;
        ldr[sn] = ps + (ps & 1);   // row-major rows padded to even length (16-B loads in k_bwd_tile)
        bnd_off[sn] = (int)bnd.size();
        pull_off[sn] = rows_total;
        if (!inc[sn]) continue;
        bnd.insert(bnd.end(), F.bnd[sn].begin(), F.bnd[sn].end());
        rows_total += ps + nbs;
        nnz_L_ += (size_t)ps * (ps + 1) / 2 + (size_t)ps * nbs;
        go += (long long)(ps + nbs) * (ps + (ps & 1));
        uo += 3LL * nbs;
        uo = (uo + 15) / 16 * 16;   // every update vector on 128-B lines of its own (streamed levels)
        dense += 0.5 * ps * (ps + 1.0);
        offd += (double)ps * nbs;
        piv += ps;
        bsum += nbs;
    }
    // G_s = [Linv ; M], M = L_BP Linv: the row-major copy Gr is formed here (every entry written,
    // so no zero fill of the 1 GB buffer), the column-major copy Gc on the device from it
    std::unique_ptr<double[]> Gr(new double[std::max<long long>(go, 1)]);
#pragma omp parallel for schedule(dynamic, 1)
    for (int sn = 0; sn < nn_; ++sn) {
        if (!inc[sn]) continue;
        const int ps = p[sn], nbs = nb[sn], R = ps + nbs, ld = ldr[sn];
        double* gr = Gr.get() + goff[sn];
        const std::vector<double>& Li = F.Linv[sn];
        const std::vector<double>& LB = F.LBP[sn];
        for (int r = 0; r < R; ++r)
            for (int c = ps; c < ld; ++c) gr[(size_t)r * ld + c] = 0.0;   // pad column
        for (int r = 0; r < ps; ++r)
            for (int c = 0; c < ps; ++c) gr[(size_t)r * ld + c] = c <= r ? Li[(size_t)r * ps + c] : 0.0;
        const bool have_m = F.M.size() == (size_t)nn_ && F.M[sn].size() == (size_t)nbs * ps;
        for (int a = 0; a < nbs; ++a) {
            double* m = gr + (size_t)(ps + a) * ld;
            if (have_m) {   // formed with the factor (dense backend)
                std::copy(F.M[sn].begin() + (size_t)a * ps, F.M[sn].begin() + (size_t)(a + 1) * ps, m);
                continue;
            }
            for (int c = 0; c < ps; ++c) m[c] = 0.0;
            for (int k = 0; k < ps; ++k) {
                const double l = LB[(size_t)a * ps + k];
                if (l == 0.0) continue;
                const double* lr = Li.data() + (size_t)k * ps;
                for (int c = 0; c <= k; ++c) m[c] += l * lr[c];
            }
        }
    }
    // children lists and ELL pull lists (front row q of a parent <- child update entries, fixed order)
    // (partitioned: the children of the top that belong to other GPUs' parts contribute nothing
    // here -- their update vectors arrive through the all-reduce of the top rows)
    std::vector<std::vector<int>> kl(nn_);
    for (int sn = 0; sn < nn_; ++sn) if (F.parent[sn] >= 0 && inc[sn]) kl[F.parent[sn]].push_back(sn);
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
    std::vector<int> ell_w(nn_, 0);
    std::vector<long long> ell_off(nn_, 0), ell;
    for (int sn = 0; sn < nn_; ++sn) {
        const int R = inc[sn] ? p[sn] + nb[sn] : 0;
        int w = 0;
        for (int q = 0; q < R; ++q) w = std::max(w, (int)pull[pull_off[sn] + q].size());
        ell_w[sn] = w;
        ell_off[sn] = (long long)ell.size();
        for (int q = 0; q < R; ++q) {
            const auto& l = pull[pull_off[sn] + q];
            for (int k = 0; k < w; ++k) ell.push_back(k < (int)l.size() ? l[k] : -1);
        }
    }
    // ---- fused bottom subtrees: the largest cut height H such that at least `min_sub`
    // subtrees root at height <= H (enough workgroups to fill the chip) and every subtree level
    // fits the LDS budget; supernodes above H are solved level by level.
    std::vector<std::vector<int>> kids(nn_);
    for (int sn = 0; sn < nn_; ++sn) if (F.parent[sn] >= 0 && inc[sn]) kids[F.parent[sn]].push_back(sn);
    const char* ms = std::getenv("AA_SOLVE_MIN_SUBTREES");
    const bool stats = std::getenv("AA_SOLVE_STATS") != nullptr;
    const char* sb = std::getenv("AA_SUB_BLOCK");
    sub_block_ = sb ? std::atoi(sb) : 1024;
    // split-K tile width (forward columns / backward rows) per level: the widest of 256 / 128 /
    // 64 that still gives the level >= min_tiles workgroups (a level of few big supernodes gets
    // narrow tiles and enough workgroups to keep loads in flight on every CU; wide tiles keep the
    // partial traffic low where there is parallelism anyway). Structure only: the same for
    // one- and two-set solves. AA_SOLVE_TILE forces one width, AA_SOLVE_MIN_TILES the target.
    const char* tw = std::getenv("AA_SOLVE_TILE");
    const char* mt = std::getenv("AA_SOLVE_MIN_TILES");
    const int min_tiles = mt ? std::atoi(mt) : 0;   // 0: 256 everywhere (narrower measured slower on C4)
    const char* wp = std::getenv("AA_SOLVE_WAVEP");
    const char* wr = std::getenv("AA_SOLVE_WAVER");
    wave_p_ = wp ? std::atoi(wp) : wave_p;
    wave_r_ = wr ? std::atoi(wr) : wave_r;
    // fused subtrees wanted: enough workgroups to fill the chip on one GPU; a partitioned GPU's
    // share of the tree is P times smaller, and its fused subtrees cost a latency chain per level
    // whatever their count, so it takes fewer, taller ones (measured)
    const int min_sub = ms ? std::atoi(ms) : (comm_ ? std::max(32, 256 / comm_->size()) : 256);
    auto roots_at = [&](int H) {
        std::vector<int> r;
        for (int sn = 0; sn < nn_; ++sn)
            if (inc[sn] && F.height[sn] <= H && (F.parent[sn] < 0 || F.height[F.parent[sn]] > H)) r.push_back(sn);
        return r;
    };
    auto collect = [&](int root) {
        std::vector<int> out, st{root};
        while (!st.empty()) { int v = st.back(); st.pop_back(); out.push_back(v); for (int c : kids[v]) st.push_back(c); }
        return out;
    };
    {   // the cut height against the launch's aggregate LDS (solve_plan.hpp; the fused kernels'
        // LDS attribute is 160 KiB, set below)
        CutPlanIn pl;
        pl.parent = &F.parent; pl.height = &F.height; pl.inc = &inc; pl.p = &p; pl.nb = &nb;
        pl.max_height = F.max_height; pl.ks = KS; pl.min_sub = min_sub; pl.seg_rows = kSubSegRows;
        pl.node_bytes = (long long)sizeof(SubNode);
        cut_height_ = choose_cut_height(pl);
    }
    std::vector<char> fused(nn_, 0);
    {
        std::vector<SubNode> snodes;
        std::vector<SubLevel> slevels;
        std::vector<SubTree> strees;
        std::vector<int> items;
        std::vector<long long> items2;
        std::vector<int> fidx(nn_, -1), bidx(nn_, -1);   // forward / backward record of every fused supernode
        std::vector<std::vector<int>> sub_all;      // supernodes of every subtree (root first)
        sub_lds_f_ = sub_lds_b_ = 0;
        if (cut_height_ >= 0) {
            for (int rt : roots_at(cut_height_)) {
                std::vector<int> all = collect(rt);
                const int H = F.height[rt];
                SubTree T{(int)slevels.size(), H + 1, (int)snodes.size(), 0};
                for (int h = 0; h <= H; ++h) {
                    SubLevel L{};
                    L.n0 = (int)snodes.size();
                    int lf = 0, lb = 0;
                    std::vector<int> lv;
                    for (int v : all) if (F.height[v] == h) lv.push_back(v);
                    std::sort(lv.begin(), lv.end());
                    for (int v : lv) {
                        fused[v] = 1;
                        SubNode nd{};
                        nd.p = p[v]; nd.nb = nb[v]; nd.beg = beg[v]; nd.bnd_off = bnd_off[v]; nd.ell_w = ell_w[v];
                        nd.lds = 0; nd.goff = goff[v]; nd.uoff = uoff[v]; nd.ell_off = ell_off[v]; nd.ldr = ldr[v];
                        nd.slot = -1;   // forward copy: LDS update-vector slot (kSubU, set below)
                        nd.xo = -1;
                        fidx[v] = (int)snodes.size();
                        snodes.push_back(nd);
                    }
                    // forward: f_P offsets, assembly items, row items
                    L.fa0 = (int)items.size();
                    for (size_t k = 0; k < lv.size(); ++k) {
                        snodes[L.n0 + k].lds = lf / 8;
                        for (int c = 0; c < p[lv[k]]; ++c) items.push_back(((int)k << 16) | c);
                        lf += 24 * p[lv[k]];
                    }
                    L.nfa = (int)items.size() - L.fa0;
                    L.fr0 = (int)items.size();
                    for (size_t k = 0; k < lv.size(); ++k)
                        for (int r = 0; r < p[lv[k]] + nb[lv[k]]; ++r) items.push_back(((int)k << 16) | r);
                    L.nfr = (int)items.size() - L.fr0;
                    // backward: the same supernodes with their [y_P ; -x_B] vectors; the LDS
                    // offsets differ, so the backward items address a second copy of the nodes
                    const int n1 = (int)snodes.size();
                    for (size_t k = 0; k < lv.size(); ++k) {
                        SubNode nd = snodes[L.n0 + k];
                        bidx[lv[k]] = (int)snodes.size();
                        nd.lds = lb / 8;
                        lb += 24 * (p[lv[k]] + nb[lv[k]]);
                        snodes.push_back(nd);
                    }
                    L.bv0 = (int)items.size();
                    for (size_t k = 0; k < lv.size(); ++k)
                        for (int r = 0; r < p[lv[k]] + nb[lv[k]]; ++r) items.push_back(((int)(k + (n1 - L.n0)) << 16) | r);
                    L.nbv = (int)items.size() - L.bv0;
                    // segment partial slots after the level's vectors; items (node, segment, column)
                    L.bs0 = (int)items2.size();
                    for (size_t k = 0; k < lv.size(); ++k) {
                        SubNode& nd = snodes[n1 + k];
                        nd.slot = lb / 8;
                        const int pp = p[lv[k]], RR = pp + nb[lv[k]];
                        for (int sg = 0; sg * kSubSegRows < RR; ++sg) {
                            const int nc = std::min(pp, (sg + 1) * kSubSegRows);
                            for (int j = 0; j < nc; ++j)
                                items2.push_back(((long long)(k + (n1 - L.n0)) << 40) | ((long long)sg << 20) | j);
                            lb += 24 * nc;
                        }
                    }
                    L.nbs = (int)items2.size() - L.bs0;
                    L.bc0 = (int)items.size();
                    for (size_t k = 0; k < lv.size(); ++k)
                        for (int j = 0; j < p[lv[k]]; ++j) items.push_back(((int)(k + (n1 - L.n0)) << 16) | j);
                    L.nbc = (int)items.size() - L.bc0;
                    sub_lds_f_ = std::max(sub_lds_f_, lf);
                    sub_lds_b_ = std::max(sub_lds_b_, lb);
                    slevels.push_back(L);
                }
                T.nnode = (int)snodes.size() - T.node0;
                sub_nodes_max_ = std::max(sub_nodes_max_, T.nnode);
                strees.push_back(T);
                sub_all.push_back(std::move(all));
            }
        }
        n_sub_ = (int)strees.size();
        plan_sub_lds(F, kids, p, nb, beg, uoff, bnd_off, ell_w, ell_off, ell, bnd, fidx, bidx, sub_all, strees, snodes, KS,
                     stats, s);
        // ---- branches (AA_SOLVE_BRANCHES, see direct_solve.hpp): disjoint subtrees of the tree
        // solved on parallel streams, the supernodes above them ("top") after the join
        plan_branches(F, inc, fused, kids, p, nb, stats);
        if (nbr_ > 1) {
            int dev = 0;
            AA_HIP(hipStreamGetDevice(s, &dev));
            for (int b = 0; b < nbr_; ++b) side_[b].create(dev);
        }
        sub_rng_.assign(nbr_ + 1, {0, 0});
        if (nbr_ > 1) {   // fused subtrees grouped by branch (a SubTree is self-contained: reorder freely)
            std::vector<int> ord(strees.size());
            for (size_t t = 0; t < ord.size(); ++t) ord[t] = (int)t;
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return brn_[sub_all[a][0]] < brn_[sub_all[b][0]]; });
            std::vector<SubTree> st2;
            for (int t : ord) st2.push_back(strees[t]);
            strees.swap(st2);
            for (size_t k = 0; k < ord.size(); ++k) {
                const int b = brn_[sub_all[ord[k]][0]];
                if (b < 0 || b >= nbr_) throw Error(ERR_STATE, "DirectSolver: fused subtree outside the branches");
                if (sub_rng_[b].second == 0) sub_rng_[b].first = (int)k;
                ++sub_rng_[b].second;
            }
        } else {
            sub_rng_[0] = {0, n_sub_};
        }
        if (stats) {
            double by = 0;
            int nsn = 0;
            for (int sn = 0; sn < nn_; ++sn)
                if (fused[sn]) { by += 8.0 * (0.5 * p[sn] * (p[sn] + 1.0) + (double)p[sn] * nb[sn]); ++nsn; }
            std::fprintf(stderr, "[solve] fused subtrees: %d (cut height %d), %d supernodes, %.2f MB/sweep, lds f %d b %d\n",
                         n_sub_, cut_height_, nsn, by / 1e6, sub_lds_f_, sub_lds_b_);
            // per height inside the subtrees: supernodes, rows, the longest forward row loop (p)
            // and bytes -- a level's time is bounded below by its longest serial loop
            for (int h = 0; h <= cut_height_; ++h) {
                long long cnt = 0, rows = 0, maxp = 0, maxR = 0;
                double bh = 0;
                for (int sn = 0; sn < nn_; ++sn) {
                    if (!fused[sn] || F.height[sn] != h) continue;
                    ++cnt; rows += p[sn] + nb[sn];
                    maxp = std::max<long long>(maxp, p[sn]); maxR = std::max<long long>(maxR, p[sn] + nb[sn]);
                    bh += 8.0 * (0.5 * p[sn] * (p[sn] + 1.0) + (double)p[sn] * nb[sn]);
                }
                std::fprintf(stderr, "[solve]   sub height %d: %lld supernodes, %.1f rows/subtree, max p %lld, max R %lld, %.2f MB\n",
                             h, cnt, n_sub_ ? (double)rows / n_sub_ : 0.0, maxp, maxR, bh / 1e6);
            }
        }
        sub_nodes_.upload(snodes, s);
        sub_levels_.upload(slevels, s);
        sub_trees_.upload(strees, s);
        sub_items_.upload(items, s);
        sub_items2_.upload(items2, s);
    }
    // levels by height and their row tasks
    // partitioned: the shared top as ONE dense root supernode (nested_dissection merge_top) is
    // split over the GPUs by rows instead of being solved whole on each
    top_sn_ = -1;
    if (comm_) {
        int ntop = 0, cand = -1;
        for (int sn = 0; sn < nn_; ++sn)
            if ((*node_part)[sn] == -1 && p[sn] > 0) { ++ntop; cand = sn; }
        if (ntop == 1 && F.parent[cand] < 0 && nb[cand] == 0 && beg[cand] == top_beg_ && p[cand] == n_ - top_beg_ &&
            !fused[cand])
            top_sn_ = cand;
    }
    std::vector<std::vector<int>> hl(F.max_height + 1);
    for (int sn = 0; sn < nn_; ++sn) if (!fused[sn] && inc[sn] && sn != top_sn_) hl[F.height[sn]].push_back(sn);
    std::vector<Task> tasks;
    std::vector<BTile> btiles;
    std::vector<BRed> breds;
    std::vector<FTile> ftiles;
    std::vector<FRed> freds;
    std::vector<int> fwid, bwid;   // tile widths (packing)
    std::vector<int> ft_sn, fr_sn, bt_sn, br_sn;   // supernode of every tile / reduction (streams)
    std::vector<int> lev_of(nn_, -1);              // level of every level-scheduled supernode
    long long poff = 0;
    auto mk = [&](int sn, int r0, int nr) {
        Task t{};
        t.node = sn; t.r0 = r0; t.nr = nr;
        t.p = p[sn]; t.nb = nb[sn]; t.beg = beg[sn]; t.bnd_off = bnd_off[sn];
        t.ell_w = ell_w[sn];
        t.goff = goff[sn]; t.uoff = uoff[sn]; t.ell_off = ell_off[sn]; t.ldr = ldr[sn];
        return t;
    };
    levels_.clear();
    kernels_ = 0;

    int max_lds = 0;
    lbr_.clear();
    for (auto& l : hl) {
        if (l.empty()) continue;
        if (nbr_ > 1)   // contiguous per branch (then the top): every launch below takes a range
            std::stable_sort(l.begin(), l.end(), [&](int a, int b) { return brn_[a] < brn_[b]; });
        Level L;
        int fr = 0, br = 0;
        bool fwave = false, bwave = false;
        for (int sn : l) {
            const int R = p[sn] + nb[sn];
            if (p[sn] <= wave_p_) fr = std::max(fr, R);
            if (R <= wave_r_) br = std::max(br, p[sn]);
        }
        (void)fwave;
        L.fblock = fr > 128 ? 256 : (fr > 64 ? 128 : 64);
        (void)bwave;
        L.bblock = br > 128 ? 256 : (br > 64 ? 128 : 64);
        L.fwd_first = (int)tasks.size();
        for (int sn : l) {
            const int R = p[sn] + nb[sn];
            if (p[sn] <= wave_p_) {
                for (int r0 = 0; r0 < R; r0 += L.fblock) tasks.push_back(mk(sn, r0, std::min(L.fblock, R - r0)));
                L.lds_fwd = std::max(L.lds_fwd, 24 * p[sn]);
            }
        }
        L.fwd_count = (int)tasks.size() - L.fwd_first;
        // tile widths of this level (see min_tiles above)
        auto pick = [&](auto count) {
            if (tw) return std::atoi(tw) >= 256 ? 256 : (std::atoi(tw) >= 128 ? 128 : 64);
            if (min_tiles <= 0) return 256;
            for (int w : {256, 128}) if (count(w) >= min_tiles) return w;
            return 64;
        };
        L.ftw = pick([&](int w) {
            long long n = 0;
            for (int sn : l) {
                if (p[sn] <= wave_p_) continue;
                const int R = p[sn] + nb[sn];
                for (int r0 = 0; r0 < R; r0 += 64) n += std::min((r0 + 63) / w + 1, (p[sn] + w - 1) / w);
            }
            return n;
        });
        L.btw = pick([&](int w) {
            long long n = 0;
            for (int sn : l) {
                const int R = p[sn] + nb[sn];
                if (R <= wave_r_) continue;
                for (int c0 = 0; c0 < p[sn]; c0 += 128) n += (R - c0 + w - 1) / w;
            }
            return n;
        });
        const int ftw = L.ftw, btw = L.btw;
        // large supernodes: split-K forward tiles (64 rows x ftw columns; tiles entirely
        // above the diagonal of L_PP^-1 are zero and skipped), one reduction task per row block
        L.ft_first = (int)ftiles.size();
        L.fr_first = (int)freds.size();
        for (int sn : l) {
            if (p[sn] <= wave_p_) continue;
            const int R = p[sn] + nb[sn];
            for (int r0 = 0; r0 < R; r0 += 64) {
                FRed rd{};
                rd.beg = beg[sn]; rd.p = p[sn]; rd.r0 = r0; rd.nr = std::min(64, R - r0);
                rd.uoff = uoff[sn]; rd.ell_off = ell_off[sn]; rd.ell_w = ell_w[sn]; rd.poff = poff;
                for (int c0 = 0; c0 < p[sn]; c0 += ftw) {
                    if (r0 + 63 < c0) break;
                    FTile ft{};
                    ft.beg = beg[sn]; ft.p = p[sn]; ft.R = R; ft.c0 = c0; ft.r0 = r0;
                    ft.nc = std::min(ftw, p[sn] - c0);
                    ft.goff = goff[sn]; ft.ell_off = ell_off[sn]; ft.ell_w = ell_w[sn]; ft.poff = poff;
                    ft.rid = (int)freds.size();
                    poff += 3 * 64;
                    ftiles.push_back(ft);
                    fwid.push_back(ftw);
                    ft_sn.push_back(sn);
                    ++rd.nt;
                }
                freds.push_back(rd);
                fr_sn.push_back(sn);
            }
        }
        L.ft_count = (int)ftiles.size() - L.ft_first;
        L.frd_count = (int)freds.size() - L.fr_first;
        L.bwd_first = (int)tasks.size();
        for (int sn : l) {
            const int R = p[sn] + nb[sn];
            if (R <= wave_r_) {
                for (int j0 = 0; j0 < p[sn]; j0 += L.bblock) tasks.push_back(mk(sn, j0, std::min(L.bblock, p[sn] - j0)));
                L.lds_bwd = std::max(L.lds_bwd, 24 * R);
            }
        }
        L.bwd_count = (int)tasks.size() - L.bwd_first;
        // large supernodes: split-K tiles (128 columns x btw rows; the tiles above the
        // diagonal of L_PP^-1 are all zero and skipped) and one reduction task per column block
        L.bt_first = (int)btiles.size();
        L.br_first = (int)breds.size();
        for (int sn : l) {
            const int R = p[sn] + nb[sn];
            if (R <= wave_r_) continue;
            for (int c0 = 0; c0 < p[sn]; c0 += 128) {
                BRed rd{};
                rd.beg = beg[sn]; rd.c0 = c0; rd.nc = std::min(128, p[sn] - c0); rd.poff = poff;
                for (int r0 = c0; r0 < R; r0 += btw) {
                    BTile bt{};
                    bt.beg = beg[sn]; bt.p = p[sn]; bt.nb = nb[sn]; bt.bnd_off = bnd_off[sn];
                    bt.c0 = c0; bt.r0 = r0; bt.nr = std::min(btw, R - r0);
                    bt.goff = goff[sn]; bt.poff = poff; bt.ldr = ldr[sn];
                    bt.rid = (int)breds.size();
                    poff += 6 * 64;
                    btiles.push_back(bt);
                    bwid.push_back(btw);
                    bt_sn.push_back(sn);
                    ++rd.nt;
                }
                breds.push_back(rd);
                br_sn.push_back(sn);
            }
        }
        L.bt_count = (int)btiles.size() - L.bt_first;
        L.br_count = (int)breds.size() - L.br_first;
        max_lds = std::max(max_lds, std::max(L.lds_fwd, L.lds_bwd));
        kernels_ += (L.fwd_count ? 1 : 0) + (L.bwd_count ? 1 : 0) + (L.bt_count ? 1 : 0) + (L.ft_count ? 1 : 0);
        {   // per branch (and the top, slot nbr_): the sub-ranges of this level's four launches
            auto ranges = [&](int first, int count, auto node_of, int BrRange::*f, int BrRange::*c, size_t base) {
                for (int k = first; k < first + count; ++k) {
                    const int b = nbr_ > 1 ? brn_[node_of(k)] : 0;
                    BrRange& r = lbr_[base + b];
                    if (r.*c == 0) r.*f = k;
                    else if (r.*f + r.*c != k) throw Error(ERR_STATE, "DirectSolver: branch ranges not contiguous");
                    ++(r.*c);
                }
            };
            const size_t base = lbr_.size();
            lbr_.resize(base + nbr_ + 1);
            ranges(L.fwd_first, L.fwd_count, [&](int k) { return tasks[k].node; }, &BrRange::fwd_first, &BrRange::fwd_count, base);
            ranges(L.ft_first, L.ft_count, [&](int k) { return ft_sn[k]; }, &BrRange::ft_first, &BrRange::ft_count, base);
            ranges(L.bwd_first, L.bwd_count, [&](int k) { return tasks[k].node; }, &BrRange::bwd_first, &BrRange::bwd_count, base);
            ranges(L.bt_first, L.bt_count, [&](int k) { return bt_sn[k]; }, &BrRange::bt_first, &BrRange::bt_count, base);
        }
        levels_.push_back(L);
        for (int sn : l) lev_of[sn] = (int)levels_.size() - 1;
        if (stats) {
            double by = 0;
            int maxp = 0, maxnb = 0, nw = 0;
            for (int sn : l) {
                by += 8.0 * (0.5 * p[sn] * (p[sn] + 1.0) + (double)p[sn] * nb[sn]);
                maxp = std::max(maxp, p[sn]); maxnb = std::max(maxnb, nb[sn]);
                nw += p[sn] > wave_p_;
            }
            std::fprintf(stderr, "[solve] level %zu: %zu supernodes (%d tiled), max p %d, max nb %d, %.2f MB/sweep, "
                         "fwd tasks %d (blk %d) fwd tiles %d (w %d) bwd tasks %d (blk %d) bwd tiles %d (w %d)\n",
                         levels_.size() - 1, l.size(), nw, maxp, maxnb, by / 1e6, L.fwd_count, L.fblock, L.ft_count, L.ftw,
                         L.bwd_count, L.bblock, L.bt_count, L.btw);
        }
    }
    if (top_sn_ >= 0) {
        // rows [top_r0_, top_r1_) of the top triangle, in kTopBlk blocks, equal areas per GPU
        const int sn = top_sn_, P = comm_->size(), me = comm_->rank(), pt = p[sn];
        const int nblk = (pt + kTopBlk - 1) / kTopBlk;
        const double total = 0.5 * pt * (pt + 1.0);
        std::vector<int> cut(P + 1, nblk);
        cut[0] = 0;
        double acc = 0;
        int r = 1;
        for (int b = 0; b < nblk && r < P; ++b) {
            const double r0 = (double)b * kTopBlk, r1 = std::min<double>(pt, r0 + kTopBlk);
            acc += 0.5 * (r1 * (r1 + 1) - r0 * (r0 + 1));
            while (r < P && acc >= total * r / P) cut[r++] = b + 1;
        }
        top_p_ = pt;
        top_r0_ = std::min(pt, cut[me] * kTopBlk);
        top_r1_ = std::min(pt, cut[me + 1] * kTopBlk);
        top_task_ = mk(sn, 0, pt);
        top_ftw_ = tw ? (std::atoi(tw) >= 256 ? 256 : (std::atoi(tw) >= 128 ? 128 : 64)) : 256;
        top_btw_ = top_ftw_;
        // forward tiles of the own rows (64-row blocks); the front is read summed from top_f_
        top_ft_first_ = (int)ftiles.size();
        for (int r0 = top_r0_; r0 < top_r1_; r0 += 64) {
            FRed rd{};
            rd.beg = beg[sn]; rd.p = pt; rd.r0 = r0; rd.nr = std::min(64, top_r1_ - r0);
            rd.uoff = uoff[sn]; rd.ell_off = 0; rd.ell_w = 0; rd.poff = poff;
            for (int c0 = 0; c0 < pt; c0 += top_ftw_) {
                if (r0 + 63 < c0) break;
                FTile ft{};
                ft.beg = beg[sn]; ft.p = pt; ft.R = pt; ft.c0 = c0; ft.r0 = r0;
                ft.nc = std::min(top_ftw_, pt - c0);
                ft.goff = goff[sn]; ft.ell_off = 0; ft.ell_w = 0; ft.poff = poff;
                ft.rid = (int)freds.size();
                poff += 3 * 64;
                ftiles.push_back(ft);
                fwid.push_back(top_ftw_);
                ft_sn.push_back(sn);
                ++rd.nt;
            }
            freds.push_back(rd);
            fr_sn.push_back(sn);
        }
        top_ft_count_ = (int)ftiles.size() - top_ft_first_;
        // backward: the products of the own rows only (partial x_top, summed over the GPUs)
        top_bt_first_ = (int)btiles.size();
        for (int c0 = 0; c0 < top_r1_; c0 += 128) {
            const int rs = std::max(c0, top_r0_);
            if (rs >= top_r1_) continue;
            BRed rd{};
            rd.beg = beg[sn]; rd.c0 = c0; rd.nc = std::min(128, pt - c0); rd.poff = poff;
            for (int r0 = rs; r0 < top_r1_; r0 += top_btw_) {
                BTile bt{};
                bt.beg = beg[sn]; bt.p = pt; bt.nb = 0; bt.bnd_off = bnd_off[sn];
                bt.c0 = c0; bt.r0 = r0; bt.nr = std::min(top_btw_, top_r1_ - r0);
                bt.goff = goff[sn]; bt.poff = poff; bt.ldr = ldr[sn];
                bt.rid = (int)breds.size();
                poff += 6 * 64;
                btiles.push_back(bt);
                bwid.push_back(top_btw_);
                bt_sn.push_back(sn);
                ++rd.nt;
            }
            breds.push_back(rd);
            br_sn.push_back(sn);
        }
        top_bt_count_ = (int)btiles.size() - top_bt_first_;
        kernels_ += 4;
        // bytes: this GPU streams its row slice of the triangle (twice), not the whole top
        const double whole = 0.5 * pt * (pt + 1.0), a0 = top_r0_, a1 = top_r1_;
        dense -= whole;
        dense += 0.5 * (a1 * (a1 + 1) - a0 * (a0 + 1));
        top_task_d_.upload(std::vector<Task>{top_task_}, s);
        top_f_.alloc(3 * (size_t)KS * pt);
        top_x_.alloc(3 * (size_t)KS * pt);
        if (stats)
            std::fprintf(stderr, "[solve] dense top: %d rows, this GPU rows [%d, %d), fwd tiles %d, bwd tiles %d\n", pt,
                         top_r0_, top_r1_, top_ft_count_, top_bt_count_);
    }
    if (n_sub_) kernels_ += 2;
    if (const char* st = std::getenv("AA_SUB_TIMING")) {
        sub_timing_ = std::atoi(st);
        if (sub_timing_ > 0 && n_sub_ > 0) { sub_clk_.alloc(2 * 64 * (size_t)n_sub_); sub_clk_.zero(s); }
        if (cut_height_ + 1 > 21) sub_timing_ = 0;   // 64 clock slots per workgroup
    }
    bnd_.upload(bnd, s);
    ell_.upload(ell, s);
    Gr_.upload(Gr.get(), (size_t)go, s);
    Gc_.alloc((size_t)go);
    {   // Gc (column-major R x p per supernode) = transpose of Gr (row-major R x ldr), 32 x 32 tiles
        std::vector<TrTile> tt;
        for (int sn = 0; sn < nn_; ++sn) {
            if (!inc[sn]) continue;
            const int R = p[sn] + nb[sn];
            for (int r0 = 0; r0 < R; r0 += 32)
                for (int c0 = 0; c0 < p[sn]; c0 += 32) tt.push_back(TrTile{goff[sn], R, ldr[sn], p[sn], r0, c0});
        }
        if (!tt.empty()) {
            DevBuf<TrTile> dt;
            dt.upload(tt, s);
            hipLaunchKernelGGL(k_gr_to_gc, dim3((unsigned)tt.size()), dim3(32, 8), 0, s, dt.p, Gr_.p, Gc_.p);
            AA_CHECK_LAUNCH();
            AA_HIP(hipStreamSynchronize(s));
        }
    }
    // packed tiles: every tile's block in consumption order (see k_fwd_ptile), built on the
    // device from Gr; AA_SOLVE_PACKED=0 keeps the tiles on the strided copies (A/B)
    {
        const char* pk = std::getenv("AA_SOLVE_PACKED");
        packed_ = !(pk && pk[0] == '0');
    }
    if (packed_ && (!ftiles.empty() || !btiles.empty())) {
        long long to = 0;
        for (size_t i = 0; i < ftiles.size(); ++i) { ftiles[i].toff = to; to += 64LL * fwid[i]; }
        for (size_t i = 0; i < btiles.size(); ++i) {   // narrow blocks (<= 64 columns): half (k_pack_btiles)
            btiles[i].toff = to;
            to += (btiles[i].p - btiles[i].c0 <= 64 ? 64LL : 128LL) * bwid[i];
        }
        Gt_.alloc((size_t)to);
        DevBuf<FTile> dft;
        DevBuf<BTile> dbt;
        DevBuf<int> dfw, dbw;
        if (!ftiles.empty()) {
            dft.upload(ftiles, s);
            dfw.upload(fwid, s);
            hipLaunchKernelGGL(k_pack_ftiles, dim3((unsigned)ftiles.size()), dim3(256), 0, s, dft.p, dfw.p, Gr_.p, Gt_.p);
            AA_CHECK_LAUNCH();
        }
        if (!btiles.empty()) {
            dbt.upload(btiles, s);
            dbw.upload(bwid, s);
            hipLaunchKernelGGL(k_pack_btiles, dim3((unsigned)btiles.size()), dim3(256), 0, s, dbt.p, dbw.p, Gr_.p, Gt_.p);
            AA_CHECK_LAUNCH();
        }
        AA_HIP(hipStreamSynchronize(s));
        if (stats) std::fprintf(stderr, "[solve] packed tiles: %zu forward, %zu backward, %.1f MB\n", ftiles.size(),
                                btiles.size(), 8e-6 * (double)to);
    } else {
        packed_ = false;
    }
    // ---- streamed tile levels (see Stream in direct_solve.hpp): maximal runs of >= 2 consecutive
    // levels with packed split-K tiles only and one tile width. Forward: a tile of supernode s waits
    // for every update-row reduction of its children in the same run; backward: for every
    // reduction of its parent in the same run (the parent's rows and, through the parent's own
    // wait, all its ancestors' rows in the run).
    {
        const char* st = std::getenv("AA_SOLVE_STREAM");
        stream_ = packed_ && st && st[0] == '1';   // measured slower on C4: opt-in
        // a gated solve that is skipped (the Anderson reject path's, most iterations) costs one
        // dependent launch (~4.6 us in a graph) per level: its tile runs as one launch each cut
        // that; taken, a streamed run is slower than its levels
        const char* sg = std::getenv("AA_SOLVE_STREAM_GATED");
        stream_gated_ = packed_ && !node_part && (sg ? sg[0] == '1' : true);   // (one GPU)
    }
    stream_plan_ = stream_ || stream_gated_;
    fstreams_.clear();
    bstreams_.clear();
    std::vector<int> forder, border, bndx(bnd.size(), -1);
    long long xs_rows = 0;
    if (stream_plan_) {
        const int nL = (int)levels_.size();
        auto runs = [&](bool fwd) {
            std::vector<std::pair<int, int>> r;
            for (int i = 0; i < nL;) {
                auto ok = [&](int l) {
                    const Level& L = levels_[l];
                    return fwd ? (L.fwd_count == 0 && L.ft_count > 0) : (L.bwd_count == 0 && L.bt_count > 0);
                };
                auto wid = [&](int l) { return fwd ? levels_[l].ftw : levels_[l].btw; };
                if (!ok(i)) { ++i; continue; }
                int j = i + 1;
                while (j < nL && ok(j) && wid(j) == wid(i)) ++j;
                if (j - i >= 2) r.push_back({i, j});
                i = j;
            }
            return r;
        };
        const auto fr = runs(true), br = runs(false);
        n_heads_ = (int)(fr.size() + br.size());
        const int CF = n_heads_, CB = n_heads_ + nn_;   // counter bases in sync_
        std::vector<int> nfr_b(nn_, 0), nbr(nn_, 0);     // per supernode: update-row / all reductions
        for (size_t i = 0; i < freds.size(); ++i)
            if (freds[i].r0 + freds[i].nr > freds[i].p) ++nfr_b[fr_sn[i]];
        for (size_t i = 0; i < breds.size(); ++i) ++nbr[br_sn[i]];
        int head = 0;
        for (const auto& run : fr) {
            const int l0 = run.first, l1 = run.second;
            auto in = [&](int sn) { return sn >= 0 && lev_of[sn] >= l0 && lev_of[sn] < l1; };
            Stream S{l0, l1, (int)forder.size(), 0, head++};
            for (int l = l0; l < l1; ++l)
                for (int k = 0; k < levels_[l].ft_count; ++k) forder.push_back(levels_[l].ft_first + k);
            S.count = (int)forder.size() - S.first;
            for (int k = S.first; k < S.first + S.count; ++k) {
                FTile& ft = ftiles[forder[k]];
                const int sn = ft_sn[forder[k]];
                int need = 0;
                for (int c : kids[sn]) if (in(c)) need += nfr_b[c];
                ft.dep = CF + sn;
                ft.need = need;
            }
            for (size_t i = 0; i < freds.size(); ++i) {
                const int sn = fr_sn[i];
                if (!in(sn)) continue;
                const int par = F.parent[sn];
                freds[i].sig = (in(par) && freds[i].r0 + freds[i].nr > freds[i].p) ? CF + par : -1;
            }
            fstreams_.push_back(S);
        }
        std::vector<int> node_sn(n_, -1), xso(nn_, -1);
        for (int sn = 0; sn < nn_; ++sn)
            for (int i = F.beg[sn]; i < F.end[sn] && i < n_; ++i) node_sn[i] = sn;
        for (auto it = br.rbegin(); it != br.rend(); ++it) {   // processing order: top runs first
            const int l0 = it->first, l1 = it->second;
            auto in = [&](int sn) { return sn >= 0 && lev_of[sn] >= l0 && lev_of[sn] < l1; };
            Stream S{l0, l1, (int)border.size(), 0, head++};
            for (int l = l1 - 1; l >= l0; --l)
                for (int k = 0; k < levels_[l].bt_count; ++k) border.push_back(levels_[l].bt_first + k);
            S.count = (int)border.size() - S.first;
            std::vector<char> has_kid(nn_, 0);
            for (int l = l0; l < l1; ++l)
                for (int k = 0; k < levels_[l].bt_count; ++k) {
                    const int sn = bt_sn[levels_[l].bt_first + k];
                    if (in(F.parent[sn])) has_kid[F.parent[sn]] = 1;
                }
            for (int k = S.first; k < S.first + S.count; ++k) {
                BTile& bt = btiles[border[k]];
                const int sn = bt_sn[border[k]], par = F.parent[sn];
                bt.dep = in(par) ? CB + par : -1;
                bt.need = in(par) ? nbr[par] : 0;
                if (has_kid[sn] && xso[sn] < 0) { xso[sn] = (int)xs_rows; xs_rows += (p[sn] + 15) / 16 * 16; }
            }
            for (size_t i = 0; i < breds.size(); ++i) {
                const int sn = br_sn[i];
                if (!in(sn)) continue;
                breds[i].sig = has_kid[sn] ? CB + sn : -1;
                breds[i].xso = xso[sn];
            }
            // boundary rows of this run's supernodes owned by supernodes of the run: read from Xs
            for (int l = l0; l < l1; ++l)
                for (int k = 0; k < levels_[l].bt_count; ++k) {
                    const int sn = bt_sn[levels_[l].bt_first + k];
                    for (int a = 0; a < nb[sn]; ++a) {
                        const int node = F.bnd[sn][a], ow = node < n_ ? node_sn[node] : -1;
                        if (ow >= 0 && in(ow) && xso[ow] >= 0) bndx[bnd_off[sn] + a] = xso[ow] + (node - beg[ow]);
                    }
                }
            bstreams_.push_back(S);
        }
        if (stats)
            for (auto& S : fstreams_)
                std::fprintf(stderr, "[solve] streamed forward levels [%d, %d): %d tiles, one launch\n", S.l0, S.l1, S.count);
        if (stats)
            for (auto& S : bstreams_)
                std::fprintf(stderr, "[solve] streamed backward levels [%d, %d): %d tiles, one launch\n", S.l0, S.l1, S.count);
        if (fstreams_.empty() && bstreams_.empty()) stream_ = stream_gated_ = stream_plan_ = false;
    }
    if (stream_plan_) {
        forder_.upload(forder.empty() ? std::vector<int>{0} : forder, s);
        border_.upload(border.empty() ? std::vector<int>{0} : border, s);
        bndx_.upload(bndx.empty() ? std::vector<int>{-1} : bndx, s);
        sync_.alloc((size_t)n_heads_ + 2 * (size_t)nn_);
        sync_.zero(s);
        Xs_.alloc(std::max<long long>(3 * KS * xs_rows, 3));
    }
    tasks_.upload(tasks, s);
    btiles_.upload(btiles, s);
    ftiles_.upload(ftiles, s);
    freds_.upload(freds, s);
    fcnt_.alloc(std::max<size_t>(freds.size(), 1)); fcnt_.zero(s);
    bcnt_.alloc(std::max<size_t>(breds.size(), 1)); bcnt_.zero(s);
    breds_.upload(breds, s);
    bpart_.alloc(std::max<long long>(KS * poff, 3));
    Y_.alloc(3 * KS * (size_t)n_);
    U_.alloc(std::max<long long>(KS * uo, 3));
    // (LDS figures above are per 3 columns; a 6-column solve needs twice as much; + the staged nodes)
    // internal assert: choose_cut_height budgets exactly this aggregate
    if (std::max(sub_lds_bytes(KS, true), sub_lds_bytes(KS, false)) > 160 * 1024)
        throw Error(ERR_STATE, "DirectSolver: internal error: fused subtrees exceed 160 KiB of LDS");
    if (std::max(sub_lds_bytes(KS, true), sub_lds_bytes(KS, false)) > 64 * 1024)
        for (const void* k : {(const void*)k_fwd_sub<256, 3, false>, (const void*)k_fwd_sub<512, 3, false>, (const void*)k_fwd_sub<1024, 3, false>,
                              (const void*)k_bwd_sub<256, 3, false>, (const void*)k_bwd_sub<512, 3, false>, (const void*)k_bwd_sub<1024, 3, false>,
                              (const void*)k_fwd_sub<256, 6, false>, (const void*)k_fwd_sub<512, 6, false>, (const void*)k_fwd_sub<1024, 6, false>,
                              (const void*)k_bwd_sub<256, 6, false>, (const void*)k_bwd_sub<512, 6, false>, (const void*)k_bwd_sub<1024, 6, false>,
                              (const void*)k_fwd_sub<256, 3, true>, (const void*)k_fwd_sub<512, 3, true>, (const void*)k_fwd_sub<1024, 3, true>,
                              (const void*)k_bwd_sub<256, 3, true>, (const void*)k_bwd_sub<512, 3, true>, (const void*)k_bwd_sub<1024, 3, true>,
                              (const void*)k_fwd_sub<256, 6, true>, (const void*)k_fwd_sub<512, 6, true>, (const void*)k_fwd_sub<1024, 6, true>,
                              (const void*)k_bwd_sub<256, 6, true>, (const void*)k_bwd_sub<512, 6, true>, (const void*)k_bwd_sub<1024, 6, true>})
            AA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (KS * max_lds > 64 * 1024) {   // large fronts: opt in to more than the default 64 KiB of LDS
        for (const void* k : {(const void*)k_fwd<64, 3, false>, (const void*)k_fwd<128, 3, false>, (const void*)k_fwd<256, 3, false>,
                              (const void*)k_bwd<64, 3, false>, (const void*)k_bwd<128, 3, false>, (const void*)k_bwd<256, 3, false>,
                              (const void*)k_fwd<64, 6, false>, (const void*)k_fwd<128, 6, false>, (const void*)k_fwd<256, 6, false>,
                              (const void*)k_bwd<64, 6, false>, (const void*)k_bwd<128, 6, false>, (const void*)k_bwd<256, 6, false>,
                              (const void*)k_fwd<64, 3, true>, (const void*)k_fwd<128, 3, true>, (const void*)k_fwd<256, 3, true>,
                              (const void*)k_bwd<64, 3, true>, (const void*)k_bwd<128, 3, true>, (const void*)k_bwd<256, 3, true>,
                              (const void*)k_fwd<64, 6, true>, (const void*)k_fwd<128, 6, true>, (const void*)k_fwd<256, 6, true>,
                              (const void*)k_bwd<64, 6, true>, (const void*)k_bwd<128, 6, true>, (const void*)k_bwd<256, 6, true>})
            AA_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    }
    // algorithmic bytes of one solve: the factor once per sweep (dense triangles + boundary
    // blocks, fp64), b/y/x (24 B per node each way) and the update vectors (write + read)
    bytes_ = 2.0 * 8.0 * (dense + offd) + 4.0 * 24.0 * piv + 3.0 * 24.0 * bsum;
    {   // non-temporal factor loads when a solve's factor stream cannot stay in the Infinity Cache
        const char* e = std::getenv("AA_FACTOR_NT");
        nt_ = e ? e[0] == '1' : 2.0 * 8.0 * (dense + offd) > kNtBytes;
        // the thread-per-row kernels (fused subtrees, row tasks) separately (AA_FACTOR_NT_ROWS):
        // their 8-B-per-lane loads cover partial lines that a neighbouring wave re-reads, which nt
        // drops from L2 (PMC, C4: fused backward 1.41 -> 1.81x its factor bytes read). Measured
        // (same-box A/B): nt on the rows costs C4 (2 GB both sweeps) 33 us and C5 (0.69 GB) 44 us
        // per solve, and saves C3 (0.28 GB) 12 us -- on only where the factor is within ~2x the
        // Infinity Cache
        const char* er = std::getenv("AA_FACTOR_NT_ROWS");
        nt_rows_ = er ? er[0] == '1' : (nt_ && 2.0 * 8.0 * (dense + offd) < kNtRowsMaxBytes);
    }
    bytes2_ = 2.0 * 8.0 * (dense + offd) + 2.0 * (4.0 * 24.0 * piv + 3.0 * 24.0 * bsum);
    AA_HIP(hipStreamSynchronize(s));
}

// dynamic LDS of a fused-subtree launch: the level vectors (K sets), the LDS-resident update
// vectors (forward) or x rows (backward), then the staged node records
size_t DirectSolver::sub_lds_bytes(int K, bool fwd) const {
    const size_t v = (size_t)K * (fwd ? sub_lds_f_ + sub_lds_u_ : sub_lds_b_ + sub_lds_x_);
    return (v + 15) / 16 * 16 + (size_t)sub_nodes_max_ * sizeof(SubNode);
}

void DirectSolver::plan_sub_lds(const SupernodalFactor& F, const std::vector<std::vector<int>>& kids,
                                const std::vector<int>& p, const std::vector<int>& nb, const std::vector<int>& beg,
                                const std::vector<long long>& uoff, const std::vector<int>& bnd_off,
                                const std::vector<int>& ell_w, const std::vector<long long>& ell_off,
                                std::vector<long long>& ell, std::vector<int>& bnd, const std::vector<int>& fidx,
                                const std::vector<int>& bidx, const std::vector<std::vector<int>>& sub_all, std::vector<SubTree>& strees,
                                std::vector<SubNode>& snodes, int KS, bool stats, hipStream_t s) {
    sub_lds_u_ = sub_lds_x_ = 0;
    const char* eu = std::getenv("AA_SUB_LDS_U");
    const char* ex = std::getenv("AA_SUB_LDS_X");
    const bool want_u = !eu || eu[0] != '0', want_x = !ex || ex[0] != '0';
    // vector bytes (KS sets) a launch may hold: 160 KiB less the staged records
    const long long cap = (160LL * 1024 - (long long)sub_nodes_max_ * (long long)sizeof(SubNode)) / 16 * 16;
    const int ubase = sub_lds_f_ / 8, xbase = sub_lds_b_ / 8;   // the regions follow the level vectors
    std::vector<int> slot(nn_, -1), xg;
    int nu = 0, nx = 0;
    for (size_t t = 0; t < sub_all.size(); ++t) {
        const std::vector<int>& all = sub_all[t];
        SubTree& T = strees[t];
        const int rt = all[0];
        if (want_u) {
            const int peak = plan_update_slots(all, kids, F.height, nb, slot);
            if ((long long)KS * (sub_lds_f_ + 24LL * peak) <= cap) {
                T.flags |= kSubU;
                ++nu;
                sub_lds_u_ = std::max(sub_lds_u_, 24 * peak);
                for (int v : all) {
                    snodes[fidx[v]].slot = slot[v] >= 0 ? ubase + 3 * slot[v] : -1;
                    // v's pull lists name its children's update entries (all inside the subtree)
                    const long long e1 = ell_off[v] + (long long)(p[v] + nb[v]) * ell_w[v];
                    for (long long i = ell_off[v]; i < e1; ++i) {
                        const long long e = ell[i];
                        if (e < 0) continue;
                        long long to = -1;
                        for (int c : kids[v])
                            if (e >= uoff[c] && e < uoff[c] + 3LL * nb[c]) { to = ubase + 3LL * slot[c] + (e - uoff[c]); break; }
                        if (to < 0) throw Error(ERR_STATE, "DirectSolver: internal error: a pull outside its fused subtree");
                        ell[i] = to;
                    }
                }
            }
        }
        if (want_x) {
            // the x rows a boundary inside the subtree can name: the columns of its inner supernodes
            // (a boundary names ancestors only, so leaves' columns never) and the root's boundary
            // (every entry leaving the subtree is one of them: fill-path property of the
            // elimination tree; checked, else the subtree keeps HBM)
            std::vector<std::pair<int, int>> inner;   // (first column, supernode), sorted
            int rows = 0;
            for (int v : all)
                if (!kids[v].empty()) { inner.emplace_back(beg[v], v); rows += p[v]; }
            std::sort(inner.begin(), inner.end());
            const std::vector<int>& rb = F.bnd[rt];
            const int nxg = (int)rb.size();
            if ((long long)KS * (sub_lds_b_ + 24LL * (rows + nxg)) <= cap) {
                std::vector<int> xo(inner.size());
                for (size_t k = 0, r = 0; k < inner.size(); r += p[inner[k].second], ++k) xo[k] = xbase + 3 * (int)r;
                std::vector<std::pair<int, int>> rw;
                bool ok = true;
                for (int v : all) {
                    for (int a = 0; a < nb[v] && ok; ++a) {
                        const int i = bnd[bnd_off[v] + a];
                        auto in = std::upper_bound(inner.begin(), inner.end(), std::make_pair(i, INT32_MAX));
                        int o = -1;
                        if (in != inner.begin()) {
                            --in;
                            const int w = in->second;
                            if (i < beg[w] + p[w]) o = xo[in - inner.begin()] + 3 * (i - beg[w]);
                        }
                        if (o < 0) {
                            auto it = std::lower_bound(rb.begin(), rb.end(), i);
                            if (it == rb.end() || *it != i) { ok = false; break; }
                            o = xbase + 3 * (rows + (int)(it - rb.begin()));
                        }
                        rw.emplace_back(bnd_off[v] + a, o);
                    }
                    if (!ok) break;
                }
                if (ok) {
                    for (const auto& q : rw) bnd[q.first] = q.second;
                    for (size_t k = 0; k < inner.size(); ++k) snodes[bidx[inner[k].second]].xo = xo[k];
                    T.flags |= kSubX;
                    ++nx;
                    T.xst = xbase + 3 * rows;
                    T.nxg = nxg;
                    T.xg_off = (int)xg.size();
                    xg.insert(xg.end(), rb.begin(), rb.end());
                    sub_lds_x_ = std::max(sub_lds_x_, 24 * (rows + nxg));
                }
            }
        }
    }
    if (xg.empty()) xg.push_back(0);
    sub_xg_.upload(xg, s);
    if (stats)
        std::fprintf(stderr, "[solve] fused subtrees in LDS: update vectors %d / %zu (%d B), x rows %d / %zu (%d B), per 3 columns\n",
                     nu, sub_all.size(), sub_lds_u_, nx, sub_all.size(), sub_lds_x_);
}

// Branches: the supernodes that head the B heaviest disjoint subtrees (found by expanding the
// heaviest non-fused node of the frontier, from the roots down, until there are B of them;
// expanded nodes form the top), dealt to B streams by decreasing factor bytes (each to the
// lightest stream so far). Every launch of a sweep below the top then runs once per branch on its
// own stream: a branch's next level starts while another branch's level still drains, so the
// levels' ramp and tail overlap instead of adding up. Same tasks, tiles and sums: bit-identical.
void DirectSolver::plan_branches(const SupernodalFactor& F, const std::vector<char>& inc, const std::vector<char>& fused,
                                 const std::vector<std::vector<int>>& kids, const std::vector<int>& p,
                                 const std::vector<int>& nb, bool stats) {
    nbr_ = 1;
    brn_.assign(nn_, 0);
    const char* er = std::getenv("AA_SOLVE_BRANCHES_REJECT");
    branch_reject_ = er && er[0] == '1';
    const char* e = std::getenv("AA_SOLVE_BRANCHES");
    const char* st = std::getenv("AA_SOLVE_STREAM");
    const int want = std::max(1, std::min(kMaxBranches, e ? std::atoi(e) : default_branches));
    if (want < 2 || (st && st[0] == '1')) return;
    // subtree weights (factor entries), children before parents by height
    std::vector<int> order;
    for (int sn = 0; sn < nn_; ++sn) if (inc[sn]) order.push_back(sn);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return F.height[a] < F.height[b]; });
    std::vector<double> wt(nn_, 0.0);
    for (int sn : order) {
        wt[sn] += 0.5 * p[sn] * (p[sn] + 1.0) + (double)p[sn] * nb[sn];
        if (F.parent[sn] >= 0 && inc[F.parent[sn]]) wt[F.parent[sn]] += wt[sn];
    }
    std::vector<int> front, top;
    for (int sn : order) if (F.parent[sn] < 0 || !inc[F.parent[sn]]) front.push_back(sn);
    while ((int)front.size() < want) {
        int best = -1;
        for (size_t k = 0; k < front.size(); ++k) {
            const int v = front[k];
            if (fused[v] || kids[v].empty()) continue;
            if (best < 0 || wt[v] > wt[front[best]]) best = (int)k;
        }
        if (best < 0) break;
        const int v = front[best];
        front.erase(front.begin() + best);
        top.push_back(v);
        for (int c : kids[v]) front.push_back(c);
    }
    if (front.size() < 2) return;
    const int B = std::min<int>(want, (int)front.size());
    std::sort(front.begin(), front.end(), [&](int a, int b) { return wt[a] > wt[b]; });
    std::vector<double> load(B, 0.0);
    for (int v : front) {
        const int b = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        load[b] += wt[v];
        std::vector<int> st2{v};
        while (!st2.empty()) {
            const int u = st2.back();
            st2.pop_back();
            brn_[u] = b;
            for (int c : kids[u]) st2.push_back(c);
        }
    }
    for (int v : top) brn_[v] = B;
    nbr_ = B;
    if (stats) {
        double tw = 0;
        for (int v : top) tw += 0.5 * p[v] * (p[v] + 1.0) + (double)p[v] * nb[v];
        std::fprintf(stderr, "[solve] branches: %d streams, %zu top supernodes (%.1f MB/sweep), branch MB/sweep:", B, top.size(),
                     8e-6 * tw);
        for (double l : load) std::fprintf(stderr, " %.1f", 8e-6 * l);
        std::fprintf(stderr, "\n");
    }
}

void DirectSolver::solve(const double* b, double* x, const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    solve_nr<3>(b, x, nullptr, nullptr, ctrl, gate_reject, s);
}

void DirectSolver::solve2(const double* b0, double* x0, const double* b1, double* x1, const Ctrl* ctrl, int gate_reject,
                          hipStream_t s) {
    if (max_sets_ < 2) throw Error(ERR_STATE, "DirectSolver::solve2 needs build(..., max_sets = 2)");
    solve_nr<6>(b0, x0, b1, x1, ctrl, gate_reject, s);
}

// one launch of split-K tiles (width w = forward columns / backward rows per tile): packed or on
// the strided copies
template <int NR>
void DirectSolver::launch_ftiles(int w, int count, int first, const double* b0, const double* b1, int ext_off,
                                 const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    if (packed_) {
        auto kf = w == 256 ? (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 256, AA_TILE_DEPTH, false, true> : k_fwd_ptile<NR, AA_FWD_CH, 256, AA_TILE_DEPTH, false, false>)
                  : w == 128 ? (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 128, AA_TILE_DEPTH, false, true> : k_fwd_ptile<NR, AA_FWD_CH, 128, AA_TILE_DEPTH, false, false>)
                             : (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 64, AA_TILE_DEPTH, false, true> : k_fwd_ptile<NR, AA_FWD_CH, 64, AA_TILE_DEPTH, false, false>);
        hipLaunchKernelGGL(kf, dim3(count), dim3(256), 0, s, ftiles_.p, first, Gt_.p, ell_.p, b0, b1, bpart_.p, freds_.p,
                           fcnt_.p, Y_.p, U_.p, ctrl, gate_reject, ext_off, nullptr, nullptr, 0);
    } else {
        auto kf = w == 256 ? k_fwd_tile<NR, AA_FWD_CH, 256> : (w == 128 ? k_fwd_tile<NR, AA_FWD_CH, 128> : k_fwd_tile<NR, AA_FWD_CH, 64>);
        hipLaunchKernelGGL(kf, dim3(count), dim3(256), 0, s, ftiles_.p, first, Gc_.p, ell_.p, b0, b1, bpart_.p, freds_.p,
                           fcnt_.p, Y_.p, U_.p, ctrl, gate_reject, ext_off);
    }
}
template <int NR>
void DirectSolver::launch_btiles(int w, int count, int first, double* x0, double* x1, int ext_off, const Ctrl* ctrl,
                                 int gate_reject, hipStream_t s) {
    if (packed_) {
        auto kb = w == 256 ? (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 256, AA_TILE_DEPTH, false, true> : k_bwd_ptile<NR, AA_BWD_CH, 256, AA_TILE_DEPTH, false, false>)
                  : w == 128 ? (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 128, AA_TILE_DEPTH, false, true> : k_bwd_ptile<NR, AA_BWD_CH, 128, AA_TILE_DEPTH, false, false>)
                             : (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 64, AA_TILE_DEPTH, false, true> : k_bwd_ptile<NR, AA_BWD_CH, 64, AA_TILE_DEPTH, false, false>);
        hipLaunchKernelGGL(kb, dim3(count), dim3(256), 0, s, btiles_.p, first, Gt_.p, bnd_.p, Y_.p, x0, x1, bpart_.p,
                           breds_.p, bcnt_.p, ctrl, gate_reject, ext_off, nullptr, nullptr, 0, nullptr, nullptr);
    } else {
        auto kb = w == 256 ? k_bwd_tile<NR, AA_BWD_CH, 256> : (w == 128 ? k_bwd_tile<NR, AA_BWD_CH, 128> : k_bwd_tile<NR, AA_BWD_CH, 64>);
        hipLaunchKernelGGL(kb, dim3(count), dim3(256), 0, s, btiles_.p, first, Gr_.p, bnd_.p, Y_.p, x0, x1, bpart_.p,
                           breds_.p, bcnt_.p, ctrl, gate_reject, ext_off);
    }
}

// one launch of a streamed run of levels (packed tiles, one width)
template <int NR>
void DirectSolver::launch_fstream(const Stream& S, const double* b0, const double* b1, const Ctrl* ctrl, int gate_reject,
                                  hipStream_t s) {
    const int w = levels_[S.l0].ftw;
    auto kf = w == 256 ? (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 256, AA_TILE_DEPTH, true, true> : k_fwd_ptile<NR, AA_FWD_CH, 256, AA_TILE_DEPTH, true, false>)
                  : w == 128 ? (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 128, AA_TILE_DEPTH, true, true> : k_fwd_ptile<NR, AA_FWD_CH, 128, AA_TILE_DEPTH, true, false>)
                             : (nt_ ? k_fwd_ptile<NR, AA_FWD_CH, 64, AA_TILE_DEPTH, true, true> : k_fwd_ptile<NR, AA_FWD_CH, 64, AA_TILE_DEPTH, true, false>);
    hipLaunchKernelGGL(kf, dim3(S.count), dim3(256), 0, s, ftiles_.p, S.first, Gt_.p, ell_.p, b0, b1, bpart_.p, freds_.p,
                       fcnt_.p, Y_.p, U_.p, ctrl, gate_reject, 0, forder_.p, sync_.p, S.head);
}
template <int NR>
void DirectSolver::launch_bstream(const Stream& S, double* x0, double* x1, const Ctrl* ctrl, int gate_reject,
                                  hipStream_t s) {
    const int w = levels_[S.l0].btw;
    auto kb = w == 256 ? (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 256, AA_TILE_DEPTH, true, true> : k_bwd_ptile<NR, AA_BWD_CH, 256, AA_TILE_DEPTH, true, false>)
                  : w == 128 ? (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 128, AA_TILE_DEPTH, true, true> : k_bwd_ptile<NR, AA_BWD_CH, 128, AA_TILE_DEPTH, true, false>)
                             : (nt_ ? k_bwd_ptile<NR, AA_BWD_CH, 64, AA_TILE_DEPTH, true, true> : k_bwd_ptile<NR, AA_BWD_CH, 64, AA_TILE_DEPTH, true, false>);
    hipLaunchKernelGGL(kb, dim3(S.count), dim3(256), 0, s, btiles_.p, S.first, Gt_.p, bnd_.p, Y_.p, x0, x1, bpart_.p,
                       breds_.p, bcnt_.p, ctrl, gate_reject, 0, border_.p, sync_.p, S.head, bndx_.p, Xs_.p);
}

template <int NR>
void DirectSolver::solve_nr(const double* b0, double* x0, const double* b1, double* x1, const Ctrl* ctrl,
                            int gate_reject, hipStream_t s) {
    constexpr int K = NR / 3;
    const Task* T = tasks_.p;
    // AA_SUB_TIMING: phase clocks of the fused subtrees, printed for the first solves (eager only)
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    AA_HIP(hipStreamIsCapturing(s, &cst));
    const bool clk_on = sub_timing_ > 0 && cst == hipStreamCaptureStatusNone && n_sub_ > 0;
    const int noff_f = (K * (sub_lds_f_ + sub_lds_u_) + 15) / 16 * 16, noff_b = (K * (sub_lds_b_ + sub_lds_x_) + 15) / 16 * 16;
    // queue heads and dependency counters of the streamed runs start from zero every solve
    const bool st_on = stream_plan_ && (stream_ || (gate_reject == 1 && stream_gated_));
    if (st_on) AA_HIP(hipMemsetAsync(sync_.p, 0, sizeof(int) * ((size_t)n_heads_ + 2 * (size_t)nn_), s));
#define SUBF(BL, T0, NT, ST) hipLaunchKernelGGL((nt_rows_ ? k_fwd_sub<BL, NR, true> : k_fwd_sub<BL, NR, false>), dim3(NT), dim3(BL), sub_lds_bytes(K, true), ST, sub_trees_.p, \
                                    sub_levels_.p, sub_nodes_.p, sub_items_.p, Gc_.p, ell_.p, b0, b1, Y_.p, U_.p, ctrl, gate_reject, \
                                    clk_on ? sub_clk_.p : nullptr, 64, noff_f, T0)
#define SUBB(BL, T0, NT, ST) hipLaunchKernelGGL((nt_rows_ ? k_bwd_sub<BL, NR, true> : k_bwd_sub<BL, NR, false>), dim3(NT), dim3(BL), sub_lds_bytes(K, false), ST, sub_trees_.p, \
                                    sub_levels_.p, sub_nodes_.p, sub_items_.p, sub_items2_.p, Gr_.p, bnd_.p, Y_.p, x0, x1, sub_xg_.p, \
                                    ctrl, gate_reject, clk_on ? sub_clk_.p + 64 * (size_t)n_sub_ : nullptr, 64, noff_b, T0)
#define FWD(BL, F0, NC, LDS, ST) hipLaunchKernelGGL((nt_rows_ ? k_fwd<BL, NR, true> : k_fwd<BL, NR, false>), dim3(NC), dim3(BL), LDS, ST, T, F0, Gc_.p, \
                                   ell_.p, b0, b1, Y_.p, U_.p, ctrl, gate_reject)
#define BWD(BL, F0, NC, LDS, ST) hipLaunchKernelGGL((nt_rows_ ? k_bwd<BL, NR, true> : k_bwd<BL, NR, false>), dim3(NC), dim3(BL), LDS, ST, T, F0, Gr_.p, \
                                   bnd_.p, Y_.p, x0, x1, ctrl, gate_reject)
    auto sub_fwd = [&](int t0, int nt, hipStream_t st) {
        if (nt) switch (sub_block_) { case 1024: SUBF(1024, t0, nt, st); break; case 512: SUBF(512, t0, nt, st); break; default: SUBF(256, t0, nt, st); break; }
    };
    auto sub_bwd = [&](int t0, int nt, hipStream_t st) {
        if (nt) switch (sub_block_) { case 1024: SUBB(1024, t0, nt, st); break; case 512: SUBB(512, t0, nt, st); break; default: SUBB(256, t0, nt, st); break; }
    };
    // one level's forward (row tasks, then split-K tiles) / backward launches over a range
    auto lvl_fwd = [&](const Level& L, const BrRange& r, hipStream_t st) {
        if (r.fwd_count) switch (L.fblock) { case 64: FWD(64, r.fwd_first, r.fwd_count, K * L.lds_fwd, st); break;
                                              case 128: FWD(128, r.fwd_first, r.fwd_count, K * L.lds_fwd, st); break;
                                              default: FWD(256, r.fwd_first, r.fwd_count, K * L.lds_fwd, st); break; }
        if (r.ft_count) launch_ftiles<NR>(L.ftw, r.ft_count, r.ft_first, b0, b1, 0, ctrl, gate_reject, st);
    };
    auto lvl_bwd = [&](const Level& L, const BrRange& r, hipStream_t st) {
        if (r.bwd_count) switch (L.bblock) { case 64: BWD(64, r.bwd_first, r.bwd_count, K * L.lds_bwd, st); break;
                                              case 128: BWD(128, r.bwd_first, r.bwd_count, K * L.lds_bwd, st); break;
                                              default: BWD(256, r.bwd_first, r.bwd_count, K * L.lds_bwd, st); break; }
        if (r.bt_count) launch_btiles<NR>(L.btw, r.bt_count, r.bt_first, x0, x1, 0, ctrl, gate_reject, st);
    };
#undef SUBF
#undef SUBB
#undef FWD
#undef BWD
    // the reject path's gated one-set solve (skipped in most iterations) on one stream unless
    // AA_SOLVE_BRANCHES_REJECT=1: a skipped solve costs its launches, twice the streams twice them
    const int NB = (gate_reject && !branch_reject_) ? 1 : nbr_;
    if (NB > 1) {
        // branches: fork, each branch's fused subtrees and levels on its stream, join, then the
        // top's levels on s (see plan_branches)
        AA_HIP(hipEventRecord(side_[0].fork_f, s));
        for (int b = 1; b < NB; ++b) AA_HIP(hipStreamWaitEvent(side_[b].st, side_[0].fork_f, 0));
        for (int b = 0; b < NB; ++b) {
            hipStream_t st = b ? side_[b].st : s;
            sub_fwd(sub_rng_[b].first, sub_rng_[b].second, st);
            for (size_t li = 0; li < levels_.size(); ++li) lvl_fwd(levels_[li], lbr_[li * (NB + 1) + b], st);
        }
        for (int b = 1; b < NB; ++b) {
            AA_HIP(hipEventRecord(side_[b].join_f, side_[b].st));
            AA_HIP(hipStreamWaitEvent(s, side_[b].join_f, 0));
        }
        for (size_t li = 0; li < levels_.size(); ++li) lvl_fwd(levels_[li], lbr_[li * (NB + 1) + NB], s);
    } else {
        sub_fwd(0, n_sub_, s);
    }
    size_t fs = 0;
    for (int li = 0; li < (int)levels_.size() && NB == 1; ++li) {
        const Level& L = levels_[li];
        if (st_on && fs < fstreams_.size() && fstreams_[fs].l0 == li) {
            launch_fstream<NR>(fstreams_[fs], b0, b1, ctrl, gate_reject, s);
            li = fstreams_[fs++].l1 - 1;
            continue;
        }
        BrRange r;
        r.fwd_first = L.fwd_first; r.fwd_count = L.fwd_count; r.ft_first = L.ft_first; r.ft_count = L.ft_count;
        lvl_fwd(L, r, s);
    }
    // partitioned: the top rows of Y hold this GPU's share of the forward result (linear in b
    // and in the update vectors); their sum over the GPUs is the full forward result. When the
    // solve is gated off the stale rows are summed too -- harmless, the next forward rewrites
    // them and the backward sweep is gated alike on every GPU.
    if (top_sn_ >= 0) {
        // dense top: sum the front over the GPUs, forward of the own rows, backward products of
        // the own rows into a partial x_top, sum it, scatter it into x
        const int pt = top_p_;
        const unsigned nb = (unsigned)((pt + 255) / 256);
        hipLaunchKernelGGL((k_top_front<NR>), dim3(nb), dim3(256), 0, s, top_task_d_.p, ell_.p, b0, b1, U_.p, top_f_.p,
                           ctrl, gate_reject);
        comm_->allreduce_sum(top_f_.p, top_f_.p, 3 * (size_t)K * pt, s);
        // the tiles address the front / x by global row beg + q: the set-major buffers hold rows
        // from beg on (ext_off)
        const int eo = top_task_.beg;
        if (top_ft_count_)
            launch_ftiles<NR>(top_ftw_, top_ft_count_, top_ft_first_, top_f_.p, top_f_.p + 3 * (size_t)pt, eo, ctrl,
                              gate_reject, s);
        AA_HIP(hipMemsetAsync(top_x_.p, 0, sizeof(double) * 3 * (size_t)K * pt, s));
        if (top_bt_count_)
            launch_btiles<NR>(top_btw_, top_bt_count_, top_bt_first_, top_x_.p, top_x_.p + 3 * (size_t)pt, eo, ctrl,
                              gate_reject, s);
        comm_->allreduce_sum(top_x_.p, top_x_.p, 3 * (size_t)K * pt, s);
        hipLaunchKernelGGL((k_top_scatter<NR>), dim3(nb), dim3(256), 0, s, top_task_d_.p, top_x_.p, x0, x1, ctrl,
                           gate_reject);
    } else if (comm_ && top_beg_ < n_) {
        comm_->allreduce_sum(Y_.p + NR * (size_t)top_beg_, Y_.p + NR * (size_t)top_beg_, NR * (size_t)(n_ - top_beg_), s);
    }
    if (NB > 1) {   // the backward mirrors the forward: the top first, then the branches
        for (int li = (int)levels_.size() - 1; li >= 0; --li) lvl_bwd(levels_[li], lbr_[li * (NB + 1) + NB], s);
        AA_HIP(hipEventRecord(side_[0].fork_b, s));
        for (int b = 1; b < NB; ++b) AA_HIP(hipStreamWaitEvent(side_[b].st, side_[0].fork_b, 0));
        for (int b = 0; b < NB; ++b) {
            hipStream_t st = b ? side_[b].st : s;
            for (int li = (int)levels_.size() - 1; li >= 0; --li) lvl_bwd(levels_[li], lbr_[li * (NB + 1) + b], st);
            sub_bwd(sub_rng_[b].first, sub_rng_[b].second, st);
        }
        for (int b = 1; b < NB; ++b) {
            AA_HIP(hipEventRecord(side_[b].join_b, side_[b].st));
            AA_HIP(hipStreamWaitEvent(s, side_[b].join_b, 0));
        }
        AA_CHECK_LAUNCH();
        if (clk_on) --sub_timing_;
        return;
    }
    size_t bs = 0;
    for (int li = (int)levels_.size() - 1; li >= 0; --li) {
        const Level& L = levels_[li];
        if (st_on && bs < bstreams_.size() && bstreams_[bs].l1 - 1 == li) {
            launch_bstream<NR>(bstreams_[bs], x0, x1, ctrl, gate_reject, s);
            li = bstreams_[bs++].l0;
            continue;
        }
        BrRange r;
        r.bwd_first = L.bwd_first; r.bwd_count = L.bwd_count; r.bt_first = L.bt_first; r.bt_count = L.bt_count;
        lvl_bwd(L, r, s);
    }
    sub_bwd(0, n_sub_, s);
    AA_CHECK_LAUNCH();
    if (clk_on) {
        --sub_timing_;
        AA_HIP(hipStreamSynchronize(s));
        std::vector<long long> h(2 * 64 * (size_t)n_sub_);
        AA_HIP(hipMemcpy(h.data(), sub_clk_.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
        std::vector<SubTree> tr(n_sub_);
        AA_HIP(hipMemcpy(tr.data(), sub_trees_.p, tr.size() * sizeof(SubTree), hipMemcpyDeviceToHost));
        const int nl = tr[0].nlvl;
        auto show = [&](const char* what, int base, int nph) {   // median / max over workgroups, us (100 MHz)
            std::fprintf(stderr, "[solve] sub timing NR=%d %s:", NR, what);
            for (int q = 1; q <= nph; ++q) {
                std::vector<double> d;
                for (int b = 0; b < n_sub_; ++b)
                    if (tr[b].nlvl == nl) d.push_back(0.01 * (double)(h[(base + b) * 64 + q] - h[(base + b) * 64 + q - 1]));
                if (d.empty()) continue;
                std::sort(d.begin(), d.end());
                std::fprintf(stderr, " %.1f/%.1f", d[d.size() / 2], d.back());
            }
            std::vector<double> tot;
            for (int b = 0; b < n_sub_; ++b)
                if (tr[b].nlvl == nl) tot.push_back(0.01 * (double)(h[(base + b) * 64 + nph] - h[(base + b) * 64]));
            std::sort(tot.begin(), tot.end());
            std::fprintf(stderr, " | total %.1f/%.1f us", tot[tot.size() / 2], tot.back());
            // every workgroup (any level count): start and end against the earliest start
            const int per = nph / nl;
            long long t0 = h[(size_t)base * 64];
            for (int b = 0; b < n_sub_; ++b) t0 = std::min(t0, h[(size_t)(base + b) * 64]);
            std::vector<double> st, en;
            std::map<int, int> by_lvl;
            for (int b = 0; b < n_sub_; ++b) {
                st.push_back(0.01 * (double)(h[(size_t)(base + b) * 64] - t0));
                en.push_back(0.01 * (double)(h[(size_t)(base + b) * 64 + per * tr[b].nlvl] - t0));
                ++by_lvl[tr[b].nlvl];
            }
            std::sort(st.begin(), st.end());
            std::sort(en.begin(), en.end());
            std::fprintf(stderr, " | start med/max %.1f/%.1f end med/max %.1f/%.1f us | subtrees by levels:", st[st.size() / 2],
                         st.back(), en[en.size() / 2], en.back());
            for (auto& kv : by_lvl) std::fprintf(stderr, " %d:%d", kv.first, kv.second);
            std::fprintf(stderr, "\n");
        };
        show("fwd (assembly, rows per level, bottom-up)", 0, 2 * nl);
        show("bwd (vector, segments, columns per level, top-down)", n_sub_, 3 * nl);
    }
}

}  // namespace aa
