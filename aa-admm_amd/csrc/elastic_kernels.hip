// HIP kernels of the admm-elastic hot path (gfx950, wave64, fp64).
//
// One thread per energy term for the local step (SoA element data -> coalesced loads; node
// positions gathered 24 B at a time from an xyz-interleaved array that stays L2/MALL
// resident), deterministic block partial sums for every residual norm, and a one-block
// control kernel that makes the reference's data-dependent decisions (Anderson reject,
// comb < eps break) on the device so the whole ADMM loop is enqueued without host syncs.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "device_lbfgs.hpp"
#include "device_prox.hpp"
#include "elastic_kernels.hpp"

namespace aa {

namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// deterministic block sum; result valid in thread 0
__device__ __forceinline__ double block_sum(double v, double* sm) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sm[wid] = v;
    __syncthreads();
    double r = 0;
    if (threadIdx.x == 0)
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += sm[i];
    __syncthreads();
    return r;
}

// deterministic block sum of red[0..nb) visible to every thread (same order in every block)
// a thread's share of nb partials, summed in index order; loads issued 8 at a time (a thread
// strides through ~15 partials on C4: one round trip each when loaded one by one)
__device__ __forceinline__ double thread_sum_strided(const double* red, int nb) {
    double a = 0;
    int i = threadIdx.x;
    const int st = blockDim.x;
    for (; i + 7 * st < nb; i += 8 * st) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = red[i + q * st];
#pragma unroll
        for (int q = 0; q < 8; ++q) a += v[q];
    }
    for (; i < nb; i += st) a += red[i];
    return a;
}

__device__ __forceinline__ double block_sum_all(const double* red, int nb, double* sm) {
    double a = thread_sum_strided(red, nb);
    a = block_sum(a, sm);
    if (threadIdx.x == 0) sm[0] = a;
    __syncthreads();
    a = sm[0];
    __syncthreads();
    return a;
}

// history row k = nrec (prim, comb, reject, device clock); true when the run-to-epsilon stop
// (comb <= eps_rel * comb of the first row) is reached. Single thread.
__device__ __forceinline__ bool record_iter(Ctrl* c, double* hp, double* hc, int* hr, double comb) {
    const int k = c->nrec;
    if (k < c->cap) {
        hp[k] = c->prim; hc[k] = comb; hr[k] = c->reject;
        if (c->hist_clock) c->hist_clock[k] = (long long)wall_clock64();
    }
    c->nrec = k + 1;
    if (k == 0) c->eps_abs = c->eps_rel * comb;
    return c->eps_rel > 0 && comb <= c->eps_abs;
}

__device__ __forceinline__ bool gated(const Ctrl* c, int gate_reject) {
    if (!c) return false;
    if (c->done) return true;
    return gate_reject && !c->reject;
}

// F = P x_full, Cp = P_pinned x_pin  (EnergyTerm::update_z's D.block*x, Solver.cpp C_fix)
template <int NV>
__device__ __forceinline__ void gather_F(const GroupDev& g, int e, const double* __restrict__ xfull, int nf, double* F,
                                         double* Cp) {
    constexpr int NC = ncol_of(NV);
#pragma unroll
    for (int i = 0; i < 3 * NC; ++i) { F[i] = 0; Cp[i] = 0; }
#pragma unroll
    for (int a = 0; a < NV; ++a) {
        const int v = g.idx[(size_t)a * g.count + e];
        const double x0 = xfull[3 * (size_t)v], x1 = xfull[3 * (size_t)v + 1], x2 = xfull[3 * (size_t)v + 2];
        const bool pin = v >= nf;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double gc = g.G[(size_t)(c * NV + a) * g.count + e];
            F[3 * c + 0] += gc * x0; F[3 * c + 1] += gc * x1; F[3 * c + 2] += gc * x2;
            if (pin) { Cp[3 * c + 0] += gc * x0; Cp[3 * c + 1] += gc * x1; Cp[3 * c + 2] += gc * x2; }
        }
    }
}

// Cp alone, for the callers that need only C_fix (the rhs slots after the gradient pass): a group without pinned nodes (g.pinned = 0, kernel-uniform) has Cp = 0 and loads
// no position; otherwise gather_F's products (F unused). A per-node `if pinned` branch instead was
// measured slower (the node id load then waits before anything else issues): C4 local_z 412 -> 430 us.
template <int NV>
__device__ __forceinline__ void gather_Cp(const GroupDev& g, int e, const double* __restrict__ xfull, int nf, double* Cp) {
    constexpr int NC = ncol_of(NV);
    if (!g.pinned) {
#pragma unroll
        for (int i = 0; i < 3 * NC; ++i) Cp[i] = 0;
        return;
    }
    double F[3 * NC];
    gather_F<NV>(g, e, xfull, nf, F, Cp);
}

template <int NV>
__device__ __forceinline__ void gather_P(const GroupDev& g, int e, const double* __restrict__ xfull, double* F) {
    constexpr int NC = ncol_of(NV);
#pragma unroll
    for (int i = 0; i < 3 * NC; ++i) F[i] = 0;
#pragma unroll
    for (int a = 0; a < NV; ++a) {
        const int v = g.idx[(size_t)a * g.count + e];
        const double x0 = xfull[3 * (size_t)v], x1 = xfull[3 * (size_t)v + 1], x2 = xfull[3 * (size_t)v + 2];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double gc = g.G[(size_t)(c * NV + a) * g.count + e];
            F[3 * c + 0] += gc * x0; F[3 * c + 1] += gc * x1; F[3 * c + 2] += gc * x2;
        }
    }
}

// Per-vertex right-hand-side contributions of one element: with y_c = w (w z_c - w Cp_c - u_c)
// (the element's rows of W z + C - u, Solver.cpp:105/175), vertex a of a free node receives
// f_a = sum_c G[c][a] y_c, scattered to its node's run of slots (spos, node order); the rhs
// kernel then streams each node's run (no coefficient array, no gathers).
// (write_slots_pre: the same with the element's slot positions and coefficients already loaded)
template <int NV>
__device__ __forceinline__ void write_slots_pre(const int* pos, const double* gk, double w, const double* zz,
                                                const double* Cp, const double* uu, double* __restrict__ y) {
    constexpr int NC = ncol_of(NV);
    double yc[3 * NC];
#pragma unroll
    for (int i = 0; i < 3 * NC; ++i) yc[i] = w * (w * zz[i] - w * Cp[i] - uu[i]);
#pragma unroll
    for (int a = 0; a < NV; ++a) {
        if (pos[a] < 0) continue;   // pinned: no rhs row
        double f0 = 0, f1 = 0, f2 = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double gc = gk[c * NV + a];
            f0 += gc * yc[3 * c]; f1 += gc * yc[3 * c + 1]; f2 += gc * yc[3 * c + 2];
        }
        double* o = y + 3 * (size_t)pos[a];
        o[0] = f0; o[1] = f1; o[2] = f2;
    }
}
template <int NV>
__device__ __forceinline__ void write_slots(const GroupDev& g, int e, int nf, double w, const double* zz,
                                            const double* Cp, const double* uu, double* __restrict__ y) {
    constexpr int NC = ncol_of(NV);
    double yc[3 * NC];
#pragma unroll
    for (int i = 0; i < 3 * NC; ++i) yc[i] = w * (w * zz[i] - w * Cp[i] - uu[i]);
    // every load before the per-node branch: a load inside `if (pos >= 0)` is issued only after
    // the branch resolves, i.e. after a wait on pos (one serialised round trip per node)
    int pos[NV];
    double gk[NC * NV];
#pragma unroll
    for (int a = 0; a < NV; ++a) pos[a] = g.spos[(size_t)a * g.count + e];
#pragma unroll
    for (int k = 0; k < NC * NV; ++k) gk[k] = g.G[(size_t)k * g.count + e];
#pragma unroll
    for (int a = 0; a < NV; ++a) {
        if (pos[a] < 0) continue;   // pinned: no rhs row
        double f0 = 0, f1 = 0, f2 = 0;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const double gc = gk[c * NV + a];
            f0 += gc * yc[3 * c]; f1 += gc * yc[3 * c + 1]; f2 += gc * yc[3 * c + 2];
        }
        double* o = y + 3 * (size_t)pos[a];
        o[0] = f0; o[1] = f1; o[2] = f2;
    }
}

// u of an element (0 without u): the null test outside the loads, so they issue together
template <int D>
__device__ __forceinline__ void load_u(const GroupDev& g, int e, const double* __restrict__ u, double* uu) {
    if (u) {
#pragma unroll
        for (int i = 0; i < D; ++i) uu[i] = u[g.zoff + (size_t)i * g.count + e];
    } else {
#pragma unroll
        for (int i = 0; i < D; ++i) uu[i] = 0.0;
    }
}

// ------------------------------------------------------------------ local step
template <int NV, int HYPER>
__global__ __launch_bounds__(kBlock) void k_local_z(GroupDev g, const double* __restrict__ xfull,
                                                    const double* __restrict__ u, double* __restrict__ z,
                                                    double* __restrict__ y, int nf, int variant, int mode, Ctrl* ctrl,
                                                    double* red, int red_off) {
    if (mode != LZ_INIT && gated(ctrl, mode == LZ_REDO)) return;
    __shared__ double sm[kBlock / 64];
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double part = 0;
    if (e < g.count) {
        double F[D], Cp[D], uu[D], vin[D], zz[D];
        gather_F<NV>(g, e, xfull, nf, F, Cp);
        const double w = g.w[e];
        load_u<D>(g, e, u, uu);
#pragma unroll
        for (int i = 0; i < D; ++i) vin[i] = F[i] + uu[i] / w;
        if constexpr (NV == 1) {
            // the (u,x) variant's candidate exactly as EnergyTerm::update_z forms it for an identity
            // row (EnergyTerm.hpp:166-178: z = W^-1 (W x + u - c), W^-1 stored as 1/w): the
            // contact decision is discrete, so the candidate is rounded like the reference's
            if (variant == 1) dev::collision_candidate(F, uu, w, vin);
            dev::collision_prox(vin, g.obs, zz);
        } else if constexpr (NV == 3) {
            dev::tri_prox(vin, zz, variant, g.lmin, g.lmax);
        } else if constexpr (HYPER == 0) {
            dev::tet_linear_prox(vin, zz);
        } else {
#pragma unroll
            for (int i = 0; i < D; ++i) zz[i] = vin[i];
            int fail = 0;
            dev::hyper_prox(g.mat, g.mu, g.lambda, g.k, g.vol[e], vin, zz, &fail);
            if (fail && ctrl) ctrl->fail = 1;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const double r = w * (F[i] - zz[i]);
            part += r * r;
            z[g.zoff + (size_t)i * g.count + e] = zz[i];
        }
        if (y) write_slots<NV>(g, e, nf, w, zz, Cp, uu, y);
    }
    if (red) {
        const double s = block_sum(part, sm);
        if (threadIdx.x == 0) red[red_off + blockIdx.x] = s;
    }
}

// NeoHookean / StVK local step without residual partials (the Z variant's update_z calls), as a
// persistent work queue: the per-element L-BFGS takes 1..100 iterations, so with one element per
// lane a wave runs as long as its slowest lane. Here every lane that finishes its element (z and
// the optional rhs slots written) takes the next one from a queue (one atomic per wave and
// refill, ballot-aggregated) and lanes advance one outer L-BFGS iteration per trip. Each
// element's arithmetic is unchanged, so the results are bit-identical to k_local_z.
// HV: where the L-BFGS history lives -- LQ_HIST_REGS (default): all of it in registers
// (dev::HyperLbfgs); LQ_HIST_YLDS: the y half in LDS (dev::HyperLbfgsLds, dynamic LDS kLqLdsBytes,
// AA_LQ_LDS=1; measured slower). Bit-identical.
// end of a work-queue launch: the last block to finish resets the queue -- claim counter
// queue[0], finished blocks queue[1] -- for the next launch, which follows a kernel boundary; this
// replaces a memset node (a fill kernel and its dependency gap) before every launch. A gated
// launch returns before claiming and leaves both at 0.
__device__ __forceinline__ void queue_reset_last(int* queue) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned d = atomicAdd(reinterpret_cast<unsigned*>(queue + 1), 1u);
        if (d == gridDim.x - 1) {
            atomicExch(queue, 0);
            atomicExch(queue + 1, 0);
        }
    }
}

// the work queue's claim. The address offset comes from an opaque VGPR so the compiler's
// wave-aggregation rewrite of a uniform-address atomic does not apply: that rewrite reads the
// result back (readfirstlane) inside the leader's branch, i.e. waits for the atomic's round trip
// at once, before the finished elements' stores and loads that it could overlap
__device__ __forceinline__ int queue_claim(int* queue, int n) {
    int off;
    asm volatile("v_mov_b32 %0, 0" : "=v"(off));
    return atomicAdd(queue + off, n);
}

template <int HV>
struct LqHist {
    using type = typename std::conditional<HV == LQ_HIST_YLDS, dev::HyperLbfgsLds, dev::HyperLbfgs>::type;
};

// CHUNK (AA_LQ_CHUNK=1): the wave claims its elements in chunks of 64 one chunk AHEAD (a
// wave-uniform range [p0, p1) plus the next chunk's base nx, claimed while the current one is
// worked on), so a refill's element ids are known without waiting for the queue atomic: the refill
// chain is node ids -> positions instead of atomic -> node ids -> positions. The last chunks (the
// queue within `margin` elements of its end) are claimed at the refill, as CHUNK = 0 does, so no
// wave sits on unstarted elements while others run dry. Same elements, same arithmetic per
// element: bit-identical outputs.
template <int NV, int HV, int CHUNK = 0>
__global__ __launch_bounds__(kBlock) void k_local_z_hq(GroupDev g, const double* __restrict__ xfull,
                                                       const double* __restrict__ u, double* __restrict__ z,
                                                       double* __restrict__ y, int nf, int mode, Ctrl* ctrl,
                                                       int* __restrict__ queue, int refill,
                                                       unsigned long long* __restrict__ stats, int margin = 0) {
    if (mode != LZ_INIT && gated(ctrl, mode == LZ_REDO)) return;
    unsigned trips = 0, refills = 0;
    __shared__ unsigned hist[101];   // diagnostics only: per-block histogram, flushed at the end
    if (stats) {
        for (int i = threadIdx.x; i < 101; i += blockDim.x) hist[i] = 0;
        __syncthreads();
    }
    constexpr int D = 3 * (NV - 1);
    const int lane = threadIdx.x & 63;
    typename LqHist<HV>::type L;
    if constexpr (HV == LQ_HIST_YLDS) {
        extern __shared__ double lq_hist[];
        L.bind(lq_hist + threadIdx.x, kBlock);
    }
    double v[D], x[D];
    double vol = 0;
    int e = -1, fail = 0;
    // pending: the lane's element is solved but its outputs are not written yet -- they are
    // written at the next refill, together with the loads of the lane's next element, so a
    // wave pays the gathers' latency once per refill instead of on every trip in which some
    // lane finishes
    bool active = false, pending = false, exhausted = false;
    // CHUNK: the wave's claimed, unstarted range [p0, p1); nxv = lane 0's last queue atomic
    // result; ahead = a 64-chunk claim is in flight; qpos = the last queue position seen
    // (nxs: nxv read back at the end of the refill that issued it -- a wait there costs nothing, the
    // refill's later gathers have returned; a read at the next refill would wait for that refill's
    // finalize stores too, the vector memory counter being in order)
    int p0 = 0, p1 = 0, nxv = 0, nxs = 0, qpos = 0;
    bool ahead = false, fresh = false;
    auto finalize = [&]() {
#pragma unroll
        for (int i = 0; i < D; ++i) z[g.zoff + (size_t)i * g.count + e] = x[i];
        if (y) {   // (gather_Cp here measured slower: local_z 410 / 412 -> 415 / 421 us on C4)
            double F[D], Cp[D], uu[D];
            gather_F<NV>(g, e, xfull, nf, F, Cp);
            load_u<D>(g, e, u, uu);
            write_slots<NV>(g, e, nf, g.w[e], x, Cp, uu, y);
        }
    };
    for (;;) {
        const bool need = !active && !exhausted;   // idle lanes, pending ones included
        const unsigned long long mask = __ballot(need);
        if (!__any(active || need)) break;
        ++trips;
        // refill only once enough lanes are idle (the init path then runs for many lanes at once)
        if (mask && (__popcll(mask) >= refill || !__any(active))) {
            ++refills;
            const int leader = __ffsll((long long)mask) - 1;
            const int k = __popcll(mask), rank = __popcll(mask & ((1ull << lane) - 1ull));
            int b = 0, my = 0;
            if constexpr (CHUNK == 0) {
                if (lane == leader) b = queue_claim(queue, k);
            } else if (!ahead && qpos + 64 <= g.count - margin) {   // the next chunk, ahead of need
                // (issued before the finalize, like CHUNK = 0's claim, so its round trip hides
                // under the finalize's gathers when this refill already needs it)
                if (lane == 0) nxv = atomicAdd(queue, 64);
                ahead = true;
                fresh = true;
            }
            if (pending) {
                finalize();
                pending = false;
            }
            if constexpr (CHUNK == 0) {
                b = __shfl(b, leader, 64);
                my = b + rank;
            } else {
                // exec is full here (the refill test is wave-uniform, all lanes stay in the loop
                // until the wave breaks), so lane 0 issues the claims and readfirstlane reads it
                const int avail = p1 - p0;
                if (avail >= k) {
                    my = p0 + rank;
                    p0 += k;
                } else {
                    int hi;
                    if (ahead) {   // the chunk claimed ahead: 64 more
                        hi = fresh ? __builtin_amdgcn_readfirstlane(nxv) : nxs;
                        p1 = hi + 64;
                    } else {       // first refill, or the tail: claim exactly what is missing, now
                        if (lane == 0) nxv = atomicAdd(queue, k - avail);
                        hi = __builtin_amdgcn_readfirstlane(nxv);
                        p1 = hi + (k - avail);
                    }
                    my = rank < avail ? p0 + rank : hi + (rank - avail);
                    p0 = hi + (k - avail);
                    qpos = hi;
                    ahead = false;
                    fresh = false;
                }
            }
            if (need) {
                if (my >= g.count) {
                    exhausted = true;
                } else {
                    e = my;
                    double F[D], Cp[D];
                    gather_F<NV>(g, e, xfull, nf, F, Cp);
                    const double w = g.w[e];
                    double uu[D];
                    load_u<D>(g, e, u, uu);
#pragma unroll
                    for (int i = 0; i < D; ++i) {
                        v[i] = F[i] + uu[i] / w;
                        x[i] = v[i];
                    }
                    vol = g.vol[e];
                    if (L.start(g.mat, g.mu, g.lambda, g.k, vol, v, x)) {
                        finalize();
                        if (stats) atomicAdd(&hist[0], 1u);
                    } else {
                        active = true;
                    }
                }
            }
            if constexpr (CHUNK != 0) {
                if (fresh) {   // claimed at this refill, not used yet: read it back now
                    nxs = __builtin_amdgcn_readfirstlane(nxv);
                    fresh = false;
                }
            }
        }
        if (active && L.iterate(g.mat, g.mu, g.lambda, g.k, vol, v, x, &fail)) {
            active = false;
            pending = true;
            if (stats) atomicAdd(&hist[min(L.k_it, 100)], 1u);
        }
    }
    if (stats) {
        if (lane == 0) {
            atomicAdd(stats + 101, (unsigned long long)trips);
            atomicAdd(stats + 102, (unsigned long long)refills);
            atomicAdd(stats + 103, 1ull);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 101; i += blockDim.x)
            if (hist[i]) atomicAdd(stats + i, (unsigned long long)hist[i]);
    }
    if (fail && ctrl) ctrl->fail = 1;
    queue_reset_last(queue);
}

// k_local_z_hq with the refill's loads regrouped (the default for the main local step; AA_LQ_FUSED=0
// the plain refill; groups with pinned nodes keep it -- their Cp needs the finished element's
// positions). The plain refill is a chain of dependent round trips: the finished element's node
// ids, its positions (for Cp, 0 without pins), then its slot positions, then the new element's
// node ids and positions (tools/isa_serial.py; 27 % of the wave's cycles parked on s_waitcnt). Here
// the loads go out in three groups, unconditionally for every lane (indices clamped; a lane without
// a finished or a new element loads valid data it does not use, so no branch splits a group):
// the queue claim with the finished element's coefficients, u, w and slot positions; the new
// element's node ids, with the finished element's stores issued while they are in flight; the new
// element's positions, coefficients, u, w and vol. A start point that already passes the gradient
// test leaves its element pending (written at the next refill) instead of writing it at once.
// Same arithmetic in the same order: bit-identical. 452 registers (one wave per SIMD, as the
// plain kernel's 402) -- too many to leave the Anderson kernels room beside it, so the concurrent
// combined-residual pass keeps the plain refill (ElasticSolver::initialize). C4 (same box, two A/B
// pairs): local_z 433 / 435 -> 422 / 418 us.
template <int NV, bool SLOTS = true>
__global__ __launch_bounds__(kBlock) void k_local_z_hqf(GroupDev g, const double* __restrict__ xfull,
                                                        const double* __restrict__ u, double* __restrict__ z,
                                                        double* __restrict__ y, int nf, int mode, Ctrl* ctrl,
                                                        int* __restrict__ queue, int refill,
                                                        unsigned long long* __restrict__ stats) {
    static_assert(NV == 4, "the fused refill is for tets");
    if (mode != LZ_INIT && gated(ctrl, mode == LZ_REDO)) return;
    unsigned trips = 0, refills = 0;
    __shared__ unsigned hist[101];
    if (stats) {
        for (int i = threadIdx.x; i < 101; i += blockDim.x) hist[i] = 0;
        __syncthreads();
    }
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int lane = threadIdx.x & 63;
    dev::HyperLbfgs L;
    double v[D], x[D];
    double vol = 0;
    int e = 0, fail = 0;
    bool active = false, pending = false, exhausted = false;
    const size_t n = g.count;
    for (;;) {
        const bool need = !active && !exhausted;
        const unsigned long long mask = __ballot(need);
        if (!__any(active || need)) break;
        ++trips;
        if (mask && (__popcll(mask) >= refill || !__any(active))) {
            ++refills;
            const int leader = __ffsll((long long)mask) - 1;
            const int rank = __popcll(mask & ((1ull << lane) - 1ull));
            int b = 0;
            if (lane == leader) b = queue_claim(queue, __popcll(mask));
            // the finished element's slot data (every lane: e is a valid element or 0)
            int so[NV];
            double go[NC * NV], uo[D], wo = 1.0;
            if (SLOTS && y) {   // kernel-uniform (SLOTS = false: a pass without slots, fewer live registers)
#pragma unroll
                for (int a = 0; a < NV; ++a) so[a] = g.spos[a * n + e];
#pragma unroll
                for (int k = 0; k < NC * NV; ++k) go[k] = g.G[k * n + e];
                load_u<D>(g, e, u, uo);
                wo = g.w[e];
            }
            b = __shfl(b, leader, 64);
            const int my = b + rank;
            const int en = min(my, g.count - 1);
            int id[NV];   // the new element's node ids first: its positions wait on them
#pragma unroll
            for (int a = 0; a < NV; ++a) id[a] = g.idx[a * n + en];
            if (pending) {   // the finished element's outputs while the ids are in flight
#pragma unroll
                for (int i = 0; i < D; ++i) z[g.zoff + (size_t)i * n + e] = x[i];
                if (SLOTS && y) {
                    double Cp[D];
#pragma unroll
                    for (int i = 0; i < D; ++i) Cp[i] = 0;
                    write_slots_pre<NV>(so, go, wo, x, Cp, uo, y);
                }
                pending = false;
            }
            double xp[3 * NV], gn[NC * NV], un[D];
#pragma unroll
            for (int a = 0; a < NV; ++a) {
                xp[3 * a] = xfull[3 * (size_t)id[a]];
                xp[3 * a + 1] = xfull[3 * (size_t)id[a] + 1];
                xp[3 * a + 2] = xfull[3 * (size_t)id[a] + 2];
            }
#pragma unroll
            for (int k = 0; k < NC * NV; ++k) gn[k] = g.G[k * n + en];
            load_u<D>(g, en, u, un);
            const double wn = g.w[en], voln = g.vol[en];
            if (need) {
                if (my >= g.count) {
                    exhausted = true;
                } else {
                    e = my;
                    double F[D];   // gather_F's sums, in its order
#pragma unroll
                    for (int i = 0; i < D; ++i) F[i] = 0;
#pragma unroll
                    for (int a = 0; a < NV; ++a)
#pragma unroll
                        for (int c = 0; c < NC; ++c) {
                            const double gc = gn[c * NV + a];
                            F[3 * c + 0] += gc * xp[3 * a]; F[3 * c + 1] += gc * xp[3 * a + 1];
                            F[3 * c + 2] += gc * xp[3 * a + 2];
                        }
#pragma unroll
                    for (int i = 0; i < D; ++i) {
                        v[i] = F[i] + un[i] / wn;
                        x[i] = v[i];
                    }
                    vol = voln;
                    if (L.start(g.mat, g.mu, g.lambda, g.k, vol, v, x)) {
                        pending = true;
                        if (stats) atomicAdd(&hist[0], 1u);
                    } else {
                        active = true;
                    }
                }
            }
        }
        if (active && L.iterate(g.mat, g.mu, g.lambda, g.k, vol, v, x, &fail)) {
            active = false;
            pending = true;
            if (stats) atomicAdd(&hist[min(L.k_it, 100)], 1u);
        }
    }
    if (stats) {
        if (lane == 0) {
            atomicAdd(stats + 101, (unsigned long long)trips);
            atomicAdd(stats + 102, (unsigned long long)refills);
            atomicAdd(stats + 103, 1ull);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 101; i += blockDim.x)
            if (hist[i]) atomicAdd(stats + i, (unsigned long long)hist[i]);
    }
    if (fail && ctrl) ctrl->fail = 1;
    queue_reset_last(queue);
}

// k_local_z_hq with each element's L-BFGS split over a lane pair (dev::HyperLbfgs2, AA_LQ_SPLIT=1,
// opt-in): a wave holds 32 elements, the state fits 256 registers, and a SIMD runs two waves -- the
// one-wave kernel spends ~27 % of its cycles waiting on the refills' dependent loads with nothing
// to hide them. Measured on C4 (profiles/r5_c4_local_step_split.json): 1.56x the VALU instructions
// per element and 196 B of spills at 256 registers, 428 -> 800 us per launch; not the default. The queue hands out elements to pairs; every branch is pair-uniform
// (both lanes hold the same decisions), so the DPP swaps always see their partner active. At a
// finalize each lane writes its half of z and the slots of two of the four vertices.
template <int NV>
__global__ __launch_bounds__(kBlock, 2) void k_local_z_hq2(GroupDev g, const double* __restrict__ xfull,
                                                           const double* __restrict__ u, double* __restrict__ z,
                                                           double* __restrict__ y, int nf, int mode, Ctrl* ctrl,
                                                           int* __restrict__ queue, int refill,
                                                           unsigned long long* __restrict__ stats) {
    static_assert(NV == 4, "the lane-pair local step is for tets");
    if (mode != LZ_INIT && gated(ctrl, mode == LZ_REDO)) return;
    constexpr int H = dev::kHalf;
    unsigned trips = 0, refills = 0;
    __shared__ unsigned hist[101];
    if (stats) {
        for (int i = threadIdx.x; i < 101; i += blockDim.x) hist[i] = 0;
        __syncthreads();
    }
    const int lane = threadIdx.x & 63, h = lane & 1;
    const unsigned long long evens = 0x5555555555555555ull;
    dev::HyperLbfgs2 L;
    double v[H], x[H];
    double vol = 0;
    int e = -1, fail = 0;
    bool active = false, pending = false, exhausted = false;
    // this lane's components of F = P x and Cp = P_pinned x_pin (the sums of gather_F, a = 0..3)
    // and of u; component 5h + j (the pad j = 4 on h = 1 reads component 8 and is not used)
    // one node at a time (not unrolled): the gathers' results would otherwise all be live at
    // once beside the lanes' L-BFGS state, past the 256 registers of two waves per SIMD
    auto gather_own = [&](double* Fo, double* Co, double* uo) {
#pragma unroll
        for (int j = 0; j < H; ++j) {
            Fo[j] = 0.0;
            Co[j] = 0.0;
            uo[j] = u ? u[g.zoff + (size_t)min(5 * h + j, 8) * g.count + e] : 0.0;
        }
#pragma unroll 1
        for (int a = 0; a < NV; ++a) {
            const int vi = g.idx[(size_t)a * g.count + e];
            const double* xa = xfull + 3 * (size_t)vi;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int i = min(5 * h + j, 8), c = i / 3, r = i - 3 * c;
                const double gc = g.G[(size_t)(c * NV + a) * g.count + e];
                const double xr = xa[r];
                Fo[j] += gc * xr;
                if (vi >= nf) Co[j] += gc * xr;
            }
        }
    };
    auto finalize = [&]() {
#pragma unroll
        for (int j = 0; j < H; ++j)
            if (h == 0 || j < 4) z[g.zoff + (size_t)(5 * h + j) * g.count + e] = x[j];
        if (y) {   // y_c = w (w z_c - w Cp_c - u_c) per own component, then the two vertices' slots
            const double w = g.w[e];
            double yo[H];
            {
                double co[H], uo[H];
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    co[j] = 0.0;
                    uo[j] = u ? u[g.zoff + (size_t)min(5 * h + j, 8) * g.count + e] : 0.0;
                }
#pragma unroll 1
                for (int a = 0; a < NV; ++a) {
                    const int vi = g.idx[(size_t)a * g.count + e];
                    if (vi < nf) continue;   // Cp: pinned nodes only
                    const double* xa = xfull + 3 * (size_t)vi;
#pragma unroll
                    for (int j = 0; j < H; ++j) {
                        const int i = min(5 * h + j, 8), c = i / 3, r = i - 3 * c;
                        co[j] += g.G[(size_t)(c * NV + a) * g.count + e] * xa[r];
                    }
                }
#pragma unroll
                for (int j = 0; j < H; ++j) yo[j] = w * (w * x[j] - w * co[j] - uo[j]);
            }
            double yc[9];
            dev::pair_full(h, yo, yc);
#pragma unroll 1
            for (int b = 0; b < 2; ++b) {
                const int a = 2 * h + b;
                const int pos = g.spos[(size_t)a * g.count + e];
                const double g0 = g.G[(size_t)(0 * NV + a) * g.count + e], g1 = g.G[(size_t)(1 * NV + a) * g.count + e],
                             g2 = g.G[(size_t)(2 * NV + a) * g.count + e];
                if (pos < 0) continue;   // pinned: no rhs row
                double* o = y + 3 * (size_t)pos;
                o[0] = g0 * yc[0] + g1 * yc[3] + g2 * yc[6];
                o[1] = g0 * yc[1] + g1 * yc[4] + g2 * yc[7];
                o[2] = g0 * yc[2] + g1 * yc[5] + g2 * yc[8];
            }
        }
    };
    for (;;) {
        const bool need = !active && !exhausted;   // the same on both lanes of a pair
        const unsigned long long mask = __ballot(need) & evens;
        if (!__any(active || need)) break;
        ++trips;
        if (mask && (__popcll(mask) >= refill || !__any(active))) {
            ++refills;
            const int leader = __ffsll((long long)mask) - 1;
            int b = 0;
            if (lane == leader) b = atomicAdd(queue, __popcll(mask));
            if (pending) {
                finalize();
                pending = false;
            }
            b = __shfl(b, leader, 64);
            if (need) {
                const int my = b + __popcll(mask & ((1ull << (lane & ~1)) - 1ull));
                if (my >= g.count) {
                    exhausted = true;
                } else {
                    e = my;
                    double Fo[H], Co[H], uo[H];
                    gather_own(Fo, Co, uo);
                    const double w = g.w[e];
#pragma unroll
                    for (int j = 0; j < H; ++j) {
                        v[j] = (h && j == 4) ? 0.0 : Fo[j] + uo[j] / w;
                        x[j] = v[j];
                    }
                    vol = g.vol[e];
                    L.begin();   // its start evaluation is this trip's
                    active = true;
                }
            }
        }
        if (active && L.trip(h, g.mat, g.mu, g.lambda, g.k, vol, v, x, &fail)) {
            active = false;
            pending = true;
            if (stats && h == 0) atomicAdd(&hist[min(L.k_it, 100)], 1u);
        }
    }
    if (stats) {
        if (lane == 0) {
            atomicAdd(stats + 101, (unsigned long long)trips);
            atomicAdd(stats + 102, (unsigned long long)refills);
            atomicAdd(stats + 103, 1ull);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 101; i += blockDim.x)
            if (hist[i]) atomicAdd(stats + i, (unsigned long long)hist[i]);
    }
    if (fail && ctrl) ctrl->fail = 1;
}

// k_local_z_hq with a one-element lookahead per lane (AA_LQ_AHEAD=1; measured 6 % slower than
// k_local_z_hq on C4). A refill of the plain queue is a chain of three dependent round trips -- the
// returning queue atomic, the element's node ids, then the node positions -- paid while the wave's
// other lanes wait (28 % of the kernel's cycles at one wave per SIMD). Here each
// lane holds its NEXT element: the claim atomic is issued at a refill and read on the next trip,
// the node ids are loaded right then, so the following refill only waits for the positions /
// coefficient / u loads, all independent (one round trip). The finalize keeps the element's node
// ids and loads positions only for pinned nodes (the only ones Cp needs). Close to the end of the
// queue (fewer than `margin` elements left) lookahead stops, so claimed-ahead elements cannot
// pile up on a few waves. Same arithmetic per element: bit-identical to k_local_z_hq.
template <int NV, int HV>
__global__ __launch_bounds__(kBlock) void k_local_z_hqa(GroupDev g, const double* __restrict__ xfull,
                                                        const double* __restrict__ u, double* __restrict__ z,
                                                        double* __restrict__ y, int nf, int mode, Ctrl* ctrl,
                                                        int* __restrict__ queue, int refill, int margin,
                                                        unsigned long long* __restrict__ stats) {
    if (mode != LZ_INIT && gated(ctrl, mode == LZ_REDO)) return;
    unsigned trips = 0, refills = 0;
    __shared__ unsigned hist[101];
    if (stats) {
        for (int i = threadIdx.x; i < 101; i += blockDim.x) hist[i] = 0;
        __syncthreads();
    }
    constexpr int D = 3 * (NV - 1), NC = NV - 1;
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (1ull << lane) - 1ull;
    typename LqHist<HV>::type L;
    if constexpr (HV == LQ_HIST_YLDS) {
        extern __shared__ double lq_hist[];
        L.bind(lq_hist + threadIdx.x, kBlock);
    }
    double v[D], x[D];
    double vol = 0;
    int e = -1, fail = 0;
    int nid[NV];                 // node ids of the lane's element
    int ex = -1, xid[NV];        // lookahead element and its node ids
    int stage = 0, ab = 0, aleader = 0;   // stage 1: a lookahead claim (atomic) is in flight
    unsigned long long amask = 0;
    bool active = false, pending = false, exhausted = false, dry = false;
#pragma unroll
    for (int a = 0; a < NV; ++a) { nid[a] = 0; xid[a] = 0; }
    auto finalize = [&]() {
#pragma unroll
        for (int i = 0; i < D; ++i) z[g.zoff + (size_t)i * g.count + e] = x[i];
        if (y) {
            double Cp[D], uu[D];
#pragma unroll
            for (int i = 0; i < D; ++i) Cp[i] = 0;
#pragma unroll
            for (int a = 0; a < NV; ++a) {   // gather_F's Cp: pinned nodes only, same order
                const int vv = nid[a];
                if (vv >= nf) {
                    const double x0 = xfull[3 * (size_t)vv], x1 = xfull[3 * (size_t)vv + 1], x2 = xfull[3 * (size_t)vv + 2];
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        const double gc = g.G[(size_t)(c * NV + a) * g.count + e];
                        Cp[3 * c + 0] += gc * x0; Cp[3 * c + 1] += gc * x1; Cp[3 * c + 2] += gc * x2;
                    }
                }
            }
            load_u<D>(g, e, u, uu);
            write_slots<NV>(g, e, nf, g.w[e], x, Cp, uu, y);
        }
    };
    auto begin = [&](int ee, const int* ids) {
        e = ee;
        double F[D];
#pragma unroll
        for (int i = 0; i < D; ++i) F[i] = 0;
#pragma unroll
        for (int a = 0; a < NV; ++a) {   // gather_F's F, same order
            nid[a] = ids[a];
            const double x0 = xfull[3 * (size_t)ids[a]], x1 = xfull[3 * (size_t)ids[a] + 1], x2 = xfull[3 * (size_t)ids[a] + 2];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const double gc = g.G[(size_t)(c * NV + a) * g.count + e];
                F[3 * c + 0] += gc * x0; F[3 * c + 1] += gc * x1; F[3 * c + 2] += gc * x2;
            }
        }
        const double w = g.w[e];
        double uu[D];
        load_u<D>(g, e, u, uu);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            v[i] = F[i] + uu[i] / w;
            x[i] = v[i];
        }
        vol = g.vol[e];
        if (L.start(g.mat, g.mu, g.lambda, g.k, vol, v, x)) {
            finalize();
            if (stats) atomicAdd(&hist[0], 1u);
        } else {
            active = true;
        }
    };
    for (;;) {
        const bool need = !active && !exhausted;
        const unsigned long long mask = __ballot(need);
        if (!__any(active || need)) break;
        ++trips;
        if (stage == 1) {   // the lookahead claim issued at the last refill has returned
            const int b = __shfl(ab, aleader, 64);
            if ((amask >> lane) & 1ull) {
                const int my = b + __popcll(amask & below);
                if (my < g.count) {
                    ex = my;
#pragma unroll
                    for (int a = 0; a < NV; ++a) xid[a] = g.idx[(size_t)a * g.count + ex];
                }
            }
            if (b + __popcll(amask) >= g.count - margin) dry = true;
            stage = 0;
        }
        if (mask && (__popcll(mask) >= refill || !__any(active))) {
            ++refills;
            const bool direct = need && ex < 0;   // no lookahead: claim now (queue start, its tail)
            const unsigned long long dmask = __ballot(direct);
            int b = 0, leader = 0;
            if (dmask) {
                leader = __ffsll((long long)dmask) - 1;
                if (lane == leader) b = atomicAdd(queue, __popcll(dmask));
            }
            if (pending) {
                finalize();
                pending = false;
            }
            int ee = -1, ids[NV];
#pragma unroll
            for (int a = 0; a < NV; ++a) ids[a] = xid[a];
            if (need && ex >= 0) { ee = ex; ex = -1; }
            if (dmask) {
                b = __shfl(b, leader, 64);
                if (direct) {
                    const int my = b + __popcll(dmask & below);
                    if (my >= g.count) {
                        exhausted = true;
                    } else {
                        ee = my;
#pragma unroll
                        for (int a = 0; a < NV; ++a) ids[a] = g.idx[(size_t)a * g.count + ee];
                    }
                }
            }
            if (ee >= 0) begin(ee, ids);
            if (!dry) {   // the next lookahead claim, for every lane without one
                const unsigned long long lm = __ballot(ex < 0 && !exhausted);
                if (lm) {
                    amask = lm;
                    aleader = __ffsll((long long)lm) - 1;
                    if (lane == aleader) ab = atomicAdd(queue, __popcll(lm));
                    stage = 1;
                }
            }
        }
        if (active && L.iterate(g.mat, g.mu, g.lambda, g.k, vol, v, x, &fail)) {
            active = false;
            pending = true;
            if (stats) atomicAdd(&hist[min(L.k_it, 100)], 1u);
        }
    }
    if (stats) {
        if (lane == 0) {
            atomicAdd(stats + 101, (unsigned long long)trips);
            atomicAdd(stats + 102, (unsigned long long)refills);
            atomicAdd(stats + 103, 1ull);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < 101; i += blockDim.x)
            if (hist[i]) atomicAdd(stats + i, (unsigned long long)hist[i]);
    }
    if (fail && ctrl) ctrl->fail = 1;
}

// r = w(P x - z): prim2 += |r|^2, dual2 += |w P (x - x_last)|^2, u += r
template <int NV>
__global__ __launch_bounds__(kBlock) void k_resid_u(GroupDev g, const double* __restrict__ xfull,
                                                    const double* __restrict__ xlast, const double* __restrict__ z,
                                                    double* __restrict__ u, int nf, Ctrl* ctrl, double* red_a,
                                                    double* red_b, int red_off) {
    if (gated(ctrl, 0)) return;
    __shared__ double sm[kBlock / 64];
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double pa = 0, pb = 0;
    if (e < g.count) {
        double F[D], Fl[D];
        gather_P<NV>(g, e, xfull, F);
        gather_P<NV>(g, e, xlast, Fl);
        const double w = g.w[e];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const size_t o = g.zoff + (size_t)i * g.count + e;
            const double r = w * (F[i] - z[o]);
            const double d = w * (F[i] - Fl[i]);
            pa += r * r;
            pb += d * d;
            u[o] += r;
        }
    }
    const double sa = block_sum(pa, sm);
    const double sb = block_sum(pb, sm);
    if (threadIdx.x == 0) { red_a[red_off + blockIdx.x] = sa; red_b[red_off + blockIdx.x] = sb; }
}

// Z variant: u update (mode 0 dual ascent, 1 = W^-1 grad E(z), 2 = keep u) then y = w (w z + c - u)
template <int NV, int HYPER>
__global__ __launch_bounds__(kBlock) void k_u_and_y(GroupDev g, const double* __restrict__ xfull,
                                                    const double* __restrict__ z, double* __restrict__ u,
                                                    double* __restrict__ y, int nf, int mode, int redo, Ctrl* ctrl) {
    if (gated(ctrl, redo)) return;
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= g.count) return;
    // the gradient (mode 1) needs only z: it runs before the element's gathers, so its
    // temporaries and the gathered G / P x never hold registers together
    double F[D], Cp[D], zz[D], uu[D];
    const double w = g.w[e];
    // the element volume with the other loads (loaded where it is used, it waited alone mid-gradient)
    const double vol = (NV == 4 && mode == 1) ? g.vol[e] : 0.0;
#pragma unroll
    for (int i = 0; i < D; ++i) zz[i] = z[g.zoff + (size_t)i * g.count + e];
    if (mode != 1) {
#pragma unroll
        for (int i = 0; i < D; ++i) uu[i] = u[g.zoff + (size_t)i * g.count + e];
    }
    if (mode == 1) {
        double gr[D];
        if constexpr (NV == 3 || NV == 1) {
            // TriEnergyTerm::get_gradient / Collision::get_gradient throw in the reference
            if (ctrl) ctrl->fail = 2;
#pragma unroll
            for (int i = 0; i < D; ++i) gr[i] = 0;
        } else if constexpr (HYPER == 0) {
            dev::tet_linear_grad(zz, g.k * vol, gr);
        } else {
            dev::hyper_psi_grad(g.mat, g.mu, g.lambda, zz, gr);
#pragma unroll
            for (int i = 0; i < D; ++i) gr[i] *= vol;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) uu[i] = gr[i] / w;
    }
    if (mode == 0) {
        gather_F<NV>(g, e, xfull, nf, F, Cp);
#pragma unroll
        for (int i = 0; i < D; ++i) uu[i] += w * F[i] - w * zz[i];
    } else {
        gather_Cp<NV>(g, e, xfull, nf, Cp);
    }
    if (mode != 2) {
#pragma unroll
        for (int i = 0; i < D; ++i) u[g.zoff + (size_t)i * g.count + e] = uu[i];
    }
    write_slots<NV>(g, e, nf, w, zz, Cp, uu, y);
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_prim_z(GroupDev g, const double* __restrict__ xfull,
                                                   const double* __restrict__ z, const double* __restrict__ zref,
                                                   int nf, int redo, Ctrl* ctrl, double* red_a, double* red_b,
                                                   int red_off) {
    if (gated(ctrl, redo)) return;
    __shared__ double sm[kBlock / 64];
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    double pa = 0, pb = 0;
    if (e < g.count) {
        double F[D];
        gather_P<NV>(g, e, xfull, F);
        const double w = g.w[e];
        double zi[D], zr[D];   // all loads first (a load under `if (zref)` waited per entry)
#pragma unroll
        for (int i = 0; i < D; ++i) zi[i] = z[g.zoff + (size_t)i * g.count + e];
        if (zref) {
#pragma unroll
            for (int i = 0; i < D; ++i) zr[i] = zref[g.zoff + (size_t)i * g.count + e];
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const double r = w * (F[i] - zi[i]);
            pa += r * r;
            if (zref) { const double d = w * (zi[i] - zr[i]); pb += d * d; }
        }
    }
    const double sa = block_sum(pa, sm);
    const double sb = block_sum(pb, sm);
    if (threadIdx.x == 0) { red_a[red_off + blockIdx.x] = sa; if (red_b) red_b[red_off + blockIdx.x] = sb; }
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_init_z(GroupDev g, const double* __restrict__ xfull, double* __restrict__ z) {
    constexpr int NC = ncol_of(NV), D = 3 * NC;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= g.count) return;
    double F[D];
    gather_P<NV>(g, e, xfull, F);
#pragma unroll
    for (int i = 0; i < D; ++i) z[g.zoff + (size_t)i * g.count + e] = F[i];
}

// ------------------------------------------------------------------ global rhs (D^T gather)
__global__ __launch_bounds__(kBlock) void k_rhs(int nf, const int* __restrict__ ptr, const int* __restrict__ row,
                                                const double* __restrict__ val, const double* __restrict__ y,
                                                const double* __restrict__ Mxbar, double pdt2, double* __restrict__ b,
                                                Ctrl* ctrl, int gate_reject, const double* __restrict__ xsrc,
                                                double* __restrict__ xlast, const double* __restrict__ red_final,
                                                int nb_final) {
    if (gated(ctrl, gate_reject)) return;
    if (red_final && blockIdx.x == 0) {   // prim after a reject recompute; prev_prim = prim
        __shared__ double sm[kBlock / 64];
        const double a = block_sum_all(red_final, nb_final, sm);
        if (threadIdx.x == 0) {
            if (ctrl->reject) ctrl->prim = sqrt(a);
            ctrl->prev_prim = ctrl->prim;
        }
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    if (xlast) {   // last_x = curr_x (Solver.cpp:170), fused here: it must follow the reject restore
        xlast[3 * (size_t)i] = xsrc[3 * (size_t)i];
        xlast[3 * (size_t)i + 1] = xsrc[3 * (size_t)i + 1];
        xlast[3 * (size_t)i + 2] = xsrc[3 * (size_t)i + 2];
    }
    double s0 = 0, s1 = 0, s2 = 0;
    if (val) {
#pragma unroll 4
        for (int k = ptr[i]; k < ptr[i + 1]; ++k) {
            const double v = val[k];
            const size_t r = 3 * (size_t)row[k];
            s0 += v * y[r]; s1 += v * y[r + 1]; s2 += v * y[r + 2];
        }
    } else {   // vertex slots (write_slots): the node's run, contiguous
        const double* q = y + 3 * (size_t)ptr[i];
#pragma unroll 4
        for (int k = ptr[i]; k < ptr[i + 1]; ++k, q += 3) { s0 += q[0]; s1 += q[1]; s2 += q[2]; }
    }
    b[3 * (size_t)i + 0] = Mxbar[3 * (size_t)i + 0] + pdt2 * s0;
    b[3 * (size_t)i + 1] = Mxbar[3 * (size_t)i + 1] + pdt2 * s1;
    b[3 * (size_t)i + 2] = Mxbar[3 * (size_t)i + 2] + pdt2 * s2;
}

// The same for the vertex-slot layout, one lane per node COMPONENT: lanes 3j, 3j+1, 3j+2 of a
// wave sum x, y, z of node 21 w + j along its run (lane 63 idles), so a wave's loads cover 21
// runs in 24-B pieces instead of 64 runs in 8-B pieces; each component is still summed in slot
// order (the same sums as k_rhs, bit for bit)
#ifndef AA_RHS_CHUNK
#define AA_RHS_CHUNK 1
#endif
__global__ __launch_bounds__(kBlock) void k_rhs_slots(int nf, const int* __restrict__ ptr, const double* __restrict__ y,
                                                      const double* __restrict__ Mxbar, double pdt2,
                                                      double* __restrict__ b, Ctrl* ctrl, int gate_reject,
                                                      const double* __restrict__ xsrc, double* __restrict__ xlast,
                                                      const double* __restrict__ red_final, int nb_final) {
    if (gated(ctrl, gate_reject)) return;
    if (red_final && blockIdx.x == 0) {   // prim after a reject recompute; prev_prim = prim
        __shared__ double sm[kBlock / 64];
        const double a = block_sum_all(red_final, nb_final, sm);
        if (threadIdx.x == 0) {
            if (ctrl->reject) ctrl->prim = sqrt(a);
            ctrl->prev_prim = ctrl->prim;
        }
    }
    const int lane = threadIdx.x & 63;
    if (lane == 63) return;
    const long long w = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
    const long long i = w * 21 + lane / 3;
    const int c = lane % 3;
    if (i >= nf) return;
    const size_t o = 3 * (size_t)i + c;
    const double mx = Mxbar[o];   // issued with the run bounds, not after the sum
    double sum = 0;
    const int k0 = ptr[i], k1 = ptr[i + 1];
    const double* q = y + 3 * (size_t)k0 + c;
#if AA_RHS_CHUNK
    // the node's slots in chunks of 8 loads issued together (clamped to the last slot, the extra
    // terms adding 0): ceil(n / 8) round trips, no serial remainder; the same sum order
    for (int k = 0; k < k1 - k0; k += 8) {
        double g[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) g[m] = q[3 * (size_t)min(k + m, k1 - k0 - 1)];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 8; ++m) sum += k + m < k1 - k0 ? g[m] : 0.0;
    }
#else
#pragma unroll 4
    for (int k = k0; k < k1; ++k, q += 3) sum += *q;
#endif
    b[o] = mx + pdt2 * sum;
    if (xlast) xlast[o] = xsrc[o];   // last_x = curr_x (Solver.cpp:170); after the sum: its load is not in the chain
}

// ------------------------------------------------------------------ control (one block)
// 1024 threads: the kernel is latency-bound on summing a few thousand block partials
constexpr int kCtlBlock = 1024;
__global__ __launch_bounds__(kCtlBlock) void k_control(int op, Ctrl* ctrl, const double* red_a, const double* red_b,
                                                    int nb, int accel, double* hist_prim, double* hist_comb,
                                                    int* hist_rej) {
    if (ctrl->done) return;
    __shared__ double sm[kCtlBlock / 64];
    double a = thread_sum_strided(red_a, nb), b = red_b ? thread_sum_strided(red_b, nb) : 0.0;
    a = block_sum(a, sm);
    b = block_sum(b, sm);
    if (threadIdx.x != 0) return;
    switch (op) {
        case CTL_PRIM_CHECK:
        case CTL_PRIM_CHECK_Z: {
            const double prim = sqrt(a);
            ctrl->prim = prim;
            ctrl->reject = (accel && ctrl->prev_prim < prim) ? 1 : 0;
            if (ctrl->reject) {
                ctrl->nrej += 1;
                if (op == CTL_PRIM_CHECK) { ctrl->aa_iter = 0; ctrl->aa_col = 0; }  // accelerator->reset
            }
            break;
        }
        case CTL_PRIM_FINAL:
        case CTL_PRIM_FINAL_Z:
            if (ctrl->reject) ctrl->prim = sqrt(a);
            ctrl->prev_prim = ctrl->prim;
            break;
        case CTL_COMB_UX: {
            const double comb = a + b;
            ctrl->iters_run += 1;
            ctrl->comb = comb;
            if (comb < kCombEps) { ctrl->done = 1; break; }
            if (record_iter(ctrl, hist_prim, hist_comb, hist_rej, comb)) ctrl->done = 1;
            break;
        }
        case CTL_COMB_Z:
        case CTL_COMB_ZP: {
            const double comb = a + b;
            ctrl->iters_run += 1;
            ctrl->comb = comb;
            const bool eps = record_iter(ctrl, hist_prim, hist_comb, hist_rej, comb);
            // ZP: decided one iteration late (pipelined): done = 2 asks for the speculative
            // next iteration's x to be rolled back (launch_copy gate 2)
            if (comb < kCombEps || eps) ctrl->done = op == CTL_COMB_ZP ? 2 : 1;
            break;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_copy(double* __restrict__ dst, const double* __restrict__ src,
                                                 long long n, const Ctrl* ctrl, int gate_reject) {
    if (gate_reject == 2) {   // only after a pipelined break (CTL_COMB_ZP)
        if (!ctrl || ctrl->done != 2) return;
    } else if (gated(ctrl, gate_reject)) {
        return;
    }
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// Streaming read (16 B per lane, eight loads in flight per thread, one store per thread): the
// measured HBM read ceiling the bench reports the (read-dominated) roofline kernel against, next
// to the spec peak (aa_ctx_bench_read)
__global__ __launch_bounds__(256) void k_stream_read(const double2* __restrict__ src, long long n, double* __restrict__ out) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    double acc = 0;
    for (; i + 7 * stride < n; i += 8 * stride) {
        double2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = src[i + k * stride];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y;
    }
    for (; i < n; i += stride) acc += src[i].x + src[i].y;
    out[blockIdx.x * (long long)blockDim.x + threadIdx.x] = acc;
}

// the same read with a contiguous chunk per workgroup (a wave reads 1 KB per instruction, 8 in
// flight per lane, consecutive instructions on consecutive KB), plain or non-temporal loads
typedef double dbl2v_ __attribute__((ext_vector_type(2)));
template <bool NT>
__global__ __launch_bounds__(256) void k_stream_read_chunk(const double2* __restrict__ src, long long n,
                                                           double* __restrict__ out) {
    const long long per = (n + gridDim.x - 1) / gridDim.x;
    const long long b0 = blockIdx.x * per, b1 = min(n, b0 + per);
    double acc = 0;
    long long i = b0 + threadIdx.x;
    for (; i + 7 * 256 < b1; i += 8 * 256) {
        dbl2v_ v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const dbl2v_* q = reinterpret_cast<const dbl2v_*>(src + i + k * 256);
            v[k] = NT ? __builtin_nontemporal_load(q) : *q;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y;
    }
    for (; i < b1; i += 256) acc += src[i].x + src[i].y;
    out[blockIdx.x * (long long)blockDim.x + threadIdx.x] = acc;
}

// UX reject test (Solver.cpp:139-146) fused with the restore (Solver.cpp:150-154): every block
// reduces the prim partials itself (identical order -> identical decision); block 0 records it.
__global__ __launch_bounds__(kBlock) void k_check_restore_ux(Ctrl* ctrl, const double* __restrict__ red, int nb,
                                                             int accel, double* __restrict__ u, double* __restrict__ x,
                                                             double* __restrict__ cur, const double* __restrict__ du,
                                                             const double* __restrict__ dx, long long nz, long long nx) {
    if (ctrl->done) return;
    __shared__ double sm[kBlock / 64];
    const double prim = sqrt(block_sum_all(red, nb, sm));
    const bool reject = accel && ctrl->prev_prim < prim;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctrl->prim = prim;
        ctrl->reject = reject ? 1 : 0;
        if (reject) { ctrl->nrej += 1; ctrl->aa_iter = 0; ctrl->aa_col = 0; }   // accelerator->reset
    }
    if (!reject) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nz + nx; i += (long long)gridDim.x * blockDim.x) {
        if (i < nz) { const double v = du[i]; u[i] = v; if (cur) cur[i] = v; }
        else { const double v = dx[i - nz]; x[i - nz] = v; if (cur) cur[i] = v; }
    }
}

// Z reject test (Solver.cpp:159-168, k_control CTL_PRIM_CHECK_Z) fused with the restore of the
// defaults (u, x, z = default_{u,x,z} of the previous iteration, Solver.cpp:170-176): one launch
// instead of the control kernel and three gated copies. Every block sums the prim partials itself
// with k_control's 1024-thread order (the same bits, so the same decision); block 0 records it.
__global__ __launch_bounds__(kCtlBlock) void k_check_restore_z(Ctrl* ctrl, const double* __restrict__ red, int nb,
                                                               int accel, double* __restrict__ u,
                                                               double* __restrict__ x, double* __restrict__ z,
                                                               const double* __restrict__ du,
                                                               const double* __restrict__ dx,
                                                               const double* __restrict__ dz, long long nz,
                                                               long long nx) {
    if (ctrl->done) return;
    __shared__ double sm[kCtlBlock / 64];
    double a = thread_sum_strided(red, nb);
    a = block_sum(a, sm);   // thread 0 holds k_control's sum
    __shared__ int rej;
    if (threadIdx.x == 0) {
        const double prim = sqrt(a);
        rej = (accel && ctrl->prev_prim < prim) ? 1 : 0;
        if (blockIdx.x == 0) {
            ctrl->prim = prim;
            ctrl->reject = rej;
            if (rej) ctrl->nrej += 1;
        }
    }
    __syncthreads();
    if (!rej) return;
    const long long n = 2 * nz + nx;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        if (i < nz) u[i] = du[i];
        else if (i < nz + nx) x[i - nz] = dx[i - nz];
        else z[i - nz - nx] = dz[i - nz - nx];
    }
}

// UX reject (Solver.cpp:150-154): (u, x) = defaults and accelerator->reset(u, x) stores them
__global__ __launch_bounds__(kBlock) void k_restore_ux(double* __restrict__ u, double* __restrict__ x,
                                                       double* __restrict__ cur, const double* __restrict__ du,
                                                       const double* __restrict__ dx, long long nz, long long nx,
                                                       const Ctrl* ctrl) {
    if (gated(ctrl, 1)) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nz + nx; i += (long long)gridDim.x * blockDim.x) {
        if (i < nz) { const double v = du[i]; u[i] = v; if (cur) cur[i] = v; }
        else { const double v = dx[i - nz]; x[i - nz] = v; if (cur) cur[i] = v; }
    }
}

__global__ __launch_bounds__(kBlock) void k_predict(int nf, double* __restrict__ xs, double* __restrict__ vs,
                                                    const double* __restrict__ mass, double dt, double gravity,
                                                    double* __restrict__ xbar, double* __restrict__ Mxbar,
                                                    double* __restrict__ xfull) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nf) return;
    if (fabs(gravity) > 0) vs[3 * (size_t)q + 1] += dt * gravity;
    const double m = mass[q];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const size_t o = 3 * (size_t)q + j;
        const double xb = xs[o] + dt * vs[o];
        xbar[o] = xb;
        Mxbar[o] = m * xb;
        xfull[o] = xb;
    }
}

__global__ __launch_bounds__(kBlock) void k_finalize(int n, int nf, const double* __restrict__ xsrc,
                                                     const double* __restrict__ xfull, double* __restrict__ xs,
                                                     double* __restrict__ vs, double dt) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double inv = 1.0 / dt;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const size_t o = 3 * (size_t)q + j;
        const double xn = q < nf ? xsrc[o] : xfull[o];
        vs[o] = (xn - xs[o]) * inv;
        xs[o] = xn;
    }
}

// ------------------------------------------------------------------ Anderson acceleration
// history columns (m x dim doubles: 0.9 GB on C4, streamed past the Infinity Cache every
// iteration) are read with non-temporal loads (AA_AA_NT=0: plain, A/B)
#ifndef AA_AA_NT
#define AA_AA_NT 1
#endif
__device__ __forceinline__ double ld_h(const double* p) {
#if AA_AA_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
// the segment is picked by address, not by branch (a load in each arm of a branch is issued only
// once the branch resolves, behind the loads before it)
__device__ __forceinline__ double seg_get(const Seg2& s, long long i) { return *(i < s.na ? s.a + i : s.b + (i - s.na)); }
__device__ __forceinline__ void seg_set(const Seg2& s, long long i, double v) { *(i < s.na ? s.a + i : s.b + (i - s.na)) = v; }

// pass 1: the partial sums for |dF_j|^2, dF_j.F, dF_j.dF_c, dF_c.F with dF_j = dF_j + F formed on
// the fly (read only: k_aa_mix forms dF_j + F and dG_j + G again and stores them, so the history
// columns are written once per iteration; the arithmetic is unchanged)
template <int MM>
__global__ __launch_bounds__(kBlock) void k_aa_reduce(Seg2 G, const double* __restrict__ cur, long long eff,
                                                      double* __restrict__ dF, double* __restrict__ dG, Ctrl* ctrl,
                                                      double* red, Seg2 copy_to, const double* comb_a,
                                                      const double* comb_b, int comb_nb, double* hist_prim,
                                                      double* hist_comb, int* hist_rej, AAMask mask) {
    if (ctrl->done || !ctrl->aa_active || ctrl->aa_skip) return;
    constexpr int NVAL = 2 + 2 * MM;
    __shared__ double sm[kBlock / 64][NVAL];
    if (comb_a) {   // combined residual + break test + record, fused (every block decides alike)
        __shared__ double sc[kBlock / 64];
        const double comb = block_sum_all(comb_a, comb_nb, sc) + block_sum_all(comb_b, comb_nb, sc);
        const bool brk = comb < kCombEps;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctrl->comb = comb;
            ctrl->iters_run += 1;
            if (brk) ctrl->done = 1;
            // run-to-epsilon stop: this iteration completes as a last one would (the default
            // copies below still happen); k_aa_solve turns eps_hit into done, gating the mix
            else if (record_iter(ctrl, hist_prim, hist_comb, hist_rej, comb)) ctrl->eps_hit = 1;
        }
        if (brk) return;
    }
    const long long dim = G.na + G.nb;
    const int iter = ctrl->aa_iter, col = ctrl->aa_col, m = ctrl->aa_m;
    const int mk = iter < m ? iter : m;
    double acc[NVAL];
#pragma unroll
    for (int t = 0; t < NVAL; ++t) acc[t] = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < dim; i += (long long)gridDim.x * blockDim.x) {
        const double g = seg_get(G, i);
        if (copy_to.a) seg_set(copy_to, i, g);
        if (iter == 0 || i >= eff) continue;
        // every load of the element first (cur, dF_j, the other history columns), then the
        // products: a load used right away serialises the loop on its latency
        const double ci = cur[i];
        const double dfo = ld_h(dF + (size_t)col * eff + i);
        // (wide windows keep the loads in the product loop: MM doubles more would cost occupancy)
        constexpr bool kPre = MM <= 16;
        double dfc[kPre ? MM : 1];
        if constexpr (kPre) {
#pragma unroll
            for (int c = 0; c < MM; ++c) dfc[c] = (c < mk && c != col) ? ld_h(dF + (size_t)c * eff + i) : 0.0;
        }
        if (i >= G.na) {
            const long long j = i - G.na;
            if (!((j >= mask.lo1 && j < mask.hi1) || (j >= mask.lo2 && j < mask.hi2))) continue;
        }
        const double f = g - ci;
        const double dfj = dfo + f;
        acc[0] += dfj * dfj;
        acc[1] += dfj * f;
#pragma unroll
        for (int c = 0; c < MM; ++c) {
            if (c < mk && c != col) {
                double d;
                if constexpr (kPre) d = dfc[c];
                else d = dF[(size_t)c * eff + i];
                acc[2 + c] += dfj * d;
                acc[2 + MM + c] += d * f;
            }
        }
    }
    if (iter == 0) return;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < NVAL; ++t) {
        const double v = wave_sum(acc[t]);
        if (lane == 0) sm[wid][t] = v;
    }
    __syncthreads();
    if (threadIdx.x < NVAL) {
        double s = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sm[w][threadIdx.x];
        red[(size_t)blockIdx.x * NVAL + threadIdx.x] = s;
    }
}

// Wide windows (m > 16, the C5 wire mesh's m = 20): the same partial sums, column-parallel. The
// row-parallel form above keeps 2 + 2 MM accumulators and the MM history loads of an entry in every
// thread's registers (221 VGPRs at MM = 32: 2 waves per SIMD, loads serialised on their latency).
// Here a block walks a contiguous row range in tiles of kAaTile rows: it first stages the tile's
// F_i = G_i - cur_i and dF_j,i + F_i in LDS (and accumulates |dF_j|^2, dF_j.F), then each wave
// takes columns c = wave, wave + 4, ... of the history and streams them coalesced over the tile --
// kAaTile / 64 independent loads per lane -- against the staged vectors: two accumulators per column
// the wave owns. The block partials keep the row-parallel kernel's layout and are summed in block
// order by k_aa_solve, so the reduction is as deterministic; the partial sums group differently, so
// the products differ from the row-parallel kernel's by rounding only (Anderson's least-squares
// coefficients, AndersonAcceleration.h:154-211, are held to the geometry goldens' tolerances).
constexpr int kAaTile = 512;
template <int MM>
__global__ __launch_bounds__(kBlock) void k_aa_reduce_cols(Seg2 G, const double* __restrict__ cur, long long eff,
                                                           double* __restrict__ dF, double* __restrict__ dG, Ctrl* ctrl,
                                                           double* red, Seg2 copy_to, const double* comb_a,
                                                           const double* comb_b, int comb_nb, double* hist_prim,
                                                           double* hist_comb, int* hist_rej, AAMask mask) {
    if (ctrl->done || !ctrl->aa_active || ctrl->aa_skip) return;
    constexpr int NVAL = 2 + 2 * MM, NW = kBlock / 64, QC = (MM + NW - 1) / NW, RL = kAaTile / 64;
    __shared__ double sm[NW][NVAL];
    __shared__ double sdf[kAaTile], sf[kAaTile];
    if (comb_a) {   // as k_aa_reduce
        __shared__ double sc[kBlock / 64];
        const double comb = block_sum_all(comb_a, comb_nb, sc) + block_sum_all(comb_b, comb_nb, sc);
        const bool brk = comb < kCombEps;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            ctrl->comb = comb;
            ctrl->iters_run += 1;
            if (brk) ctrl->done = 1;
            else if (record_iter(ctrl, hist_prim, hist_comb, hist_rej, comb)) ctrl->eps_hit = 1;
        }
        if (brk) return;
    }
    const long long dim = G.na + G.nb;
    const int iter = ctrl->aa_iter, col = ctrl->aa_col, m = ctrl->aa_m;
    const int mk = iter < m ? iter : m;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // this block's rows: a contiguous range, whole tiles
    const long long per = ((dim + gridDim.x - 1) / gridDim.x + kAaTile - 1) / kAaTile * kAaTile;
    const long long r0 = (long long)blockIdx.x * per, r1 = r0 + per < dim ? r0 + per : dim;
    double a0 = 0, a1 = 0, ac[QC], bc[QC];
#pragma unroll
    for (int q = 0; q < QC; ++q) { ac[q] = 0; bc[q] = 0; }
    for (long long t0 = r0; t0 < r1; t0 += kAaTile) {
        for (int k = threadIdx.x; k < kAaTile; k += kBlock) {
            const long long i = t0 + k;
            double dfj = 0, f = 0;
            if (i < r1) {
                const double g = seg_get(G, i);
                if (copy_to.a) seg_set(copy_to, i, g);
                bool in = iter != 0 && i < eff;
                if (in && i >= G.na) {
                    const long long j = i - G.na;
                    in = (j >= mask.lo1 && j < mask.hi1) || (j >= mask.lo2 && j < mask.hi2);
                }
                if (in) {
                    f = g - cur[i];
                    dfj = ld_h(dF + (size_t)col * eff + i) + f;
                    a0 += dfj * dfj;
                    a1 += dfj * f;
                }
            }
            sdf[k] = dfj;
            sf[k] = f;
        }
        __syncthreads();
        if (iter != 0) {
#pragma unroll
            for (int q = 0; q < QC; ++q) {
                const int c = wid + NW * q;
                if (c < mk && c != col) {   // wave-uniform
                    const double* src = dF + (size_t)c * eff;
                    double d[RL];
#pragma unroll
                    for (int j = 0; j < RL; ++j) {
                        const long long i = t0 + lane + 64 * j;
                        d[j] = i < r1 && i < eff ? ld_h(src + i) : 0.0;
                    }
#pragma unroll
                    for (int j = 0; j < RL; ++j) {
                        ac[q] += sdf[lane + 64 * j] * d[j];
                        bc[q] += d[j] * sf[lane + 64 * j];
                    }
                }
            }
        }
        __syncthreads();
    }
    if (iter == 0) return;
    a0 = wave_sum(a0);
    a1 = wave_sum(a1);
    if (lane == 0) { sm[wid][0] = a0; sm[wid][1] = a1; }
#pragma unroll
    for (int q = 0; q < QC; ++q) {
        const double x = wave_sum(ac[q]), y = wave_sum(bc[q]);
        const int c = wid + NW * q;
        if (lane == 0 && c < MM) {
            for (int w = 0; w < NW; ++w)
                if (w != wid) { sm[w][2 + c] = 0; sm[w][2 + MM + c] = 0; }
            sm[wid][2 + c] = x;
            sm[wid][2 + MM + c] = y;
        }
    }
    __syncthreads();
    if (threadIdx.x < NVAL) {
        double s2 = 0;
        for (int w = 0; w < NW; ++w) s2 += sm[w][threadIdx.x];
        red[(size_t)blockIdx.x * NVAL + threadIdx.x] = s2;
    }
}

// Eigen CompleteOrthogonalDecomposition::solve of the small normal equations, block-cooperative:
// column-pivoted Householder QR with LAPACK norm downdating (Eigen/src/QR/ColPivHouseholderQR.h
// :482-579), rank = #|R_ii| > eps*n*|maxpivot| (:255-263), RZ step + minimum-norm solve
// (Eigen/src/QR/CompleteOrthogonalDecomposition.h:410-525). All state lives in LDS; each column
// update / norm downdate runs on its own thread with the same operation order as the serial
// algorithm, so the result is the serial result bit for bit.
struct CodLds {
    double A[kMaxM * kMaxM];   // column-major n x n
    double hc[kMaxM], nu[kMaxM], nd[kMaxM], zc[kMaxM], c[kMaxM], y[kMaxM];
    double bc[4];              // beta, tau, c0 broadcast
    int tr[kMaxM], perm[kMaxM], big, rank;
};

__device__ void cod_solve_block(int n, CodLds& S, const double* b, double* x) {
    const int t = threadIdx.x;
#define QR(r, cc) S.A[(cc) * n + (r)]
    if (t < n) {
        double s = 0;
        for (int r = 0; r < n; ++r) s += QR(r, t) * QR(r, t);
        S.nd[t] = S.nu[t] = sqrt(s);
    }
    __syncthreads();
    const double ddt = sqrt(2.220446049250313e-16);
    double maxpivot = 0;   // tracked by thread 0
    for (int k = 0; k < n; ++k) {
        if (t == 0) {
            int big = k;
            for (int j = k + 1; j < n; ++j) if (S.nu[j] > S.nu[big]) big = j;
            S.tr[k] = big;
            S.big = big;
            if (big != k) {
                double tt = S.nu[k]; S.nu[k] = S.nu[big]; S.nu[big] = tt;
                tt = S.nd[k]; S.nd[k] = S.nd[big]; S.nd[big] = tt;
            }
        }
        __syncthreads();
        const int big = S.big;
        if (big != k && t < n) { const double tt = QR(t, k); QR(t, k) = QR(t, big); QR(t, big) = tt; }
        __syncthreads();
        if (t == 0) {
            const double c0 = QR(k, k);
            double tail = 0;
            for (int r = k + 1; r < n; ++r) tail += QR(r, k) * QR(r, k);
            double beta, tau;
            if (tail <= 2.2250738585072014e-308) { tau = 0; beta = c0; }
            else { beta = sqrt(c0 * c0 + tail); if (c0 >= 0) beta = -beta; tau = (beta - c0) / beta; }
            S.bc[0] = beta; S.bc[1] = tau; S.bc[2] = c0; S.bc[3] = tail;
            maxpivot = fmax(maxpivot, fabs(beta));
        }
        __syncthreads();
        const double beta = S.bc[0], tau = S.bc[1], c0 = S.bc[2];
        const bool zero_tail = S.bc[3] <= 2.2250738585072014e-308;
        if (t > k && t < n) QR(t, k) = zero_tail ? 0.0 : QR(t, k) / (c0 - beta);
        __syncthreads();
        if (t == 0) { S.hc[k] = tau; QR(k, k) = beta; }
        if (tau != 0 && t > k && t < n) {   // apply H_k to column t
            double tt = QR(k, t);
            for (int r = k + 1; r < n; ++r) tt += QR(r, k) * QR(r, t);
            QR(k, t) -= tau * tt;
            for (int r = k + 1; r < n; ++r) QR(r, t) -= tau * QR(r, k) * tt;
        }
        __syncthreads();
        if (t > k && t < n && S.nu[t] != 0) {   // norm downdate of column t
            double tt = fabs(QR(k, t)) / S.nu[t];
            tt = (1.0 + tt) * (1.0 - tt);
            tt = tt < 0 ? 0 : tt;
            const double r2 = S.nu[t] / S.nd[t];
            if (tt * r2 * r2 <= ddt) {
                double s = 0;
                for (int r = k + 1; r < n; ++r) s += QR(r, t) * QR(r, t);
                S.nd[t] = S.nu[t] = sqrt(s);
            } else S.nu[t] *= sqrt(tt);
        }
        __syncthreads();
    }
    if (t == 0) {   // rank, RZ (rank-deficient only), Q^T b, triangular solve, Z^T, permutation
        for (int i = 0; i < n; ++i) S.perm[i] = i;
        for (int k = 0; k < n; ++k) { const int tt = S.perm[k]; S.perm[k] = S.perm[S.tr[k]]; S.perm[S.tr[k]] = tt; }
        const double thr = fabs(maxpivot) * 2.220446049250313e-16 * n;
        int rank = 0;
        for (int i = 0; i < n; ++i) rank += fabs(QR(i, i)) > thr;
        for (int i = 0; i < n; ++i) S.zc[i] = 0;
        if (rank == 0) {
            for (int i = 0; i < n; ++i) x[i] = 0;
        } else {
            if (rank < n) {
                for (int k = rank - 1; k >= 0; --k) {
                    if (k != rank - 1) for (int r = 0; r <= k; ++r) { const double tt = QR(r, k); QR(r, k) = QR(r, rank - 1); QR(r, rank - 1) = tt; }
                    const double c0 = QR(k, rank - 1);
                    double tail = 0;
                    for (int cc = rank; cc < n; ++cc) tail += QR(k, cc) * QR(k, cc);
                    double beta, tau;
                    if (tail <= 2.2250738585072014e-308) { tau = 0; beta = c0; for (int cc = rank; cc < n; ++cc) QR(k, cc) = 0; }
                    else {
                        beta = sqrt(c0 * c0 + tail);
                        if (c0 >= 0) beta = -beta;
                        for (int cc = rank; cc < n; ++cc) QR(k, cc) /= (c0 - beta);
                        tau = (beta - c0) / beta;
                    }
                    S.zc[k] = tau;
                    QR(k, rank - 1) = beta;
                    if (k > 0 && tau != 0)
                        for (int r = 0; r < k; ++r) {
                            double tt = QR(r, rank - 1);
                            for (int cc = rank; cc < n; ++cc) tt += QR(r, cc) * QR(k, cc);
                            QR(r, rank - 1) -= tau * tt;
                            for (int cc = rank; cc < n; ++cc) QR(r, cc) -= tau * tt * QR(k, cc);
                        }
                    if (k != rank - 1) for (int r = 0; r <= k; ++r) { const double tt = QR(r, k); QR(r, k) = QR(r, rank - 1); QR(r, rank - 1) = tt; }
                }
            }
            for (int i = 0; i < n; ++i) S.c[i] = b[i];
            for (int k = 0; k < rank; ++k) {
                if (S.hc[k] == 0) continue;
                double tt = S.c[k];
                for (int r = k + 1; r < n; ++r) tt += QR(r, k) * S.c[r];
                S.c[k] -= S.hc[k] * tt;
                for (int r = k + 1; r < n; ++r) S.c[r] -= S.hc[k] * QR(r, k) * tt;
            }
            for (int i = 0; i < n; ++i) S.y[i] = 0;
            for (int i = rank - 1; i >= 0; --i) {
                double s = S.c[i];
                for (int j = i + 1; j < rank; ++j) s -= QR(i, j) * S.y[j];
                S.y[i] = s / QR(i, i);
            }
            if (rank < n) {
                for (int k = 0; k < rank; ++k) {
                    if (k != rank - 1) { const double tt = S.y[k]; S.y[k] = S.y[rank - 1]; S.y[rank - 1] = tt; }
                    if (S.zc[k] != 0) {
                        double tt = S.y[rank - 1];
                        for (int cc = rank; cc < n; ++cc) tt += QR(k, cc) * S.y[cc];
                        S.y[rank - 1] -= S.zc[k] * tt;
                        for (int cc = rank; cc < n; ++cc) S.y[cc] -= S.zc[k] * QR(k, cc) * tt;
                    }
                    if (k != rank - 1) { const double tt = S.y[k]; S.y[k] = S.y[rank - 1]; S.y[rank - 1] = tt; }
                }
            }
            for (int i = 0; i < n; ++i) x[S.perm[i]] = S.y[i];
        }
    }
    __syncthreads();
#undef QR
}

// 1024 threads: summing up to 2048 x NVAL block partials is latency-bound
// 256 threads (one wave per SIMD): the block then fits on a CU beside the NeoHookean local step's
// one 402-register wave per SIMD, so the Anderson step of iteration k is not held back until the
// concurrent combined-residual pass's local step retires (a 1024-thread block, 4 waves per SIMD,
// needs a CU of its own). The block partials are still summed in kSolveChunks chunks per value
// (the 1024-thread layout), so the sums -- and the coefficients -- are unchanged.
constexpr int kSolveBlock = 256;
constexpr int kSolveThreads1024 = 1024;
template <int MM>
__global__ __launch_bounds__(kSolveBlock) void k_aa_solve(Ctrl* ctrl, const double* red, int nb) {
    if (ctrl->done || !ctrl->aa_active || ctrl->aa_skip) return;
    if (ctrl->eps_hit) {   // run-to-epsilon stop recorded by k_aa_reduce (one block: no race)
        __syncthreads();
        if (threadIdx.x == 0) ctrl->done = 1;
        return;
    }
    constexpr int NVAL = 2 + 2 * MM;
    constexpr int NCH = kSolveThreads1024 / NVAL;   // block partials are split into NCH chunks per value
    __shared__ double tot[NVAL];
    __shared__ double part[NCH * NVAL];
    const int iter = ctrl->aa_iter;
    if (iter > 0) {
        // item (chunk c, value v) sums partials c, c+NCH, ... of value v: independent loads,
        // fixed order -> deterministic; a thread takes items w, w + blockDim, ...
        for (int w = threadIdx.x; w < NCH * NVAL; w += blockDim.x) {
            const int v = w % NVAL, c = w / NVAL;
            double s = 0;
#pragma unroll 8
            for (int b = c; b < nb; b += NCH) s += red[(size_t)b * NVAL + v];
            part[c * NVAL + v] = s;
        }
        __syncthreads();
        if (threadIdx.x < NVAL) {
            double s = 0;
            for (int c = 0; c < NCH; ++c) s += part[c * NVAL + threadIdx.x];
            tot[threadIdx.x] = s;
        }
    }
    __syncthreads();
    __shared__ CodLds S;
    __shared__ double sb[kMaxM], sx[kMaxM];
    __shared__ int s_mk;
    const int m = ctrl->aa_m, col = ctrl->aa_col;
    if (iter == 0) {
        if (threadIdx.x == 0) {
            ctrl->aa_first = 1; ctrl->aa_j = 0; ctrl->aa_jn = 0; ctrl->aa_mk = 0;
            ctrl->aa_iter = 1;
        }
        return;
    }
    const int mk = iter < m ? iter : m;
    const double eps = 1e-14;
    const double s = fmax(eps, sqrt(tot[0]));
    // the normal-equation matrix and the column scales live in Ctrl (device memory) between
    // iterations; they are staged through LDS here so the serial parts below never wait on a
    // global load (thread 0 reading back what it just stored cost ~25 us per call)
    __shared__ double sM[kMaxM * kMaxM], ssc[kMaxM];
    for (int q = threadIdx.x; q < mk * mk; q += blockDim.x) sM[(q / mk) * m + q % mk] = ctrl->M[(q / mk) * m + q % mk];
    if ((int)threadIdx.x < mk) ssc[threadIdx.x] = ctrl->scale[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) {
        ssc[col] = s;
        if (mk == 1) {
            sx[0] = 0;
            const double sq = tot[0] / (s * s);
            sM[0] = sq;
            const double dn = sqrt(sq);
            if (dn > eps) sx[0] = (tot[1] / s) / (dn * dn);
        } else {
            for (int c = 0; c < mk; ++c) {
                if (c == col) continue;
                const double v = tot[2 + c] / s;
                sM[c * m + col] = v;
                sM[col * m + c] = v;
                sb[c] = tot[2 + MM + c];
            }
            sM[col * m + col] = tot[0] / (s * s);
            sb[col] = tot[1] / s;
            for (int c = 0; c < mk; ++c)
                for (int r = 0; r < mk; ++r) S.A[c * mk + r] = sM[c * m + r];
        }
        s_mk = mk;
    }
    __syncthreads();
    if (s_mk > 1) cod_solve_block(s_mk, S, sb, sx);
    // write back in parallel: row/column col of M, scale[col], the coefficients
    if ((int)threadIdx.x < mk) {
        const int c = threadIdx.x;
        ctrl->M[c * m + col] = sM[c * m + col];
        ctrl->M[col * m + c] = sM[col * m + c];
        ctrl->coef[c] = sx[c] / ssc[c];
        if (c == col) ctrl->scale[col] = s;
    }
    if (threadIdx.x != 0) return;
    ctrl->aa_first = 0;
    ctrl->aa_j = col;
    ctrl->aa_jn = (col + 1) % m;
    ctrl->aa_mk = mk;
    ctrl->aa_s = s;
    ctrl->aa_col = (col + 1) % m;
    ctrl->aa_iter = iter + 1;
}

// pass 2: dG_j += G, dF_j = (dF_j + F) / scale, u = G - dG theta/scale, start the next column with
// -F / -G. With out.a == cur (the Z variant mixes z in place) the output is written once.
template <int MM>
__global__ __launch_bounds__(kBlock) void k_aa_mix(Seg2 G, double* cur, long long eff,
                                                   double* __restrict__ dF, double* __restrict__ dG, Ctrl* ctrl,
                                                   Seg2 out) {
    if (ctrl->done || !ctrl->aa_active || ctrl->aa_skip) return;
    const long long dim = G.na + G.nb;
    const int first = ctrl->aa_first, j = ctrl->aa_j, jn = ctrl->aa_jn, mk = ctrl->aa_mk;
    const double s = ctrl->aa_s;
    const bool inplace = out.a == cur && out.nb == 0;
    double coef[MM];
#pragma unroll
    for (int c = 0; c < MM; ++c) coef[c] = c < mk ? ctrl->coef[c] : 0.0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < dim; i += (long long)gridDim.x * blockDim.x) {
        // loads first (G, cur, dF_j, the dG columns), then the arithmetic and the stores
        const double g = seg_get(G, i);
        const bool in_eff = i < eff;
        const double ci = in_eff ? cur[i] : 0.0;
        const double dfo = (!first && in_eff) ? ld_h(dF + (size_t)j * eff + i) : 0.0;
        constexpr bool kPre = MM <= 16;   // as in k_aa_reduce
        double dgc[kPre ? MM : 1];
        if constexpr (kPre) {
#pragma unroll
            for (int c = 0; c < MM; ++c) dgc[c] = (!first && c < mk) ? ld_h(dG + (size_t)c * dim + i) : 0.0;
        }
        const double f = in_eff ? g - ci : 0.0;
        double res;
        if (first) {
            res = g;
        } else {
            double acc = 0, dgj = 0;
#pragma unroll
            for (int c = 0; c < MM; ++c)
                if (c < mk) {
                    double d;
                    if constexpr (kPre) d = dgc[c];
                    else d = dG[(size_t)c * dim + i];
                    if (c == j) { d += g; dgj = d; }
                    acc += d * coef[c];
                }
            dG[(size_t)j * dim + i] = dgj;
            res = g - acc;
            if (in_eff) dF[(size_t)j * eff + i] = (dfo + f) / s;
        }
        if (i < eff) dF[(size_t)jn * eff + i] = -f;
        dG[(size_t)jn * dim + i] = -g;
        if (!inplace) seg_set(out, i, res);
        cur[i] = res;
    }
}

inline int grid_for(long long n) { long long b = (n + kBlock - 1) / kBlock; return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048); }

// ---- element-level test hooks: the device prox / COD functions on given inputs (tests only)
// op 0 linear tet (9), 1 NeoHookean, 2 StVK (prm: E, nu, h -> vol = h^3/6), 3 tri H prox, 4 tri X
// prox (prm: -, -, limit_min, limit_max)
__global__ void k_test_prox(int op, double E, double nu, double p2, double p3, const double* __restrict__ in, int n,
                            double* __restrict__ out, int* __restrict__ iters) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const int D = op >= 3 ? 6 : 9;
    double v[9], z[9];
    for (int i = 0; i < D; ++i) v[i] = in[(size_t)e * D + i];
    int it = 0;
    if (op == 0) {
        dev::tet_linear_prox(v, z);
    } else if (op <= 2) {
        const double mu = E / (2.0 * (1.0 + nu)), lam = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu));
        for (int i = 0; i < 9; ++i) z[i] = v[i];
        int fail = 0;
        it = dev::hyper_prox(op, mu, lam, lam + 2.0 * mu / 3.0, p2 * p2 * p2 / 6.0, v, z, &fail);
        if (fail) it = -1;
    } else {
        dev::tri_prox(v, z, op == 3 ? 1 : 0, p2, p3);
    }
    for (int i = 0; i < D; ++i) out[(size_t)e * D + i] = z[i];
    if (iters) iters[e] = it;
}

__global__ __launch_bounds__(kSolveBlock) void k_test_cod(int n, const double* __restrict__ M, const double* __restrict__ b,
                                                          double* __restrict__ x) {
    __shared__ CodLds S;
    __shared__ double sb[kMaxM], sx[kMaxM];
    for (int q = threadIdx.x; q < n * n; q += blockDim.x) S.A[q] = M[q];
    if ((int)threadIdx.x < n) sb[threadIdx.x] = b[threadIdx.x];
    __syncthreads();
    cod_solve_block(n, S, sb, sx);
    __syncthreads();
    if ((int)threadIdx.x < n) x[threadIdx.x] = sx[threadIdx.x];
}

}  // namespace

// ============================================================================ launchers
// per solver (initialize): the resident grid of the work-queue kernel on `device` and the refill
// threshold (AA_LQ_REFILL, default 60 idle lanes)
LocalQueue make_local_queue(int device, int* counter) {
    LocalQueue q;
    q.counter = counter;
    int cus = 0, per = 0;
    AA_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const char* r = std::getenv("AA_LQ_REFILL");
    const char* ah = std::getenv("AA_LQ_AHEAD");
    const char* lh = std::getenv("AA_LQ_LDS");
    q.ahead = ah && ah[0] == '1';   // opt-in: measured slower on C4
    q.hist = (lh && lh[0] == '1') ? LQ_HIST_YLDS : LQ_HIST_REGS;   // opt-in: no faster on C4
    const char* sp = std::getenv("AA_LQ_SPLIT");
    q.split = sp ? sp[0] == '1' : false;
    if (q.split) q.ahead = false, q.hist = LQ_HIST_REGS;
    const char* ck = std::getenv("AA_LQ_CHUNK");
    q.chunk = ck && ck[0] == '1' && !q.split && !q.ahead && q.hist == LQ_HIST_REGS;
    const char* fu = std::getenv("AA_LQ_FUSED");
    // default on (AA_LQ_FUSED=0: the plain refill); the caller turns it off for the concurrent pass
    q.fused = (fu ? fu[0] == '1' : true) && !q.split && !q.ahead && !q.chunk && q.hist == LQ_HIST_REGS;
    const void* kq = q.fused ? (const void*)k_local_z_hqf<4>
                   : q.chunk ? (const void*)k_local_z_hq<4, LQ_HIST_REGS, 1>
                   : q.split ? (const void*)k_local_z_hq2<4>
                   : q.ahead ? (q.hist == LQ_HIST_YLDS ? (const void*)k_local_z_hqa<4, LQ_HIST_YLDS>
                                                       : (const void*)k_local_z_hqa<4, LQ_HIST_REGS>)
                             : (q.hist == LQ_HIST_YLDS ? (const void*)k_local_z_hq<4, LQ_HIST_YLDS>
                                                       : (const void*)k_local_z_hq<4, LQ_HIST_REGS>);
    const size_t lds = q.hist == LQ_HIST_YLDS ? kLqLdsBytes : 0;
    q.lds_bytes = lds;
    if (lds) AA_HIP(hipFuncSetAttribute(kq, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    AA_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kq, kBlock, lds));
    q.resident = std::max(1, cus * std::max(1, per));
    q.refill = r ? std::atoi(r) : 60;
    if (q.split) q.refill = std::max(1, (q.refill + 1) / 2);   // in pairs (elements) per wave
    // lookahead stops once fewer elements than this are left (AA_LQ_MARGIN: in resident lanes)
    const char* mg = std::getenv("AA_LQ_MARGIN");
    q.margin = (int)(std::max(0.0, mg ? std::atof(mg) : 1.0) * q.resident * kBlock);
    return q;
}

void launch_local_z(const GroupDev& g, const double* xfull, const double* u, double* z, double* y, int nf,
                    int variant, int mode, Ctrl* ctrl, double* red, int red_off, hipStream_t s, const LocalQueue* queue) {
    if (g.count == 0) return;
    const int nb = blocks_for(g.count);
    if (g.kind == 0 && g.mat != 0 && !red && queue && queue->counter) {   // hyperelastic, no partials: work queue
        // k_local_z_hq / k_local_z_hqf reset the queue themselves (queue_reset_last)
        if (queue->split || queue->ahead) AA_HIP(hipMemsetAsync(queue->counter, 0, sizeof(int), s));
        const int resident = std::max(1, queue->resident), refill = queue->refill;
        const dim3 grid(std::min(nb, resident));
        const size_t lds = queue->lds_bytes;
        if (queue->split) {   // two lanes per element: half the elements per block
            const dim3 grid2(std::min(blocks_for(2LL * g.count), resident));
            hipLaunchKernelGGL((k_local_z_hq2<4>), grid2, dim3(kBlock), 0, s, g, xfull, u, z, y, nf, mode, ctrl,
                               queue->counter, refill, queue->stats);
        } else if (queue->ahead && queue->hist == LQ_HIST_YLDS)
            hipLaunchKernelGGL((k_local_z_hqa<4, LQ_HIST_YLDS>), grid, dim3(kBlock), lds, s, g, xfull, u, z, y, nf, mode,
                               ctrl, queue->counter, refill, queue->margin, queue->stats);
        else if (queue->ahead)
            hipLaunchKernelGGL((k_local_z_hqa<4, LQ_HIST_REGS>), grid, dim3(kBlock), 0, s, g, xfull, u, z, y, nf, mode,
                               ctrl, queue->counter, refill, queue->margin, queue->stats);
        else if (queue->fused && !g.pinned)   // pinned groups keep the plain refill (their Cp needs positions)
        {
            if (y) hipLaunchKernelGGL((k_local_z_hqf<4, true>), grid, dim3(kBlock), 0, s, g, xfull, u, z, y, nf, mode,
                                      ctrl, queue->counter, refill, queue->stats);
            else hipLaunchKernelGGL((k_local_z_hqf<4, false>), grid, dim3(kBlock), 0, s, g, xfull, u, z, y, nf, mode,
                                    ctrl, queue->counter, refill, queue->stats);
        }
        else if (queue->chunk)
            hipLaunchKernelGGL((k_local_z_hq<4, LQ_HIST_REGS, 1>), grid, dim3(kBlock), 0, s, g, xfull, u, z, y, nf,
                               mode, ctrl, queue->counter, refill, queue->stats, queue->margin);
        else if (queue->hist == LQ_HIST_YLDS)
            hipLaunchKernelGGL((k_local_z_hq<4, LQ_HIST_YLDS>), grid, dim3(kBlock), lds, s, g, xfull, u, z, y, nf, mode,
                               ctrl, queue->counter, refill, queue->stats);
        else
            hipLaunchKernelGGL((k_local_z_hq<4, LQ_HIST_REGS>), grid, dim3(kBlock), 0, s, g, xfull, u, z, y, nf, mode,
                               ctrl, queue->counter, refill, queue->stats);
        AA_CHECK_LAUNCH();
        return;
    }
    if (g.kind == 2) hipLaunchKernelGGL((k_local_z<1, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, u, z, y, nf, variant, mode, ctrl, red, red_off);
    else if (g.kind == 1) hipLaunchKernelGGL((k_local_z<3, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, u, z, y, nf, variant, mode, ctrl, red, red_off);
    else if (g.mat == 0) hipLaunchKernelGGL((k_local_z<4, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, u, z, y, nf, variant, mode, ctrl, red, red_off);
    else hipLaunchKernelGGL((k_local_z<4, 1>), dim3(nb), dim3(kBlock), 0, s, g, xfull, u, z, y, nf, variant, mode, ctrl, red, red_off);
    AA_CHECK_LAUNCH();
}

void launch_resid_update_u(const GroupDev& g, const double* xfull, const double* xlast, const double* z, double* u,
                           int nf, Ctrl* ctrl, double* red_a, double* red_b, int red_off, hipStream_t s) {
    if (g.count == 0) return;
    const int nb = blocks_for(g.count);
    if (g.kind == 2) hipLaunchKernelGGL(k_resid_u<1>, dim3(nb), dim3(kBlock), 0, s, g, xfull, xlast, z, u, nf, ctrl, red_a, red_b, red_off);
    else if (g.kind == 1) hipLaunchKernelGGL(k_resid_u<3>, dim3(nb), dim3(kBlock), 0, s, g, xfull, xlast, z, u, nf, ctrl, red_a, red_b, red_off);
    else hipLaunchKernelGGL(k_resid_u<4>, dim3(nb), dim3(kBlock), 0, s, g, xfull, xlast, z, u, nf, ctrl, red_a, red_b, red_off);
    AA_CHECK_LAUNCH();
}

void launch_u_and_y(const GroupDev& g, const double* xfull, const double* z, double* u, double* y, int nf, int mode,
                    int redo, Ctrl* ctrl, hipStream_t s) {
    if (g.count == 0) return;
    const int nb = blocks_for(g.count);
    if (g.kind == 2) hipLaunchKernelGGL((k_u_and_y<1, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, z, u, y, nf, mode, redo, ctrl);
    else if (g.kind == 1) hipLaunchKernelGGL((k_u_and_y<3, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, z, u, y, nf, mode, redo, ctrl);
    else if (g.mat == 0) hipLaunchKernelGGL((k_u_and_y<4, 0>), dim3(nb), dim3(kBlock), 0, s, g, xfull, z, u, y, nf, mode, redo, ctrl);
    else hipLaunchKernelGGL((k_u_and_y<4, 1>), dim3(nb), dim3(kBlock), 0, s, g, xfull, z, u, y, nf, mode, redo, ctrl);
    AA_CHECK_LAUNCH();
}

void launch_prim_z(const GroupDev& g, const double* xfull, const double* z, const double* zref, int nf, int redo,
                   Ctrl* ctrl, double* red_a, double* red_b, int red_off, hipStream_t s) {
    if (g.count == 0) return;
    const int nb = blocks_for(g.count);
    if (g.kind == 2) hipLaunchKernelGGL(k_prim_z<1>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z, zref, nf, redo, ctrl, red_a, red_b, red_off);
    else if (g.kind == 1) hipLaunchKernelGGL(k_prim_z<3>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z, zref, nf, redo, ctrl, red_a, red_b, red_off);
    else hipLaunchKernelGGL(k_prim_z<4>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z, zref, nf, redo, ctrl, red_a, red_b, red_off);
    AA_CHECK_LAUNCH();
}

void launch_init_z(const GroupDev& g, const double* xfull, double* z, hipStream_t s) {
    if (g.count == 0) return;
    const int nb = blocks_for(g.count);
    if (g.kind == 2) hipLaunchKernelGGL(k_init_z<1>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z);
    else if (g.kind == 1) hipLaunchKernelGGL(k_init_z<3>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z);
    else hipLaunchKernelGGL(k_init_z<4>, dim3(nb), dim3(kBlock), 0, s, g, xfull, z);
    AA_CHECK_LAUNCH();
}

void launch_rhs(int nf, const int* ptr, const int* row, const double* val, const double* y, const double* Mxbar,
                double pdt2, double* b, Ctrl* ctrl, int gate_reject, hipStream_t s, const double* xsrc,
                double* xlast, const double* red_final, int nb_final) {
    if (nf == 0) return;
    if (!val)
        hipLaunchKernelGGL(k_rhs_slots, dim3(blocks_for(64 * ((nf + 20) / 21LL))), dim3(kBlock), 0, s, nf, ptr, y, Mxbar,
                           pdt2, b, ctrl, gate_reject, xsrc, xlast, red_final, nb_final);
    else
        hipLaunchKernelGGL(k_rhs, dim3(blocks_for(nf)), dim3(kBlock), 0, s, nf, ptr, row, val, y, Mxbar, pdt2, b, ctrl,
                           gate_reject, xsrc, xlast, red_final, nb_final);
    AA_CHECK_LAUNCH();
}

void launch_control(int op, Ctrl* ctrl, const double* red_a, const double* red_b, int nblocks, int accel,
                    double* hist_prim, double* hist_comb, int* hist_rej, hipStream_t s) {
    hipLaunchKernelGGL(k_control, dim3(1), dim3(kCtlBlock), 0, s, op, ctrl, red_a, red_b, nblocks, accel, hist_prim, hist_comb, hist_rej);
    AA_CHECK_LAUNCH();
}

__global__ void k_stamp(Ctrl* ctrl) { ctrl->clock0 = (long long)wall_clock64(); }

// Concurrent combined-residual pass (ElasticSolver::enqueue_iteration_z): the
// pass of iteration k-1 runs on a second stream beside iteration k, on its own copy of the
// control block. Fork: the copy is taken once everything before it on the main stream is done
// (the prim / reject of k-1 it records, done, fail, the record counters).
__global__ __launch_bounds__(256) void k_ctrl_fork(const Ctrl* __restrict__ ctrl, Ctrl* __restrict__ side) {
    const int* a = reinterpret_cast<const int*>(ctrl);
    int* b = reinterpret_cast<int*>(side);
    for (int i = threadIdx.x; i < (int)(sizeof(Ctrl) / sizeof(int)); i += blockDim.x) b[i] = a[i];
    __syncthreads();
    if (threadIdx.x == 0) side->pad_ = ctrl->done;   // done at the fork: a join acts only on a pass that ran
}

// Join: the pass's records become the solver's; a break (comb < 1e-20 or the eps stop, the
// side's done) ends the step as the sequential order would have -- before the iteration(s)
// enqueued since the fork: done = 2, x restored to curr_x of the pass's iteration (dx), and what
// those iterations changed that outlives the step is taken back (their reject count, a prox
// failure of their local steps). Every block decides from the side block alone (written before
// this kernel, read-only here), so the restore happens exactly once, at the join that found the
// break -- a later pass forked with done set is inert.
__global__ __launch_bounds__(256) void k_ctrl_join(Ctrl* __restrict__ ctrl, const Ctrl* __restrict__ side,
                                                   double* __restrict__ x, const double* __restrict__ dx, long long n) {
    const bool ran = side->pad_ == 0, brk = ran && side->done != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && ran) {
        ctrl->nrec = side->nrec;
        ctrl->iters_run = side->iters_run;
        ctrl->comb = side->comb;
        ctrl->eps_abs = side->eps_abs;
        if (brk) {
            ctrl->done = 2;
            ctrl->nrej = side->nrej;
            ctrl->fail = side->fail;
        } else {
            ctrl->fail = ctrl->fail ? ctrl->fail : side->fail;
        }
    }
    if (!brk) return;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        x[i] = dx[i];
}

// WindForce::project (ExplicitForce.cpp:47-104; helper::triangle_norm :28-39), Wejchert-Haumann
// normal force, one workgroup sweeping the triangle levels (see launch_wind); Eigen's operation
// order (squaredNorm (a + b) + c, normalized = n / sqrt(squaredNorm), dot (a + b) + c), no FMA.
__global__ __launch_bounds__(1024) void k_wind(const int* __restrict__ tris3, const int* __restrict__ ord,
                                               const int* __restrict__ lvl_ptr, int nlvl, const double* __restrict__ x,
                                               double* __restrict__ v, double d0, double d1, double d2, double dt) {
#pragma clang fp contract(off)
    const double dir[3] = {d0, d1, d2};
    for (int l = 0; l < nlvl; ++l) {
        for (int k = lvl_ptr[l] + (int)threadIdx.x; k < lvl_ptr[l + 1]; k += blockDim.x) {
            const int t = ord[k];
            const size_t i0 = 3 * (size_t)tris3[3 * t], i1 = 3 * (size_t)tris3[3 * t + 1], i2 = 3 * (size_t)tris3[3 * t + 2];
            double vr[3], a[3], b[3];
            for (int c = 0; c < 3; ++c) {
                vr[c] = (v[i0 + c] + v[i1 + c] + v[i2 + c]) / 3.0 - dir[c];
                a[c] = x[i1 + c] - x[i0 + c];
                b[c] = x[i2 + c] - x[i0 + c];
            }
            double n[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
            const double z2 = (n[0] * n[0] + n[1] * n[1]) + n[2] * n[2];
            const double nrm = sqrt(z2);
            double nu[3] = {n[0], n[1], n[2]};
            if (z2 > 0.0) { nu[0] = n[0] / nrm; nu[1] = n[1] / nrm; nu[2] = n[2] / nrm; }
            const double area = 0.5 * nrm;
            const double alpha_n = 1000.0;
            const double vn = (nu[0] * vr[0] + nu[1] * vr[1]) + nu[2] * vr[2];
            const double sc = -alpha_n * area * vn * fabs(vn);
            double f[3];
            for (int c = 0; c < 3; ++c) { f[c] = sc * nu[c]; f[c] *= 0.33; f[c] *= dt; }
            for (int c = 0; c < 3; ++c) v[i0 + c] += f[c];
            for (int c = 0; c < 3; ++c) v[i1 + c] += f[c];
            for (int c = 0; c < 3; ++c) v[i2 + c] += f[c];
        }
        __syncthreads();
    }
}

void launch_stamp(Ctrl* ctrl, hipStream_t s) {
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(1), 0, s, ctrl);
    AA_CHECK_LAUNCH();
}

void launch_ctrl_fork(const Ctrl* ctrl, Ctrl* side, hipStream_t s) {
    hipLaunchKernelGGL(k_ctrl_fork, dim3(1), dim3(256), 0, s, ctrl, side);
    AA_CHECK_LAUNCH();
}

void launch_ctrl_join(Ctrl* ctrl, const Ctrl* side, double* x, const double* dx, long long n, hipStream_t s) {
    hipLaunchKernelGGL(k_ctrl_join, dim3(std::max(1, grid_for(n))), dim3(256), 0, s, ctrl, side, x, dx, n);
    AA_CHECK_LAUNCH();
}

void launch_copy(double* dst, const double* src, long long n, const Ctrl* ctrl, int gate_reject, hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_copy, dim3(grid_for(n)), dim3(kBlock), 0, s, dst, src, n, ctrl, gate_reject);
    AA_CHECK_LAUNCH();
}

void launch_check_restore_ux(Ctrl* ctrl, const double* red, int nb, int accel, double* u, double* x, double* cur,
                             const double* du, const double* dx, long long nz, long long nx, hipStream_t s) {
    const int grid = accel ? grid_for(nz + nx) : 1;
    hipLaunchKernelGGL(k_check_restore_ux, dim3(grid), dim3(kBlock), 0, s, ctrl, red, nb, accel, u, x, cur, du, dx, nz, nx);
    AA_CHECK_LAUNCH();
}

void launch_check_restore_z(Ctrl* ctrl, const double* red, int nb, int accel, double* u, double* x, double* z,
                            const double* du, const double* dx, const double* dz, long long nz, long long nx,
                            hipStream_t s) {
    // 512 blocks: each sums the ~4k partials (L2 hits) before its share of the copy
    const int grid = accel ? 512 : 1;
    hipLaunchKernelGGL(k_check_restore_z, dim3(grid), dim3(kCtlBlock), 0, s, ctrl, red, nb, accel, u, x, z, du, dx, dz,
                       nz, nx);
    AA_CHECK_LAUNCH();
}

void launch_restore_ux(double* u, double* x, double* cur, const double* du, const double* dx, long long nz,
                       long long nx, const Ctrl* ctrl, hipStream_t s) {
    hipLaunchKernelGGL(k_restore_ux, dim3(grid_for(nz + nx)), dim3(kBlock), 0, s, u, x, cur, du, dx, nz, nx, ctrl);
    AA_CHECK_LAUNCH();
}

void launch_predict(int n, int nf, double* xstate, double* vstate, const double* mass, double dt, double gravity,
                    double* xbar, double* Mxbar, double* xfull, hipStream_t s) {
    (void)n;
    if (nf == 0) return;
    hipLaunchKernelGGL(k_predict, dim3(blocks_for(nf)), dim3(kBlock), 0, s, nf, xstate, vstate, mass, dt, gravity, xbar, Mxbar, xfull);
    AA_CHECK_LAUNCH();
}

void launch_finalize(int n, int nf, const double* xsrc, const double* xfull, double* xstate, double* vstate, double dt,
                     hipStream_t s) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_finalize, dim3(blocks_for(n)), dim3(kBlock), 0, s, n, nf, xsrc, xfull, xstate, vstate, dt);
    AA_CHECK_LAUNCH();
}

int aa_reduce_blocks(long long dim) {   // more partials only pay off on large vectors (k_aa_solve sums them)
    static const int cap_env = std::getenv("AA_AA_BLOCKS") ? std::atoi(std::getenv("AA_AA_BLOCKS")) : 0;
    const int cap = cap_env > 0 ? cap_env : (dim > (4LL << 20) ? 2048 : 512);
    return grid_for(dim) < cap ? grid_for(dim) : cap;
}

// m <= 12 (C3's m = 10) has its own bucket: k_aa_reduce<12> 125 VGPRs / k_aa_mix<12> 110 against
// 157 / 135 at 16 -- 4 waves per SIMD instead of 3 (AA_AA_MM12=0: the 16 bucket, for the A/B)
int aa_window_bucket(int m) {
    static const bool b12 = !(std::getenv("AA_AA_MM12") && std::getenv("AA_AA_MM12")[0] == '0');
    return m <= 8 ? 8 : (b12 && m <= 12 ? 12 : (m <= 16 ? 16 : 32));
}
static int mm_bucket(int m) { return aa_window_bucket(m); }

static bool aa_cols() {
    static const bool on = !(std::getenv("AA_AA_COLS") && std::getenv("AA_AA_COLS")[0] == '0');
    return on;
}

void launch_aa_reduce(Seg2 G, const double* cur, long long eff, double* dF, double* dG, Ctrl* ctrl, double* red,
                      int nblocks, Seg2 copy_to, int m, hipStream_t s, const double* comb_a, const double* comb_b,
                      int comb_nb, double* hist_prim, double* hist_comb, int* hist_rej, AAMask mask) {
#define AA_RED_ARGS G, cur, eff, dF, dG, ctrl, red, copy_to, comb_a, comb_b, comb_nb, hist_prim, hist_comb, hist_rej, mask
    switch (mm_bucket(m)) {
        case 8: hipLaunchKernelGGL(k_aa_reduce<8>, dim3(nblocks), dim3(kBlock), 0, s, AA_RED_ARGS); break;
        case 12: hipLaunchKernelGGL(k_aa_reduce<12>, dim3(nblocks), dim3(kBlock), 0, s, AA_RED_ARGS); break;
        case 16: hipLaunchKernelGGL(k_aa_reduce<16>, dim3(nblocks), dim3(kBlock), 0, s, AA_RED_ARGS); break;
        default:   // m > 16: column-parallel (AA_AA_COLS=0: the row-parallel kernel)
            if (aa_cols()) hipLaunchKernelGGL(k_aa_reduce_cols<32>, dim3(nblocks), dim3(kBlock), 0, s, AA_RED_ARGS);
            else hipLaunchKernelGGL(k_aa_reduce<32>, dim3(nblocks), dim3(kBlock), 0, s, AA_RED_ARGS);
            break;
    }
#undef AA_RED_ARGS
    AA_CHECK_LAUNCH();
}

void launch_aa_solve(Ctrl* ctrl, const double* red, int nblocks, int m, hipStream_t s) {
    switch (mm_bucket(m)) {
        case 8: hipLaunchKernelGGL(k_aa_solve<8>, dim3(1), dim3(kSolveBlock), 0, s, ctrl, red, nblocks); break;
        case 12: hipLaunchKernelGGL(k_aa_solve<12>, dim3(1), dim3(kSolveBlock), 0, s, ctrl, red, nblocks); break;
        case 16: hipLaunchKernelGGL(k_aa_solve<16>, dim3(1), dim3(kSolveBlock), 0, s, ctrl, red, nblocks); break;
        default: hipLaunchKernelGGL(k_aa_solve<32>, dim3(1), dim3(kSolveBlock), 0, s, ctrl, red, nblocks); break;
    }
    AA_CHECK_LAUNCH();
}

void launch_aa_mix(Seg2 G, double* cur, long long eff, double* dF, double* dG, Ctrl* ctrl, Seg2 out, int m,
                   hipStream_t s) {
    const long long dim = G.na + G.nb;
    switch (mm_bucket(m)) {
        case 8: hipLaunchKernelGGL(k_aa_mix<8>, dim3(grid_for(dim)), dim3(kBlock), 0, s, G, cur, eff, dF, dG, ctrl, out); break;
        case 12: hipLaunchKernelGGL(k_aa_mix<12>, dim3(grid_for(dim)), dim3(kBlock), 0, s, G, cur, eff, dF, dG, ctrl, out); break;
        case 16: hipLaunchKernelGGL(k_aa_mix<16>, dim3(grid_for(dim)), dim3(kBlock), 0, s, G, cur, eff, dF, dG, ctrl, out); break;
        default: hipLaunchKernelGGL(k_aa_mix<32>, dim3(grid_for(dim)), dim3(kBlock), 0, s, G, cur, eff, dF, dG, ctrl, out); break;
    }
    AA_CHECK_LAUNCH();
}

void launch_test_prox(int op, const double* prm4, const double* in, int n, double* out, int* iters, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_test_prox, dim3((n + 63) / 64), dim3(64), 0, s, op, prm4[0], prm4[1], prm4[2], prm4[3], in, n, out,
                       iters);
    AA_CHECK_LAUNCH();
}

void launch_test_cod(int n, const double* M, const double* b, double* x, hipStream_t s) {
    hipLaunchKernelGGL(k_test_cod, dim3(1), dim3(kSolveBlock), 0, s, n, M, b, x);
    AA_CHECK_LAUNCH();
}

void launch_wind(const int* tris3, const int* tri_ord, const int* lvl_ptr, int nlvl, const double* x, double* v,
                 double dir0, double dir1, double dir2, double dt, hipStream_t s) {
    if (nlvl <= 0) return;
    hipLaunchKernelGGL(k_wind, dim3(1), dim3(1024), 0, s, tris3, tri_ord, lvl_ptr, nlvl, x, v, dir0, dir1, dir2, dt);
    AA_CHECK_LAUNCH();
}

double bench_stream_read(long long bytes, int reps, hipStream_t s) {
    const long long n = bytes / 16;
    const int grid = 256 * 8;
    DevBuf<double2> a((size_t)n);
    DevBuf<double> out((size_t)grid * 256);
    AA_HIP(hipMemsetAsync(a.p, 0, (size_t)n * 16, s));
    hipEvent_t e0, e1;
    AA_HIP(hipEventCreate(&e0));
    AA_HIP(hipEventCreate(&e1));
    // three forms (grid-stride; contiguous chunk per workgroup, plain and non-temporal loads): the
    // ceiling reported is the fastest
    double best = 0;
    for (int form = 0; form < 3; ++form) {
        auto run = [&] {
            if (form == 0) hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, s, a.p, n, out.p);
            else if (form == 1) hipLaunchKernelGGL(k_stream_read_chunk<false>, dim3(grid), dim3(256), 0, s, a.p, n, out.p);
            else hipLaunchKernelGGL(k_stream_read_chunk<true>, dim3(grid), dim3(256), 0, s, a.p, n, out.p);
        };
        run();   // warm-up
        AA_HIP(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) run();
        AA_HIP(hipEventRecord(e1, s));
        AA_HIP(hipEventSynchronize(e1));
        float ms = 0;
        AA_HIP(hipEventElapsedTime(&ms, e0, e1));
        best = std::max(best, 16.0 * (double)n * reps / (ms * 1e-3) / 1e9);   // GB/s read
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return best;
}

}  // namespace aa
