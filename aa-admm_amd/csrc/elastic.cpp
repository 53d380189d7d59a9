// Host orchestration of the admm-elastic hot path (see elastic.hpp).
//
// Reference call stack being replaced:
//   Solver::initialize  admm_anderson_hard_zxu/src/Solver.cpp:361-491 (X: xzu/src/Solver.cpp:373-498)
//   Solver::step        admm_anderson_hard_zxu/src/Solver.cpp:34-234  (X: xzu/src/Solver.cpp:34-263)
// All per-iteration work is enqueued on one HIP stream; the data-dependent branches of the
// reference (Anderson reject, comb < 1e-20 break) are evaluated by device control kernels
// and gate the following kernels, so a time step needs exactly one host synchronisation.
#include "elastic.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <set>

#include "dense_gpu.hpp"
#include "spd_direct.hpp"

namespace aa {

ElasticSolver::~ElasticSolver() {
    drop_graph();
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    if (side_) (void)hipStreamDestroy(side_);
    for (auto& kv : kstats_)
        for (auto e : kv.second.ev) (void)hipEventDestroy(e);
}

void ElasticSolver::drop_graph() {
    if (gexec_) (void)hipGraphExecDestroy(gexec_);
    if (graph_) (void)hipGraphDestroy(graph_);
    gexec_ = nullptr;
    graph_ = nullptr;
}

int ElasticSolver::add_nodes(const double* x3, const double* m3, int n) {
    if (n < 0 || (n > 0 && (!x3 || !m3))) throw Error(ERR_ARG, "add_nodes: bad input");
    if (initialized_) throw Error(ERR_STATE, "add_nodes after initialize is not supported");
    x_.insert(x_.end(), x3, x3 + 3 * (size_t)n);
    v_.insert(v_.end(), 3 * (size_t)n, 0.0);
    m3_.insert(m3_.end(), m3, m3 + 3 * (size_t)n);
    return (int)(x_.size() / 3);
}

// TetEnergyTerm ctor + get_reduction (TetEnergyTerm.cpp:32-72), TriEnergyTerm ctor +
// get_reduction (TriEnergyTerm.cpp:30-72), EnergyTerm::get_reduction weight check (EnergyTerm.hpp:135-153)
void ElasticSolver::add_elements(int kind, int material, const double* verts3, const int* idx, int count,
                                 const aa_lame& lame, int vertex_offset) {
    if (count < 0 || (count > 0 && (!verts3 || !idx))) throw Error(ERR_ARG, "add_elements: bad input");
    if (initialized_) throw Error(ERR_STATE, "adding energy terms after initialize is not supported");
    if (kind == 1) {
        if (lame.limit_min > 1.0) throw Error(ERR_ARG, "**TriEnergyTerm Error: Strain limit min should be -inf to 1");
        if (lame.limit_max < 1.0) throw Error(ERR_ARG, "**TriEnergyTerm Error: Strain limit max should be 1 to inf");
        material = AA_LINEAR;
    } else if (material < 0 || material > 2) {
        throw Error(ERR_ARG, "add_tets: unknown material");
    }
    HostGroup g;
    g.kind = kind; g.material = material; g.lame = lame;
    g.nv = kind == 0 ? 4 : 3; g.ncol = g.nv - 1;
    const double k = lame.lambda + (2.0 / 3.0) * lame.mu;
    g.idx.resize((size_t)count * g.nv);
    g.G.resize((size_t)count * g.ncol * g.nv);
    g.vol.resize(count); g.w.resize(count);
    for (int t = 0; t < count; ++t) {
        const double* P[4];
        for (int a = 0; a < g.nv; ++a) {
            const int li = idx[(size_t)t * g.nv + a];
            if (li < 0) throw Error(ERR_ARG, "add_elements: negative index");
            P[a] = verts3 + 3 * (size_t)li;
            g.idx[(size_t)t * g.nv + a] = li + vertex_offset;
        }
        double* G = &g.G[(size_t)t * g.ncol * g.nv];
        double vol;
        if (kind == 0) {
            double B[9];
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) B[r * 3 + c] = P[c + 1][r] - P[0][r];
            double cof[9];
            cof[0] = B[4] * B[8] - B[5] * B[7]; cof[1] = B[5] * B[6] - B[3] * B[8]; cof[2] = B[3] * B[7] - B[4] * B[6];
            cof[3] = B[2] * B[7] - B[1] * B[8]; cof[4] = B[0] * B[8] - B[2] * B[6]; cof[5] = B[1] * B[6] - B[0] * B[7];
            cof[6] = B[1] * B[5] - B[2] * B[4]; cof[7] = B[2] * B[3] - B[0] * B[5]; cof[8] = B[0] * B[4] - B[1] * B[3];
            const double det = B[0] * cof[0] + B[1] * cof[1] + B[2] * cof[2];
            double Bi[9];
            for (int r = 0; r < 3; ++r) for (int c = 0; c < 3; ++c) Bi[r * 3 + c] = cof[c * 3 + r] / det;
            vol = det / 6.0;
            if (vol < 0) throw Error(ERR_NUMERIC, "**TetEnergyTerm Error: Inverted initial tet");
            for (int r = 0; r < 3; ++r) {
                G[r * 4 + 0] = -Bi[0 * 3 + r] - Bi[1 * 3 + r] - Bi[2 * 3 + r];
                for (int a = 1; a < 4; ++a) G[r * 4 + a] = Bi[(a - 1) * 3 + r];
            }
        } else {
            double e12[3], e13[3], n1[3], n2[3];
            for (int r = 0; r < 3; ++r) { e12[r] = P[1][r] - P[0][r]; e13[r] = P[2][r] - P[0][r]; }
            double l = std::sqrt(e12[0] * e12[0] + e12[1] * e12[1] + e12[2] * e12[2]);
            for (int r = 0; r < 3; ++r) n1[r] = e12[r] / l;
            const double d = e13[0] * n1[0] + e13[1] * n1[1] + e13[2] * n1[2];
            for (int r = 0; r < 3; ++r) n2[r] = e13[r] - d * n1[r];
            l = std::sqrt(n2[0] * n2[0] + n2[1] * n2[1] + n2[2] * n2[2]);
            for (int r = 0; r < 3; ++r) n2[r] /= l;
            auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
            const double b00 = dot(n1, e12), b01 = dot(n1, e13), b10 = dot(n2, e12), b11 = dot(n2, e13);
            const double det = b00 * b11 - b01 * b10;
            const double invdet = 1.0 / det;
            const double R[2][2] = {{b11 * invdet, -b01 * invdet}, {-b10 * invdet, b00 * invdet}};
            vol = 0.5 * det;
            if (vol < 0) throw Error(ERR_NUMERIC, "**TriEnergyTerm Error: Inverted initial pose");
            for (int c = 0; c < 2; ++c) {
                G[c * 3 + 0] = -R[0][c] - R[1][c];
                G[c * 3 + 1] = R[0][c];
                G[c * 3 + 2] = R[1][c];
            }
        }
        const double w = std::sqrt(k * vol);
        if (!(w > 0.0)) throw Error(ERR_NUMERIC, "**EnergyTerm::get_reduction Error: Some weight leq 0");
        g.vol[t] = vol;
        g.w[t] = w;
    }
    hgroups_.push_back(std::move(g));
}

// Solver::add_obstacle (admm_anderson_hard_zxu/src/Solver.cpp:346-348) with the passive objects of
// PassiveObject.hpp:32-136. The collision terms read the obstacle table every iteration, so
// obstacles may be added after initialize (as in the reference, whose prox walks the collider's
// list each time).
void ElasticSolver::add_obstacle(int type, const double* prm) {
    if (!prm) throw Error(ERR_ARG, "add_obstacle: null parameters");
    if (type < OBS_FLOOR || type > OBS_CYLINDER) throw Error(ERR_ARG, "add_obstacle: unknown obstacle type");
    if ((int)obstacles_.size() >= kMaxObstacles) throw Error(ERR_ARG, "add_obstacle: too many obstacles");
    std::array<double, kObsStride> o{};
    o[0] = type;
    const int np = type == OBS_FLOOR ? 1 : (type == OBS_SLIDE_FLOOR ? 6 : 4);
    for (int k = 0; k < np; ++k) o[1 + k] = prm[k];
    if (type == OBS_SLIDE_FLOOR) {   // SlideFloor ctor: normal.normalize() (Eigen: / sqrt(squaredNorm))
        const double z2 = (o[4] * o[4] + o[5] * o[5]) + o[6] * o[6];
        if (z2 > 0.0) { const double nr = std::sqrt(z2); o[4] /= nr; o[5] /= nr; o[6] /= nr; }
    }
    obstacles_.push_back(o);
    if (initialized_) upload_obstacles();
}

void ElasticSolver::upload_obstacles() {
    if (!obs_dev_.p) return;
    std::vector<double> h(1 + kObsStride * obstacles_.size());
    h[0] = (double)obstacles_.size();
    for (size_t k = 0; k < obstacles_.size(); ++k) std::copy(obstacles_[k].begin(), obstacles_[k].end(), h.begin() + 1 + kObsStride * k);
    AA_HIP(hipMemcpyAsync(obs_dev_.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s()));
    AA_HIP(hipStreamSynchronize(s()));
}

// Solver::set_collisions (admm_anderson_hard_zxu/src/Solver.cpp:318-344): one Collision term
// (CollisionEnergyTerm.hpp:41-117) per listed node, created at initialize after the other
// terms, in node order (the reference's std::map). Called after initialize it changes nothing
// (the reference only re-activates the terms it already made).
void ElasticSolver::set_collisions(const int* inds, int n) {
    if (n < 0 || (n > 0 && !inds)) throw Error(ERR_ARG, "**Solver::set_collisions Error: Bad input.");
    const int nodes = num_nodes();
    std::set<int> s;
    for (int i = 0; i < n; ++i) {
        if (inds[i] < 0 || inds[i] >= nodes) throw Error(ERR_ARG, "**Solver::set_collisions Error: Bad input.");
        s.insert(inds[i]);
    }
    if (initialized_) return;
    coll_nodes_.assign(s.begin(), s.end());
}

// WindForce (admm_anderson_hard_zxu/src/ExplicitForce.{hpp,cpp}) pushed to Solver::ext_forces:
// applied to v at the start of every step, before gravity (Solver.cpp:49-53)
int ElasticSolver::add_wind(const int* tris3, int ntris, const double* dir3) {
    if (ntris < 0 || (ntris > 0 && !tris3) || !dir3) throw Error(ERR_ARG, "add_wind: bad input");
    const int nodes = num_nodes();
    auto w = std::make_unique<Wind>();
    w->tris.assign(tris3, tris3 + 3 * (size_t)ntris);
    for (int i : w->tris) if (i < 0 || i >= nodes) throw Error(ERR_ARG, "add_wind: triangle references a node that does not exist");
    for (int c = 0; c < 3; ++c) w->dir[c] = dir3[c];
    if (initialized_) build_wind(*w);
    winds_.push_back(std::move(w));
    return (int)winds_.size() - 1;
}

void ElasticSolver::set_wind(int id, const double* dir3) {
    if (id < 0 || id >= (int)winds_.size() || !dir3) throw Error(ERR_ARG, "set_wind: bad wind id");
    for (int c = 0; c < 3; ++c) winds_[id]->dir[c] = dir3[c];
}

// level schedule of the triangles (internal node ids): level(t) = 1 + the highest level of an
// earlier triangle sharing one of its vertices
void ElasticSolver::build_wind(Wind& w) {
    const int nt = (int)(w.tris.size() / 3);
    std::vector<int> tri(3 * (size_t)nt), lvl(nt), last(num_nodes(), -1);
    int nl = 0;
    for (int t = 0; t < nt; ++t) {
        int l = 0;
        for (int j = 0; j < 3; ++j) {
            const int q = node2int_[w.tris[3 * (size_t)t + j]];
            tri[3 * (size_t)t + j] = q;
            l = std::max(l, last[q] + 1);
        }
        for (int j = 0; j < 3; ++j) last[tri[3 * (size_t)t + j]] = l;
        lvl[t] = l;
        nl = std::max(nl, l + 1);
    }
    std::vector<int> ptr(nl + 1, 0), ord(nt);
    for (int t = 0; t < nt; ++t) ++ptr[lvl[t] + 1];
    for (int l = 0; l < nl; ++l) ptr[l + 1] += ptr[l];
    std::vector<int> fill(ptr.begin(), ptr.end() - 1);
    for (int t = 0; t < nt; ++t) ord[fill[lvl[t]]++] = t;
    w.dtris.upload(tri, s());
    w.dord.upload(ord, s());
    w.dlvl.upload(ptr, s());
    w.nlvl = nl;
    AA_HIP(hipStreamSynchronize(s()));
}

// Solver::set_pins (admm_anderson_hard_zxu/src/Solver.cpp:280-315). Pins are kept in a map
// (like ConstraintSet::pins); each pinned node gets ITS OWN point. (The reference pairs the
// i-th given point with the i-th pin in sorted order -- identical whenever inds are sorted.)
void ElasticSolver::set_pins(const int* inds, const double* pts3, int n) {
    if (n < 0 || (n > 0 && !inds)) throw Error(ERR_ARG, "**Solver::set_pins Error: Bad input.");
    const bool in_place = pts3 == nullptr;
    const int nodes = num_nodes();
    if (nodes == 0 && in_place && n > 0) throw Error(ERR_ARG, "**Solver::set_pins Error: Bad input.");
    std::map<int, std::array<double, 3>> pins;
    for (int i = 0; i < n; ++i) {
        const int id = inds[i];
        if (id < 0 || id >= nodes) throw Error(ERR_ARG, "**Solver::set_pins Error: Bad input.");
        std::array<double, 3> p;
        for (int j = 0; j < 3; ++j) p[j] = in_place ? x_[3 * (size_t)id + j] : pts3[3 * i + j];
        pins[id] = p;
    }
    if (initialized_) {
        bool same = pins.size() == pins_.size();
        for (auto it = pins.begin(), jt = pins_.begin(); same && it != pins.end(); ++it, ++jt) same = it->first == jt->first;
        if (!same) throw Error(ERR_STATE, "set_pins: the pinned node set cannot change after initialize");
    }
    pins_ = std::move(pins);
    pins_dirty_ = true;
}

void ElasticSolver::initialize(const aa_settings& s_in) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::pair<const char*, double>> phases;   // AA_SETUP_TIMES=1: printed to stderr
    auto stamp = [&](const char* what) {
        phases.push_back({what, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count()});
    };
    drop_graph();
    if (const char* g = std::getenv("AA_ADMM_NO_GRAPH")) use_graph_ = !(g[0] == '1');
    if (comm_ && !comm_->capturable()) use_graph_ = false;
    st_ = s_in;
    if (st_.timestep_s <= 0.0) st_.timestep_s = 1.0 / 24.0;  // Solver.cpp:369-373
    const int n = num_nodes();
    if (!((int)m3_.size() == 3 * n && 3 * n >= 3)) throw Error(ERR_ARG, "**Solver Error: Problem with node data!");
    for (int i = 0; i < n; ++i)
        if (m3_[3 * i] != m3_[3 * i + 1] || m3_[3 * i] != m3_[3 * i + 2])
            throw Error(ERR_ARG, "initialize: per-node masses must be equal in x, y and z (A = A_s (x) I3)");
    const bool accel = st_.acceleration_type == 1;
    if (accel && (st_.anderson_m <= 0 || st_.anderson_m > kMaxM))
        throw Error(ERR_ARG, "initialize: Anderson window must be in [1, 32]");
    if (st_.variant != AA_VARIANT_Z && st_.variant != AA_VARIANT_UX) throw Error(ERR_ARG, "initialize: bad variant");
    if (st_.admm_iters < 0) throw Error(ERR_ARG, "initialize: admm_iters < 0");
    std::fill(v_.begin(), v_.end(), 0.0);
    if (st_.variant == AA_VARIANT_Z && !obstacles_.empty())   // admm_anderson_xzu/src/Solver.cpp:485-489
        throw Error(ERR_ARG, "**Solver::add_obstacle Error: No collisions with LDLT solver");
    if (st_.variant == AA_VARIANT_Z && !coll_nodes_.empty())
        throw Error(ERR_ARG, "set_collisions: energy-based collisions exist in the (u,x) variant only (admm_anderson_hard_zxu)");
    // collision terms (Solver.cpp:386-392): after the other terms, one per node in node order;
    // Lame::soft_rubber (EnergyTerm.hpp:38), weight sqrt(2 k), volume 2 (CollisionEnergyTerm.hpp:63-70)
    hgroups_.erase(std::remove_if(hgroups_.begin(), hgroups_.end(), [](const HostGroup& g) { return g.kind == 2; }),
                   hgroups_.end());
    if (!coll_nodes_.empty()) {
        HostGroup g;
        g.kind = 2; g.material = AA_LINEAR; g.nv = 1; g.ncol = 1;
        const double E = 10000000.0, nu = 0.399;
        g.lame = aa_lame{};
        g.lame.mu = E / (2.0 * (1.0 + nu));
        g.lame.lambda = E * nu / ((1.0 + nu) * (1.0 - 2.0 * nu));
        g.lame.limit_min = -100.0; g.lame.limit_max = 100.0;
        const double wt = std::sqrt((g.lame.lambda + (2.0 / 3.0) * g.lame.mu) * 2.0);
        g.idx = coll_nodes_;
        g.G.assign(coll_nodes_.size(), 1.0);
        g.vol.assign(coll_nodes_.size(), 2.0);
        g.w.assign(coll_nodes_.size(), wt);
        hgroups_.push_back(std::move(g));
    }

    n_ = n;
    np_ = (int)pins_.size();
    nf_ = n - np_;
    // ---- free / pinned split and nested-dissection order of the free nodes
    std::vector<int> free_nodes;
    std::vector<int> is_pin(n, 0);
    for (auto& kv : pins_) is_pin[kv.first] = 1;
    for (int i = 0; i < n; ++i) if (!is_pin[i]) free_nodes.push_back(i);
    std::vector<int> node2free(n, -1);
    for (int k = 0; k < nf_; ++k) node2free[free_nodes[k]] = k;
    std::vector<std::vector<int>> adjl(nf_);
    for (auto& g : hgroups_)
        for (size_t t = 0; t < g.idx.size() / g.nv; ++t)
            for (int a = 0; a < g.nv; ++a) {
                const int na = g.idx[t * g.nv + a];
                if (na < 0 || na >= n) throw Error(ERR_ARG, "energy term references a node that does not exist");
                const int fa = node2free[na];
                if (fa < 0) continue;
                for (int b = 0; b < g.nv; ++b) {
                    const int fb = node2free[g.idx[t * g.nv + b]];
                    if (fb >= 0 && fb != fa) adjl[fa].push_back(fb);
                }
            }
    std::vector<int> aptr(nf_ + 1, 0), aj;
    for (int k = 0; k < nf_; ++k) {
        auto& l = adjl[k];
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
        aptr[k + 1] = aptr[k] + (int)l.size();
        aj.insert(aj.end(), l.begin(), l.end());
    }
    std::vector<double> coords(3 * (size_t)nf_);
    for (int k = 0; k < nf_; ++k)
        for (int j = 0; j < 3; ++j) coords[3 * k + j] = x_[3 * (size_t)free_nodes[k] + j];
    // partitioned: the top bisections of the nested dissection (P parts, any P) are
    // forced; part r (a contiguous range of free nodes) belongs to rank r, the separators of
    // those bisections (the "top") are shared by all ranks
    const int P = comm_ ? comm_->size() : 1;
    // the shared top separators as one dense root split over the ranks (AA_TOP_DENSE=0: one
    // supernode per separator, replicated on every rank -- the round-1 layout)
    const bool top_dense = !(std::getenv("AA_TOP_DENSE") && std::getenv("AA_TOP_DENSE")[0] == '0');
    // ... and each part's own upper levels amalgamated into one dense supernode of up to this many
    // rows (AA_PART_TOP_ROWS)
    const int part_top_rows = std::getenv("AA_PART_TOP_ROWS") ? std::atoi(std::getenv("AA_PART_TOP_ROWS"))
                                                              : DirectSolver::kPartTopRows;
    const int nd_leaf = default_nd_leaf(nf_);
    stamp("adjacency");
    NdTree tree = nested_dissection(nf_, coords.data(), aptr, aj, nd_leaf, P > 1 ? 0 : DirectSolver::top_rows(nf_), P > 1 ? P : 0, top_dense,
                                     part_top_rows);
    stamp("nested dissection");
    node2int_.assign(n, -1);
    int2node_.assign(n, -1);
    for (int q = 0; q < nf_; ++q) { node2int_[free_nodes[tree.perm[q]]] = q; int2node_[q] = free_nodes[tree.perm[q]]; }
    {
        int q = nf_;
        for (auto& kv : pins_) { node2int_[kv.first] = q; int2node_[q] = kv.first; ++q; }
    }
    top_beg_ = P > 1 ? tree.top_beg : nf_;
    own_beg_ = P > 1 ? tree.part_beg[rank_] : 0;
    own_end_ = P > 1 ? tree.part_end[rank_] : nf_;
    if (P > 1) {   // every rank must have been handed the same scene
        double h[5] = {(double)n, (double)nf_, 0, 0, 0};
        for (auto& g : hgroups_) h[2] += (double)g.idx.size();
        for (size_t i = 0; i < x_.size(); ++i) { h[3] += x_[i]; h[4] += m3_[i]; }
        double r[5];
        std::copy(h, h + 5, r);
        comm_->allreduce_sum_host(r, 5);
        for (int i = 0; i < 5; ++i)
            if (std::fabs(r[i] - P * h[i]) > 1e-12 * std::fabs(P * h[i]))
                throw Error(ERR_ARG, "initialize: the ranks were given different scenes (nodes, elements or pins differ)");
    }
    // ---- global matrix A_s = M + pdt2 * sum_e w^2 G^T G  (Solver.cpp:466-467)
    const double dt2 = st_.timestep_s * st_.timestep_s;
    pdt2_ = (st_.variant == AA_VARIANT_UX ? st_.penalty : 1.0) * dt2;
    // rows in parallel: each free node sums its mass and its incident elements' w^2 G^T G
    // entries in (group, element) order -- a fixed order, independent of the thread count
    struct Inc { int g, t, a; };
    std::vector<int> iptr(nf_ + 1, 0);
    for (auto& g : hgroups_)
        for (size_t t = 0; t < g.idx.size() / g.nv; ++t)
            for (int a = 0; a < g.nv; ++a) {
                const int qa = node2int_[g.idx[t * g.nv + a]];
                if (qa < nf_) ++iptr[qa + 1];
            }
    for (int q = 0; q < nf_; ++q) iptr[q + 1] += iptr[q];
    std::vector<Inc> inc(iptr[nf_]);
    {
        std::vector<int> fill(iptr.begin(), iptr.end() - 1);
        for (int gi = 0; gi < (int)hgroups_.size(); ++gi) {
            const auto& g = hgroups_[gi];
            for (size_t t = 0; t < g.idx.size() / g.nv; ++t)
                for (int a = 0; a < g.nv; ++a) {
                    const int qa = node2int_[g.idx[t * g.nv + a]];
                    if (qa < nf_) inc[fill[qa]++] = Inc{gi, (int)t, a};
                }
        }
    }
    std::vector<std::vector<std::pair<int, double>>> rows(nf_);
#pragma omp parallel for schedule(dynamic, 256)
    for (int q = 0; q < nf_; ++q) {
        std::vector<std::pair<int, double>> r;
        r.reserve(1 + 4 * (size_t)(iptr[q + 1] - iptr[q]));
        r.push_back({q, m3_[3 * (size_t)int2node_[q]]});
        for (int k = iptr[q]; k < iptr[q + 1]; ++k) {
            const auto& g = hgroups_[inc[k].g];
            const size_t t = inc[k].t;
            const int a = inc[k].a;
            const double w2 = g.w[t] * g.w[t];
            const double* G = &g.G[t * g.ncol * g.nv];
            for (int b = 0; b < g.nv; ++b) {
                const int qb = node2int_[g.idx[t * g.nv + b]];
                if (qb >= nf_) continue;
                double sacc = 0;
                for (int c = 0; c < g.ncol; ++c) sacc += G[c * g.nv + a] * G[c * g.nv + b];
                r.push_back({qb, pdt2_ * w2 * sacc});
            }
        }
        std::stable_sort(r.begin(), r.end(), [](const std::pair<int, double>& x, const std::pair<int, double>& y) { return x.first < y.first; });
        std::vector<std::pair<int, double>> out;
        for (size_t k = 0; k < r.size();) {
            size_t k2 = k;
            double v = 0;
            while (k2 < r.size() && r[k2].first == r[k].first) v += r[k2++].second;
            out.push_back({r[k].first, v});
            k = k2;
        }
        rows[q] = std::move(out);
    }
    CsrMatrix A;
    A.n = nf_;
    A.ptr.assign(nf_ + 1, 0);
    for (int q = 0; q < nf_; ++q) A.ptr[q + 1] = A.ptr[q] + (int)rows[q].size();
    A.col.resize(A.ptr[nf_]);
    A.val.resize(A.ptr[nf_]);
#pragma omp parallel for schedule(static)
    for (int q = 0; q < nf_; ++q)
        for (size_t k = 0; k < rows[q].size(); ++k) { A.col[A.ptr[q] + k] = rows[q][k].first; A.val[A.ptr[q] + k] = rows[q][k].second; }
    std::vector<std::vector<std::pair<int, double>>>().swap(rows);
    stamp("assembly of A_s");
    SupernodalFactor F;
    try {
        auto pf = make_part_factor(P > 1 ? comm_ : nullptr, rank_, s());   // no rank factors another's part
        F = factor_on_device(A, tree, s(), pf.get());
    } catch (const Error&) {
        throw;   // device / allocation failures keep their own status
    } catch (const std::runtime_error& e) {
        throw Error(ERR_NUMERIC, e.what());   // not positive definite / singular block
    }
    // Z variant with Anderson: the combined-residual solve is batched with the next iteration's
    // solve (enqueue_iteration_z); AA_Z_PIPELINE=0 restores the sequential order
    pipe_z_ = st_.variant == AA_VARIANT_Z && st_.acceleration_type == 1;
    if (const char* e = std::getenv("AA_Z_PIPELINE")) pipe_z_ = pipe_z_ && e[0] != '0';
    // the pipelined pass on a second stream (one GPU: a partitioned pass would put collectives
    // on two streams); AA_CONCURRENT=0 keeps it in line
    conc_ = pipe_z_ && !comm_;
    if (const char* e = std::getenv("AA_CONCURRENT")) conc_ = conc_ && e[0] != '0';
    conc_fork_ = std::getenv("AA_CONC_FORK") ? std::atoi(std::getenv("AA_CONC_FORK")) : 1;
    // Z variant + Anderson: the two-set layout whether pipelined or not (same sums, same bits)
    stamp("factor");
    // the sweeps as two parallel branches (DirectSolver::plan_branches): measured on C4 (one GPU,
    // Z variant) 407-408 -> 412-416 it/s; three or four branches, and the geometry configs, slower
    // 
    solver_.default_branches = (P == 1 && st_.variant == AA_VARIANT_Z) ? 2 : 1;
    solver_.build(F, s(), P > 1 ? &tree.part : nullptr, rank_, top_beg_, comm_, pipe_z_ ? 2 : 1,
                  st_.variant == AA_VARIANT_Z && st_.acceleration_type == 1);
    stamp("solver build + upload");

    // ---- element ownership (partitioned): an element touching a node of part r belongs to
    // rank r (it cannot touch another part: the separators split the mesh); elements whose free
    // nodes are all separator nodes go round-robin. Every rank computes the same assignment.
    std::vector<HostGroup> owned;
    nbg_ = 0;
    long long zmax = 0;
    if (P > 1) {
        std::vector<int> qpart(n, -1);
        for (int r = 0; r < P; ++r) for (int q = tree.part_beg[r]; q < tree.part_end[r]; ++q) qpart[q] = r;
        std::vector<long long> zr(P, 0);
        std::vector<int> br(P, 0);
        long long rr = 0;
        for (auto& hg : hgroups_) {
            const int cnt = (int)(hg.idx.size() / hg.nv);
            std::vector<int> c(P, 0);
            HostGroup lg;
            lg.kind = hg.kind; lg.material = hg.material; lg.nv = hg.nv; lg.ncol = hg.ncol; lg.lame = hg.lame;
            for (int t = 0; t < cnt; ++t) {
                int o = -1;
                for (int a = 0; a < hg.nv && o < 0; ++a) o = qpart[node2int_[hg.idx[(size_t)t * hg.nv + a]]];
                if (o < 0) o = (int)(rr++ % P);
                ++c[o];
                if (o != rank_) continue;
                lg.idx.insert(lg.idx.end(), hg.idx.begin() + (size_t)t * hg.nv, hg.idx.begin() + (size_t)(t + 1) * hg.nv);
                lg.G.insert(lg.G.end(), hg.G.begin() + (size_t)t * hg.ncol * hg.nv, hg.G.begin() + (size_t)(t + 1) * hg.ncol * hg.nv);
                lg.vol.push_back(hg.vol[t]);
                lg.w.push_back(hg.w[t]);
            }
            for (int r = 0; r < P; ++r) { br[r] += blocks_for(c[r]); zr[r] += 3LL * hg.ncol * c[r]; }
            owned.push_back(std::move(lg));
        }
        for (int r = 0; r < P; ++r) { nbg_ = std::max(nbg_, br[r]); zmax = std::max(zmax, zr[r]); }
    }
    const std::vector<HostGroup>& dgroups = P > 1 ? owned : hgroups_;
    // ---- device element groups (internal node ids), z/u offsets, D^T gather rows
    groups_.clear();
    groups_.resize(dgroups.size());
    long long zoff = 0, yrow = 0;
    red_blocks_ = 0;
    std::vector<std::vector<long long>> dtr(nf_);   // per free node: its vertex slots
    for (size_t gi = 0; gi < dgroups.size(); ++gi) {
        auto& hg = dgroups[gi];
        auto& dg = groups_[gi];
        const int cnt = (int)(hg.idx.size() / hg.nv);
        std::vector<int> idx((size_t)hg.nv * cnt);
        std::vector<double> G((size_t)hg.ncol * hg.nv * cnt);
        for (int t = 0; t < cnt; ++t) {
            for (int a = 0; a < hg.nv; ++a) idx[(size_t)a * cnt + t] = node2int_[hg.idx[(size_t)t * hg.nv + a]];
            for (int c = 0; c < hg.ncol; ++c)
                for (int a = 0; a < hg.nv; ++a)
                    G[(size_t)(c * hg.nv + a) * cnt + t] = hg.G[((size_t)t * hg.ncol + c) * hg.nv + a];
            for (int a = 0; a < hg.nv; ++a) {
                const int q = node2int_[hg.idx[(size_t)t * hg.nv + a]];
                if (q >= nf_) continue;
                dtr[q].push_back(yrow + (long long)t * hg.nv + a);
            }
        }
        dg.idx.upload(idx, s());
        dg.G.upload(G, s());
        dg.w.upload(hg.w, s());
        dg.vol.upload(hg.vol, s());
        GroupDev& d = dg.d;
        d.kind = hg.kind; d.mat = hg.material; d.count = cnt; d.nv = hg.nv; d.ncol = hg.ncol; d.dim = 3 * hg.ncol;
        d.pinned = std::any_of(idx.begin(), idx.end(), [&](int q) { return q >= nf_; }) ? 1 : 0;
        d.zoff = zoff; d.yrow = yrow;
        d.idx = dg.idx.p; d.G = dg.G.p; d.w = dg.w.p; d.vol = dg.vol.p;
        d.mu = hg.lame.mu; d.lambda = hg.lame.lambda; d.k = hg.lame.lambda + (2.0 / 3.0) * hg.lame.mu;
        d.lmin = hg.lame.limit_min; d.lmax = hg.lame.limit_max;
        if (hg.kind == 2) {   // the obstacle table the collision prox reads (fixed address: graph-safe)
            if (!obs_dev_.p) obs_dev_.alloc(1 + (size_t)kObsStride * kMaxObstacles);
            d.obs = obs_dev_.p;
        } else {
            d.obs = nullptr;
        }
        zoff += (long long)d.dim * cnt;
        yrow += (long long)d.nv * cnt;
        red_blocks_ += blocks_for(cnt);
    }
    Z_ = zoff;
    if (P == 1) { nbg_ = red_blocks_; zmax = Z_; }
    {
        // vertex slots in node order: the element kernels scatter each vertex contribution to its
        // node's run (spos), the rhs kernel streams every node's run contiguously
        std::vector<int> ptr(nf_ + 1, 0);
        std::vector<std::vector<int>> spos(groups_.size());
        std::vector<long long> gfirst(groups_.size());
        for (size_t gi = 0; gi < groups_.size(); ++gi) {
            spos[gi].assign((size_t)groups_[gi].d.nv * groups_[gi].d.count, -1);
            gfirst[gi] = groups_[gi].d.yrow;
        }
        long long pos = 0;
        for (int q = 0; q < nf_; ++q) {
            auto& r = dtr[q];
            std::sort(r.begin(), r.end());
            for (long long key : r) {   // key = group's first slot + t * nv + a
                const size_t gi = (size_t)(std::upper_bound(gfirst.begin(), gfirst.end(), key) - gfirst.begin()) - 1;
                const long long local = key - gfirst[gi];
                const int nv = groups_[gi].d.nv, cnt = groups_[gi].d.count;
                spos[gi][(size_t)(local % nv) * cnt + (size_t)(local / nv)] = (int)pos++;
            }
            if (pos > 0x7fffffffLL) throw Error(ERR_ARG, "initialize: too many element vertices");
            ptr[q + 1] = (int)pos;
            std::vector<long long>().swap(r);
        }
        dt_ptr_.upload(ptr, s());
        for (size_t gi = 0; gi < groups_.size(); ++gi) {
            groups_[gi].spos.upload(spos[gi], s());
            groups_[gi].d.spos = groups_[gi].spos.p;
        }
        Yslots_ = pos;
    }
    // ---- state and work buffers
    std::vector<double> xs(3 * (size_t)n), ms(n);
    for (int q = 0; q < n; ++q) {
        for (int j = 0; j < 3; ++j) xs[3 * (size_t)q + j] = x_[3 * (size_t)int2node_[q] + j];
        ms[q] = m3_[3 * (size_t)int2node_[q]];
    }
    xs_.upload(xs, s());
    vs_.alloc(3 * (size_t)n); vs_.zero(s());
    mass_.upload(ms, s());
    xfull_.alloc(3 * (size_t)n); xlast_.alloc(3 * (size_t)n); cxfull_.alloc(3 * (size_t)n);
    xfull_.zero(s()); xlast_.zero(s()); cxfull_.zero(s());
    xbar_.alloc(3 * (size_t)nf_); Mxbar_.alloc(3 * (size_t)nf_); b_.alloc(3 * (size_t)nf_);
    if (pipe_z_) b2_.alloc(3 * (size_t)nf_); dx_.alloc(3 * (size_t)nf_);
    z_.alloc(Z_); u_.alloc(Z_); y_.alloc(3 * std::max<long long>(1, Yslots_)); du_.alloc(Z_);
    if (st_.variant == AA_VARIANT_Z) { dz_.alloc(Z_); lastz_.alloc(Z_); cz_.alloc(Z_); }
    if (conc_) {
        du2_.alloc(Z_); dz2_.alloc(Z_); dx2_.alloc(3 * (size_t)nf_);
        ctrl_c_.alloc(1);
        lzq2_.alloc(2);   // claim counter, finished blocks (queue_reset_last)
        AA_HIP(hipMemset(lzq2_.p, 0, 2 * sizeof(int)));
        if (!side_) AA_HIP(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
        if (!ev_fork_) AA_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
        if (!ev_join_) AA_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    }
    // residual block partials [a | b], padded to the largest rank's block count (zeros beyond
    // this rank's blocks), and their all-rank sums (the same buffer on one GPU)
    nbg_ = std::max(1, nbg_);
    red_ab_.alloc(2 * (size_t)nbg_); red_ab_.zero(s());
    if (conc_) { red_c_.alloc(2 * (size_t)nbg_); red_c_.zero(s()); }
    pa_ = red_ab_.p; pb_ = red_ab_.p + nbg_;
    if (comm_) { red_gab_.alloc(2 * (size_t)nbg_); red_gab_.zero(s()); ga_ = red_gab_.p; gb_ = red_gab_.p + nbg_; }
    else { ga_ = pa_; gb_ = pb_; }
    ctrl_.alloc(1);
    lzq_.alloc(2);   // claim counter, finished blocks (queue_reset_last)
    AA_HIP(hipMemset(lzq_.p, 0, 2 * sizeof(int)));
    if (const char* q = std::getenv("AA_LOCAL_QUEUE")) use_queue_ = q[0] != '0';
    lq_ = make_local_queue(ctx_->device, lzq_.p);
    if (conc_) {
        lq2_ = make_local_queue(ctx_->device, lzq2_.p);
        // the concurrent pass writes no rhs slots, so it runs the fused refill without their loads
        // (k_local_z_hqf<4, false>: 412 registers, room beside it for the Anderson kernels; the
        // slot-writing form's 452 leave none -- C4 with that on both passes: the main step 25 us
        // faster, the iteration 100 us slower). Same box, 8 steps: 457.7 / 459.8 -> 459.2 / 464.8
        // it/s. AA_LQ_FUSED_CONC=0: the plain refill here
        const char* fc = std::getenv("AA_LQ_FUSED_CONC");
        lq2_.fused = lq2_.fused && (fc ? fc[0] == '1' : true);
    }
    if (const char* q = std::getenv("AA_LQ_STATS"); q && q[0] == '1') {
        lq_stats_.alloc(kLqStats);
        lq_stats_.zero(s());
        lq_.stats = lq_stats_.p;
    }
    if (conc_) lq2_.stats = lq_.stats;
    hist_cap_ = std::max(1, st_.admm_iters);
    hist_prim_.alloc(hist_cap_); hist_comb_.alloc(hist_cap_); hist_rej_.alloc(hist_cap_);
    hist_clock_.alloc(hist_cap_ + 1);
    {
        int khz = 0;
        AA_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx_->device));
        if (khz > 0) clock_khz_ = khz;
    }
    if (!(st_.eps_rel >= 0.0)) throw Error(ERR_ARG, "initialize: eps_rel must be >= 0");
    if (accel) {
        const int m = st_.anderson_m;
        const long long dim = st_.variant == AA_VARIANT_UX ? Z_ + 3LL * nf_ : Z_;
        // the Z variant mixes z in place: the accelerator's current iterate is z itself (z == the
        // last Anderson output or, after a reject, default_z -- accelerator.replace)
        if (st_.variant == AA_VARIANT_UX) aa_cur_.alloc(dim);
        aa_dF_.alloc((size_t)m * Z_); aa_dF_.zero(s());
        aa_dG_.alloc((size_t)m * dim); aa_dG_.zero(s());
        // same grid on every rank (the largest rank's) so the partial layouts line up
        aa_blocks_ = aa_reduce_blocks(st_.variant == AA_VARIANT_UX ? zmax + 3LL * nf_ : zmax);
        (void)dim;
        const int mm = aa_window_bucket(m);
        aa_red_.alloc((size_t)aa_blocks_ * (2 + 2 * mm)); aa_red_.zero(s());
        if (comm_) { aa_red_g_.alloc(aa_red_.n); aa_red_g_.zero(s()); aag_ = aa_red_g_.p; }
        else aag_ = aa_red_.p;
    }
    AA_HIP(hipStreamSynchronize(s()));
    initialized_ = true;
    upload_obstacles();
    for (auto& w : winds_) build_wind(*w);
    pins_dirty_ = true;
    rt_ = aa_runtime{};
    rt_.nnz_factor = (long long)F.nnz_L;
    rt_.n_free = nf_; rt_.n_pinned = np_;
    rt_.n_elements = 0;
    for (auto& g : groups_) rt_.n_elements += g.d.count;
    rt_.z_dim = (int)Z_;
    rt_.setup_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stamp("elements + buffers");
    setup_phases_.clear();
    {
        double prev = 0;
        for (auto& ph : phases) { setup_phases_.push_back({ph.first, ph.second - prev}); prev = ph.second; }
    }
    if (const char* e = std::getenv("AA_SETUP_TIMES"); e && e[0] == '1')
        for (auto& ph : setup_phases_) std::fprintf(stderr, "[setup] %-24s %8.1f ms\n", ph.first.c_str(), ph.second);
    // algorithmic bytes per launch class (DESIGN.md "roofline accounting")
    kstats_.clear();
    double lz = 0, rs = 0;
    for (auto& g : groups_) {
        const double per = 4.0 * g.d.nv + 8.0 * g.d.ncol * g.d.nv + 8.0;
        lz += g.d.count * (per + 2 * 8.0 * g.d.dim + 28.0 * g.d.nv);   // u in, z out, slot positions + slots out
        rs += g.d.count * (per + 3 * 8.0 * g.d.dim);
    }
    kstats_["local_z"].bytes = lz + 24.0 * n;
    kstats_["resid"].bytes = rs + 48.0 * n;
    kstats_["solve"].bytes = pipe_z_ ? solver_.bytes_per_solve2() : solver_.bytes_per_solve();
    kstats_["solve1"].bytes = solver_.bytes_per_solve();
    kstats_["rhs"].bytes = 24.0 * (double)Yslots_ + 4.0 * nf_ + 48.0 * nf_;   // 3 doubles per slot; ptr, Mxbar, b
    // Z variant: u = W^-1 grad E(z) and the vertex slots (reads idx, G, w, z; writes u, slots),
    // prim (reads idx, G, w, z, u; writes block partials)
    double gy = 0, pr = 0;
    for (auto& g : groups_) {
        const double per = 4.0 * g.d.nv + 8.0 * g.d.ncol * g.d.nv + 8.0;
        gy += g.d.count * (per + 8.0 * 2 * g.d.dim + 28.0 * g.d.nv);
        pr += g.d.count * (per + 8.0 * 2 * g.d.dim);
    }
    kstats_["grad"].bytes = gy + 24.0 * n;
    kstats_["prim"].bytes = pr + 24.0 * n;
    if (accel) {   // Anderson: ~ 8 d (2m + 8) bytes per iteration (history read/write + vectors)
        const double d = st_.variant == AA_VARIANT_UX ? (double)Z_ + 3.0 * nf_ : (double)Z_;
        kstats_["aa"].bytes = 8.0 * d * (2.0 * st_.anderson_m + 8.0);
    }
}

void ElasticSolver::set_comm(Comm* c) {
    if (initialized_) throw Error(ERR_STATE, "set_comm after initialize is not supported");
    comm_ = c;   // size 1 runs the reductions through the transport too (plumbing checks)
    rank_ = comm_ ? comm_->rank() : 0;
}

// all-rank sums of the residual block partials (no-op on one GPU: ga_/gb_ alias pa_/pb_)
void ElasticSolver::reduce_partials() {
    if (comm_) comm_->allreduce_sum(red_ab_.p, red_gab_.p, 2 * (size_t)nbg_, s());
}

void ElasticSolver::reduce_aa() {
    if (comm_) comm_->allreduce_sum(aa_red_.p, aa_red_g_.p, aa_red_.n, s());
}

// Partitioned: after a step each rank holds valid positions/velocities for its own part, the
// shared top and the pins. Zero everything else (the top and pins on ranks > 0) and sum over
// the ranks, so every rank ends the step with the full state (Solver::m_x / m_v).
void ElasticSolver::gather_state(DevBuf<double>& v) {
    if (!comm_) return;
    auto zero = [&](int q0, int q1) {
        if (q1 > q0) AA_HIP(hipMemsetAsync(v.p + 3 * (size_t)q0, 0, 3 * sizeof(double) * (size_t)(q1 - q0), s()));
    };
    zero(0, own_beg_);
    zero(own_end_, top_beg_);
    if (rank_ != 0) zero(top_beg_, n_);
    comm_->allreduce_sum(v.p, v.p, 3 * (size_t)n_, s());
}

void ElasticSolver::upload_pins() {
    if (!pins_dirty_) return;
    std::vector<double> p(3 * (size_t)np_);
    int q = 0;
    for (auto& kv : pins_) { for (int j = 0; j < 3; ++j) p[3 * q + j] = kv.second[j]; ++q; }
    if (np_) {
        const size_t off = 3 * (size_t)nf_;
        AA_HIP(hipMemcpyAsync(xfull_.p + off, p.data(), p.size() * 8, hipMemcpyHostToDevice, s()));
        AA_HIP(hipMemcpyAsync(xlast_.p + off, p.data(), p.size() * 8, hipMemcpyHostToDevice, s()));
        AA_HIP(hipMemcpyAsync(cxfull_.p + off, p.data(), p.size() * 8, hipMemcpyHostToDevice, s()));
        AA_HIP(hipStreamSynchronize(s()));
    }
    pins_dirty_ = false;
}

void ElasticSolver::ev_begin(const char* name) {
    if (!instrument_) return;
    hipEvent_t e;
    AA_HIP(hipEventCreate(&e));
    AA_HIP(hipEventRecord(e, s()));
    kstats_[name].ev.push_back(e);
}
void ElasticSolver::ev_end(const char* name) { ev_begin(name); }

void ElasticSolver::local_z_all(const double* xfull, const double* u, double* z, double* y, int mode, bool red) {
    int off = 0;
    const bool timed = mode == LZ_NORMAL && red;
    if (timed) ev_begin("local_z");
    for (auto& g : groups_) {
        launch_local_z(g.d, xfull, u, z, y, nf_, st_.variant, mode, ctrl_.p, red ? pa_ : nullptr, off, s(),
                       use_queue_ ? &lq_ : nullptr);
        off += blocks_for(g.d.count);
    }
    if (timed) ev_end("local_z");
}

// the element prox of every group on stream st with control block c (no partials, no slots)
void ElasticSolver::local_z_on(const double* xfull, const double* u, double* z, int mode, hipStream_t st, Ctrl* c,
                               const LocalQueue* q) {
    for (auto& g : groups_)
        launch_local_z(g.d, xfull, u, z, nullptr, nf_, st_.variant, mode, c, nullptr, 0, st, use_queue_ ? q : nullptr);
}

void ElasticSolver::prologue() {
    upload_pins();
    const bool accel = st_.acceleration_type == 1;
    Ctrl c;
    std::memset(&c, 0, sizeof(c));
    c.prev_prim = 1e20;
    c.cap = hist_cap_;
    c.aa_m = accel ? st_.anderson_m : 0;
    c.aa_active = accel ? 1 : 0;
    c.hist_clock = hist_clock_.p;
    c.eps_rel = st_.eps_rel;
    AA_HIP(hipMemcpyAsync(ctrl_.p, &c, sizeof(Ctrl), hipMemcpyHostToDevice, s()));
    launch_stamp(ctrl_.p, s());
    for (auto& w : winds_)   // explicit forces before gravity (Solver.cpp:49-53), on the step's start state
        launch_wind(w->dtris.p, w->dord.p, w->dlvl.p, w->nlvl, xs_.p, vs_.p, w->dir[0], w->dir[1], w->dir[2],
                    st_.timestep_s, s());
    launch_predict(n_, nf_, xs_.p, vs_.p, mass_.p, st_.timestep_s, st_.gravity, xbar_.p, Mxbar_.p, xfull_.p, s());
    // partitioned: the mass term of a shared separator row enters the right-hand side once
    // (rank 0); the other ranks contribute only their elements' D^T rows to it
    if (comm_ && rank_ != 0 && top_beg_ < nf_)
        AA_HIP(hipMemsetAsync(Mxbar_.p + 3 * (size_t)top_beg_, 0, 3 * sizeof(double) * (size_t)(nf_ - top_beg_), s()));
    for (auto& g : groups_) launch_init_z(g.d, xfull_.p, z_.p, s());
    u_.zero(s());
    const long long nx = 3LL * nf_;
    if (st_.variant == AA_VARIANT_UX) {
        local_z_all(xfull_.p, u_.p, z_.p, y_.p, LZ_INIT, false);
        launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, nullptr, 0, s());
        solver_.solve(b_.p, xfull_.p, nullptr, 0, s());
        {
            int off = 0;
            for (auto& g : groups_) {
                launch_resid_update_u(g.d, xfull_.p, xlast_.p, z_.p, u_.p, nf_, ctrl_.p, pa_, pb_, off, s());
                off += blocks_for(g.d.count);
            }
        }
        launch_copy(du_.p, u_.p, Z_, nullptr, 0, s());
        launch_copy(dx_.p, xfull_.p, nx, nullptr, 0, s());
        if (accel) {
            launch_copy(aa_cur_.p, u_.p, Z_, nullptr, 0, s());
            launch_copy(aa_cur_.p + Z_, xfull_.p, nx, nullptr, 0, s());
        }
    } else {
        for (auto& g : groups_) launch_u_and_y(g.d, xfull_.p, z_.p, u_.p, y_.p, nf_, 2, 0, ctrl_.p, s());
        launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, nullptr, 0, s());
        solver_.solve(b_.p, xfull_.p, nullptr, 0, s());
        local_z_all(xfull_.p, u_.p, z_.p, nullptr, LZ_INIT, false);
        // default_{z,x,u} of "iteration -1" (the parity buffers of the concurrent pass)
        launch_copy(dz_at(-1), z_.p, Z_, nullptr, 0, s());
        launch_copy(dx_at(-1), xfull_.p, nx, nullptr, 0, s());
        launch_copy(du_at(-1), u_.p, Z_, nullptr, 0, s());
        // (Z variant: the accelerator's current iterate is z_ itself)
    }
}

// admm_anderson_hard_zxu/src/Solver.cpp:130-214
void ElasticSolver::enqueue_iteration_ux(bool accel) {
    const long long nx = 3LL * nf_;
    Ctrl* c = ctrl_.p;
    local_z_all(xfull_.p, u_.p, z_.p, y_.p, LZ_NORMAL, true);
    reduce_partials();
    launch_check_restore_ux(c, ga_, nbg_, accel, u_.p, xfull_.p, accel ? aa_cur_.p : nullptr, du_.p, dx_.p,
                            Z_, nx, s());
    if (accel) {
        local_z_all(xfull_.p, u_.p, z_.p, y_.p, LZ_REDO, true);
        reduce_partials();
    }
    ev_begin("rhs");
    launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, c, 0, s(), xfull_.p, xlast_.p,
               ga_, nbg_);
    ev_end("rhs");
    ev_begin("solve");
    solver_.solve(b_.p, xfull_.p, c, 0, s());
    ev_end("solve");
    ev_begin("resid");
    {
        int off = 0;
        for (auto& g : groups_) {
            launch_resid_update_u(g.d, xfull_.p, xlast_.p, z_.p, u_.p, nf_, c, pa_, pb_, off, s());
            off += blocks_for(g.d.count);
        }
    }
    ev_end("resid");
    reduce_partials();
    if (accel) {
        const int m = st_.anderson_m;
        Seg2 G{u_.p, Z_, xfull_.p, nx};
        Seg2 cp{du_.p, Z_, dx_.p, nx};
        ev_begin("aa");
        launch_aa_reduce(G, aa_cur_.p, Z_, aa_dF_.p, aa_dG_.p, c, aa_red_.p, aa_blocks_, cp, m, s(), ga_, gb_, nbg_,
                         hist_prim_.p, hist_comb_.p, hist_rej_.p);
        reduce_aa();
        launch_aa_solve(c, aag_, aa_blocks_, m, s());
        launch_aa_mix(G, aa_cur_.p, Z_, aa_dF_.p, aa_dG_.p, c, G, m, s());
        ev_end("aa");
    } else {
        launch_control(CTL_COMB_UX, c, ga_, gb_, nbg_, accel, hist_prim_.p, hist_comb_.p, hist_rej_.p, s());
    }
}

// admm_anderson_xzu/src/Solver.cpp:122-251
//
// Pipelined combined residual (pipe_z_): the "for drawing figures" pass of iteration k
// (Solver.cpp:217-233: x_c = A^-1 b(default_z_k, u_k), z_c = update_z(x_c), comb_k) needs a
// solve that does not depend on iteration k+1, and iteration k+1's main solve does not depend
// on it -- so the two run as one two-set solve (DirectSolver::solve2, the factor streamed once).
// comb_k's update_z / residual / break test follow that solve, before iteration k+1 records or
// changes anything the test depends on: its inputs are default_z (dz_), default_u (du_, equal
// to curr_u_k: the Anderson step leaves u alone) and x_c, none of which iteration k+1 writes
// before that point. A break at comb_k (done = 2) rolls back the one speculative write that
// survives the step, x (restored from default_x = curr_x_k); everything after is gated off.
// The last iteration's pass runs alone (enqueue_comb_tail_z). Results are bit-identical to
// the unpipelined order (same kernels, same operands; the batched solve sums each column in
// the same order).
void ElasticSolver::enqueue_iteration_z(bool accel, int it) {
    const long long nx = 3LL * nf_;
    Ctrl* c = ctrl_.p;
    const bool pipe = accel && pipe_z_;
    // default_{u,z,x}: this iteration's (written below) and the previous one's (read by the
    // reject restore, the previous iteration's combined-residual pass and its rollback)
    double *duc = du_at(it), *dzc = dz_at(it), *dxc = dx_at(it);
    double *dup = du_at(it - 1), *dzp = dz_at(it - 1), *dxp = dx_at(it - 1);
    // concurrent pass (conc_): iteration k-1's combined residual on its own control block, forked
    // and joined (the rollback of a break then happens once, at the join); on side_ beside this
    // iteration's Anderson step -- in line on the solver's stream in the instrumented
    // (per-kernel-class timing) pass
    const bool side = pipe && it > 0 && conc_;
    hipStream_t sst = instrument_ ? s() : side_;
    // k-1's pass beside this iteration's work: its local step (one wave per SIMD) leaves room for
    // memory-bound waves beside it. Where it forks (AA_CONC_FORK, same-box A/B on C4): after the
    // local step (0) 412 / 412 it/s, after the Anderson reduce (1: the reduce then streams at full
    // occupancy) 415 / 419, after the mix (2) 393 / 396, in line 399 / 400; right after the
    // two-set solve (-1: the pass's local step would fill the GPU while this iteration's prim check
    // and gated reject branch -- ~20 launches that exit at once, ~110 us -- go by) 404 / 404 against
    // 426 / 423: the Anderson step then runs alone, and that overlap was worth more)
    // (the instrumented pass runs it in line before the Anderson step, outside its timing bracket)
    auto fork_side = [&](int at) {
        if (!side || at != (instrument_ ? 0 : conc_fork_)) return;
        if (sst != s()) {
            AA_HIP(hipEventRecord(ev_fork_, s()));
            AA_HIP(hipStreamWaitEvent(sst, ev_fork_, 0));
        }
        if (sst == s()) ev_begin("comb");
        comb_finish_z(CTL_COMB_ZP, sst, ctrl_c_.p, red_c_.p, red_c_.p + nbg_, &lq2_, dup, dzp);
        if (sst == s()) ev_end("comb");
        if (sst != s()) AA_HIP(hipEventRecord(ev_join_, sst));
        join_wait_ = sst != s();
    };
    ev_begin("grad");
    for (auto& g : groups_) launch_u_and_y(g.d, xfull_.p, z_.p, u_.p, y_.p, nf_, accel ? 1 : 0, 0, c, s());
    ev_end("grad");
    ev_begin("rhs");
    launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, c, 0, s());
    ev_end("rhs");
    if (pipe && it > 0) {
        ev_begin("solve");
        solver_.solve2(b_.p, xfull_.p, b2_.p, cxfull_.p, c, 0, s());
        ev_end("solve");
        if (side) {   // the pass's control block: k-1's prim / reject, before this iteration's
            launch_ctrl_fork(c, ctrl_c_.p, s());   // check; its nrej / fail for a rollback
            fork_side(-1);
        } else {
            ev_begin("comb");
            comb_finish_z(CTL_COMB_ZP, s(), c, pa_, pb_, &lq_, dup, dzp);
            launch_copy(xfull_.p, dxp, nx, c, 2, s());   // break at comb_{k-1}: x back to curr_x_{k-1}
            ev_end("comb");
        }
    } else {
        ev_begin(pipe ? "solve1" : "solve");
        solver_.solve(b_.p, xfull_.p, c, 0, s());
        ev_end(pipe ? "solve1" : "solve");
    }
    auto prim_all = [&](const double* xf, const double* z, const double* zref, int redo) {
        int off = 0;
        for (auto& g : groups_) {
            launch_prim_z(g.d, xf, z, zref, nf_, redo, c, pa_, zref ? pb_ : nullptr, off, s());
            off += blocks_for(g.d.count);
        }
    };
    ev_begin("prim");
    prim_all(xfull_.p, z_.p, nullptr, 0);
    ev_end("prim");
    reduce_partials();
    // the reject test with the restore of the defaults fused (gated on the device: copies only
    // when prim increased)
    launch_check_restore_z(c, ga_, nbg_, accel, u_.p, xfull_.p, z_.p, dup, dxp, dzp, Z_, nx, s());
    if (accel) {   // reject branch (gated on the device; a no-op unless prim increased)
        ev_begin("reject");
        // accelerator.replace(curr_z): the accelerator's iterate is z_ (restored above)
        for (auto& g : groups_) launch_u_and_y(g.d, xfull_.p, z_.p, u_.p, y_.p, nf_, 0, 1, c, s());
        launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, c, 1, s());
        solver_.solve(b_.p, xfull_.p, c, 1, s());
        prim_all(xfull_.p, z_.p, nullptr, 1);
        reduce_partials();
        ev_end("reject");
    }
    launch_control(CTL_PRIM_FINAL_Z, c, ga_, nullptr, nbg_, accel, hist_prim_.p, hist_comb_.p, hist_rej_.p, s());
    if (accel) {
        const int m = st_.anderson_m;
        // default_x / default_u (Solver.cpp:194-195): nothing reads them before the combined-residual
        // pass, so they are copied after the Anderson reduce, beside the concurrent pass's local
        // step instead of on the critical path (the instrumented pass times them here, on their own)
        auto copy_defaults = [&]() {
            ev_begin("copy");
            launch_copy(dxc, xfull_.p, nx, c, 0, s());
            launch_copy(duc, u_.p, Z_, c, 0, s());
            ev_end("copy");
        };
        if (instrument_) copy_defaults();
        // default_z = update_z(curr_x, curr_u) (Solver.cpp:196-199); the same pass writes the
        // rhs slots of the combined-residual solve, w (w default_z + C - curr_u)
        // (Solver.cpp:220): curr_u is final for this iteration and the AA step does not touch it
        ev_begin("local_z");
        local_z_all(xfull_.p, u_.p, dzc, y_.p, LZ_NORMAL, false);
        ev_end("local_z");
        fork_side(0);
        Seg2 G{dzc, Z_, nullptr, 0};
        Seg2 out{z_.p, Z_, nullptr, 0};
        Seg2 none{nullptr, 0, nullptr, 0};
        ev_begin("aa");
        launch_aa_reduce(G, z_.p, Z_, aa_dF_.p, aa_dG_.p, c, aa_red_.p, aa_blocks_, none, m, s());
        reduce_aa();
        fork_side(1);
        if (!instrument_) copy_defaults();
        launch_aa_solve(c, aag_, aa_blocks_, m, s());
        launch_aa_mix(G, z_.p, Z_, aa_dF_.p, aa_dG_.p, c, out, m, s());   // in place (out == cur)
        fork_side(2);
        ev_end("aa");
        // combined residual "for drawing figures" (Solver.cpp:217-233): extra solve + update_z
        if (pipe) {   // its rhs now (the next iteration overwrites the slots); the rest next iteration
            ev_begin("rhs");
            launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b2_.p, c, 0, s());
            ev_end("rhs");
            if (side) {   // join: the pass's records, and a break at comb_{k-1} undoes this iteration
                join_dx_ = dxp;
                join_side();
            }
            return;
        }
        ev_begin("comb");
        launch_rhs(nf_, dt_ptr_.p, nullptr, nullptr, y_.p, Mxbar_.p, pdt2_, b_.p, c, 0, s());
        solver_.solve(b_.p, cxfull_.p, c, 0, s());
        comb_finish_z(CTL_COMB_Z, s(), c, pa_, pb_, &lq_, duc, dzc);
        ev_end("comb");
        return;
    }
    launch_copy(lastz_.p, z_.p, Z_, c, 0, s());
    ev_begin("local_z");
    local_z_all(xfull_.p, u_.p, z_.p, nullptr, LZ_NORMAL, false);
    ev_end("local_z");
    prim_all(xfull_.p, z_.p, lastz_.p, 0);
    reduce_partials();
    launch_control(CTL_COMB_Z, c, ga_, gb_, nbg_, accel, hist_prim_.p, hist_comb_.p, hist_rej_.p, s());
}

// comb pass after its solve: z_c = update_z(x_c, curr_u) into cz_, dual = W (z_c - default_z),
// prim = D x_c - W z_c - C, comb = |prim|^2 + |dual|^2 and the break test (Solver.cpp:224-246).
// du / dz: curr_u and default_z of the iteration the pass belongs to (when pipelined, u_ already
// holds the next iteration's u). On stream st with control block c and partials pa / pb: the
// solver's own, or (concurrent pass) the side stream's copies, summed only there -- one GPU.
void ElasticSolver::comb_finish_z(int op, hipStream_t st, Ctrl* c, double* pa, double* pb, const LocalQueue* q,
                                  const double* du, const double* dz) {
    local_z_on(cxfull_.p, du, cz_.p, LZ_NORMAL, st, c, q);
    int off = 0;
    for (auto& g : groups_) {
        launch_prim_z(g.d, cxfull_.p, cz_.p, dz, nf_, 0, c, pa, pb, off, st);
        off += blocks_for(g.d.count);
    }
    if (st == s()) {
        reduce_partials();
        launch_control(op, c, ga_, gb_, nbg_, 1, hist_prim_.p, hist_comb_.p, hist_rej_.p, st);
    } else {
        launch_control(op, c, pa, pb, nbg_, 1, hist_prim_.p, hist_comb_.p, hist_rej_.p, st);
    }
}

// the last iteration's combined-residual pass (pipelined Z variant)
// the concurrent pass's join, at the end of the iteration that forked it: its records merged, a
// break at its comb undoing that iteration (done = 2, x back to the pass's curr_x). Measured: a
// join delayed to the next iteration's two-set solve (the pass also beside that iteration's
// gradient and rhs) gains nothing (415.9 / 416.3 vs 414.9 / 417.0 it/s on C4)
void ElasticSolver::join_side() {
    if (join_wait_) AA_HIP(hipStreamWaitEvent(s(), ev_join_, 0));
    launch_ctrl_join(ctrl_.p, ctrl_c_.p, xfull_.p, join_dx_, 3LL * nf_, s());
}

void ElasticSolver::enqueue_comb_tail_z(int iters) {
    ev_begin("comb");
    solver_.solve(b2_.p, cxfull_.p, ctrl_.p, 0, s());
    comb_finish_z(CTL_COMB_Z, s(), ctrl_.p, pa_, pb_, &lq_, du_at(iters - 1), dz_at(iters - 1));
    ev_end("comb");
}

void ElasticSolver::enqueue_iterations(int iters, bool accel) {
    // AA_EAGER_SYNC=n (diagnostics, eager launches only): drain the stream every n iterations,
    // bounding the depth of unsynchronised dispatches (profiler runs)
    static const int eager_sync = [] { const char* e = std::getenv("AA_EAGER_SYNC"); return e ? std::atoi(e) : 0; }();
    hipStreamCaptureStatus cst = hipStreamCaptureStatusNone;
    if (eager_sync > 0) AA_HIP(hipStreamIsCapturing(s(), &cst));
    for (int it = 0; it < iters; ++it) {
        if (st_.variant == AA_VARIANT_UX) enqueue_iteration_ux(accel);
        else enqueue_iteration_z(accel, it);
        if (eager_sync > 0 && cst == hipStreamCaptureStatusNone && (it + 1) % eager_sync == 0)
            AA_HIP(hipStreamSynchronize(s()));
    }
    if (st_.variant != AA_VARIANT_UX && accel && pipe_z_ && iters > 0) enqueue_comb_tail_z(iters);
}

void ElasticSolver::epilogue_enqueue(bool accel) {
    const double* src = (st_.variant == AA_VARIANT_UX && accel) ? dx_.p : xfull_.p;
    launch_finalize(n_, nf_, src, xfull_.p, xs_.p, vs_.p, st_.timestep_s, s());
}

void ElasticSolver::fetch_results() {
    Ctrl c;
    AA_HIP(hipMemcpyAsync(&c, ctrl_.p, sizeof(Ctrl), hipMemcpyDeviceToHost, s()));
    AA_HIP(hipStreamSynchronize(s()));
    nrec_ = std::min(c.nrec, hist_cap_);
    h_prim_.resize(nrec_); h_comb_.resize(nrec_); h_rej_.resize(nrec_);
    if (nrec_) {
        AA_HIP(hipMemcpy(h_prim_.data(), hist_prim_.p, nrec_ * 8, hipMemcpyDeviceToHost));
        AA_HIP(hipMemcpy(h_comb_.data(), hist_comb_.p, nrec_ * 8, hipMemcpyDeviceToHost));
        AA_HIP(hipMemcpy(h_rej_.data(), hist_rej_.p, nrec_ * 4, hipMemcpyDeviceToHost));
        std::vector<long long> clk(nrec_);
        AA_HIP(hipMemcpy(clk.data(), hist_clock_.p, nrec_ * sizeof(long long), hipMemcpyDeviceToHost));
        h_time_.resize(nrec_);
        for (int i = 0; i < nrec_; ++i) h_time_[i] = (double)(clk[i] - c.clock0) / clock_khz_;
    } else {
        h_time_.clear();
    }
    rt_.iterations = c.iters_run;
    rt_.rejects = c.nrej;
    if (comm_) {   // a failing element prox lives on one rank: agree before throwing
        double f[2] = {c.fail == 1 ? 1.0 : 0.0, c.fail == 2 ? 1.0 : 0.0};
        comm_->allreduce_sum_host(f, 2);
        c.fail = f[0] > 0 ? 1 : (f[1] > 0 ? 2 : 0);
        if (comm_->rehearsal()) c.fail = 0;   // the other parts are absent: positions are not physical
    }
    if (c.fail == 1) throw Error(ERR_NUMERIC, "the line search step became smaller than the minimum value allowed");
    if (c.fail == 2) throw Error(ERR_NUMERIC, "**TriEnergyTerm TODO: gradient function");
}

void ElasticSolver::step() {
    if (!initialized_) throw Error(ERR_STATE, "step() before initialize()");
    auto t0 = std::chrono::steady_clock::now();
    const bool accel = st_.acceleration_type == 1;
    bool graph = use_graph_ && st_.admm_iters > 0;
    if (graph && !gexec_) {   // pointers and control flow are fixed after initialize: capture once,
        // before the prologue starts the step's device clock (capture is host work)
        bool ok = capture_graph(s(), [&] { enqueue_iterations(st_.admm_iters, accel); }, &graph_, &gexec_);
        if (comm_) {   // the ranks replay or launch eagerly together
            double f = ok ? 0.0 : 1.0;
            comm_->allreduce_sum_host(&f, 1);
            if (f > 0 && ok) { drop_graph(); ok = false; }
        }
        if (!ok) {
            use_graph_ = graph = false;
            std::fprintf(stderr, "[aa_admm] step graph capture failed: launching eagerly\n");
        }
    }
    prologue();
    if (graph) {
        AA_HIP(hipGraphLaunch(gexec_, s()));
    } else {
        enqueue_iterations(st_.admm_iters, accel);
    }
    epilogue_enqueue(accel);
    gather_state(xs_);
    gather_state(vs_);
    fetch_results();
    // host mirrors of m_x / m_v
    std::vector<double> xs(3 * (size_t)n_), vs(3 * (size_t)n_);
    AA_HIP(hipMemcpy(xs.data(), xs_.p, xs.size() * 8, hipMemcpyDeviceToHost));
    AA_HIP(hipMemcpy(vs.data(), vs_.p, vs.size() * 8, hipMemcpyDeviceToHost));
    for (int q = 0; q < n_; ++q)
        for (int j = 0; j < 3; ++j) { x_[3 * (size_t)int2node_[q] + j] = xs[3 * (size_t)q + j]; v_[3 * (size_t)int2node_[q] + j] = vs[3 * (size_t)q + j]; }
    rt_.step_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void ElasticSolver::get_x(double* out) { std::copy(x_.begin(), x_.end(), out); }
void ElasticSolver::get_v(double* out) { std::copy(v_.begin(), v_.end(), out); }
// Solver::m_x assignment between steps (the reference's public member): the next step starts
// from these positions
void ElasticSolver::set_x(const double* x3) {
    std::copy(x3, x3 + x_.size(), x_.begin());
    if (initialized_) {
        std::vector<double> xs(3 * (size_t)n_);
        for (int q = 0; q < n_; ++q) for (int j = 0; j < 3; ++j) xs[3 * (size_t)q + j] = x_[3 * (size_t)int2node_[q] + j];
        AA_HIP(hipMemcpy(xs_.p, xs.data(), xs.size() * 8, hipMemcpyHostToDevice));
    }
}

void ElasticSolver::set_v(const double* v3) {
    std::copy(v3, v3 + v_.size(), v_.begin());
    if (initialized_) {
        std::vector<double> vs(3 * (size_t)n_);
        for (int q = 0; q < n_; ++q) for (int j = 0; j < 3; ++j) vs[3 * (size_t)q + j] = v_[3 * (size_t)int2node_[q] + j];
        AA_HIP(hipMemcpy(vs_.p, vs.data(), vs.size() * 8, hipMemcpyHostToDevice));
    }
}

int ElasticSolver::history(double* prim, double* comb, int* rej, int cap) const {
    const int n = std::min(cap, nrec_);
    for (int i = 0; i < n; ++i) {
        if (prim) prim[i] = h_prim_[i];
        if (comb) comb[i] = h_comb_[i];
        if (rej) rej[i] = h_rej_[i];
    }
    return nrec_;
}

// run limits of later steps (bench: a run-to-epsilon leg after the fixed-iteration steps,
// without re-factoring): drops the captured graph, grows the history if needed
void ElasticSolver::set_iterations(int admm_iters, double eps_rel) {
    if (!initialized_) throw Error(ERR_STATE, "set_iterations before initialize()");
    if (admm_iters < 0 || !(eps_rel >= 0.0)) throw Error(ERR_ARG, "set_iterations: admm_iters >= 0 and eps_rel >= 0");
    drop_graph();
    st_.admm_iters = admm_iters;
    st_.eps_rel = eps_rel;
    if (std::max(1, admm_iters) > hist_cap_) {
        hist_cap_ = admm_iters;
        hist_prim_.alloc(hist_cap_); hist_comb_.alloc(hist_cap_); hist_rej_.alloc(hist_cap_);
        hist_clock_.alloc(hist_cap_ + 1);
    }
}

int ElasticSolver::times(double* time_ms, int cap) const {
    const int n = std::min(cap, (int)h_time_.size());
    for (int i = 0; i < n && time_ms; ++i) time_ms[i] = h_time_[i];
    return (int)h_time_.size();
}

double ElasticSolver::bench_iterations(int iters) {
    if (!initialized_) throw Error(ERR_STATE, "bench before initialize()");
    const bool accel = st_.acceleration_type == 1;
    for (auto& kv : kstats_) { for (auto e : kv.second.ev) (void)hipEventDestroy(e); kv.second.ev.clear(); }
    prologue();
    AA_HIP(hipStreamSynchronize(s()));
    instrument_ = true;
    hipEvent_t e0, e1;
    AA_HIP(hipEventCreate(&e0)); AA_HIP(hipEventCreate(&e1));
    AA_HIP(hipEventRecord(e0, s()));
    enqueue_iterations(iters, accel);
    AA_HIP(hipEventRecord(e1, s()));
    AA_HIP(hipEventSynchronize(e1));
    instrument_ = false;
    float ms = 0;
    AA_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    for (auto& kv : kstats_) {
        KStat& k = kv.second;
        k.total_ms = 0; k.launches = 0;
        for (size_t i = 0; i + 1 < k.ev.size(); i += 2) {
            float t = 0;
            AA_HIP(hipEventElapsedTime(&t, k.ev[i], k.ev[i + 1]));
            k.total_ms += t; k.launches += 1;
        }
    }
    Ctrl c;
    AA_HIP(hipMemcpy(&c, ctrl_.p, sizeof(Ctrl), hipMemcpyDeviceToHost));
    rt_.iterations = c.iters_run;
    rt_.rejects = c.nrej;
    return ms;
}

bool ElasticSolver::kernel_stats(const std::string& name, double* avg_ms, double* bytes, int* launches) const {
    auto it = kstats_.find(name);
    if (it == kstats_.end()) return false;
    const KStat& k = it->second;
    if (avg_ms) *avg_ms = k.launches ? k.total_ms / k.launches : 0.0;
    if (bytes) *bytes = k.bytes;
    if (launches) *launches = k.launches;
    return true;
}

int ElasticSolver::local_stats(long long* out, int cap, bool reset) {
    const int n = std::min(cap, kLqStats);
    if (!lq_stats_.p) {
        for (int i = 0; i < n; ++i) out[i] = 0;
        return n;
    }
    std::vector<unsigned long long> h(kLqStats);
    AA_HIP(hipMemcpyAsync(h.data(), lq_stats_.p, kLqStats * sizeof(unsigned long long), hipMemcpyDeviceToHost, s()));
    AA_HIP(hipStreamSynchronize(s()));
    for (int i = 0; i < n; ++i) out[i] = (long long)h[i];
    if (reset) lq_stats_.zero(s());
    return n;
}

}  // namespace aa
