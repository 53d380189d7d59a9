// aa_admm.hpp -- header-only C++ facade over the C ABI (aa_admm.h) that keeps the reference's
// admm-elastic plugin API shape (admm_anderson_hard_zxu/src/Solver.hpp:39-262,
// EnergyTerm.hpp:35-129, TetEnergyTerm.hpp:36-51, TriEnergyTerm.hpp:33-47) so existing scene
// code ports by changing includes:
//
//   admm::Solver solver;                               // one MI355X (device 0) by default
//   solver.add_nodes(x, m, n);                         // Solver::add_nodes
//   admm::create_tets_from_mesh<float, admm::NeoHookeanTet>(solver.energyterms, verts, inds, n, lame, off);
//   admm::create_tris_from_mesh<float, admm::TriEnergyTerm>(solver.energyterms, verts, inds, n, lame, off);
//   solver.set_pins(pins, points);                     // Solver::set_pins
//   solver.add_obstacle(std::make_shared<admm::Floor>(-1.0)); solver.set_collisions(inds);  // (u,x) variant
//   solver.ext_forces.push_back(std::make_shared<admm::WindForce>(faces));                    // wind
//   solver.initialize(settings);                       // Solver::initialize (returns bool)
//   solver.step();                                     // Solver::step; solver.m_x / m_v updated
//
// Energy terms are descriptors of the built-in element kinds (batched SoA on the device);
// user-defined EnergyTerm subclasses with arbitrary prox() are not supported (no host
// callbacks on the GPU path). Errors are re-raised as std::runtime_error like the reference.
#ifndef AA_ADMM_HPP
#define AA_ADMM_HPP

#include <algorithm>
#include <array>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "aa_admm.h"

namespace admm {

inline void check(int rc) {
    if (rc != AA_OK) throw std::runtime_error(aa_last_error());
}

// EnergyTerm.hpp:35-61
class Lame {
public:
    static Lame rubber() { return Lame(10000000, 0.499); }
    static Lame soft_rubber() { return Lame(10000000, 0.399); }
    static Lame very_soft_rubber() { return Lame(1000000, 0.299); }
    double mu = 0, lambda = 0;
    double limit_min = -100.0, limit_max = 100.0;
    double bulk_modulus() const { return lambda + (2.0 / 3.0) * mu; }
    Lame(double k, double v) : mu(k / (2.0 * (1.0 + v))), lambda(k * v / ((1.0 + v) * (1.0 - 2.0 * v))) {}
    Lame() {}
    aa_lame c() const { return aa_lame{mu, lambda, limit_min, limit_max}; }
};

// Descriptors of the built-in energy terms (one per create_*_from_mesh call).
class EnergyTerm {
public:
    virtual ~EnergyTerm() {}
    int kind = 0, material = AA_LINEAR;   // kind 0 tet, 1 tri
    Lame lame;
    std::vector<double> verts;   // rest shape (as given to create_*_from_mesh)
    std::vector<int> inds;
    int count = 0, vertex_offset = 0;
};
struct TetEnergyTerm { static constexpr int material = AA_LINEAR; };
struct NeoHookeanTet { static constexpr int material = AA_NEOHOOKEAN; };
struct StVKTet { static constexpr int material = AA_STVK; };
struct TriEnergyTerm { static constexpr int material = AA_LINEAR; };

// TetEnergyTerm.hpp:36-51 (one descriptor holds the whole mesh instead of n objects)
template <typename IN_SCALAR, typename TYPE>
inline void create_tets_from_mesh(std::vector<std::shared_ptr<EnergyTerm>>& energyterms, const IN_SCALAR* verts,
                                  const int* inds, int n_tets, const Lame& lame, const int vertex_offset) {
    auto e = std::make_shared<EnergyTerm>();
    e->kind = 0;
    e->material = TYPE::material;
    e->lame = lame;
    int nv = 0;
    for (int i = 0; i < 4 * n_tets; ++i) nv = std::max(nv, inds[i] + 1);
    e->verts.assign(verts, verts + 3 * (size_t)nv);
    e->inds.assign(inds, inds + 4 * (size_t)n_tets);
    e->count = n_tets;
    e->vertex_offset = vertex_offset;
    energyterms.push_back(e);
}

// TriEnergyTerm.hpp:33-47
template <typename IN_SCALAR, typename TYPE>
inline void create_tris_from_mesh(std::vector<std::shared_ptr<EnergyTerm>>& energyterms, const IN_SCALAR* verts,
                                  const int* inds, int n_tris, const Lame& lame, const int vertex_offset) {
    auto e = std::make_shared<EnergyTerm>();
    e->kind = 1;
    e->material = AA_LINEAR;
    e->lame = lame;
    int nv = 0;
    for (int i = 0; i < 3 * n_tris; ++i) nv = std::max(nv, inds[i] + 1);
    e->verts.assign(verts, verts + 3 * (size_t)nv);
    e->inds.assign(inds, inds + 3 * (size_t)n_tris);
    e->count = n_tris;
    e->vertex_offset = vertex_offset;
    energyterms.push_back(e);
}

typedef std::array<double, 3> Vec3d;

// Passive obstacles (admm_anderson_hard_zxu/src/PassiveObject.hpp:32-136, Collider.hpp:63-82):
// shape descriptors, tested on the device by the collision terms
class PassiveCollision {
public:
    virtual ~PassiveCollision() {}
    int type = AA_OBS_FLOOR;
    double params[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};
class Floor : public PassiveCollision {
public:
    explicit Floor(double y) { type = AA_OBS_FLOOR; params[0] = y; }
};
class SlideFloor : public PassiveCollision {
public:
    SlideFloor(const Vec3d& c, const Vec3d& n) {
        type = AA_OBS_SLIDE_FLOOR;
        for (int i = 0; i < 3; ++i) { params[i] = c[i]; params[3 + i] = n[i]; }
    }
};
class Sphere : public PassiveCollision {
public:
    Sphere(const Vec3d& c, double r) { type = AA_OBS_SPHERE; for (int i = 0; i < 3; ++i) params[i] = c[i]; params[3] = r; }
};
class PlaneAndHalfSphere : public PassiveCollision {
public:
    PlaneAndHalfSphere(const Vec3d& c, double r) {
        type = AA_OBS_PLANE_HALF_SPHERE;
        for (int i = 0; i < 3; ++i) params[i] = c[i];
        params[3] = r;
    }
};
class Cylinder : public PassiveCollision {
public:
    Cylinder(const Vec3d& c, double r) { type = AA_OBS_CYLINDER; for (int i = 0; i < 3; ++i) params[i] = c[i]; params[3] = r; }
};

// Explicit forces (ExplicitForce.hpp:33-47): WindForce on a list of triangles (flat, 3 per face);
// `direction` may be changed between steps (windyflag.cpp's intensity keys)
class ExplicitForce {
public:
    virtual ~ExplicitForce() {}
};
class WindForce : public ExplicitForce {
public:
    explicit WindForce(std::vector<int>& tris_) : tris(tris_), direction{{0, 0, 0}} {}
    std::vector<int> tris;
    Vec3d direction;
    int id = -1;   // device handle once registered
};

class Solver {
public:
    typedef std::vector<double> VecX;      // Eigen::VectorXd in the reference (no Eigen dependency here)
    typedef std::array<double, 3> Vec3;

    // Solver::Settings (Solver.hpp:45-67); `variant` selects the reference copy
    struct Settings {
        enum AccelationType { NOACC = 0, ANDERSON = 1 };
        double timestep_s;
        int verbose;
        int admm_iters;
        double gravity;
        double constraint_w;
        int Anderson_m;
        double penalty;
        AccelationType acceleration_type;
        int variant;
        Settings() : timestep_s(1.0 / 30.0), verbose(1), admm_iters(500), gravity(-9.8), constraint_w(-1),
                     Anderson_m(2), penalty(1.0), acceleration_type(NOACC), variant(AA_VARIANT_UX) {}
    };
    struct RuntimeData : aa_runtime {};

    VecX m_x, m_v, m_masses;   // scaled x3, as the reference
    std::vector<std::shared_ptr<EnergyTerm>> energyterms;
    std::vector<std::shared_ptr<ExplicitForce>> ext_forces;   // Solver.hpp:90

    explicit Solver(int device = 0) {
        check(aa_ctx_create(device, &ctx_));
        check(aa_elastic_create(ctx_, &h_));
    }
    ~Solver() {
        if (h_) aa_elastic_destroy(h_);
        if (ctx_) aa_ctx_destroy(ctx_);
    }
    Solver(const Solver&) = delete;
    Solver& operator=(const Solver&) = delete;

    template <typename T>
    int add_nodes(T* x, T* m, int n_verts) {
        const int prev = (int)m_x.size();
        m_x.resize(prev + 3 * n_verts);
        m_v.resize(prev + 3 * n_verts);
        m_masses.resize(prev + 3 * n_verts);
        for (int i = 0; i < 3 * n_verts; ++i) { m_x[prev + i] = x[i]; m_v[prev + i] = 0; m_masses[prev + i] = m[i]; }
        return (prev + 3 * n_verts) / 3;
    }

    void set_pins(const std::vector<int>& inds, const std::vector<Vec3>& points = std::vector<Vec3>()) {
        pins_ = inds;
        pin_pts_.clear();
        if (points.size() == inds.size())
            for (auto& p : points) { pin_pts_.push_back(p[0]); pin_pts_.push_back(p[1]); pin_pts_.push_back(p[2]); }
        if (initialized_) push_pins();
    }

    // Solver::add_obstacle (Solver.cpp:346-348): takes effect at once, also between steps
    void add_obstacle(std::shared_ptr<PassiveCollision> obj) { check(aa_elastic_add_obstacle(h_, obj->type, obj->params)); }
    // Solver::set_collisions (Solver.cpp:318-344): the points are not used by the prox
    void set_collisions(const std::vector<int>& inds, const std::vector<Vec3>& points = std::vector<Vec3>()) {
        (void)points;
        check(aa_elastic_set_collisions(h_, inds.data(), (int)inds.size()));
    }

    // Nodes and energy terms are handed to the device solver on the FIRST initialize(); a later
    // initialize() re-runs only the device setup with the new settings (the reference rebuilds
    // its matrices from the same members).
    bool initialize(const Settings& s) {
        settings_ = s;
        if (!bound_) {
            int total = 0;
            if (aa_elastic_add_nodes(h_, m_x.data(), m_masses.data(), (int)m_x.size() / 3, &total) != AA_OK) return false;
            for (auto& e : energyterms) {
                aa_lame l = e->lame.c();
                const int rc = e->kind == 0
                    ? aa_elastic_add_tets(h_, e->verts.data(), e->inds.data(), e->count, e->material, &l, e->vertex_offset)
                    : aa_elastic_add_tris(h_, e->verts.data(), e->inds.data(), e->count, &l, e->vertex_offset);
                if (rc != AA_OK) return false;
            }
            bound_ = true;
        }
        push_pins();
        aa_settings cs{s.timestep_s, s.verbose, s.admm_iters, s.gravity, s.constraint_w, s.Anderson_m, s.penalty,
                       (int)s.acceleration_type, s.variant, 0.0};
        if (aa_elastic_initialize(h_, &cs) != AA_OK) return false;
        initialized_ = true;
        x_seen_.clear();
        v_seen_.clear();
        return true;
    }

    // m_x / m_v edited by the caller between steps (the reference reads them directly) are pushed
    // to the device first.
    void step() {
        for (auto& f : ext_forces) {   // register new forces, push the current wind directions
            auto w = std::dynamic_pointer_cast<WindForce>(f);
            if (!w) throw std::runtime_error("ext_forces: only WindForce is provided");
            if (w->id < 0) check(aa_elastic_add_wind(h_, w->tris.data(), (int)w->tris.size() / 3, w->direction.data(), &w->id));
            else check(aa_elastic_set_wind(h_, w->id, w->direction.data()));
        }
        if (!x_seen_.empty() && x_seen_ != m_x) check(aa_elastic_set_x(h_, m_x.data()));
        if (!v_seen_.empty() && v_seen_ != m_v) check(aa_elastic_set_v(h_, m_v.data()));
        check(aa_elastic_step(h_));
        check(aa_elastic_get_x(h_, m_x.data()));
        check(aa_elastic_get_v(h_, m_v.data()));
        x_seen_ = m_x;
        v_seen_ = m_v;
        save(true);
    }

    // Solver::save() (Solver.hpp:130-155, called at the end of every step, Solver.cpp:232/262):
    // ./result/residual-<m>.txt (or residual-no.txt) with one row per iteration of the last step:
    // time (ms since the step started; device clock), prim, comb and -- (u,x) variant
    // (admm_anderson_hard_zxu) only -- the reject flag, %.16g as `ofs << setprecision(16)`.
    // quiet: skip silently when ./result does not exist (the reference prints "Cannot open").
    bool save(bool quiet = false) const {
        const std::string file = settings_.acceleration_type ? "./result/residual-" + std::to_string(settings_.Anderson_m) + ".txt"
                                                             : std::string("./result/residual-no.txt");
        std::FILE* f = std::fopen(file.c_str(), "w");
        if (!f) {
            if (!quiet) std::printf("Cannot open: %s\n", file.c_str());
            return false;
        }
        std::vector<double> prim, comb, t;
        std::vector<int> rej;
        const int n = history(prim, comb, rej);
        int nt = 0;
        check(aa_elastic_get_times(h_, nullptr, 0, &nt));
        t.assign(std::max(n, nt), 0.0);
        if (nt) check(aa_elastic_get_times(h_, t.data(), nt, &nt));
        for (int i = 0; i < n; ++i) {
            if (settings_.variant == AA_VARIANT_UX) std::fprintf(f, "%.16g\t%.16g\t%.16g\t%d\n", t[i], prim[i], comb[i], rej[i]);
            else std::fprintf(f, "%.16g\t%.16g\t%.16g\n", t[i], prim[i], comb[i]);
        }
        std::fclose(f);
        return true;
    }

    const Settings& settings() const { return settings_; }
    RuntimeData runtime_data() const {
        RuntimeData r;
        check(aa_elastic_runtime(h_, &r));
        return r;
    }
    // the (prim, comb, reject) rows Solver::save() writes (Solver.hpp:130-155)
    int history(std::vector<double>& prim, std::vector<double>& comb, std::vector<int>& rej) const {
        int n = 0;
        check(aa_elastic_get_history(h_, nullptr, nullptr, nullptr, 0, &n));
        prim.resize(n); comb.resize(n); rej.resize(n);
        check(aa_elastic_get_history(h_, prim.data(), comb.data(), rej.data(), n, &n));
        return n;
    }

private:
    void push_pins() {
        check(aa_elastic_set_pins(h_, pins_.data(), pin_pts_.empty() ? nullptr : pin_pts_.data(), (int)pins_.size()));
    }
    aa_ctx ctx_ = nullptr;
    aa_elastic h_ = nullptr;
    Settings settings_;
    bool initialized_ = false, bound_ = false;
    VecX x_seen_, v_seen_;
    std::vector<int> pins_;
    std::vector<double> pin_pts_;
};

}  // namespace admm

#endif  // AA_ADMM_HPP
