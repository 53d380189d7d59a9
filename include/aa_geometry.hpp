// aa_geometry.hpp -- header-only C++ facade over the C ABI (aa_admm.h) with the shape of the
// reference's Geometry API (bldeng/AA-ADMM Geometry/Constraint.h:48-414,
// Geometry/ALMGeometrySolver.h:59-320, Geometry/LinearRegularization.h:47-87,
// Geometry/TriMeshAABB.h:38-69, Geometry/SolverCommon.h:34-38), so optimize_mesh-style caller
// code ports by changing includes:
//
//   ALMGeometrySolver<3> solver;                                   // one MI355X (device 0)
//   auto aabb = std::make_shared<TriMeshAABB>(ref_V, ref_F);       // reference surface
//   solver.add_soft_constraint(new PointToRefSurfaceConstraint(i, 1.0, aabb));
//   solver.add_relative_uniform_laplacian(ring, 0.1, ref_points);
//   solver.add_hard_constraint(new PlaneConstraint(face_vertices, 1.0));
//   solver.setup_ADMM(n_points, 1e5, LDLT_SOLVER);
//   solver.solve_ADMM(init_x, rel_eps, max_iter, Anderson_m);
//   const Matrix3X& x = solver.get_solution();   solver.function_values_ / elapsed_time_
//
// Point sets are 3 x n column-major (the layout of the reference's Matrix3X); any matrix type
// with data() and cols() over contiguous column-major doubles (e.g. Eigen::Matrix3Xd) is
// accepted wherever the reference takes a MatrixNX. Constraints are descriptors of the
// built-in projection types (batched per type on the device); user-defined Constraint
// subclasses with an arbitrary project_impl() are not supported. The solver owns (deletes)
// the constraints handed to it, as the reference's destructor does (ALMGeometrySolver.h:67-79).
#ifndef AA_GEOMETRY_HPP
#define AA_GEOMETRY_HPP

#include <cmath>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "aa_admm.h"

typedef double Scalar;

enum SPDSolverType { LDLT_SOLVER = AA_SPD_LDLT, LLT_SOLVER = AA_SPD_LLT };   // SolverCommon.h:34-38

// 3 x n column-major point matrix (x, y, z of point i at data()[3 i .. 3 i + 2])
class Matrix3X {
public:
    Matrix3X() {}
    explicit Matrix3X(int n) : v_(3 * (size_t)n, 0.0) {}
    template <class M> static Matrix3X from(const M& m) {
        Matrix3X r((int)m.cols());
        for (size_t i = 0; i < r.v_.size(); ++i) r.v_[i] = m.data()[i];
        return r;
    }
    int rows() const { return 3; }
    int cols() const { return (int)(v_.size() / 3); }
    double* data() { return v_.data(); }
    const double* data() const { return v_.data(); }
    double& operator()(int r, int c) { return v_[3 * (size_t)c + r]; }
    double operator()(int r, int c) const { return v_[3 * (size_t)c + r]; }

private:
    std::vector<double> v_;
};

// 3 x n column-major index matrix (the reference's Eigen::Matrix3Xi of face vertex ids)
class Matrix3Xi {
public:
    Matrix3Xi() {}
    explicit Matrix3Xi(int n) : v_(3 * (size_t)n, 0) {}
    int rows() const { return 3; }
    int cols() const { return (int)(v_.size() / 3); }
    int* data() { return v_.data(); }
    const int* data() const { return v_.data(); }
    int& operator()(int r, int c) { return v_[3 * (size_t)c + r]; }

private:
    std::vector<int> v_;
};

// TriMeshAABB.h:38-69: the closest-point structure over a reference triangle mesh; here the
// mesh itself (the BVH is built on the GPU when the solver is set up). F is 3 x nf vertex ids.
class TriMeshAABB {
public:
    template <class MV, class MF>
    TriMeshAABB(const MV& V, const MF& F) {
        V_.assign(V.data(), V.data() + 3 * (size_t)V.cols());
        F_.assign(F.data(), F.data() + 3 * (size_t)F.cols());
    }
    TriMeshAABB(const std::vector<double>& V3, const std::vector<int>& F3) : V_(V3), F_(F3) {}
    std::vector<double> V_;
    std::vector<int> F_;
};

template <unsigned int N>
class Constraint {   // Constraint.h:48-192 (descriptor)
public:
    static_assert(N == 3, "the MI355X path implements Constraint<3>");
    virtual ~Constraint() {}
    int type = 0;
    std::vector<int> idI_;
    Scalar weight_ = 1;
    std::vector<double> params_;
    std::shared_ptr<TriMeshAABB> surface_;

protected:
    Constraint(int t, std::vector<int> idI, Scalar w) : type(t), idI_(std::move(idI)), weight_(w) {}
};

template <unsigned int N>
class EdgeLengthConstraint : public Constraint<N> {   // Constraint.h:194-218
public:
    EdgeLengthConstraint(int idx1, int idx2, Scalar weight, Scalar target_length)
        : Constraint<N>(AA_CON_EDGE, {idx1, idx2}, weight) { this->params_ = {target_length}; }
};

template <unsigned int N>
class AngleConstraint : public Constraint<N> {   // Constraint.h:220-296
public:
    AngleConstraint(int tip_idx, int side_idx1, int side_idx2, Scalar weight, Scalar min_radian, Scalar max_radian)
        : Constraint<N>(AA_CON_ANGLE, {tip_idx, side_idx1, side_idx2}, weight) {
        this->params_ = {min_radian, max_radian};
    }
};

template <unsigned int N>
class ClosenessConstraint : public Constraint<N> {   // Constraint.h:299-326
public:
    template <class V>
    ClosenessConstraint(int idx, Scalar weight, const V& target_pos) : Constraint<N>(AA_CON_CLOSENESS, {idx}, weight) {
        this->params_ = {target_pos[0], target_pos[1], target_pos[2]};
    }
};

class PointToRefSurfaceConstraint : public Constraint<3> {   // Constraint.h:328-349
public:
    PointToRefSurfaceConstraint(int pt_idx, Scalar weight, const std::shared_ptr<TriMeshAABB>& aabb)
        : Constraint<3>(AA_CON_POINT_TO_REF, {pt_idx}, weight) { surface_ = aabb; }
};

class ReferenceSurfceConstraint : public Constraint<3> {   // Constraint.h:351-394 (points 0..n-1)
public:
    template <class MV, class MF>
    ReferenceSurfceConstraint(int n_points, Scalar weight, const MV& ref_surface_vtx, const MF& ref_surface_faces)
        : Constraint<3>(AA_CON_REF_SURFACE, {}, weight) {
        idI_.resize(n_points);
        for (int i = 0; i < n_points; ++i) idI_[i] = i;
        surface_ = std::make_shared<TriMeshAABB>(ref_surface_vtx, ref_surface_faces);
    }
};

class PlaneConstraint : public Constraint<3> {   // Constraint.h:396-414
public:
    PlaneConstraint(const std::vector<int>& idI, Scalar weight) : Constraint<3>(AA_CON_PLANE, idI, weight) {}
};

namespace detail {
// The two reference solvers share their public surface; KIND selects the device loop
// (AA_GEOM_ALM: ALMGeometrySolver.h:59-320, AA_GEOM_PLAIN: GeometrySolver.h:57-464).
template <unsigned int N, int KIND>
class GeometrySolverFacade {
public:
    static_assert(N == 3, "the MI355X path implements the N = 3 geometry solvers");
    explicit GeometrySolverFacade(int device = 0) {
        check(aa_ctx_create(device, &ctx_));
        check(aa_geom_create_kind(ctx_, KIND, &h_));
    }
    ~GeometrySolverFacade() {
        for (auto* c : hard_) delete c;
        for (auto* c : soft_) delete c;
        if (h_) aa_geom_destroy(h_);
        if (ctx_) aa_ctx_destroy(ctx_);
    }
    GeometrySolverFacade(const GeometrySolverFacade&) = delete;
    GeometrySolverFacade& operator=(const GeometrySolverFacade&) = delete;

    void add_hard_constraint(Constraint<N>* c) { hard_.push_back(c); }
    void add_soft_constraint(Constraint<N>* c) { soft_.push_back(c); }
    template <class V>
    void add_closeness(int idx, Scalar weight, const V& target_pt) {
        const double t[3] = {target_pt[0], target_pt[1], target_pt[2]};
        check(aa_geom_add_closeness(h_, idx, weight, t));
    }
    // LinearRegularization.h:47-53: coefficients 1, -1/(k-1), ..., first index = centre
    void add_uniform_laplacian(const std::vector<int>& indices, Scalar weight) {
        add_laplacian(indices, uniform(indices.size()), weight);
    }
    void add_laplacian(const std::vector<int>& indices, const std::vector<Scalar> coefs, Scalar weight) {
        check(aa_geom_add_laplacian(h_, indices.data(), coefs.data(), (int)indices.size(), weight, nullptr));
    }
    template <class M>
    void add_relative_uniform_laplacian(const std::vector<int>& indices, Scalar weight, const M& ref_points) {
        add_relative_laplacian(indices, uniform(indices.size()), weight, ref_points);
    }
    template <class M>
    void add_relative_laplacian(const std::vector<int>& indices, const std::vector<Scalar> coefs, Scalar weight,
                                const M& ref_points) {
        check(aa_geom_add_laplacian(h_, indices.data(), coefs.data(), (int)indices.size(), weight, ref_points.data()));
    }

    // ALMGeometrySolver.h:81-161: constraint rows in insertion order (consecutive constraints of
    // one type and weight go down as one batch); returns false like the reference on failure
    bool setup_ADMM(int n_points, Scalar penalty_param, SPDSolverType spd_solver_type = LDLT_SOLVER) {
        try {
            flush(hard_, 1);
            flush(soft_, 0);
            check(aa_geom_setup(h_, n_points, penalty_param, (int)spd_solver_type));
            n_ = n_points;
            return true;
        } catch (const std::exception&) {
            return false;
        }
    }
    // ALMGeometrySolver.h:163-283 (init_x: 3 x n column-major)
    template <class M>
    void solve_ADMM(const M& init_x, Scalar rel_residual_eps, int max_iter, int Anderson_m) {
        check(aa_geom_solve(h_, init_x.data(), rel_residual_eps, max_iter, Anderson_m));
        x_ = Matrix3X(n_);
        check(aa_geom_get_solution(h_, x_.data()));
        int k = 0;
        check(aa_geom_get_history(h_, nullptr, nullptr, 0, &k));
        function_values_.assign(k, 0.0);
        elapsed_time_.assign(k, 0.0);
        if (k) check(aa_geom_get_history(h_, function_values_.data(), elapsed_time_.data(), k, &k));
    }
    const Matrix3X& get_solution() const { return x_; }
    // extension (aa_geom_set_stop): run later solves to the residual_eps the reference computes
    // (ALMGeometrySolver.h:172) but never tests, and/or to eps_rel * the first comb
    void set_stop_at_eps(bool stop_at_eps, Scalar eps_rel = 0) { check(aa_geom_set_stop(h_, stop_at_eps ? 1 : 0, eps_rel)); }

    // save(Anderson_m) (ALMGeometrySolver.h:343-365, GeometrySolver.h:322-346): "elapsed\tvalue"
    // rows, 16 digits, to ./result/residual-<m>.txt or ./result/residual-no.txt
    void save(int Anderson_m) const {
        const std::string file = Anderson_m > 0 ? "./result/residual-" + std::to_string(Anderson_m) + ".txt"
                                                : std::string("./result/residual-no.txt");
        std::ofstream ofs(file, std::ios::out | std::ios::ate);
        if (!ofs.is_open()) { std::cout << "Cannot open: " << file << std::endl; return; }
        ofs << std::setprecision(16);
        for (size_t i = 0; i < elapsed_time_.size(); i++) ofs << elapsed_time_[i] << '\t' << function_values_[i] << std::endl;
    }

    std::vector<Scalar> function_values_;   // residual per (accepted) iteration
    std::vector<Scalar> elapsed_time_;      // seconds since the loop started

private:
    aa_ctx ctx_ = nullptr;
    aa_geom h_ = nullptr;
    int n_ = 0;
    Matrix3X x_;
    std::vector<Constraint<N>*> hard_, soft_;
    std::vector<std::pair<const TriMeshAABB*, int>> surfaces_;

    static void check(int rc) {
        if (rc != AA_OK) throw std::runtime_error(aa_last_error());
    }
    static std::vector<Scalar> uniform(size_t k) {
        std::vector<Scalar> c(1, Scalar(1));
        c.insert(c.end(), k - 1, Scalar(-1.0 / double(k - 1)));
        return c;
    }
    int surface_id(const std::shared_ptr<TriMeshAABB>& s) {
        for (auto& e : surfaces_) if (e.first == s.get()) return e.second;
        int id = -1;
        check(aa_geom_add_ref_surface(h_, s->V_.data(), (int)(s->V_.size() / 3), s->F_.data(), (int)(s->F_.size() / 3), &id));
        surfaces_.push_back({s.get(), id});
        return id;
    }
    void flush(const std::vector<Constraint<N>*>& cs, int hard) {
        size_t i = 0;
        while (i < cs.size()) {
            const Constraint<N>* c0 = cs[i];
            const int t = c0->type;
            if (t == AA_CON_REF_SURFACE) {   // one constraint over points 0..n-1
                const std::vector<double> sid(c0->idI_.size(), (double)surface_id(c0->surface_));   // [count][1]
                check(aa_geom_add_constraints(h_, hard, t, nullptr, 1, (int)c0->idI_.size(), c0->weight_, sid.data()));
                ++i;
                continue;
            }
            const size_t k = c0->idI_.size();
            std::vector<int> idx;
            std::vector<double> prm;
            size_t j = i;
            for (; j < cs.size(); ++j) {
                const Constraint<N>* c = cs[j];
                if (c->type != t || c->weight_ != c0->weight_ || c->idI_.size() != k) break;
                idx.insert(idx.end(), c->idI_.begin(), c->idI_.end());
                if (t == AA_CON_POINT_TO_REF) prm.push_back(surface_id(c->surface_));
                else prm.insert(prm.end(), c->params_.begin(), c->params_.end());
            }
            check(aa_geom_add_constraints(h_, hard, t, idx.data(), (int)k, (int)(j - i), c0->weight_,
                                          prm.empty() ? nullptr : prm.data()));
            i = j;
        }
    }
};
}  // namespace detail

// ALMGeometrySolver<3> (Geometry/ALMGeometrySolver.h): hard constraints through the augmented
// Lagrangian, weighted soft rows, combined residual, accept/reject with Anderson reset
template <unsigned int N>
class ALMGeometrySolver : public detail::GeometrySolverFacade<N, AA_GEOM_ALM> {
public:
    explicit ALMGeometrySolver(int device = 0) : detail::GeometrySolverFacade<N, AA_GEOM_ALM>(device) {}
};

// GeometrySolver<3> (Geometry/GeometrySolver.h): all rows unweighted x penalty, soft constraints
// through Constraint::project_and_combine, residual |Dx - z|, Anderson on (u, x) with `replace`
template <unsigned int N>
class GeometrySolver : public detail::GeometrySolverFacade<N, AA_GEOM_PLAIN> {
public:
    explicit GeometrySolver(int device = 0) : detail::GeometrySolverFacade<N, AA_GEOM_PLAIN>(device) {}
};

#endif  // AA_GEOMETRY_HPP
