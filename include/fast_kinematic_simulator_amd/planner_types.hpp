/*
 * planner_types.hpp — host value types of the planner-facing interface
 * (include/fast_kinematic_simulator_amd/simulator_interface.hpp).
 *
 * The reference's SimulatorInterface (uncertainty_planning_core, re-declared here
 * from its overrides at SPCS:446-1416) carries Eigen and ROS message types:
 * Eigen::VectorXd control inputs (SPCS:719, 1546), Eigen::Vector4d points
 * (SPCS:776), Eigen::Isometry3d SE(3) configurations, std_msgs::ColorRGBA and
 * visualization_msgs::Marker/MarkerArray display representations (SPCS:559-786).
 * Neither Eigen nor ROS is part of this repository, so this header
 * defines the value types the re-declared interface is written over.  They keep the
 * reference's member names where the simulator uses them (MarkerArray::markers,
 * Marker::points/colors/scale/color, ColorRGBA::r/g/b/a, Isometry3d::matrix()(r, c),
 * VectorXd::size()/operator()), so a planner built against the real libraries swaps
 * this one header for aliases ("Planner-facing C++ interface").
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_PLANNER_TYPES_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_PLANNER_TYPES_HPP

#include <array>
#include <cstdint>
#include <initializer_list>
#include <string>
#include <vector>

namespace fks_planner_types {

/* Eigen::VectorXd: dynamic column vector of doubles */
class VectorXd {
  public:
    VectorXd() {}
    explicit VectorXd(size_t n) : v_(n, 0.0) {}
    VectorXd(std::initializer_list<double> values) : v_(values) {}
    explicit VectorXd(const std::vector<double>& values) : v_(values) {}
    static VectorXd Zero(size_t n) { return VectorXd(n); }
    int64_t size() const { return (int64_t)v_.size(); }
    void resize(size_t n) { v_.resize(n, 0.0); }
    double& operator()(int64_t i) { return v_[(size_t)i]; }
    double operator()(int64_t i) const { return v_[(size_t)i]; }
    double& operator[](int64_t i) { return v_[(size_t)i]; }
    double operator[](int64_t i) const { return v_[(size_t)i]; }
    const double* data() const { return v_.data(); }
    double* data() { return v_.data(); }
    const std::vector<double>& values() const { return v_; }
    bool operator==(const VectorXd& o) const { return v_ == o.v_; }

  private:
    std::vector<double> v_;
};

/* Eigen::Matrix<double, N, 1> for N = 3, 4 */
template <int N>
class FixedVector {
  public:
    FixedVector() : v_{} {}
    template <typename... T>
    FixedVector(double a, T... rest) : v_{{a, (double)rest...}} {
        static_assert(sizeof...(T) + 1 == N, "one value per coefficient");
    }
    double& operator()(int i) { return v_[(size_t)i]; }
    double operator()(int i) const { return v_[(size_t)i]; }
    double& operator[](int i) { return v_[(size_t)i]; }
    double operator[](int i) const { return v_[(size_t)i]; }
    double x() const { return v_[0]; }
    double y() const { return v_[1]; }
    double z() const { return v_[2]; }
    static constexpr int64_t size() { return N; }
    const double* data() const { return v_.data(); }
    bool operator==(const FixedVector& o) const { return v_ == o.v_; }

  private:
    std::array<double, N> v_;
};
typedef FixedVector<3> Vector3d;
typedef FixedVector<4> Vector4d;

/* Eigen::Isometry3d: the affine 3x4 part [R | t] of the 4x4 matrix, row-major */
class Isometry3d {
  public:
    Isometry3d() : m_{{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}} {}
    static Isometry3d Identity() { return Isometry3d(); }
    static Isometry3d FromRowMajor34(const double* m) {
        Isometry3d t;
        for (int i = 0; i < 12; ++i) t.m_[(size_t)i] = m[i];
        return t;
    }
    /* matrix()(r, c) for r < 3 (the bottom row is [0 0 0 1]) */
    struct MatrixView {
        const Isometry3d* t;
        double operator()(int r, int c) const { return r < 3 ? t->m_[(size_t)(4 * r + c)] : (c == 3 ? 1.0 : 0.0); }
    };
    MatrixView matrix() const { return MatrixView{this}; }
    Vector3d translation() const { return Vector3d(m_[3], m_[7], m_[11]); }
    const double* data34() const { return m_.data(); }
    double* data34() { return m_.data(); }
    bool operator==(const Isometry3d& o) const { return m_ == o.m_; }

  private:
    std::array<double, 12> m_;
};

/* std_msgs::ColorRGBA */
struct ColorRGBA {
    float r = 0.0f, g = 0.0f, b = 0.0f, a = 0.0f;
};

/* geometry_msgs::Point / Vector3 */
struct Point {
    double x = 0.0, y = 0.0, z = 0.0;
};

/* visualization_msgs::Marker (the fields the reference's display helpers fill) */
struct Marker {
    enum Type { LINE_LIST = 5, CUBE_LIST = 6, SPHERE_LIST = 7 };
    enum Action { ADD = 0 };
    std::string ns;
    int32_t id = 0;
    int32_t type = SPHERE_LIST;
    int32_t action = ADD;
    std::string frame_id;
    bool frame_locked = false;
    Point scale;
    ColorRGBA color;
    std::vector<Point> points;
    std::vector<ColorRGBA> colors;
};

/* visualization_msgs::MarkerArray */
struct MarkerArray {
    std::vector<Marker> markers;
};

}  // namespace fks_planner_types

#endif
