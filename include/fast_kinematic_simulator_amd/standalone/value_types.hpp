/*
 * standalone/value_types.hpp — stand-ins for the Eigen and ROS message value types of
 * the planner-facing interface, used only when the planner's own libraries are absent
 * (fks_external_types.hpp selects; never include this header directly).
 *
 * The reference's SimulatorInterface (uncertainty_planning_core, re-declared in
 * standalone/planner_libraries.hpp from its overrides at SPCS:446-1416) carries Eigen
 * and ROS message types: Eigen::VectorXd control inputs (SPCS:719, 1546),
 * Eigen::Vector4d points (SPCS:776), Eigen::Isometry3d SE(3) configurations stored with
 * Eigen::aligned_allocator (UPC.cpp:131), std_msgs::ColorRGBA and
 * visualization_msgs::Marker/MarkerArray display representations (SPCS:559-786).  These
 * classes live in their own namespace (fks_standalone) so they can never collide with
 * Eigen or ROS; fks_external_types.hpp maps fks_planner_types:: onto them or onto the
 * real types.  They keep the real member names the simulator uses (Marker::header.frame_id,
 * Marker::points/colors/scale/color, ColorRGBA::r/g/b/a, Isometry3d::matrix()(r, c),
 * VectorXd::size()/operator()), so the code above them is written once for both.
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_STANDALONE_VALUE_TYPES_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_STANDALONE_VALUE_TYPES_HPP

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <initializer_list>
#include <new>
#include <string>
#include <vector>

namespace fks_standalone {

/* Eigen::VectorXd: dynamic column vector of doubles */
class VectorXd {
  public:
    VectorXd() {}
    explicit VectorXd(int64_t n) : v_((size_t)n, 0.0) {}
    VectorXd(std::initializer_list<double> values) : v_(values) {}
    static VectorXd Zero(int64_t n) { return VectorXd(n); }
    int64_t size() const { return (int64_t)v_.size(); }
    void resize(int64_t n) { v_.resize((size_t)n, 0.0); }
    double& operator()(int64_t i) { return v_[(size_t)i]; }
    double operator()(int64_t i) const { return v_[(size_t)i]; }
    double& operator[](int64_t i) { return v_[(size_t)i]; }
    double operator[](int64_t i) const { return v_[(size_t)i]; }
    const double* data() const { return v_.data(); }
    double* data() { return v_.data(); }
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

/* Eigen::Isometry3d: a 4x4 homogeneous matrix whose bottom row is [0 0 0 1]; matrix()
 * gives (r, c) access like Eigen's Matrix4d */
class Isometry3d {
  public:
    class Matrix4 {
      public:
        double& operator()(int r, int c) { return m_[(size_t)(4 * r + c)]; }
        double operator()(int r, int c) const { return m_[(size_t)(4 * r + c)]; }
        bool operator==(const Matrix4& o) const { return m_ == o.m_; }

      private:
        std::array<double, 16> m_{{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}};
    };
    Isometry3d() {}
    static Isometry3d Identity() { return Isometry3d(); }
    Matrix4& matrix() { return m_; }
    const Matrix4& matrix() const { return m_; }
    Vector3d translation() const { return Vector3d(m_(0, 3), m_(1, 3), m_(2, 3)); }
    bool operator==(const Isometry3d& o) const { return m_ == o.m_; }

  private:
    Matrix4 m_;
};

/* Eigen::Quaterniond: (w, x, y, z) coefficients, the constructor order of Eigen's */
class Quaterniond {
  public:
    Quaterniond() : w_(1.0), x_(0.0), y_(0.0), z_(0.0) {}
    Quaterniond(double w, double x, double y, double z) : w_(w), x_(x), y_(y), z_(z) {}
    double w() const { return w_; }
    double x() const { return x_; }
    double y() const { return y_; }
    double z() const { return z_; }

  private:
    double w_, x_, y_, z_;
};

/* Eigen::aligned_allocator: 16-byte aligned storage for fixed-size vectorisable types
 * (the reference stores SE(3) configurations with it, UPC.cpp:131) */
template <typename T>
class aligned_allocator {
  public:
    typedef T value_type;
    aligned_allocator() noexcept {}
    template <typename U>
    aligned_allocator(const aligned_allocator<U>&) noexcept {}
    T* allocate(size_t n) {
        const size_t bytes = ((n * sizeof(T) + 15u) / 16u) * 16u;
        void* p = std::aligned_alloc(16, bytes ? bytes : 16u);
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) noexcept { std::free(p); }
    template <typename U>
    struct rebind {
        typedef aligned_allocator<U> other;
    };
    template <typename U>
    bool operator==(const aligned_allocator<U>&) const noexcept { return true; }
    template <typename U>
    bool operator!=(const aligned_allocator<U>&) const noexcept { return false; }
};

/* std_msgs::ColorRGBA */
struct ColorRGBA {
    float r = 0.0f, g = 0.0f, b = 0.0f, a = 0.0f;
};

/* geometry_msgs::Point / geometry_msgs::Vector3 */
struct Point {
    double x = 0.0, y = 0.0, z = 0.0;
};
typedef Point Vector3;

/* std_msgs::Header (the field the display helpers set) */
struct Header {
    std::string frame_id;
};

/* visualization_msgs::Marker (the fields the reference's display helpers fill) */
struct Marker {
    enum Type { LINE_LIST = 5, CUBE_LIST = 6, SPHERE_LIST = 7 };
    enum Action { ADD = 0 };
    Header header;
    std::string ns;
    int32_t id = 0;
    int32_t type = SPHERE_LIST;
    int32_t action = ADD;
    bool frame_locked = false;
    Vector3 scale;
    ColorRGBA color;
    std::vector<Point> points;
    std::vector<ColorRGBA> colors;
};

/* visualization_msgs::MarkerArray */
struct MarkerArray {
    std::vector<Marker> markers;
};

}  // namespace fks_standalone

#endif
