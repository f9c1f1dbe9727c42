/* Mock of the arc_utilities robot models the reference derives from (test only;
 * tests/cpp/mock_workspace/README.md): the interface the simulator receives (SPCS:377),
 * the configuration types (UPC.cpp:81-82, 131), the joint model / RobotLink / RobotJoint
 * (TNUVA:486-493, 548-559), PointSphereGeometry (SPCS:600-601) and the
 * PointSphereBasic*Robot bases with the constructor arguments TNUVA passes them
 * (TNUVA:115-119, 299-303, 494-500).  The interface carries more pure virtuals than the
 * simulator calls, as the real one does; the bases implement them. */
#ifndef MOCK_ARC_UTILITIES_SIMPLE_ROBOT_MODELS
#define MOCK_ARC_UTILITIES_SIMPLE_ROBOT_MODELS
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#include <Eigen/Geometry>

namespace EigenHelpers {
typedef std::vector<Eigen::Vector4d, Eigen::aligned_allocator<Eigen::Vector4d>> VectorVector4d;
}

namespace simple_robot_model_interface {
template <typename Configuration, typename ConfigAlloc = std::allocator<Configuration>>
class SimpleRobotModelInterface {
  public:
    virtual ~SimpleRobotModelInterface() {}
    virtual SimpleRobotModelInterface<Configuration, ConfigAlloc>* Clone() const = 0;
    virtual const Configuration& GetPosition() const = 0;
    virtual const Configuration& SetPosition(const Configuration& config) = 0;
    virtual std::vector<std::string> GetLinkNames() const = 0;
    virtual double ComputeConfigurationDistanceTo(const Configuration& target) const = 0;
    virtual Eigen::VectorXd ComputePerDimensionConfigurationSignedDistance(const Configuration& config1,
                                                                            const Configuration& config2) const = 0;
};
}  // namespace simple_robot_model_interface

namespace simple_se2_robot_model {
typedef Eigen::Matrix<double, 3, 1> SimpleSE2Configuration;
typedef std::allocator<Eigen::Matrix<double, 3, 1>> SimpleSE2ConfigAlloc;
}  // namespace simple_se2_robot_model

namespace simple_se3_robot_model {
typedef Eigen::Isometry3d SimpleSE3Configuration;
typedef Eigen::aligned_allocator<Eigen::Isometry3d> SimpleSE3ConfigAlloc;
}  // namespace simple_se3_robot_model

namespace simple_linked_robot_model {
class SimpleJointModel {
  public:
    enum JOINT_TYPE : uint32_t { PRISMATIC = 4, REVOLUTE = 1, CONTINUOUS = 2, FIXED = 0 };
    SimpleJointModel() {}
    SimpleJointModel(const std::pair<double, double>& limits, const double value, const JOINT_TYPE type)
        : limits_(limits), type_(type) {
        SetValue(value);
    }
    double GetValue() const { return value_; }
    JOINT_TYPE GetType() const { return type_; }
    const std::pair<double, double>& GetLimits() const { return limits_; }
    bool IsFixed() const { return type_ == FIXED; }
    bool IsContinuous() const { return type_ == CONTINUOUS; }
    bool IsRevolute() const { return type_ == REVOLUTE || type_ == CONTINUOUS; }
    bool IsPrismatic() const { return type_ == PRISMATIC; }
    SimpleJointModel CopyWithNewValue(const double value) const { return SimpleJointModel(limits_, value, type_); }

  private:
    void SetValue(double v) {
        if (type_ == CONTINUOUS) {
            v = std::remainder(v, 2.0 * M_PI);
        } else if (type_ != FIXED) {
            v = v < limits_.first ? limits_.first : (v > limits_.second ? limits_.second : v);
        }
        value_ = v;
    }
    std::pair<double, double> limits_{0.0, 0.0};
    JOINT_TYPE type_ = FIXED;
    double value_ = 0.0;
};
typedef std::vector<SimpleJointModel> SimpleLinkedConfiguration;
typedef std::allocator<SimpleLinkedConfiguration> SimpleLinkedConfigAlloc;
struct RobotLink {
    std::shared_ptr<EigenHelpers::VectorVector4d> link_points;
    std::string link_name;
};
struct RobotJoint {
    std::string name;
    int64_t parent_link_index = -1;
    int64_t child_link_index = -1;
    Eigen::Isometry3d joint_transform;
    Eigen::Vector3d joint_axis;
    SimpleJointModel joint_model;
};
}  // namespace simple_linked_robot_model

namespace simple_robot_models {
class PointSphereGeometry {
  public:
    enum MODEL_GEOMETRY_TYPE { POINTS, SPHERES };
    PointSphereGeometry() : type_(POINTS), points_(new EigenHelpers::VectorVector4d()) {}
    PointSphereGeometry(const MODEL_GEOMETRY_TYPE type, const std::shared_ptr<const EigenHelpers::VectorVector4d>& points)
        : type_(type), points_(points) {}
    const MODEL_GEOMETRY_TYPE& GeometryType() const { return type_; }
    const std::shared_ptr<const EigenHelpers::VectorVector4d>& Geometry() const { return points_; }

  private:
    MODEL_GEOMETRY_TYPE type_;
    std::shared_ptr<const EigenHelpers::VectorVector4d> points_;
};

template <typename Configuration, typename ConfigAlloc>
class PointSphereBasicRobot : public simple_robot_model_interface::SimpleRobotModelInterface<Configuration, ConfigAlloc> {
  public:
    const Configuration& GetPosition() const override { return config_; }
    const Configuration& SetPosition(const Configuration& config) override {
        config_ = config;
        return config_;
    }
    std::vector<std::string> GetLinkNames() const override {
        std::vector<std::string> names;
        for (const auto& g : link_geometries_) names.push_back(g.first);
        return names;
    }
    double ComputeConfigurationDistanceTo(const Configuration&) const override { return 0.0; }
    Eigen::VectorXd ComputePerDimensionConfigurationSignedDistance(const Configuration&, const Configuration&) const override {
        return Eigen::VectorXd();
    }
    const std::vector<std::pair<std::string, PointSphereGeometry>>& GetLinkGeometries() const { return link_geometries_; }

  protected:
    std::vector<std::pair<std::string, PointSphereGeometry>> link_geometries_;
    Configuration config_;
};

class PointSphereBasicSE2Robot
    : public PointSphereBasicRobot<simple_se2_robot_model::SimpleSE2Configuration, simple_se2_robot_model::SimpleSE2ConfigAlloc> {
  public:
    PointSphereBasicSE2Robot(const simple_se2_robot_model::SimpleSE2Configuration& initial_position, const double, const double,
                             const std::string& link_name, const PointSphereGeometry& geometry) {
        link_geometries_.emplace_back(link_name, geometry);
        SetPosition(initial_position);
    }
};

class PointSphereBasicSE3Robot
    : public PointSphereBasicRobot<simple_se3_robot_model::SimpleSE3Configuration, simple_se3_robot_model::SimpleSE3ConfigAlloc> {
  public:
    PointSphereBasicSE3Robot(const simple_se3_robot_model::SimpleSE3Configuration& initial_position, const double, const double,
                             const std::string& link_name, const PointSphereGeometry& geometry) {
        link_geometries_.emplace_back(link_name, geometry);
        SetPosition(initial_position);
    }
};

class PointSphereBasicLinkedRobot
    : public PointSphereBasicRobot<simple_linked_robot_model::SimpleLinkedConfiguration, simple_linked_robot_model::SimpleLinkedConfigAlloc> {
  public:
    PointSphereBasicLinkedRobot(const Eigen::Isometry3d&, const std::vector<simple_linked_robot_model::RobotLink>&,
                                const std::vector<simple_linked_robot_model::RobotJoint>& joints,
                                const simple_linked_robot_model::SimpleLinkedConfiguration& initial_position, const std::vector<double>&,
                                const std::vector<std::pair<std::string, PointSphereGeometry>>& link_geometries,
                                const std::vector<std::pair<size_t, size_t>>&) {
        for (const auto& j : joints) num_active_joints_ += j.joint_model.IsFixed() ? 0u : 1u;
        link_geometries_ = link_geometries;
        SetPosition(initial_position);
    }

  protected:
    size_t num_active_joints_ = 0;
};
}  // namespace simple_robot_models
#endif
