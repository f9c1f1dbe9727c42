/*
 * tnuva_robot_models.hpp — the robot models the planner hands the simulator.
 *
 * Reference: tnuva_robot_models::TnuvaSE2Robot / TnuvaSE3Robot / TnuvaLinkedRobot
 * (TNUVA:26-615): arc_utilities PointSphereBasic*Robot models (TNUVA:27, 202, 416) plus
 * per-DOF SimplePIDController + TruncatedNormalUncertainVelocityActuator groups.  Here each
 * class derives from the same arc_utilities base (the real one in a planner workspace, the
 * stand-in otherwise: fks_external_types.hpp), passes it the same constructor arguments
 * (TNUVA:109-132, 293-325, 486-517), and instead of the host controllers and actuators
 * carries what the GPU simulates from: the flattened fks::RobotDescription built once in
 * the constructor (HipDescription(), shared by clones and owned through a shared_ptr, so
 * a simulator may keep it as its cache key) and the controller state a mutable robot
 * carries between simulator calls (ResetPosition zeroes it, TNUVA:524-536).
 * The TnuvaRobot control interface (TNUVA:15-23) steps one robot by hand, as execution
 * and demonstration code does: GenerateControlAction (the robot's PID controllers and
 * actuator clamp), ApplyControlInput(u) and ApplyControlInput(u, rng) (the actuators'
 * truncated-normal noise drawn from the caller's generator, one
 * std::normal_distribution per actuator as TruncatedNormalDistribution keeps,
 * UNC:61/77-90), and the virtual ResetControllers.  They run on the host through the
 * C-ABI (fks_robot_control_action / fks_robot_apply_control_input) with the simulation
 * kernels' arithmetic.
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_TNUVA_ROBOT_MODELS_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_TNUVA_ROBOT_MODELS_HPP

#include <algorithm>
#include <array>
#include <cmath>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/fks_external_types.hpp"
#include "fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp"
#include "fast_kinematic_simulator_amd/truncated_normal.hpp"

namespace tnuva_robot_models {

namespace detail {
inline std::vector<double> flatten_points(const simple_robot_models::PointSphereGeometry& g) {
    std::vector<double> xyzw;
    for (const auto& p : *g.Geometry()) xyzw.insert(xyzw.end(), {p(0), p(1), p(2), p(3)});
    return xyzw;
}
inline void row_major34(const fks_planner_types::Isometry3d& T, double* out) {
    const std::array<double, 12> m = fks_ext::iso_to_row_major34(T);
    std::copy(m.begin(), m.end(), out);
}
/* the per-axis gains of an SE2/SE3_ROBOT_CONFIG (TNUVA:43-107, 227-291) */
template <typename C>
fks_dof_controller translation(const C& c) {
    return fks_dof_controller{c.kp, c.ki, c.kd, c.integral_clamp, c.velocity_limit, c.acceleration_limit,
                              c.max_sensor_noise, c.max_actuator_proportional_noise, c.max_actuator_minimum_noise};
}
template <typename C>
fks_dof_controller rotation(const C& c) {
    return fks_dof_controller{c.r_kp, c.r_ki, c.r_kd, c.r_integral_clamp, c.r_velocity_limit, c.r_acceleration_limit,
                              c.r_max_sensor_noise, c.r_max_actuator_proportional_noise, c.r_max_actuator_minimum_noise};
}
}  // namespace detail

/* gains of the translational (kp ...) and rotational (r_kp ...) axes, TNUVA:43-107 / 227-291 */
struct AXIS_ROBOT_CONFIG {
    double kp = 0.0, ki = 0.0, kd = 0.0, integral_clamp = 0.0, velocity_limit = 0.0, acceleration_limit = 0.0,
           max_sensor_noise = 0.0, max_actuator_proportional_noise = 0.0, max_actuator_minimum_noise = 0.0;
    double r_kp = 0.0, r_ki = 0.0, r_kd = 0.0, r_integral_clamp = 0.0, r_velocity_limit = 0.0, r_acceleration_limit = 0.0,
           r_max_sensor_noise = 0.0, r_max_actuator_proportional_noise = 0.0, r_max_actuator_minimum_noise = 0.0;
    AXIS_ROBOT_CONFIG() {}
    AXIS_ROBOT_CONFIG(double in_kp, double in_ki, double in_kd, double in_integral_clamp, double in_velocity_limit,
                      double in_acceleration_limit, double in_max_sensor_noise, double in_max_actuator_proportional_noise,
                      double in_max_actuator_minimum_noise, double in_r_kp, double in_r_ki, double in_r_kd,
                      double in_r_integral_clamp, double in_r_velocity_limit, double in_r_acceleration_limit,
                      double in_r_max_sensor_noise, double in_r_max_actuator_proportional_noise,
                      double in_r_max_actuator_minimum_noise)
        : kp(in_kp), ki(in_ki), kd(in_kd), integral_clamp(in_integral_clamp), velocity_limit(in_velocity_limit),
          acceleration_limit(in_acceleration_limit), max_sensor_noise(in_max_sensor_noise),
          max_actuator_proportional_noise(in_max_actuator_proportional_noise),
          max_actuator_minimum_noise(in_max_actuator_minimum_noise), r_kp(in_r_kp), r_ki(in_r_ki), r_kd(in_r_kd),
          r_integral_clamp(in_r_integral_clamp), r_velocity_limit(in_r_velocity_limit),
          r_acceleration_limit(in_r_acceleration_limit), r_max_sensor_noise(in_r_max_sensor_noise),
          r_max_actuator_proportional_noise(in_r_max_actuator_proportional_noise),
          r_max_actuator_minimum_noise(in_r_max_actuator_minimum_noise) {}
};

/* What the HIP simulator needs from a DerivedRobotType: the flattened description (owned,
 * immutable after construction), the PID state (per dof: error integral, then per dof:
 * last error) and the conversion of configurations to and from the flat form of fks_capi.h. */
template <typename Configuration>
class HipRobotState {
  public:
    virtual ~HipRobotState() {}
    /* TnuvaRobot (TNUVA:15-23); Generator is the robot class's template argument */
    virtual const Configuration& ResetPosition(const Configuration& position) = 0;
    const fks::RobotDescription& HipDescription() const { return *desc_; }
    const std::shared_ptr<const fks::RobotDescription>& SharedHipDescription() const { return desc_; }
    const std::vector<double>& ControllerState() const { return pid_; }
    void SetControllerState(const std::vector<double>& state) {
        if (state.size() != pid_.size()) throw std::invalid_argument("controller state has the wrong size");
        pid_ = state;
    }
    /* TNUVA:145-150, 338-346, 530-536: every controller's integral and last error to zero */
    virtual void ResetControllers() { std::fill(pid_.begin(), pid_.end(), 0.0); }
    bool ControllersAreZero() const {
        for (double v : pid_)
            if (v != 0.0) return false;
        return true;
    }
    virtual std::vector<double> ToFlat(const Configuration& config) const = 0;
    virtual Configuration FromFlat(const double* flat) const = 0;

  protected:
    void InitState(const std::shared_ptr<const fks::RobotDescription>& desc) {
        desc_ = desc;
        pid_.assign(2 * (size_t)desc->NumDofs(), 0.0);
        /* TruncatedNormalUncertainVelocityActuator(..., 0.5): TN(0, 0.5) on [-1, 1] (TNUVA:130, 322, 469) */
        noise_.assign((size_t)desc->NumDofs(), fks::TruncatedNormalDistribution(0.0, 0.5, -1.0, 1.0));
    }
    static void Check(fks_status st, const char* what) {
        if (st != FKS_OK) throw std::runtime_error(std::string(what) + ": " + fks_status_string(st));
    }
    /* GenerateControlAction from the current flat configuration (TNUVA:179-198, 384-412, 598-614) */
    fks_planner_types::VectorXd ControlAction(const std::vector<double>& current, const std::vector<double>& target,
                                              double controller_interval) {
        const fks_robot_desc d = desc_->View();
        std::vector<double> u((size_t)desc_->NumDofs());
        Check(fks_robot_control_action(&d, current.data(), target.data(), controller_interval, pid_.data(), u.data()),
              "GenerateControlAction");
        return fks_ext::vecx(u);
    }
    /* ApplyControlInput: the new flat configuration (TNUVA:152-177, 348-382, 538-596) */
    std::vector<double> Applied(const std::vector<double>& current, const fks_planner_types::VectorXd& input,
                                const std::vector<double>* unit_noise) {
        const std::vector<double> u = fks_ext::vecx_values(input);
        if (u.size() != (size_t)desc_->NumDofs()) throw std::invalid_argument("ApplyControlInput: one input per dof");
        const fks_robot_desc d = desc_->View();
        std::vector<double> out(current.size());
        Check(fks_robot_apply_control_input(&d, current.data(), u.data(), unit_noise ? unit_noise->data() : nullptr, out.data()),
              "ApplyControlInput");
        return out;
    }
    /* one draw of each actuator's TruncatedNormalDistribution(0, 0.5, -1, 1) (UNC:61, 86), in dof
     * order: fks::TruncatedNormalDistribution (truncated_normal.hpp; arc_helpers' sampler
     * restated, parity unpinned), whose standardised bounds [-2, 2] take the naive
     * accept-reject of each actuator's own normal draws */
    template <typename RNG>
    std::vector<double> DrawNoise(RNG& rng) {
        std::vector<double> n(noise_.size());
        for (size_t k = 0; k < noise_.size(); ++k) n[k] = noise_[k](rng);
        return n;
    }
    std::shared_ptr<const fks::RobotDescription> desc_;
    std::vector<double> pid_;
    std::vector<fks::TruncatedNormalDistribution> noise_;
};

/* ---------------------------------------------------------------- SE(2) (TNUVA:26-199) */
template <typename Generator>
class TnuvaSE2Robot : public simple_robot_models::PointSphereBasicSE2Robot,
                      public HipRobotState<simple_se2_robot_model::SimpleSE2Configuration> {
  public:
    typedef simple_se2_robot_model::SimpleSE2Configuration Configuration;
    typedef AXIS_ROBOT_CONFIG SE2_ROBOT_CONFIG;

    /* TNUVA:109-132 */
    TnuvaSE2Robot(const Configuration& initial_position, const double position_distance_weight,
                  const double rotation_distance_weight, const std::string& link_name,
                  const simple_robot_models::PointSphereGeometry& geometry, const SE2_ROBOT_CONFIG& robot_config)
        : simple_robot_models::PointSphereBasicSE2Robot(initial_position, position_distance_weight, rotation_distance_weight,
                                                        link_name, geometry) {
        auto d = std::make_shared<fks::RobotDescription>();
        d->type = FKS_ROBOT_SE2;
        d->num_links = 1;
        d->num_dofs = 3;
        d->AddGeometry(0, detail::flatten_points(geometry));
        d->controllers = {detail::translation(robot_config), detail::translation(robot_config), detail::rotation(robot_config)};
        d->distance_weights = {position_distance_weight, rotation_distance_weight};
        InitState(d);
    }
    simple_robot_model_interface::SimpleRobotModelInterface<Configuration, simple_se2_robot_model::SimpleSE2ConfigAlloc>* Clone()
        const override {
        return new TnuvaSE2Robot(*this);
    }
    /* TNUVA:139-150 */
    const Configuration& ResetPosition(const Configuration& position) override {
        this->ResetControllers();
        return SetPosition(position);
    }
    /* TnuvaRobot::ApplyControlInput(u), ApplyControlInput(u, rng), GenerateControlAction */
    void ApplyControlInput(const fks_planner_types::VectorXd& input) {
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, nullptr).data()));
    }
    void ApplyControlInput(const fks_planner_types::VectorXd& input, Generator& rng) {
        const std::vector<double> noise = this->DrawNoise(rng);
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, &noise).data()));
    }
    fks_planner_types::VectorXd GenerateControlAction(const Configuration& target, const double controller_interval) {
        return this->ControlAction(ToFlat(GetPosition()), ToFlat(target), controller_interval);
    }
    std::vector<double> ToFlat(const Configuration& c) const override { return {c(0), c(1), c(2)}; }
    Configuration FromFlat(const double* f) const override { return Configuration(f[0], f[1], f[2]); }
};

/* ---------------------------------------------------------------- SE(3) (TNUVA:201-413) */
template <typename Generator>
class TnuvaSE3Robot : public simple_robot_models::PointSphereBasicSE3Robot,
                      public HipRobotState<simple_se3_robot_model::SimpleSE3Configuration> {
  public:
    typedef simple_se3_robot_model::SimpleSE3Configuration Configuration;
    typedef AXIS_ROBOT_CONFIG SE3_ROBOT_CONFIG;

    /* TNUVA:293-325: x, y, z use the translational gains, rx, ry, rz the rotational */
    TnuvaSE3Robot(const Configuration& initial_position, const double position_distance_weight,
                  const double rotation_distance_weight, const std::string& link_name,
                  const simple_robot_models::PointSphereGeometry& geometry, const SE3_ROBOT_CONFIG& robot_config)
        : simple_robot_models::PointSphereBasicSE3Robot(initial_position, position_distance_weight, rotation_distance_weight,
                                                        link_name, geometry) {
        auto d = std::make_shared<fks::RobotDescription>();
        d->type = FKS_ROBOT_SE3;
        d->num_links = 1;
        d->num_dofs = 6;
        d->AddGeometry(0, detail::flatten_points(geometry));
        const fks_dof_controller t = detail::translation(robot_config), r = detail::rotation(robot_config);
        d->controllers = {t, t, t, r, r, r};
        d->distance_weights = {position_distance_weight, rotation_distance_weight};
        InitState(d);
    }
    simple_robot_model_interface::SimpleRobotModelInterface<Configuration, simple_se3_robot_model::SimpleSE3ConfigAlloc>* Clone()
        const override {
        return new TnuvaSE3Robot(*this);
    }
    /* TNUVA:332-336 */
    const Configuration& ResetPosition(const Configuration& position) override {
        this->ResetControllers();
        return SetPosition(position);
    }
    /* TnuvaRobot::ApplyControlInput(u), ApplyControlInput(u, rng), GenerateControlAction */
    void ApplyControlInput(const fks_planner_types::VectorXd& input) {
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, nullptr).data()));
    }
    void ApplyControlInput(const fks_planner_types::VectorXd& input, Generator& rng) {
        const std::vector<double> noise = this->DrawNoise(rng);
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, &noise).data()));
    }
    fks_planner_types::VectorXd GenerateControlAction(const Configuration& target, const double controller_interval) {
        return this->ControlAction(ToFlat(GetPosition()), ToFlat(target), controller_interval);
    }
    /* the 3x4 row-major [R | t] */
    std::vector<double> ToFlat(const Configuration& c) const override {
        const std::array<double, 12> m = fks_ext::iso_to_row_major34(c);
        return std::vector<double>(m.begin(), m.end());
    }
    Configuration FromFlat(const double* f) const override { return fks_ext::iso_from_row_major34(f); }
};

/* ---------------------------------------------------------------- linked (TNUVA:415-615) */
template <typename Generator>
class TnuvaLinkedRobot : public simple_robot_models::PointSphereBasicLinkedRobot,
                         public HipRobotState<simple_linked_robot_model::SimpleLinkedConfiguration> {
  public:
    typedef simple_linked_robot_model::SimpleLinkedConfiguration Configuration;

    /* TNUVA:420-457 */
    struct LINKED_ROBOT_CONFIG {
        double kp = 0.0, ki = 0.0, kd = 0.0, integral_clamp = 0.0, velocity_limit = 0.0, acceleration_limit = 0.0,
               max_sensor_noise = 0.0, max_actuator_proportional_noise = 0.0, max_actuator_minimum_noise = 0.0;
        LINKED_ROBOT_CONFIG() {}
        LINKED_ROBOT_CONFIG(double in_kp, double in_ki, double in_kd, double in_integral_clamp, double in_velocity_limit,
                            double in_acceleration_limit, double in_max_sensor_noise, double in_max_actuator_proportional_noise,
                            double in_max_actuator_minimum_noise)
            : kp(in_kp), ki(in_ki), kd(in_kd), integral_clamp(in_integral_clamp), velocity_limit(in_velocity_limit),
              acceleration_limit(in_acceleration_limit), max_sensor_noise(in_max_sensor_noise),
              max_actuator_proportional_noise(in_max_actuator_proportional_noise),
              max_actuator_minimum_noise(in_max_actuator_minimum_noise) {}
    };

    /* TNUVA:486-517.  Geometries are attached to links by name; allowed self-collision
     * pairs index link_geometries (the indices CheckIfSelfCollisionAllowed receives,
     * SPCS:1008, 1193).  Throws std::invalid_argument when the joint-config count differs
     * from the active-joint count (TNUVA:515). */
    TnuvaLinkedRobot(const fks_planner_types::Isometry3d& base_transform,
                     const std::vector<simple_linked_robot_model::RobotLink>& links,
                     const std::vector<simple_linked_robot_model::RobotJoint>& joints, const Configuration& initial_position,
                     const std::vector<double>& joint_distance_weights,
                     const std::vector<std::pair<std::string, simple_robot_models::PointSphereGeometry>>& link_geometries,
                     const std::vector<std::pair<size_t, size_t>>& allowed_self_collisions,
                     const std::vector<LINKED_ROBOT_CONFIG>& joint_configs)
        : simple_robot_models::PointSphereBasicLinkedRobot(base_transform, links, joints, initial_position, joint_distance_weights,
                                                           link_geometries, allowed_self_collisions) {
        auto d = std::make_shared<fks::RobotDescription>();
        d->type = FKS_ROBOT_LINKED;
        d->num_links = (int32_t)links.size();
        detail::row_major34(base_transform, d->base_transform);
        int32_t active = 0;
        for (const auto& j : joints) {
            fks_joint_desc jd{};
            jd.parent_link = (int32_t)j.parent_link_index;
            jd.child_link = (int32_t)j.child_link_index;
            jd.type = (int32_t)j.joint_model.GetType();
            detail::row_major34(j.joint_transform, jd.origin);
            for (int i = 0; i < 3; ++i) jd.axis[i] = j.joint_axis(i);
            jd.limit_lower = j.joint_model.GetLimits().first;
            jd.limit_upper = j.joint_model.GetLimits().second;
            d->joints.push_back(jd);
            if (!j.joint_model.IsFixed()) {
                active++;
                joint_models_.push_back(j.joint_model);
            }
        }
        if ((size_t)active != joint_configs.size())
            throw std::invalid_argument("Number of joint configs must match number of active joints");
        d->num_dofs = active;
        for (const auto& g : link_geometries) {
            int32_t link = -1;
            for (size_t l = 0; l < links.size(); ++l)
                if (links[l].link_name == g.first) link = (int32_t)l;
            if (link < 0) throw std::invalid_argument("link geometry names an unknown link: " + g.first);
            d->AddGeometry(link, detail::flatten_points(g.second));
        }
        for (const auto& p : allowed_self_collisions) d->AllowSelfCollision((int32_t)p.first, (int32_t)p.second);
        for (const auto& c : joint_configs)
            d->controllers.push_back(fks_dof_controller{c.kp, c.ki, c.kd, c.integral_clamp, c.velocity_limit, c.acceleration_limit,
                                                        c.max_sensor_noise, c.max_actuator_proportional_noise,
                                                        c.max_actuator_minimum_noise});
        d->distance_weights = joint_distance_weights;
        if (d->distance_weights.size() != (size_t)active) throw std::invalid_argument("one distance weight per active joint");
        InitState(d);
    }
    simple_robot_model_interface::SimpleRobotModelInterface<Configuration, simple_linked_robot_model::SimpleLinkedConfigAlloc>* Clone()
        const override {
        return new TnuvaLinkedRobot(*this);
    }
    /* TNUVA:524-536 */
    const Configuration& ResetPosition(const Configuration& position) override {
        this->ResetControllers();
        return SetPosition(position);
    }
    /* TnuvaRobot::ApplyControlInput(u), ApplyControlInput(u, rng), GenerateControlAction */
    void ApplyControlInput(const fks_planner_types::VectorXd& input) {
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, nullptr).data()));
    }
    void ApplyControlInput(const fks_planner_types::VectorXd& input, Generator& rng) {
        const std::vector<double> noise = this->DrawNoise(rng);
        SetPosition(FromFlat(this->Applied(ToFlat(GetPosition()), input, &noise).data()));
    }
    fks_planner_types::VectorXd GenerateControlAction(const Configuration& target, const double controller_interval) {
        return this->ControlAction(ToFlat(GetPosition()), ToFlat(target), controller_interval);
    }

    std::vector<double> ToFlat(const Configuration& c) const override {
        std::vector<double> f;
        for (const auto& j : c) f.push_back(j.GetValue());
        return f;
    }
    /* each active joint's model with the value (limits / wrap enforced, TNUVA:556) */
    Configuration FromFlat(const double* f) const override {
        Configuration c;
        for (size_t k = 0; k < joint_models_.size(); ++k) c.push_back(joint_models_[k].CopyWithNewValue(f[k]));
        return c;
    }

  private:
    std::vector<simple_linked_robot_model::SimpleJointModel> joint_models_; /* active joints, in order */
};

}  // namespace tnuva_robot_models

#endif
