/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle/README.md).
 *
 * Restatement of the reference's robot, controller and noise models:
 *   simple_pid_controller::SimplePIDController        PID:53-136
 *   TruncatedNormalUncertainVelocityActuator           UNC:48-121
 *   SampledUncertainVelocityActuator, GetMatchingBin   UNC:123-281
 *   arc_helpers::TruncatedNormalDistribution           (absent dependency; TYPE_1
 *       naive accept-reject restated, the only case the actuator reaches: bounds
 *       [-1,1] at sigma 0.5 -> standardized [-2,2], UNC:61, TNUVA:469)
 *   TnuvaLinkedRobot / TnuvaSE2Robot / TnuvaSE3Robot  TNUVA:26-615 over the
 *       absent arc_utilities PointSphereBasic{Linked,SE2,SE3}Robot models.
 * The robots keep the reference's object structure (Clone() = deep copy,
 * name-based GetLinkTransform, std::vector configurations) because the oracle
 * doubles as the timed CPU baseline of the reference path.
 */
#ifndef FKS_ORACLE_MODELS_H
#define FKS_ORACLE_MODELS_H

#include <stdint.h>

#include <memory>
#include <random>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "fks_capi.h"
#include "fks_portable_math.h"
#include "oracle_geometry.h"
#include "oracle_rng.h"

namespace oracle {

typedef std::vector<double> Config;

/* ---------------- PID (PID:53-136) ---------------- */
class SimplePIDController {
  public:
    SimplePIDController() : kp_(0), ki_(0), kd_(0), integral_clamp_(0), error_integral_(0), last_error_(0) {}
    SimplePIDController(double kp, double ki, double kd, double integral_clamp) { Initialize(kp, ki, kd, integral_clamp); }
    void Zero() {
        last_error_ = 0.0;
        error_integral_ = 0.0;
    }
    void Initialize(double kp, double ki, double kd, double integral_clamp) {
        kp_ = fks_math::dabs(kp);
        ki_ = fks_math::dabs(ki);
        kd_ = fks_math::dabs(kd);
        integral_clamp_ = fks_math::dabs(integral_clamp);
        error_integral_ = 0.0;
        last_error_ = 0.0;
    }
    double ComputeFeedbackTerm(double current_error, double timestep) {
        const double timestep_error_integral = ((current_error * 0.5) + (last_error_ * 0.5)) * timestep;
        const double new_error_integral = error_integral_ + timestep_error_integral;
        error_integral_ = fks_math::dmax(-integral_clamp_, fks_math::dmin(integral_clamp_, new_error_integral));
        const double error_derivative = (current_error - last_error_) / timestep;
        last_error_ = current_error;
        return (current_error * kp_) + (error_integral_ * ki_) + (error_derivative * kd_);
    }
    /* the controller state a mutable robot carries between calls (fks_forward_simulate_mutable) */
    double ErrorIntegral() const { return error_integral_; }
    double LastError() const { return last_error_; }
    void SetState(double error_integral, double last_error) {
        error_integral_ = error_integral;
        last_error_ = last_error;
    }

  private:
    double kp_, ki_, kd_, integral_clamp_, error_integral_, last_error_;
};

/* ---------------- noise sources ---------------- */
enum RngMode { RNG_COUNTER = 0, RNG_REFERENCE = 1 };

/* The "rng" argument of ApplyControlInput(input, rng).  In counter (parity) mode
 * it identifies the draw (particle, controller step, microstep); in reference
 * mode it is the per-OpenMP-thread std::mt19937_64 of SPCS:391,850. */
struct NoiseContext {
    int mode;
    uint32_t key0, key1;
    uint64_t particle;
    uint32_t step, micro;
    std::mt19937_64* mt;
    uint32_t* error_flags;
};

/* counter-mode truncated normal: TN(mean 0, sigma 0.5) on [-1,1] sampled by the
 * TYPE_1 naive accept-reject of TruncatedNormalDistribution over Marsaglia-polar
 * normal draws (the libstdc++ std::normal_distribution algorithm) fed by
 * Philox uniforms.  DESIGN.md §RNG. */
inline double counter_truncated_normal(const NoiseContext& ctx, uint32_t dof, double mean, double stddev,
                                       double std_lower, double std_upper) {
    for (uint32_t attempt = 0; attempt < 64; ++attempt) {
        Philox4 c;
        c.v[0] = (uint32_t)ctx.particle;
        c.v[1] = ctx.step;
        c.v[2] = ctx.micro;
        c.v[3] = ((uint32_t)(ctx.particle >> 32) << 16) | ((dof & 0xffu) << 8) | attempt;
        const Philox4 r = philox4x32_10(c, ctx.key0, ctx.key1);
        const double x = 2.0 * u53(r.v[0], r.v[1]) - 1.0;
        const double y = 2.0 * u53(r.v[2], r.v[3]) - 1.0;
        const double r2 = x * x + y * y;
        if (r2 > 1.0 || r2 == 0.0) continue;
        const double mult = fks_math::dsqrt(-2.0 * fks_math::log(r2) / r2);
        const double n1 = (y * mult) * 1.0 + 0.0;
        const double n2 = (x * mult) * 1.0 + 0.0;
        if ((n1 <= std_upper) && (n1 >= std_lower)) return mean + stddev * n1;
        if ((n2 <= std_upper) && (n2 >= std_lower)) return mean + stddev * n2;
    }
    *ctx.error_flags |= FKS_PARTICLE_ERR_RNG_EXHAUSTED;
    return 0.0;
}

/* arc_helpers::TruncatedNormalDistribution (reference mode keeps the libstdc++
 * normal_distribution member, whose saved polar value is copied by Clone()). */
class TruncatedNormalDistribution {
  public:
    TruncatedNormalDistribution() : TruncatedNormalDistribution(0.0, 1.0, 0.0, 0.0) {}
    TruncatedNormalDistribution(double mean, double stddev, double lower, double upper)
        : mean_(mean), stddev_(stddev), normal_dist_(0.0, 1.0) {
        if (fks_math::dabs(stddev_) == 0.0) {
            std_lower_ = lower;
            std_upper_ = upper;
        } else {
            std_lower_ = (lower - mean_) / stddev_;
            std_upper_ = (upper - mean_) / stddev_;
        }
    }
    double Sample(NoiseContext& ctx, uint32_t dof) {
        if (!((std_lower_ <= 0.0) && (std_upper_ >= 0.0))) {
            /* TYPE_2..4 are unreachable from the actuator (bounds straddle the mean) */
            *ctx.error_flags |= FKS_PARTICLE_ERR_RNG_EXHAUSTED;
            return 0.0;
        }
        if (ctx.mode == RNG_COUNTER) return counter_truncated_normal(ctx, dof, mean_, stddev_, std_lower_, std_upper_);
        while (true) {
            const double draw = normal_dist_(*ctx.mt);
            if ((draw <= std_upper_) && (draw >= std_lower_)) return mean_ + stddev_ * draw;
        }
    }

  private:
    double mean_, stddev_, std_lower_, std_upper_;
    std::normal_distribution<double> normal_dist_;
};

/* ---------------- actuator (UNC:48-121) ---------------- */
class TruncatedNormalUncertainVelocityActuator {
  public:
    TruncatedNormalUncertainVelocityActuator() : velocity_limit_(0), acceleration_limit_(0), proportional_noise_bound_(0), minimum_noise_bound_(0) {}
    TruncatedNormalUncertainVelocityActuator(double velocity_limit, double acceleration_limit, double proportional_noise_bound,
                                            double minimum_noise_bound, double percent_variance)
        : noise_distribution_(0.0, fks_math::clamp(fks_math::dabs(percent_variance), 0.0, 1.0), -1.0, 1.0),
          velocity_limit_(fks_math::dabs(velocity_limit)),
          acceleration_limit_(fks_math::dabs(acceleration_limit)),
          proportional_noise_bound_(fks_math::dabs(proportional_noise_bound)),
          minimum_noise_bound_(fks_math::dabs(minimum_noise_bound)) {}
    double GetControlValue(double control_input) const {
        return fks_math::clamp(control_input, -velocity_limit_, velocity_limit_);
    }
    double GetControlValue(double control_input, NoiseContext& ctx, uint32_t dof) {
        const double real_control_input = GetControlValue(control_input);
        const double real_proportional_noise_bound = proportional_noise_bound_ * fks_math::dabs(real_control_input);
        const double real_minimum_noise_bound = minimum_noise_bound_ * velocity_limit_;
        const double real_noise_bound = fks_math::dmax(real_proportional_noise_bound, real_minimum_noise_bound);
        const double real_noise = noise_distribution_.Sample(ctx, dof) * real_noise_bound;
        return real_control_input + real_noise;
    }

  private:
    TruncatedNormalDistribution noise_distribution_;
    double velocity_limit_, acceleration_limit_, proportional_noise_bound_, minimum_noise_bound_;
};

/* ---------------- sampled actuator (UNC:123-281) ---------------- */
/* JointUncertaintySampleModel (UNC:123): ((lower, upper), velocity errors) per bin */
typedef std::vector<std::pair<std::pair<double, double>, std::vector<double>>> JointUncertaintySampleModel;

/* GetMatchingBin (UNC:140-154): first bin whose closed interval holds the value;
 * the reference asserts when none does (here: error flag, returns false) */
inline bool GetMatchingBin(const JointUncertaintySampleModel& bins, double commanded_velocity, size_t* idx) {
    for (size_t i = 0; i < bins.size(); ++i) {
        const std::pair<double, double>& bin_bounds = bins[i].first;
        if (commanded_velocity >= bin_bounds.first && commanded_velocity <= bin_bounds.second) {
            *idx = i;
            return true;
        }
    }
    return false;
}

/* counter-mode uniform_int_distribution(0, size - 1): first Philox block of the
 * (particle, step, micro, dof) counter, as the HIP kernel's sampled_pick */
inline size_t counter_pick(const NoiseContext& ctx, uint32_t dof, size_t size) {
    Philox4 c;
    c.v[0] = (uint32_t)ctx.particle;
    c.v[1] = ctx.step;
    c.v[2] = ctx.micro;
    c.v[3] = ((uint32_t)(ctx.particle >> 32) << 16) | ((dof & 0xffu) << 8);
    const Philox4 r = philox4x32_10(c, ctx.key0, ctx.key1);
    uint32_t pick = (uint32_t)(u53(r.v[0], r.v[1]) * (double)(uint32_t)size);
    if (pick >= (uint32_t)size) pick = (uint32_t)size - 1u;
    return (size_t)pick;
}

class SampledUncertainVelocityActuator {
  public:
    SampledUncertainVelocityActuator(std::shared_ptr<const JointUncertaintySampleModel> model_ptr, double max_velocity)
        : actuator_limit_(fks_math::dabs(max_velocity)), model_ptr_(model_ptr) {}
    /* UNC:257-264 */
    double GetControlValue(double control_input) const {
        double real_control_input = fks_math::dmin(actuator_limit_, control_input);
        real_control_input = fks_math::dmax(-actuator_limit_, real_control_input);
        return real_control_input;
    }
    /* UNC:266-279 */
    double GetControlValue(double control_input, NoiseContext& ctx, uint32_t dof) const {
        const double real_control_input = GetControlValue(control_input);
        const double noise = GetNoiseValue(real_control_input, ctx, dof);
        return real_control_input + noise;
    }

  private:
    /* UNC:228-243.  The reference takes the RNG BY VALUE, so reference mode draws
     * from a copy and leaves the thread's generator where it was. */
    double GetNoiseValue(double commanded_velocity, NoiseContext& ctx, uint32_t dof) const {
        if (!model_ptr_) return 0.0;
        size_t bin_idx = 0;
        if (!GetMatchingBin(*model_ptr_, commanded_velocity, &bin_idx)) {
            *ctx.error_flags |= FKS_PARTICLE_ERR_NO_NOISE_BIN;
            return 0.0;
        }
        const std::vector<double>& best_match_bin = (*model_ptr_)[bin_idx].second;
        size_t pick_idx;
        if (ctx.mode == RNG_COUNTER) {
            pick_idx = counter_pick(ctx, dof, best_match_bin.size());
        } else {
            std::mt19937_64 rng = *ctx.mt;
            std::uniform_int_distribution<size_t> pick_dist(0, best_match_bin.size() - 1);
            pick_idx = pick_dist(rng);
        }
        return best_match_bin[pick_idx];
    }
    double actuator_limit_;
    std::shared_ptr<const JointUncertaintySampleModel> model_ptr_;
};

/* the dof's actuator: truncated-normal (TNUVA:128-130, 318-323, 469) or, when the
 * robot description carries one, the sampled actuator */
class ActuatorModel {
  public:
    ActuatorModel() {}
    ActuatorModel(const fks_dof_controller& c, const fks_sampled_actuator* sa)
        : tn_(c.velocity_limit, c.acceleration_limit, c.max_actuator_proportional_noise, c.max_actuator_minimum_noise, 0.5) {
        if (sa && sa->num_bins > 0) {
            std::shared_ptr<JointUncertaintySampleModel> m(new JointUncertaintySampleModel());
            for (uint32_t b = 0; b < sa->num_bins; ++b) {
                std::vector<double> samples(sa->bin_samples + (size_t)b * sa->bin_elements,
                                            sa->bin_samples + (size_t)(b + 1) * sa->bin_elements);
                m->push_back(std::make_pair(std::make_pair(sa->bin_bounds[2 * b], sa->bin_bounds[2 * b + 1]), samples));
            }
            sampled_ = std::make_shared<SampledUncertainVelocityActuator>(m, c.velocity_limit);
        }
    }
    double GetControlValue(double control_input) const {
        return sampled_ ? sampled_->GetControlValue(control_input) : tn_.GetControlValue(control_input);
    }
    double GetControlValue(double control_input, NoiseContext& ctx, uint32_t dof) {
        return sampled_ ? sampled_->GetControlValue(control_input, ctx, dof) : tn_.GetControlValue(control_input, ctx, dof);
    }

  private:
    TruncatedNormalUncertainVelocityActuator tn_;
    std::shared_ptr<const SampledUncertainVelocityActuator> sampled_;
};

struct JointControllerGroup {
    SimplePIDController controller;
    ActuatorModel actuator;
    JointControllerGroup() {}
    JointControllerGroup(const fks_dof_controller& c, const fks_sampled_actuator* sa)
        : controller(c.kp, c.ki, c.kd, c.integral_clamp), actuator(c, sa) {}
};

/* PointSphereGeometry with POINTS */
struct PointSphereGeometry {
    std::shared_ptr<std::vector<V4>> points;
};
typedef std::vector<std::pair<std::string, PointSphereGeometry>> LinkGeometries;

/* ---------------- robot base ---------------- */
class RobotModel {
  public:
    virtual ~RobotModel() {}
    virtual RobotModel* Clone() const = 0;
    virtual const Config& SetPosition(const Config& position) = 0;
    virtual const Config& GetPosition() const = 0;
    virtual Iso GetLinkTransform(const std::string& link_name) const = 0;
    /* 3 x D row-major */
    virtual std::vector<double> ComputeLinkPointTranslationJacobian(const std::string& link_name, const V4& p) const = 0;
    virtual double ComputeConfigurationDistanceTo(const Config& target) const = 0;
    virtual void ApplyControlInput(const std::vector<double>& input) = 0;
    virtual void ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) = 0;
    virtual std::vector<double> GenerateControlAction(const Config& target, double controller_interval) = 0;
    virtual const Config& ResetPosition(const Config& position) = 0;
    virtual bool CheckIfSelfCollisionAllowed(size_t a, size_t b) const = 0;
    virtual const LinkGeometries& GetLinkGeometries() const = 0;
    virtual size_t NumDofs() const = 0;
    /* PID state per dof: out[d] = error integral, out[D + d] = last error */
    void GetControllerState(double* out) const {
        const size_t D = NumDofs();
        for (size_t d = 0; d < D; ++d) {
            out[d] = Controller(d).ErrorIntegral();
            out[D + d] = Controller(d).LastError();
        }
    }
    void SetControllerState(const double* in) {
        const size_t D = NumDofs();
        for (size_t d = 0; d < D; ++d) Controller(d).SetState(in[d], in[D + d]);
    }

  protected:
    virtual SimplePIDController& Controller(size_t dof) = 0;
    const SimplePIDController& Controller(size_t dof) const { return const_cast<RobotModel*>(this)->Controller(dof); }
};

/* ---------------- linked robot (TNUVA:415-615 over PointSphereBasicLinkedRobot) ---------------- */
struct SimpleJointModel {
    int type;
    double lower, upper;
    bool IsFixed() const { return type == FKS_JOINT_FIXED; }
    bool IsContinuous() const { return type == FKS_JOINT_CONTINUOUS; }
    bool IsRevolute() const { return type == FKS_JOINT_REVOLUTE || type == FKS_JOINT_CONTINUOUS; }
    bool IsPrismatic() const { return type == FKS_JOINT_PRISMATIC; }
    double EnforceLimits(double v) const {
        if (IsContinuous()) return fks_math::enforce_continuous_revolute_bounds(v);
        return fks_math::clamp(v, lower, upper);
    }
    /* SimpleJointModel::SignedDistance: continuous -> shortest wrapped angle */
    double SignedDistance(double v1, double v2) const {
        if (IsContinuous()) return fks_math::enforce_continuous_revolute_bounds(v2 - v1);
        return v2 - v1;
    }
};

struct RobotJoint {
    int64_t parent, child;
    Iso origin;
    V3 axis;
    SimpleJointModel model;
    double value;
};

class LinkedRobot : public RobotModel {
  public:
    LinkedRobot(const fks_robot_desc& d);
    RobotModel* Clone() const override { return new LinkedRobot(*this); }
    const Config& SetPosition(const Config& position) override;
    const Config& GetPosition() const override { return config_; }
    Iso GetLinkTransform(const std::string& link_name) const override;
    std::vector<double> ComputeLinkPointTranslationJacobian(const std::string& link_name, const V4& p) const override;
    double ComputeConfigurationDistanceTo(const Config& target) const override;
    void ApplyControlInput(const std::vector<double>& input) override;
    void ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) override;
    std::vector<double> GenerateControlAction(const Config& target, double controller_interval) override;
    const Config& ResetPosition(const Config& position) override;
    bool CheckIfSelfCollisionAllowed(size_t a, size_t b) const override;
    const LinkGeometries& GetLinkGeometries() const override { return link_geometries_; }
    size_t NumDofs() const override { return num_active_joints_; }

  protected:
    SimplePIDController& Controller(size_t dof) override { return joint_controller_groups_[dof].controller; }

  private:
    void UpdateTransforms();
    bool IsAncestorOrSelf(int64_t maybe_ancestor, int64_t link) const;
    Iso base_transform_;
    std::vector<std::string> link_names_;
    std::vector<Iso> link_transforms_;
    std::vector<int64_t> link_parent_;
    std::vector<RobotJoint> joints_;
    LinkGeometries link_geometries_;
    std::set<std::pair<size_t, size_t>> allowed_self_collisions_;
    std::vector<JointControllerGroup> joint_controller_groups_;
    std::vector<double> joint_distance_weights_;
    size_t num_active_joints_;
    Config config_;
};

/* ---------------- SE(2) robot (TNUVA:26-199) ---------------- */
class SE2Robot : public RobotModel {
  public:
    SE2Robot(const fks_robot_desc& d);
    RobotModel* Clone() const override { return new SE2Robot(*this); }
    const Config& SetPosition(const Config& position) override;
    const Config& GetPosition() const override { return config_; }
    Iso GetLinkTransform(const std::string& link_name) const override;
    std::vector<double> ComputeLinkPointTranslationJacobian(const std::string& link_name, const V4& p) const override;
    double ComputeConfigurationDistanceTo(const Config& target) const override;
    void ApplyControlInput(const std::vector<double>& input) override;
    void ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) override;
    std::vector<double> GenerateControlAction(const Config& target, double controller_interval) override;
    const Config& ResetPosition(const Config& position) override;
    bool CheckIfSelfCollisionAllowed(size_t, size_t) const override { return true; }
    const LinkGeometries& GetLinkGeometries() const override { return link_geometries_; }
    size_t NumDofs() const override { return 3; }

  protected:
    SimplePIDController& Controller(size_t dof) override { return axis_[dof].controller; }

  private:
    LinkGeometries link_geometries_;
    JointControllerGroup axis_[3];
    double position_weight_, rotation_weight_;
    Config config_;
    Iso pose_;
};

/* ---------------- SE(3) robot (TNUVA:201-413) ---------------- */
class SE3Robot : public RobotModel {
  public:
    SE3Robot(const fks_robot_desc& d);
    RobotModel* Clone() const override { return new SE3Robot(*this); }
    const Config& SetPosition(const Config& position) override;
    const Config& GetPosition() const override { return config_; }
    Iso GetLinkTransform(const std::string& link_name) const override;
    std::vector<double> ComputeLinkPointTranslationJacobian(const std::string& link_name, const V4& p) const override;
    double ComputeConfigurationDistanceTo(const Config& target) const override;
    void ApplyControlInput(const std::vector<double>& input) override;
    void ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) override;
    std::vector<double> GenerateControlAction(const Config& target, double controller_interval) override;
    const Config& ResetPosition(const Config& position) override;
    bool CheckIfSelfCollisionAllowed(size_t, size_t) const override { return true; }
    const LinkGeometries& GetLinkGeometries() const override { return link_geometries_; }
    size_t NumDofs() const override { return 6; }

  protected:
    SimplePIDController& Controller(size_t dof) override { return axis_[dof].controller; }

  private:
    LinkGeometries link_geometries_;
    JointControllerGroup axis_[6];
    double position_weight_, rotation_weight_;
    Config config_;
    Iso pose_;
};

LinkGeometries make_link_geometries(const fks_robot_desc& d, const std::vector<std::string>& link_names);

}  // namespace oracle

#endif
