/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle (see oracle/README.md).
 * Robot models: TNUVA:26-615 restated over the absent arc_utilities models.
 */
#include "oracle_models.h"

#include <cstring>

namespace oracle {

LinkGeometries make_link_geometries(const fks_robot_desc& d, const std::vector<std::string>& link_names) {
    LinkGeometries geoms;
    for (int32_t g = 0; g < d.num_geometries; ++g) {
        PointSphereGeometry geom;
        geom.points = std::make_shared<std::vector<V4>>();
        for (uint32_t i = d.geometry_point_offset[g]; i < d.geometry_point_offset[g + 1]; ++i) {
            const double* p = d.points + 4 * (size_t)i;
            geom.points->push_back(V4{p[0], p[1], p[2], p[3]});
        }
        geoms.emplace_back(link_names[(size_t)d.geometry_link[g]], geom);
    }
    return geoms;
}

/* ================= linked ================= */
LinkedRobot::LinkedRobot(const fks_robot_desc& d) {
    base_transform_ = iso_from12(d.base_transform);
    for (int32_t l = 0; l < d.num_links; ++l) link_names_.push_back("link_" + std::to_string(l));
    link_transforms_.assign((size_t)d.num_links, iso_identity());
    link_parent_.assign((size_t)d.num_links, -1);
    num_active_joints_ = 0;
    for (int32_t j = 0; j < d.num_joints; ++j) {
        const fks_joint_desc& jd = d.joints[j];
        RobotJoint rj;
        rj.parent = jd.parent_link;
        rj.child = jd.child_link;
        rj.origin = iso_from12(jd.origin);
        rj.axis = V3{jd.axis[0], jd.axis[1], jd.axis[2]};
        rj.model.type = jd.type;
        rj.model.lower = jd.limit_lower;
        rj.model.upper = jd.limit_upper;
        rj.value = 0.0;
        link_parent_[(size_t)jd.child_link] = jd.parent_link;
        if (!rj.model.IsFixed()) num_active_joints_++;
        joints_.push_back(rj);
    }
    link_geometries_ = make_link_geometries(d, link_names_);
    for (int32_t i = 0; i < d.num_allowed_pairs; ++i)
        allowed_self_collisions_.insert(
            std::make_pair((size_t)d.allowed_pairs[2 * i], (size_t)d.allowed_pairs[2 * i + 1]));
    for (size_t k = 0; k < num_active_joints_; ++k) {
        joint_controller_groups_.push_back(
            JointControllerGroup(d.controllers[k], d.sampled_actuators ? d.sampled_actuators + k : nullptr));
        joint_distance_weights_.push_back(d.distance_weights ? d.distance_weights[k] : 1.0);
    }
    config_.assign(num_active_joints_, 0.0);
    SetPosition(config_);
}

const Config& LinkedRobot::SetPosition(const Config& position) {
    /* SetConfig: copy values into the active joints (SetValue enforces limits) */
    size_t config_idx = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        RobotJoint& joint = joints_[idx];
        if (!joint.model.IsFixed()) {
            joint.value = joint.model.EnforceLimits(position[config_idx]);
            config_[config_idx] = joint.value;
            config_idx++;
        }
    }
    UpdateTransforms();
    return config_;
}

void LinkedRobot::UpdateTransforms() {
    link_transforms_[0] = base_transform_;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        const RobotJoint& joint = joints_[idx];
        const Iso& parent_transform = link_transforms_[(size_t)joint.parent];
        const Iso parent_joint = compose(parent_transform, joint.origin);
        if (joint.model.IsRevolute()) {
            Iso motion;
            const double axis[3] = {joint.axis.x, joint.axis.y, joint.axis.z};
            angle_axis_matrix(joint.value, axis, motion.r);
            motion.t[0] = motion.t[1] = motion.t[2] = 0.0;
            link_transforms_[(size_t)joint.child] = compose(parent_joint, motion);
        } else if (joint.model.IsPrismatic()) {
            Iso motion = iso_identity();
            motion.t[0] = joint.axis.x * joint.value;
            motion.t[1] = joint.axis.y * joint.value;
            motion.t[2] = joint.axis.z * joint.value;
            link_transforms_[(size_t)joint.child] = compose(parent_joint, motion);
        } else {
            link_transforms_[(size_t)joint.child] = parent_joint;
        }
    }
}

Iso LinkedRobot::GetLinkTransform(const std::string& link_name) const {
    for (size_t idx = 0; idx < link_names_.size(); ++idx)
        if (link_names_[idx] == link_name) return link_transforms_[idx];
    return iso_identity();
}

bool LinkedRobot::IsAncestorOrSelf(int64_t maybe_ancestor, int64_t link) const {
    while (link >= 0) {
        if (link == maybe_ancestor) return true;
        link = link_parent_[(size_t)link];
    }
    return false;
}

std::vector<double> LinkedRobot::ComputeLinkPointTranslationJacobian(const std::string& link_name, const V4& p) const {
    const size_t D = num_active_joints_;
    std::vector<double> J(3 * D, 0.0);
    int64_t link_index = -1;
    for (size_t idx = 0; idx < link_names_.size(); ++idx)
        if (link_names_[idx] == link_name) link_index = (int64_t)idx;
    if (link_index <= 0) return J; /* root link cannot move */
    const V4 x4 = xform4(link_transforms_[(size_t)link_index], p);
    const V3 x{x4.x, x4.y, x4.z};
    size_t joint_idx = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        const RobotJoint& joint = joints_[idx];
        if (joint.model.IsFixed()) continue;
        if (IsAncestorOrSelf(joint.child, link_index)) {
            const Iso& joint_transform = link_transforms_[(size_t)joint.child];
            const V3 axis_w = rotate(joint_transform, joint.axis);
            V3 col;
            if (joint.model.IsRevolute()) {
                const V3 d{x.x - joint_transform.t[0], x.y - joint_transform.t[1], x.z - joint_transform.t[2]};
                col = cross(axis_w, d);
            } else {
                col = axis_w;
            }
            J[0 * D + joint_idx] = J[0 * D + joint_idx] + col.x;
            J[1 * D + joint_idx] = J[1 * D + joint_idx] + col.y;
            J[2 * D + joint_idx] = J[2 * D + joint_idx] + col.z;
        }
        joint_idx++;
    }
    return J;
}

double LinkedRobot::ComputeConfigurationDistanceTo(const Config& target) const {
    double sum = 0.0;
    size_t k = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        if (joints_[idx].model.IsFixed()) continue;
        const double d = joint_distance_weights_[k] * fks_math::dabs(joints_[idx].model.SignedDistance(config_[k], target[k]));
        sum = sum + d * d;
        k++;
    }
    return fks_math::dsqrt(sum);
}

void LinkedRobot::ApplyControlInput(const std::vector<double>& input) {
    Config new_config;
    new_config.reserve(num_active_joints_);
    size_t input_idx = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        const RobotJoint& joint = joints_[idx];
        if (joint.model.IsFixed()) continue;
        const double real_input_val = joint_controller_groups_[input_idx].actuator.GetControlValue(input[input_idx]);
        const double raw_new_val = joint.value + real_input_val;
        new_config.push_back(joint.model.EnforceLimits(raw_new_val));
        input_idx++;
    }
    SetPosition(new_config);
}

void LinkedRobot::ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) {
    Config new_config;
    new_config.reserve(num_active_joints_);
    size_t input_idx = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        const RobotJoint& joint = joints_[idx];
        if (joint.model.IsFixed()) continue;
        const double noisy_input_val =
            joint_controller_groups_[input_idx].actuator.GetControlValue(input[input_idx], rng, (uint32_t)input_idx);
        const double noisy_new_val = joint.value + noisy_input_val;
        new_config.push_back(joint.model.EnforceLimits(noisy_new_val));
        input_idx++;
    }
    SetPosition(new_config);
}

std::vector<double> LinkedRobot::GenerateControlAction(const Config& target, double controller_interval) {
    std::vector<double> control_action(num_active_joints_, 0.0);
    size_t k = 0;
    for (size_t idx = 0; idx < joints_.size(); ++idx) {
        if (joints_[idx].model.IsFixed()) continue;
        const double joint_error = joints_[idx].model.SignedDistance(config_[k], target[k]);
        const double joint_term = joint_controller_groups_[k].controller.ComputeFeedbackTerm(joint_error, controller_interval);
        control_action[k] = joint_controller_groups_[k].actuator.GetControlValue(joint_term);
        k++;
    }
    return control_action;
}

const Config& LinkedRobot::ResetPosition(const Config& position) {
    for (size_t idx = 0; idx < joint_controller_groups_.size(); ++idx) joint_controller_groups_[idx].controller.Zero();
    return SetPosition(position);
}

bool LinkedRobot::CheckIfSelfCollisionAllowed(size_t a, size_t b) const {
    if (a == b) return true;
    return allowed_self_collisions_.count(std::make_pair(a, b)) > 0 ||
           allowed_self_collisions_.count(std::make_pair(b, a)) > 0;
}

/* ================= SE(2) ================= */
SE2Robot::SE2Robot(const fks_robot_desc& d) {
    std::vector<std::string> names{"link_0"};
    link_geometries_ = make_link_geometries(d, names);
    for (int i = 0; i < 3; ++i)
        axis_[i] = JointControllerGroup(d.controllers[i], d.sampled_actuators ? d.sampled_actuators + i : nullptr);
    position_weight_ = d.distance_weights ? d.distance_weights[0] : 1.0;
    rotation_weight_ = d.distance_weights ? d.distance_weights[1] : 1.0;
    config_.assign(3, 0.0);
    SetPosition(config_);
}

const Config& SE2Robot::SetPosition(const Config& position) {
    config_[0] = position[0];
    config_[1] = position[1];
    config_[2] = fks_math::enforce_continuous_revolute_bounds(position[2]);
    const double z[3] = {0.0, 0.0, 1.0};
    angle_axis_matrix(config_[2], z, pose_.r);
    pose_.t[0] = config_[0];
    pose_.t[1] = config_[1];
    pose_.t[2] = 0.0;
    return config_;
}

Iso SE2Robot::GetLinkTransform(const std::string&) const { return pose_; }

std::vector<double> SE2Robot::ComputeLinkPointTranslationJacobian(const std::string&, const V4& p) const {
    std::vector<double> J(9, 0.0);
    const V4 x4 = xform4(pose_, p);
    /* X and Y prismatic joints */
    J[0 * 3 + 0] = J[0 * 3 + 0] + 1.0;
    J[1 * 3 + 1] = J[1 * 3 + 1] + 1.0;
    /* Z revolute joint about (x, y, 0) */
    const V3 axis{0.0, 0.0, 1.0};
    const V3 d{x4.x - config_[0], x4.y - config_[1], x4.z - 0.0};
    const V3 c = cross(axis, d);
    J[0 * 3 + 2] = J[0 * 3 + 2] + c.x;
    J[1 * 3 + 2] = J[1 * 3 + 2] + c.y;
    J[2 * 3 + 2] = J[2 * 3 + 2] + c.z;
    return J;
}

double SE2Robot::ComputeConfigurationDistanceTo(const Config& target) const {
    const double dx = target[0] - config_[0];
    const double dy = target[1] - config_[1];
    const double dr = fks_math::enforce_continuous_revolute_bounds(target[2] - config_[2]);
    return position_weight_ * fks_math::dsqrt(dx * dx + dy * dy) + rotation_weight_ * fks_math::dabs(dr);
}

void SE2Robot::ApplyControlInput(const std::vector<double>& input) {
    Config new_config(3);
    for (int i = 0; i < 3; ++i) new_config[i] = config_[i] + axis_[i].actuator.GetControlValue(input[i]);
    SetPosition(new_config);
}

void SE2Robot::ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) {
    double noisy[3];
    for (int i = 0; i < 3; ++i) noisy[i] = axis_[i].actuator.GetControlValue(input[i], rng, (uint32_t)i);
    Config new_config(3);
    for (int i = 0; i < 3; ++i) new_config[i] = config_[i] + noisy[i];
    SetPosition(new_config);
}

std::vector<double> SE2Robot::GenerateControlAction(const Config& target, double controller_interval) {
    double err[3];
    err[0] = target[0] - config_[0];
    err[1] = target[1] - config_[1];
    err[2] = fks_math::enforce_continuous_revolute_bounds(target[2] - config_[2]);
    std::vector<double> u(3);
    for (int i = 0; i < 3; ++i) {
        const double term = axis_[i].controller.ComputeFeedbackTerm(err[i], controller_interval);
        u[i] = axis_[i].actuator.GetControlValue(term);
    }
    return u;
}

const Config& SE2Robot::ResetPosition(const Config& position) {
    for (int i = 0; i < 3; ++i) axis_[i].controller.Zero();
    return SetPosition(position);
}

/* ================= SE(3) ================= */
SE3Robot::SE3Robot(const fks_robot_desc& d) {
    std::vector<std::string> names{"link_0"};
    link_geometries_ = make_link_geometries(d, names);
    for (int i = 0; i < 6; ++i)
        axis_[i] = JointControllerGroup(d.controllers[i], d.sampled_actuators ? d.sampled_actuators + i : nullptr);
    position_weight_ = d.distance_weights ? d.distance_weights[0] : 1.0;
    rotation_weight_ = d.distance_weights ? d.distance_weights[1] : 1.0;
    config_.assign(12, 0.0);
    double I12[12];
    iso_to12(iso_identity(), I12);
    SetPosition(Config(I12, I12 + 12));
}

const Config& SE3Robot::SetPosition(const Config& position) {
    for (int i = 0; i < 12; ++i) config_[i] = position[i];
    pose_ = iso_from12(config_.data());
    return config_;
}

Iso SE3Robot::GetLinkTransform(const std::string&) const { return pose_; }

std::vector<double> SE3Robot::ComputeLinkPointTranslationJacobian(const std::string&, const V4& p) const {
    /* body-twist Jacobian: translation columns R e_i, rotation columns (R e_i) x (x - t) */
    std::vector<double> J(18, 0.0);
    const V4 x4 = xform4(pose_, p);
    const V3 d{x4.x - pose_.t[0], x4.y - pose_.t[1], x4.z - pose_.t[2]};
    for (int i = 0; i < 3; ++i) {
        const V3 axis{pose_.r[0 * 3 + i], pose_.r[1 * 3 + i], pose_.r[2 * 3 + i]};
        J[0 * 6 + i] = J[0 * 6 + i] + axis.x;
        J[1 * 6 + i] = J[1 * 6 + i] + axis.y;
        J[2 * 6 + i] = J[2 * 6 + i] + axis.z;
        const V3 c = cross(axis, d);
        J[0 * 6 + 3 + i] = J[0 * 6 + 3 + i] + c.x;
        J[1 * 6 + 3 + i] = J[1 * 6 + 3 + i] + c.y;
        J[2 * 6 + 3 + i] = J[2 * 6 + 3 + i] + c.z;
    }
    return J;
}

double SE3Robot::ComputeConfigurationDistanceTo(const Config& target) const {
    const Iso tgt = iso_from12(target.data());
    const double dx = tgt.t[0] - pose_.t[0], dy = tgt.t[1] - pose_.t[1], dz = tgt.t[2] - pose_.t[2];
    double tw[6];
    log_twist(compose(inverse(pose_), tgt), tw);
    const double angle = fks_math::dsqrt((tw[3] * tw[3] + tw[4] * tw[4]) + tw[5] * tw[5]);
    return position_weight_ * fks_math::dsqrt((dx * dx + dy * dy) + dz * dz) + rotation_weight_ * angle;
}

void SE3Robot::ApplyControlInput(const std::vector<double>& input) {
    double twist[6];
    for (int i = 0; i < 6; ++i) twist[i] = axis_[i].actuator.GetControlValue(input[i]);
    const Iso next = compose(pose_, exp_twist(twist));
    double m[12];
    iso_to12(next, m);
    SetPosition(Config(m, m + 12));
}

void SE3Robot::ApplyControlInput(const std::vector<double>& input, NoiseContext& rng) {
    double twist[6];
    for (int i = 0; i < 6; ++i) twist[i] = axis_[i].actuator.GetControlValue(input[i], rng, (uint32_t)i);
    const Iso next = compose(pose_, exp_twist(twist));
    double m[12];
    iso_to12(next, m);
    SetPosition(Config(m, m + 12));
}

std::vector<double> SE3Robot::GenerateControlAction(const Config& target, double controller_interval) {
    double twist[6];
    log_twist(compose(inverse(pose_), iso_from12(target.data())), twist);
    std::vector<double> u(6);
    for (int i = 0; i < 6; ++i) {
        const double term = axis_[i].controller.ComputeFeedbackTerm(twist[i], controller_interval);
        u[i] = axis_[i].actuator.GetControlValue(term);
    }
    return u;
}

const Config& SE3Robot::ResetPosition(const Config& position) {
    for (int i = 0; i < 6; ++i) axis_[i].controller.Zero();
    return SetPosition(position);
}

}  // namespace oracle
