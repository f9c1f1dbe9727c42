/*
 * fks_robot_control.cpp — one robot stepped by hand on the host: the TnuvaRobot control
 * interface (TNUVA:15-23) the planner's execution and demonstration code calls on a single
 * robot between simulator calls.
 *
 *   fks_robot_control_action       -> GenerateControlAction (TNUVA:179-198, 384-412, 598-614):
 *                                     per-dof error, SimplePIDController::ComputeFeedbackTerm
 *                                     (PID:122-135), actuator clamp (UNC:70-75)
 *   fks_robot_apply_control_input  -> ApplyControlInput(u) (TNUVA:152-163, 348-364, 538-566) and,
 *                                     with per-dof unit noise samples, ApplyControlInput(u, rng)
 *                                     (TNUVA:165-177, 366-382, 568-596; UNC:77-90)
 *
 * These are not the batch path (that is the GPU's, fks_forward_simulate): they evaluate the
 * same expression trees as the kernel's control_action / apply_input (fks_kernels.hip), with
 * the shared portable libm and SE(3) primitives (fks_portable_math.h, fks_se3.h), so a robot
 * stepped by hand agrees bit for bit with the particles the simulator runs.
 */
#include <stdint.h>

#include <vector>

#include "fks_capi.h"
#include "fks_control.h"
#include "fks_portable_math.h"
#include "fks_se3.h"

namespace {

using fks_math::clamp;
using fks_math::dabs;
using fks_math::dmax;
using fks_math::dmin;

struct DofJoint {
    int32_t type;
    double lo, hi;
};

/* the robot's dofs (linked: its non-fixed joints in joint order, as fks_set_robot numbers
 * them) and its flat configuration width; FKS_ERR_INVALID_ARGUMENT for a malformed robot */
fks_status robot_dofs(const fks_robot_desc* d, std::vector<DofJoint>* dofs, int* width) {
    if (!d || !d->controllers) return FKS_ERR_INVALID_ARGUMENT;
    dofs->clear();
    if (d->robot_type == FKS_ROBOT_LINKED) {
        if (d->num_joints < 0 || (d->num_joints > 0 && !d->joints)) return FKS_ERR_INVALID_ARGUMENT;
        for (int32_t j = 0; j < d->num_joints; ++j) {
            const fks_joint_desc& jd = d->joints[j];
            if (jd.type == FKS_JOINT_FIXED) continue;
            dofs->push_back(DofJoint{jd.type, jd.limit_lower, jd.limit_upper});
        }
        if ((int32_t)dofs->size() != d->num_dofs || d->num_dofs < 1) return FKS_ERR_INVALID_ARGUMENT;
        *width = d->num_dofs;
        return FKS_OK;
    }
    if (d->robot_type == FKS_ROBOT_SE2 && d->num_dofs == 3) {
        *width = 3;
        return FKS_OK;
    }
    if (d->robot_type == FKS_ROBOT_SE3 && d->num_dofs == 6) {
        *width = 12;
        return FKS_OK;
    }
    return FKS_ERR_INVALID_ARGUMENT;
}

bool sampled(const fks_robot_desc* d, int k) {
    return d->sampled_actuators && d->sampled_actuators[k].num_bins > 0;
}

}  // namespace

extern "C" fks_status fks_robot_control_action(const fks_robot_desc* robot, const double* config, const double* target,
                                               double controller_interval, double* pid_state, double* out_control) {
    std::vector<DofJoint> dofs;
    int W = 0;
    const fks_status st = robot_dofs(robot, &dofs, &W);
    if (st != FKS_OK) return st;
    if (!config || !target || !pid_state || !out_control) return FKS_ERR_INVALID_ARGUMENT;
    const int D = robot->num_dofs;
    /* the per-dof error (TNUVA:184, 389, 603) */
    std::vector<double> err((size_t)D, 0.0);
    if (robot->robot_type == FKS_ROBOT_LINKED) {
        for (int k = 0; k < D; ++k)
            err[(size_t)k] = (dofs[(size_t)k].type == FKS_JOINT_CONTINUOUS)
                                 ? fks_math::enforce_continuous_revolute_bounds(target[k] - config[k])
                                 : target[k] - config[k];
    } else if (robot->robot_type == FKS_ROBOT_SE2) {
        err[0] = target[0] - config[0];
        err[1] = target[1] - config[1];
        err[2] = fks_math::enforce_continuous_revolute_bounds(target[2] - config[2]);
    } else {
        double Pi[12], Dm[12];
        fks_se3::inverse34(config, Pi);
        fks_se3::compose34(Pi, target, Dm);
        fks_se3::log_twist34(Dm, err.data());
    }
    /* SimplePIDController::ComputeFeedbackTerm (PID:122-135), gains made positive (PID:104-113),
     * then the actuator's clamp (UNC:70-75) */
    for (int k = 0; k < D; ++k) {
        const fks_dof_controller& ct = robot->controllers[k];
        double& integral = pid_state[k];
        double& last = pid_state[D + k];
        const double term = fks_control::pid_feedback_term(dabs(ct.kp), dabs(ct.ki), dabs(ct.kd), dabs(ct.integral_clamp), &integral,
                                                           &last, err[(size_t)k], controller_interval);
        out_control[k] = fks_control::actuator_clamp(term, dabs(ct.velocity_limit));
    }
    return FKS_OK;
}

extern "C" fks_status fks_robot_apply_control_input(const fks_robot_desc* robot, const double* config, const double* input,
                                                    const double* unit_noise, double* out_config) {
    std::vector<DofJoint> dofs;
    int W = 0;
    const fks_status st = robot_dofs(robot, &dofs, &W);
    if (st != FKS_OK) return st;
    if (!config || !input || !out_config) return FKS_ERR_INVALID_ARGUMENT;
    const int D = robot->num_dofs;
    std::vector<double> real((size_t)D);
    for (int k = 0; k < D; ++k) {
        const fks_dof_controller& ct = robot->controllers[k];
        const double vmax = dabs(ct.velocity_limit);
        double r = fks_control::actuator_clamp(input[k], vmax); /* GetControlValue(u) (UNC:70-75) */
        if (unit_noise) {
            /* GetControlValue(u, rng) (UNC:77-90): the caller drew the truncated-normal sample */
            if (sampled(robot, k)) return FKS_ERR_UNSUPPORTED;
            r = r + unit_noise[k] * fks_control::actuator_noise_bound(r, dabs(ct.max_actuator_proportional_noise),
                                                                     dabs(ct.max_actuator_minimum_noise), vmax);
        }
        real[(size_t)k] = r;
    }
    if (robot->robot_type == FKS_ROBOT_LINKED) {
        /* CopyWithNewValue, then SetPosition's own enforcement (TNUVA:556-565) */
        for (int k = 0; k < D; ++k) {
            const DofJoint& jd = dofs[(size_t)k];
            const double raw = config[k] + real[(size_t)k];
            double v;
            if (jd.type == FKS_JOINT_CONTINUOUS) {
                v = fks_math::enforce_continuous_revolute_bounds(raw);
                v = fks_math::enforce_continuous_revolute_bounds(v);
            } else {
                v = clamp(raw, jd.lo, jd.hi);
                v = clamp(v, jd.lo, jd.hi);
            }
            out_config[k] = v;
        }
    } else if (robot->robot_type == FKS_ROBOT_SE2) {
        /* GetPosition() + real_input, SetPosition wraps the angle (TNUVA:160-162) */
        out_config[0] = config[0] + real[0];
        out_config[1] = config[1] + real[1];
        out_config[2] = fks_math::enforce_continuous_revolute_bounds(config[2] + real[2]);
    } else {
        /* GetPosition() * ExpTwist(twist, 1.0) (TNUVA:360-361) */
        double M[12], C[12];
        fks_se3::exp_twist34(real.data(), M);
        fks_se3::compose34(config, M, C);
        for (int e = 0; e < 12; ++e) out_config[e] = C[e];
    }
    return FKS_OK;
}
