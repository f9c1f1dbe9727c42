/*
 * fks_control.h — the controller and actuator arithmetic of one dof, written once for every
 * place that evaluates it: the simulation kernels (fks_kernels.hip, control_action /
 * actuator_noisy), the host robot-control entry points (fks_robot_control.cpp) and the
 * planner-facing SimplePIDController / TruncatedNormalUncertainVelocityActuator
 * (fast_kinematic_simulator_amd/simple_pid_controller.hpp, simple_uncertainty_models.hpp).
 * One expression tree per quantity, compiled for host and device, so a controller stepped on
 * the host and a particle simulated on the GPU agree bit for bit.
 */
#ifndef FKS_CONTROL_H
#define FKS_CONTROL_H

#include "fks_portable_math.h"

namespace fks_control {

/* SimplePIDController::ComputeFeedbackTerm(current_error, timestep) (PID:122-135): trapezoidal
 * error integral clamped to +-integral_clamp, backward-difference derivative, then
 * kp e + ki I + kd de/dt.  The gains and the clamp are the magnitudes Initialize() stores
 * (PID:104-113).  Updates the controller's error integral and last error in place. */
FKS_HD inline double pid_feedback_term(double kp, double ki, double kd, double integral_clamp, double* error_integral, double* last_error,
                                       double current_error, double timestep) {
    const double timestep_error_integral = ((current_error * 0.5) + (*last_error * 0.5)) * timestep;
    const double new_error_integral = *error_integral + timestep_error_integral;
    *error_integral = fks_math::dmax(-integral_clamp, fks_math::dmin(integral_clamp, new_error_integral));
    const double error_derivative = (current_error - *last_error) / timestep;
    *last_error = current_error;
    return (current_error * kp) + (*error_integral * ki) + (error_derivative * kd);
}

/* TruncatedNormalUncertainVelocityActuator::GetControlValue(u) (UNC:70-75): the command
 * clamped to the velocity limit (a magnitude) */
FKS_HD inline double actuator_clamp(double control_input, double velocity_limit) {
    return fks_math::clamp(control_input, -velocity_limit, velocity_limit);
}

/* the noise bound of GetControlValue(u, rng) (UNC:77-90): proportional to the clamped command
 * with a floor at minimum_noise_bound x velocity_limit (all three bounds are magnitudes); the
 * noisy command is real + unit_noise x bound */
FKS_HD inline double actuator_noise_bound(double real_control_input, double proportional_noise_bound, double minimum_noise_bound,
                                          double velocity_limit) {
    const double real_proportional_noise_bound = proportional_noise_bound * fks_math::dabs(real_control_input);
    const double real_minimum_noise_bound = minimum_noise_bound * velocity_limit;
    return fks_math::dmax(real_proportional_noise_bound, real_minimum_noise_bound);
}

}  // namespace fks_control

#endif
