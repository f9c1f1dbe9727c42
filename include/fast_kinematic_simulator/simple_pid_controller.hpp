/* <fast_kinematic_simulator/simple_pid_controller.hpp> — the include path planner and execution code use for the
 * reference's header of this name, forwarded to this package's header so the #include lines
 * stay as they are ("Swapping it in under the planner"). */
#ifndef FKS_FORWARD_SIMPLE_PID_CONTROLLER_HPP
#define FKS_FORWARD_SIMPLE_PID_CONTROLLER_HPP
#include "fast_kinematic_simulator_amd/simple_pid_controller.hpp"
#endif
