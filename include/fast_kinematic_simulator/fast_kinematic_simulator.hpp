/* <fast_kinematic_simulator/fast_kinematic_simulator.hpp> — the include path the planner uses for the
 * reference's FKS.hpp, forwarded to this package's header so the planner's #include lines
 * stay as they are ("Swapping it in under the planner"). */
#ifndef FKS_FORWARD_FAST_KINEMATIC_SIMULATOR_HPP
#define FKS_FORWARD_FAST_KINEMATIC_SIMULATOR_HPP
#include "fast_kinematic_simulator_amd/fast_kinematic_simulator.hpp"
#endif
