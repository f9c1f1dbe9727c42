/* <fast_kinematic_simulator/simulator_environment_builder.hpp> — the include path the planner uses for the
 * reference's SEB.hpp, forwarded to this package's header so the planner's #include lines
 * stay as they are ("Swapping it in under the planner"). */
#ifndef FKS_FORWARD_SIMULATOR_ENVIRONMENT_BUILDER_HPP
#define FKS_FORWARD_SIMULATOR_ENVIRONMENT_BUILDER_HPP
#include "fast_kinematic_simulator_amd/environment.hpp"
#endif
