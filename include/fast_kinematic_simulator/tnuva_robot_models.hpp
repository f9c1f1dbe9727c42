/* <fast_kinematic_simulator/tnuva_robot_models.hpp> — the include path the planner uses for the
 * reference's TNUVA, forwarded to this package's header so the planner's #include lines
 * stay as they are ("Swapping it in under the planner"). */
#ifndef FKS_FORWARD_TNUVA_ROBOT_MODELS_HPP
#define FKS_FORWARD_TNUVA_ROBOT_MODELS_HPP
#include "fast_kinematic_simulator_amd/tnuva_robot_models.hpp"
#endif
