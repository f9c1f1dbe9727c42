/* <fast_kinematic_simulator/simple_particle_contact_simulator.hpp> — the include path the planner uses for the
 * reference's SPCS, forwarded to this package's header so the planner's #include lines
 * stay as they are ("Swapping it in under the planner"). */
#ifndef FKS_FORWARD_SIMPLE_PARTICLE_CONTACT_SIMULATOR_HPP
#define FKS_FORWARD_SIMPLE_PARTICLE_CONTACT_SIMULATOR_HPP
#include "fast_kinematic_simulator_amd/fast_kinematic_simulator.hpp"
#endif
