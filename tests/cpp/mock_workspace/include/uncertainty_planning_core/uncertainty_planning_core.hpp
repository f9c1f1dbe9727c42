/* Mock of uncertainty_planning_core's typedefs (test only; tests/cpp/mock_workspace/README.md):
 * the return types of FKS.hpp:18-22 and the allocators of UPC.cpp:81-82, 131. */
#ifndef MOCK_UPC_UNCERTAINTY_PLANNING_CORE
#define MOCK_UPC_UNCERTAINTY_PLANNING_CORE
#include <memory>
#include <random>
#include <uncertainty_planning_core/simple_simulator_interface.hpp>
namespace uncertainty_planning_core {
typedef std::mt19937_64 PRNG;
typedef Eigen::Matrix<double, 3, 1> SE2Config;
typedef std::allocator<Eigen::Matrix<double, 3, 1>> SE2ConfigAlloc;
typedef Eigen::Isometry3d SE3Config;
typedef Eigen::aligned_allocator<Eigen::Isometry3d> SE3ConfigAlloc;
typedef simple_linked_robot_model::SimpleLinkedConfiguration LinkedConfig;
typedef simple_linked_robot_model::SimpleLinkedConfigAlloc LinkedConfigAlloc;
typedef simple_simulator_interface::SimulatorInterface<SE2Config, PRNG, SE2ConfigAlloc> SE2Simulator;
typedef simple_simulator_interface::SimulatorInterface<SE3Config, PRNG, SE3ConfigAlloc> SE3Simulator;
typedef simple_simulator_interface::SimulatorInterface<LinkedConfig, PRNG, LinkedConfigAlloc> LinkedSimulator;
typedef std::shared_ptr<SE2Simulator> SE2SimulatorPtr;
typedef std::shared_ptr<SE3Simulator> SE3SimulatorPtr;
typedef std::shared_ptr<LinkedSimulator> LinkedSimulatorPtr;
}  // namespace uncertainty_planning_core
#endif
