/* Mock of uncertainty_planning_core's simulator interface (test only;
 * tests/cpp/mock_workspace/README.md), with the virtuals the reference overrides
 * (SPCS:446-1416), the result and trace types it fills (SPCS:918, 1583-1595) and the color
 * helper it calls (SPCS:1727). */
#ifndef MOCK_UPC_SIMPLE_SIMULATOR_INTERFACE
#define MOCK_UPC_SIMPLE_SIMULATOR_INTERFACE
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include <Eigen/Geometry>
#include <arc_utilities/simple_robot_models.hpp>
#include <std_msgs/ColorRGBA.h>
#include <visualization_msgs/MarkerArray.h>

namespace simple_simulator_interface {
template <typename Configuration>
struct SimulationResult {
    Configuration result_config;
    Configuration target_config;
    bool did_contact = false;
    bool outcome_is_valid = false;
    SimulationResult() {}
    SimulationResult(const Configuration& result, const Configuration& target, const bool contact, const bool valid)
        : result_config(result), target_config(target), did_contact(contact), outcome_is_valid(valid) {}
};

template <typename Configuration, typename ConfigAlloc = std::allocator<Configuration>>
struct ForwardSimulationContactResolverStepTrace {
    std::vector<Configuration, ConfigAlloc> contact_resolution_steps;
};

template <typename Configuration, typename ConfigAlloc = std::allocator<Configuration>>
struct ForwardSimulationResolverTrace {
    Eigen::VectorXd control_input;
    Eigen::VectorXd control_input_step;
    std::vector<ForwardSimulationContactResolverStepTrace<Configuration, ConfigAlloc>> contact_resolver_steps;
};

template <typename Configuration, typename ConfigAlloc = std::allocator<Configuration>>
struct ForwardSimulationStepTrace {
    std::vector<ForwardSimulationResolverTrace<Configuration, ConfigAlloc>> resolver_steps;
    void Reset() { resolver_steps.clear(); }
};

template <typename Configuration, typename RNG, typename ConfigAlloc = std::allocator<Configuration>>
class SimulatorInterface {
  public:
    typedef simple_robot_model_interface::SimpleRobotModelInterface<Configuration, ConfigAlloc> BaseRobotType;
    typedef simple_simulator_interface::SimulationResult<Configuration> SimulationResult;
    typedef simple_simulator_interface::ForwardSimulationStepTrace<Configuration, ConfigAlloc> ForwardSimulationStepTrace;
    typedef std::function<void(const visualization_msgs::MarkerArray&)> DisplayFn;
    virtual ~SimulatorInterface() {}
    virtual int32_t GetDebugLevel() const = 0;
    virtual int32_t SetDebugLevel(const int32_t debug_level) = 0;
    virtual RNG& GetRandomGenerator() = 0;
    virtual std::map<std::string, double> GetStatistics() const = 0;
    virtual void ResetStatistics() = 0;
    virtual std::string GetFrame() const = 0;
    virtual visualization_msgs::MarkerArray MakeEnvironmentDisplayRep() const = 0;
    virtual visualization_msgs::MarkerArray MakeConfigurationDisplayRep(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                                        const Configuration& configuration, const std_msgs::ColorRGBA& color,
                                                                        const int32_t starting_index, const std::string& config_marker_ns) const = 0;
    virtual visualization_msgs::MarkerArray MakeControlInputDisplayRep(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                                       const Configuration& configuration, const Eigen::VectorXd& control_input,
                                                                       const std_msgs::ColorRGBA& color, const int32_t starting_index,
                                                                       const std::string& control_input_marker_ns) const = 0;
    virtual Eigen::Vector4d Get3dPointForConfig(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& config) const = 0;
    virtual std::vector<SimulationResult> ForwardSimulateRobots(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                                const std::vector<Configuration, ConfigAlloc>& start_positions,
                                                                const std::vector<Configuration, ConfigAlloc>& target_positions,
                                                                const bool allow_contacts, const DisplayFn& display_fn) = 0;
    virtual std::vector<SimulationResult> ReverseSimulateRobots(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                                const std::vector<Configuration, ConfigAlloc>& start_positions,
                                                                const std::vector<Configuration, ConfigAlloc>& target_positions,
                                                                const bool allow_contacts, const DisplayFn& display_fn) = 0;
    virtual SimulationResult ForwardSimulateRobot(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& start_position,
                                                  const Configuration& target_position, const bool allow_contacts,
                                                  ForwardSimulationStepTrace& trace, const bool enable_tracing, const DisplayFn& display_fn) = 0;
    virtual SimulationResult ReverseSimulateRobot(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& start_position,
                                                  const Configuration& target_position, const bool allow_contacts,
                                                  ForwardSimulationStepTrace& trace, const bool enable_tracing, const DisplayFn& display_fn) = 0;
    virtual SimulationResult ReverseSimulateMutableRobot(const std::shared_ptr<BaseRobotType>& robot, const Configuration& target_position,
                                                         const bool allow_contacts, ForwardSimulationStepTrace& trace,
                                                         const bool enable_tracing, const DisplayFn& display_fn) = 0;
    virtual SimulationResult ForwardSimulateMutableRobot(const std::shared_ptr<BaseRobotType>& robot, const Configuration& target_position,
                                                         const bool allow_contacts, ForwardSimulationStepTrace& trace,
                                                         const bool enable_tracing, const DisplayFn& display_fn) = 0;
    virtual bool CheckConfigCollision(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& config,
                                      const double inflation_ratio) const = 0;
    static std_msgs::ColorRGBA MakeColor(const float r, const float g, const float b, const float a) {
        std_msgs::ColorRGBA c;
        c.r = r;
        c.g = g;
        c.b = b;
        c.a = a;
        return c;
    }
};
}  // namespace simple_simulator_interface
#endif
