/*
 * hip_particle_contact_simulator.hpp — C++ host mirror of the reference
 * simulator interface over the C-ABI in fks_capi.h (header-only, C++17).
 *
 * Mirrors simple_particle_contact_simulator::SimpleParticleContactSimulator as the
 * planner sees it through uncertainty_planning_core's SimulatorInterface
 * (reference: include/fast_kinematic_simulator/simple_particle_contact_simulator.hpp,
 * "SPCS") and the factories of fast_kinematic_simulator.hpp/.cpp ("FKS").  Method
 * names, argument meaning and result layout follow the reference; configurations
 * are flat double vectors (linked robot: joint values; SE(2): x, y, theta;
 * SE(3): 3x4 row-major pose) because the reference's Eigen / arc_utilities types
 * are not part of this repository.  INTEGRATION.md shows the conversion a
 * maintainer adds on the reference side.
 *
 * Every simulation runs on the GPU through libfks_hip.so; there is no CPU
 * fallback.  Errors from the C-ABI are raised as fks::SimulatorError.
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_HIP_PARTICLE_CONTACT_SIMULATOR_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_HIP_PARTICLE_CONTACT_SIMULATOR_HPP

#include <algorithm>
#include <array>
#include <cstdint>
#include <limits>
#include <random>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/device_set.hpp"
#include "fks_capi.h"

namespace fks {

inline void check(fks_status st, const fks_context* ctx, const char* what) {
    if (st == FKS_OK) return;
    std::string msg = std::string(what) + ": " + fks_status_string(st);
    if (ctx) {
        const char* detail = fks_get_last_error(ctx);
        if (detail && detail[0]) msg += std::string(" (") + detail + ")";
    }
    throw SimulatorError(st, msg);
}

using Configuration = std::vector<double>;

/* simple_simulator_interface::SimulationResult as built at SPCS:918 */
struct SimulationResult {
    Configuration result_config;
    Configuration target_config;
    bool did_contact = false;
    bool outcome_is_valid = true;
    uint32_t microsteps = 0;
    uint32_t resolver_iterations = 0;
    uint32_t error_flags = 0; /* FKS_PARTICLE_ERR_* */
};

/* simple_simulator_interface::ForwardSimulationStepTrace as filled at SPCS:1583-1595,
 * 1615-1618, 1701-1704, 1712-1715, 1776-1779.  `kinds` tags each configuration
 * with the FKS_TRACE_* push site it came from. */
struct ForwardSimulationContactResolverStepTrace {
    std::vector<Configuration> contact_resolution_steps;
    std::vector<uint32_t> kinds;
};
struct ForwardSimulationResolverTrace {
    std::vector<double> control_input;      /* real_control_input = u * dt (SPCS:1549) */
    std::vector<double> control_input_step; /* real_control_input / microsteps (SPCS:1568) */
    std::vector<ForwardSimulationContactResolverStepTrace> contact_resolver_steps;
};
struct ForwardSimulationStepTrace {
    std::vector<ForwardSimulationResolverTrace> resolver_steps;
    bool truncated = false; /* records beyond the trace capacity were dropped */
};

/* visualization_msgs::Marker reduced to plain data (ROS is not part of this
 * repository): what the reference's display helpers fill in */
struct Marker {
    std::string ns;
    int32_t id = 0;
    std::string type; /* "SPHERE_LIST", "LINE_LIST" */
    std::string frame_id;
    std::array<double, 3> scale{{0.0, 0.0, 0.0}};
    std::array<float, 4> color{{0.0f, 0.0f, 0.0f, 1.0f}};
    std::vector<std::array<double, 3>> points;
    std::vector<std::array<float, 4>> colors;
};

/* fast_kinematic_simulator::GetDefaultSolverParameters (FKS.hpp:13-16) */
inline fks_solver_params GetDefaultSolverParameters() {
    fks_solver_params p;
    check(fks_default_solver_params(&p), nullptr, "GetDefaultSolverParameters");
    return p;
}

/* A flattened robot (fks_robot_desc) that owns its arrays: the immutable_robot
 * argument of ForwardSimulateRobots (SPCS:788).  Build it once per robot. */
class RobotDescription {
  public:
    fks_robot_type type = FKS_ROBOT_LINKED;
    int32_t num_links = 1;
    int32_t num_dofs = 0;
    double base_transform[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    std::vector<fks_joint_desc> joints;
    std::vector<int32_t> geometry_link;
    std::vector<uint32_t> geometry_point_offset{0};
    std::vector<double> points; /* x, y, z, w per point */
    std::vector<int32_t> allowed_pairs; /* geometry index pairs */
    std::vector<fks_dof_controller> controllers;
    std::vector<double> distance_weights;
    /* empty, or one per dof: SampledUncertainVelocityActuator bins (num_bins 0 = truncated
     * normal); the bound/sample arrays they point to must outlive the simulator calls */
    std::vector<fks_sampled_actuator> sampled_actuators;

    /* geometry `g` of link `link`: points as (x, y, z, w) quadruples */
    int32_t AddGeometry(int32_t link, const std::vector<double>& xyzw) {
        if (xyzw.size() % 4 != 0) throw std::invalid_argument("points are x, y, z, w quadruples");
        geometry_link.push_back(link);
        points.insert(points.end(), xyzw.begin(), xyzw.end());
        geometry_point_offset.push_back((uint32_t)(points.size() / 4));
        return (int32_t)geometry_link.size() - 1;
    }
    void AllowSelfCollision(int32_t geometry_a, int32_t geometry_b) {
        allowed_pairs.push_back(geometry_a);
        allowed_pairs.push_back(geometry_b);
    }
    /* dof `dof` draws its actuation noise from `bins` (SampledUncertainVelocityActuator,
     * UNC:224-281; simple_uncertainty_models::SetSampledActuator builds them from a LoadModel
     * result); `owner` keeps the arrays the bins point to alive with this description */
    void SetSampledActuator(int32_t dof, const fks_sampled_actuator& bins, std::shared_ptr<const void> owner) {
        if (dof < 0 || dof >= NumDofs()) throw std::invalid_argument("SetSampledActuator: dof out of range");
        if (sampled_actuators.size() != (size_t)NumDofs()) sampled_actuators.assign((size_t)NumDofs(), fks_sampled_actuator{});
        sampled_actuators[(size_t)dof] = bins;
        sampled_owners_.push_back(std::move(owner));
    }
    int32_t NumDofs() const { return type == FKS_ROBOT_SE2 ? 3 : (type == FKS_ROBOT_SE3 ? 6 : num_dofs); }
    int32_t ConfigurationWidth() const {
        return type == FKS_ROBOT_SE2 ? 3 : (type == FKS_ROBOT_SE3 ? 12 : num_dofs);
    }
    /* every byte the simulator receives (fields, tables and the sampled-actuator bins the
     * pointers reach): equal fingerprints mean the same robot for the GPU */
    std::vector<unsigned char> Fingerprint() const {
        std::vector<unsigned char> out;
        auto put = [&out](const void* p, size_t n) {
            const unsigned char* b = static_cast<const unsigned char*>(p);
            out.insert(out.end(), b, b + n);
        };
        auto put_size = [&put](size_t n) {
            const uint64_t v = (uint64_t)n;
            put(&v, sizeof(v));
        };
        put(&type, sizeof(type));
        put(&num_links, sizeof(num_links));
        put(&num_dofs, sizeof(num_dofs));
        put(base_transform, sizeof(base_transform));
        put_size(joints.size());
        put(joints.data(), joints.size() * sizeof(fks_joint_desc));
        put_size(geometry_link.size());
        put(geometry_link.data(), geometry_link.size() * sizeof(int32_t));
        put_size(geometry_point_offset.size());
        put(geometry_point_offset.data(), geometry_point_offset.size() * sizeof(uint32_t));
        put_size(points.size());
        put(points.data(), points.size() * sizeof(double));
        put_size(allowed_pairs.size());
        put(allowed_pairs.data(), allowed_pairs.size() * sizeof(int32_t));
        put_size(controllers.size());
        put(controllers.data(), controllers.size() * sizeof(fks_dof_controller));
        put_size(distance_weights.size());
        put(distance_weights.data(), distance_weights.size() * sizeof(double));
        put_size(sampled_actuators.size());
        for (const fks_sampled_actuator& a : sampled_actuators) {
            put(&a.num_bins, sizeof(a.num_bins));
            put(&a.bin_elements, sizeof(a.bin_elements));
            if (a.num_bins && a.bin_bounds) put(a.bin_bounds, 2 * (size_t)a.num_bins * sizeof(double));
            if (a.num_bins && a.bin_samples) put(a.bin_samples, (size_t)a.num_bins * a.bin_elements * sizeof(double));
        }
        return out;
    }
  private:
    std::vector<std::shared_ptr<const void>> sampled_owners_;

  public:
    fks_robot_desc View() const {
        fks_robot_desc d{};
        d.robot_type = type;
        d.num_links = num_links;
        d.num_joints = (int32_t)joints.size();
        d.num_geometries = (int32_t)geometry_link.size();
        d.num_dofs = num_dofs;
        d.num_allowed_pairs = (int32_t)(allowed_pairs.size() / 2);
        for (int i = 0; i < 12; ++i) d.base_transform[i] = base_transform[i];
        d.joints = joints.empty() ? nullptr : joints.data();
        d.geometry_link = geometry_link.data();
        d.geometry_point_offset = geometry_point_offset.data();
        d.points = points.data();
        d.allowed_pairs = allowed_pairs.empty() ? nullptr : allowed_pairs.data();
        d.controllers = controllers.data();
        d.distance_weights = distance_weights.empty() ? nullptr : distance_weights.data();
        d.sampled_actuators = sampled_actuators.empty() ? nullptr : sampled_actuators.data();
        return d;
    }
};

/* SimpleParticleContactSimulator on one or several MI355X devices (DeviceSet: a batch is
 * sharded by particle id over as many devices as keep at least ShardThreshold() particles
 * each, bit-identical to one device).  The stacked-Jacobian resolver is always used, as the reference factories
 * hard-wire (FKS.cpp:22,45,68). */
class HipParticleContactSimulator {
  public:
    using DisplayFn = std::function<void(const void*)>;

    HipParticleContactSimulator(const fks_environment& environment, const fks_solver_params& solver_config,
                                double simulation_controller_frequency, uint64_t prng_seed, int32_t debug_level,
                                const std::vector<int32_t>& devices)
        : dev_(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, devices) {
        ctx_ = dev_.primary();
        forward_steps_ = (uint32_t)std::max(1.0, solver_config.forward_simulation_time * simulation_controller_frequency);
        resolution_ = environment.collision_map.resolution;
        /* ResetGenerators (SPCS:457-471): the first per-thread generator */
        std::mt19937_64 prng(prng_seed);
        std::uniform_int_distribution<uint64_t> seed_dist(0, std::numeric_limits<uint64_t>::max());
        rng_ = std::mt19937_64(seed_dist(prng));
    }
    HipParticleContactSimulator(const fks_environment& environment, const fks_solver_params& solver_config,
                                double simulation_controller_frequency, uint64_t prng_seed, int32_t debug_level,
                                int32_t device = 0)
        : HipParticleContactSimulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level,
                                      std::vector<int32_t>{device}) {}

    const std::vector<int32_t>& Devices() const { return dev_.devices(); }
    void SetShardThreshold(uint64_t particles_per_device) { dev_.set_shard_threshold(particles_per_device); }
    uint64_t ShardThreshold() const { return dev_.shard_threshold(); }
    bool LastBatchSharded() const { return dev_.last_sharded(); }
    int32_t LastBatchDevices() const { return dev_.last_devices(); }
    /* build `robot`'s shape-specialised kernel on every device now (see
     * fast_kinematic_simulator.hpp PrepareKernels); never throws on a failed build */
    fks::SpecializationStatus PrepareKernels(const RobotDescription& robot) {
        SetRobot(robot);
        return dev_.prepare_kernels(FKS_SPECIALIZE_ON);
    }
    fks::SpecializationStatus SpecializationStatus() const { return dev_.specialization_status(); }

    /* GetFrame (SPCS:517-520) */
    std::string GetFrame() const { return frame_; }
    void SetFrame(const std::string& frame) { frame_ = frame; }
    /* GetRandomGenerator (SPCS:473-481), for the caller's own sampling; the simulation's
     * noise is the counter RNG keyed by (seed, call, particle, step, microstep, dof) */
    std::mt19937_64& GetRandomGenerator() { return rng_; }

    /* fks_kinematics over a batch: FKS_KIN_LINK_TRANSFORMS -> links x 12 per config,
     * FKS_KIN_POINTS -> points x 3, FKS_KIN_APPLY_CONTROL_INPUT -> config width */
    std::vector<double> Kinematics(const RobotDescription& robot, int32_t mode, const std::vector<Configuration>& configs,
                                   const std::vector<std::vector<double>>& inputs = {}) {
        SetRobot(robot);
        int32_t links = 0, points = 0, dofs = 0, width = 0;
        check(fks_robot_sizes(ctx_, &links, &points, &dofs, &width), ctx_, "fks_robot_sizes");
        const size_t n = configs.size(), W = (size_t)width;
        std::vector<double> c(n * W), u;
        for (size_t i = 0; i < n; ++i) {
            if (configs[i].size() != W) throw std::invalid_argument("configuration has the wrong width");
            std::copy(configs[i].begin(), configs[i].end(), c.begin() + i * W);
        }
        if (mode == FKS_KIN_APPLY_CONTROL_INPUT) {
            if (inputs.size() != n) throw std::invalid_argument("one control input per configuration");
            for (const auto& in : inputs) {
                if (in.size() != (size_t)dofs) throw std::invalid_argument("control input has the wrong width");
                u.insert(u.end(), in.begin(), in.end());
            }
        }
        const size_t per = mode == FKS_KIN_LINK_TRANSFORMS ? 12u * (size_t)links : (mode == FKS_KIN_POINTS ? 3u * (size_t)points : W);
        std::vector<double> out(n * per);
        check(fks_kinematics(ctx_, mode, c.data(), n, u.empty() ? nullptr : u.data(), out.data()), ctx_,
              "fks_kinematics");
        return out;
    }

    /* Get3dPointForConfig (SPCS:776-786): origin of the last geometry's link, w = 1 */
    std::array<double, 4> Get3dPointForConfig(const RobotDescription& immutable_robot, const Configuration& config) {
        const std::vector<double> T = Kinematics(immutable_robot, FKS_KIN_LINK_TRANSFORMS, {config});
        const size_t l = (size_t)immutable_robot.geometry_link.back();
        return {{T[12 * l + 3], T[12 * l + 7], T[12 * l + 11], 1.0}};
    }

    /* MakeConfigurationDisplayRep for POINTS geometries (SPCS:634-688) */
    std::vector<Marker> MakeConfigurationDisplayRep(const RobotDescription& immutable_robot, const Configuration& configuration,
                                                    const std::array<float, 4>& color, int32_t starting_index,
                                                    const std::string& config_marker_ns) {
        const std::vector<double> pts = Kinematics(immutable_robot, FKS_KIN_POINTS, {configuration});
        Marker m;
        m.ns = config_marker_ns;
        m.id = starting_index;
        m.type = "SPHERE_LIST";
        m.frame_id = frame_;
        m.scale = {{resolution_, resolution_, resolution_}};
        m.color = color;
        for (size_t i = 0; i < pts.size() / 3; ++i) {
            m.points.push_back({{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}});
            const double* p = immutable_robot.points.data() + 4 * i;
            const bool zero = (p[0] * p[0] + p[1] * p[1] + p[2] * p[2] + p[3] * p[3]) == 0.0;
            m.colors.push_back(zero ? std::array<float, 4>{{0.0f, 0.0f, 0.0f, 1.0f}} : color);
        }
        return {m};
    }

    /* MakeControlInputDisplayRep (SPCS:719-774): each point before and after the clean input */
    std::vector<Marker> MakeControlInputDisplayRep(const RobotDescription& immutable_robot, const Configuration& configuration,
                                                   const std::vector<double>& control_input, const std::array<float, 4>& color,
                                                   int32_t starting_index, const std::string& control_input_marker_ns) {
        const std::vector<double> after = Kinematics(immutable_robot, FKS_KIN_APPLY_CONTROL_INPUT, {configuration}, {control_input});
        const std::vector<double> pts =
            Kinematics(immutable_robot, FKS_KIN_POINTS, {configuration, Configuration(after.begin(), after.end())});
        const size_t P = pts.size() / 6;
        Marker m;
        m.ns = control_input_marker_ns;
        m.id = starting_index;
        m.type = "LINE_LIST";
        m.frame_id = frame_;
        m.scale = {{resolution_ * 0.5, resolution_ * 0.5, resolution_ * 0.5}};
        m.color = color;
        for (size_t i = 0; i < P; ++i) {
            m.points.push_back({{pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]}});
            m.points.push_back({{pts[3 * (P + i)], pts[3 * (P + i) + 1], pts[3 * (P + i) + 2]}});
            m.colors.push_back(color);
            m.colors.push_back(color);
        }
        return {m};
    }

    /* SPCS:446-455 */
    int32_t GetDebugLevel() const { return fks_get_debug_level(ctx_); }
    int32_t SetDebugLevel(int32_t debug_level) { return dev_.set_debug_level(debug_level); }

    /* SPCS:488-512: the eight resolve counters, by the reference's names */
    std::vector<std::pair<std::string, double>> GetStatistics() const {
        const fks_statistics s = dev_.statistics();
        return {{"successful_resolves", (double)s.successful_resolves},
                {"unsuccessful_resolves", (double)s.unsuccessful_resolves},
                {"free_resolves", (double)s.free_resolves},
                {"collision_resolves", (double)s.collision_resolves},
                {"fallback_resolves", (double)s.fallback_resolves},
                {"unsuccessful_env_collision_resolves", (double)s.unsuccessful_env_collision_resolves},
                {"unsuccessful_self_collision_resolves", (double)s.unsuccessful_self_collision_resolves},
                {"recovered_unsuccessful_resolves", (double)s.recovered_unsuccessful_resolves}};
    }
    void ResetStatistics() { dev_.reset_statistics(); }
    /* SPCS:457-471 */
    void ResetGenerators(uint64_t prng_seed) { dev_.reset_generators(prng_seed); }

    /* ForwardSimulateRobots (SPCS:788-804).  display_fn is accepted for interface
     * parity; the batch path never draws (SPCS:801 passes enable_tracing=false). */
    std::vector<SimulationResult> ForwardSimulateRobots(const RobotDescription& immutable_robot,
                                                        const std::vector<Configuration>& start_positions,
                                                        const std::vector<Configuration>& target_positions,
                                                        bool allow_contacts, const DisplayFn& display_fn = {}) {
        (void)display_fn;
        return Simulate(immutable_robot, start_positions, target_positions, allow_contacts, false);
    }
    /* ReverseSimulateRobots (SPCS:806-822) == forward simulation (SPCS:838-841) */
    std::vector<SimulationResult> ReverseSimulateRobots(const RobotDescription& immutable_robot,
                                                        const std::vector<Configuration>& start_positions,
                                                        const std::vector<Configuration>& target_positions,
                                                        bool allow_contacts, const DisplayFn& display_fn = {}) {
        (void)display_fn;
        return Simulate(immutable_robot, start_positions, target_positions, allow_contacts, true);
    }
    /* ForwardSimulateRobot (SPCS:824-829) as a batch of one */
    SimulationResult ForwardSimulateRobot(const RobotDescription& immutable_robot, const Configuration& start_position,
                                          const Configuration& target_position, bool allow_contacts) {
        return Simulate(immutable_robot, {start_position}, {target_position}, allow_contacts, false).front();
    }
    /* ForwardSimulateRobot(..., trace, enable_tracing, display_fn) (SPCS:824-829): the
     * traced kernel records the trace; without enable_tracing this is the call above */
    SimulationResult ForwardSimulateRobot(const RobotDescription& immutable_robot, const Configuration& start_position,
                                          const Configuration& target_position, bool allow_contacts,
                                          ForwardSimulationStepTrace& trace, bool enable_tracing,
                                          const DisplayFn& display_fn = {}, uint32_t config_capacity = 4096) {
        (void)display_fn;
        if (!enable_tracing) return ForwardSimulateRobot(immutable_robot, start_position, target_position, allow_contacts);
        SetRobot(immutable_robot);
        const size_t W = (size_t)immutable_robot.ConfigurationWidth(), D = (size_t)immutable_robot.NumDofs();
        if (start_position.size() != W || target_position.size() != W)
            throw std::invalid_argument("configuration has the wrong width");
        const uint32_t step_cap = forward_steps_, cfg_cap = config_capacity;
        std::vector<double> inputs((size_t)step_cap * 2 * D), configs((size_t)cfg_cap * W), out(W);
        std::vector<uint32_t> micro(step_cap), tags((size_t)cfg_cap * 3);
        uint32_t num_steps = 0, num_configs = 0, microsteps = 0, resolver = 0, errors = 0;
        uint8_t collided = 0;
        fks_trace t{step_cap, cfg_cap, inputs.data(), micro.data(), configs.data(), tags.data(), &num_steps, &num_configs};
        check(fks_forward_simulate_traced(ctx_, start_position.data(), 1, target_position.data(), 1, allow_contacts ? 1 : 0,
                                          out.data(), &collided, &microsteps, &resolver, &errors, &t),
              ctx_, "ForwardSimulateRobot");
        trace.truncated = trace.truncated || num_steps > step_cap || num_configs > cfg_cap;
        const size_t base = trace.resolver_steps.size(); /* the reference appends to the caller's trace */
        for (uint32_t k = 0; k < num_steps && k < step_cap; ++k) {
            ForwardSimulationResolverTrace rs;
            rs.control_input.assign(inputs.begin() + (size_t)k * 2 * D, inputs.begin() + (size_t)k * 2 * D + D);
            rs.control_input_step.assign(inputs.begin() + (size_t)k * 2 * D + D, inputs.begin() + (size_t)(k + 1) * 2 * D);
            trace.resolver_steps.push_back(std::move(rs));
        }
        int64_t last_step = -1, last_micro = -1;
        for (uint32_t k = 0; k < num_configs && k < cfg_cap; ++k) {
            const uint32_t st = tags[3 * k], mi = tags[3 * k + 1];
            if (base + st >= trace.resolver_steps.size()) break;
            ForwardSimulationResolverTrace& rs = trace.resolver_steps[base + st];
            if ((int64_t)st != last_step || (int64_t)mi != last_micro) rs.contact_resolver_steps.emplace_back();
            last_step = st;
            last_micro = mi;
            rs.contact_resolver_steps.back().contact_resolution_steps.emplace_back(configs.begin() + (size_t)k * W,
                                                                                   configs.begin() + (size_t)(k + 1) * W);
            rs.contact_resolver_steps.back().kinds.push_back(tags[3 * k + 2]);
        }
        SimulationResult r;
        r.result_config = out;
        r.target_config = target_position;
        r.did_contact = collided != 0;
        r.microsteps = microsteps;
        r.resolver_iterations = resolver;
        r.error_flags = errors;
        return r;
    }
    /* ReverseSimulateRobot (SPCS:831-836) */
    SimulationResult ReverseSimulateRobot(const RobotDescription& immutable_robot, const Configuration& start_position,
                                          const Configuration& target_position, bool allow_contacts) {
        return Simulate(immutable_robot, {start_position}, {target_position}, allow_contacts, true).front();
    }

    /* CheckConfigCollision (SPCS:1398-1416) */
    bool CheckConfigCollision(const RobotDescription& immutable_robot, const Configuration& config, double inflation_ratio) {
        return CheckConfigCollisions(immutable_robot, {config}, inflation_ratio).front();
    }
    /* the same check for a batch of configurations in one launch */
    std::vector<bool> CheckConfigCollisions(const RobotDescription& immutable_robot, const std::vector<Configuration>& configs,
                                            double inflation_ratio) {
        SetRobot(immutable_robot);
        const size_t W = (size_t)immutable_robot.ConfigurationWidth();
        const size_t n = configs.size();
        std::vector<double> c(n * W);
        for (size_t i = 0; i < n; ++i) {
            if (configs[i].size() != W) throw std::invalid_argument("configuration has the wrong width");
            std::copy(configs[i].begin(), configs[i].end(), c.begin() + i * W);
        }
        std::vector<uint8_t> collided(n);
        dev_.check_configs(c.data(), n, inflation_ratio, collided.data(), nullptr, "CheckConfigCollision");
        return std::vector<bool>(collided.begin(), collided.end());
    }

    fks_context* context() { return ctx_; }

  private:
    DeviceSet dev_;
    fks_context* ctx_ = nullptr; /* devices[0] */
    std::vector<unsigned char> robot_fingerprint_; /* the robot set last (RobotDescription::Fingerprint) */
    uint32_t forward_steps_ = 1; /* controller steps per simulation (SPCS:856): the trace's step capacity */
    double resolution_ = 0.0;
    std::string frame_ = "world";
    std::mt19937_64 rng_;

    /* RobotDescription is a mutable value the caller owns, so the robot set last is
     * recognised by content, never by address (a freed robot's address may be reused) */
    void SetRobot(const RobotDescription& robot) {
        std::vector<unsigned char> fp = robot.Fingerprint();
        if (!robot_fingerprint_.empty() && fp == robot_fingerprint_) return;
        robot_fingerprint_.clear();
        const fks_robot_desc d = robot.View();
        dev_.set_robot(d);
        robot_fingerprint_ = std::move(fp);
    }

    std::vector<SimulationResult> Simulate(const RobotDescription& robot, const std::vector<Configuration>& starts,
                                           const std::vector<Configuration>& targets, bool allow_contacts, bool reverse) {
        /* SPCS:792: one target per particle or one shared target */
        if (!starts.empty() && targets.size() != 1 && targets.size() != starts.size())
            throw std::invalid_argument("target_positions must hold 1 or start_positions.size() configurations");
        SetRobot(robot);
        const size_t W = (size_t)robot.ConfigurationWidth();
        const size_t n = starts.size();
        std::vector<double> s(n * W), t(targets.size() * W), out(n * W);
        for (size_t i = 0; i < n; ++i) {
            if (starts[i].size() != W) throw std::invalid_argument("start configuration has the wrong width");
            std::copy(starts[i].begin(), starts[i].end(), s.begin() + i * W);
        }
        for (size_t i = 0; i < targets.size(); ++i) {
            if (targets[i].size() != W) throw std::invalid_argument("target configuration has the wrong width");
            std::copy(targets[i].begin(), targets[i].end(), t.begin() + i * W);
        }
        std::vector<uint8_t> collided(n);
        std::vector<uint32_t> micro(n), resolver(n), errors(n);
        dev_.simulate(reverse, s.data(), n, t.data(), targets.size(), allow_contacts, out.data(), collided.data(), micro.data(),
                      resolver.data(), errors.data(), reverse ? "ReverseSimulateRobots" : "ForwardSimulateRobots");
        std::vector<SimulationResult> results(n);
        for (size_t i = 0; i < n; ++i) {
            SimulationResult& r = results[i];
            r.result_config.assign(out.begin() + i * W, out.begin() + (i + 1) * W);
            r.target_config = targets.size() == n ? targets[i] : targets[0];
            r.did_contact = collided[i] != 0;
            r.outcome_is_valid = true;
            r.microsteps = micro[i];
            r.resolver_iterations = resolver[i];
            r.error_flags = errors[i];
        }
        return results;
    }
};

/* fast_kinematic_simulator::Make{SE2,SE3,Linked}Simulator (FKS.cpp:4-71).  Without a device
 * argument the simulator runs on every visible MI355X (batches sharded by particle); `device`
 * or `devices` select them explicitly. */
inline std::shared_ptr<HipParticleContactSimulator> MakeSimulator(const fks_environment& environment, const fks_solver_params& solver_config,
                                                                  double simulation_controller_frequency, uint64_t prng_seed,
                                                                  int32_t debug_level, const std::vector<int32_t>& devices) {
    return std::make_shared<HipParticleContactSimulator>(environment, solver_config, simulation_controller_frequency, prng_seed,
                                                         debug_level, devices);
}
#define FKS_WRAPPER_FACTORY(NAME)                                                                                                 \
    inline std::shared_ptr<HipParticleContactSimulator> NAME(const fks_environment& environment, const fks_solver_params& solver_config, \
                                                             double simulation_controller_frequency, uint64_t prng_seed,        \
                                                             int32_t debug_level, const std::vector<int32_t>& devices) {       \
        return MakeSimulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level, devices);     \
    }                                                                                                                            \
    inline std::shared_ptr<HipParticleContactSimulator> NAME(const fks_environment& environment, const fks_solver_params& solver_config, \
                                                             double simulation_controller_frequency, uint64_t prng_seed,        \
                                                             int32_t debug_level, int32_t device) {                            \
        return MakeSimulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level,               \
                             std::vector<int32_t>{device});                                                                     \
    }                                                                                                                            \
    inline std::shared_ptr<HipParticleContactSimulator> NAME(const fks_environment& environment, const fks_solver_params& solver_config, \
                                                             double simulation_controller_frequency, uint64_t prng_seed,        \
                                                             int32_t debug_level) {                                             \
        return MakeSimulator(environment, solver_config, simulation_controller_frequency, prng_seed, debug_level,               \
                             AllVisibleDevices());                                                                              \
    }
FKS_WRAPPER_FACTORY(MakeSE2Simulator)
FKS_WRAPPER_FACTORY(MakeSE3Simulator)
FKS_WRAPPER_FACTORY(MakeLinkedSimulator)
#undef FKS_WRAPPER_FACTORY

}  // namespace fks

#endif
