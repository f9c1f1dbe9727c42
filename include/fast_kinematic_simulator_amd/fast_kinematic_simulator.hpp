/*
 * fast_kinematic_simulator.hpp — the planner-facing drop-in: the HIP-backed particle
 * simulator behind simple_simulator_interface::SimulatorInterface, and the
 * fast_kinematic_simulator factories with the reference's parameter lists.
 *
 *   simple_particle_contact_simulator::SimulatorSolverParameters   SPCS:345-369
 *   simple_particle_contact_simulator::HipParticleContactSimulator
 *       <DerivedRobotType, Configuration, RNG, ConfigAlloc>           SPCS:371-1999 (the
 *       class the factories instantiate), every SimulatorInterface virtual overridden
 *   fast_kinematic_simulator::SolverParameters / GetDefaultSolverParameters   FKS.hpp:11-16
 *   fast_kinematic_simulator::Make{SE2,SE3,Linked}Simulator                    FKS.hpp:18-22,
 *       FKS.cpp:4-71 (simulate_with_individual_jacobians = false, as there)
 *
 * Batch, traced, mutable-robot and validity calls all run on the GPU through the
 * C-ABI (include/fks_capi.h); there is no CPU path.  The robot a call receives is the
 * planner's BaseRobotType, static_cast to DerivedRobotType as the reference does
 * (SPCS:868); DerivedRobotType is one of tnuva_robot_models::Tnuva{SE2,SE3,Linked}Robot
 * (tnuva_robot_models.hpp), which carry the flattened description and the controller
 * state.  Differences from the reference, by design:
 *   - actuation noise comes from the counter RNG keyed by (seed, call, particle, step,
 *     microstep, dof), not from GetRandomGenerator()'s stream, which is
 *     still provided for the caller's own sampling;
 *   - the reference's per-particle asserts (SPCS:1570-1575, 1882) become error bits,
 *     available from LastParticleErrors() after a batch call;
 *   - display_fn is accepted and never called (the batch path never draws, SPCS:801).
 * The Eigen / ROS / sdf_tools / uncertainty_planning_core types in the signatures are the
 * planner workspace's own when its headers are on the include path, stand-ins otherwise
 * (fks_external_types.hpp).
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_FAST_KINEMATIC_SIMULATOR_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_FAST_KINEMATIC_SIMULATOR_HPP

#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "fast_kinematic_simulator_amd/device_set.hpp"
#include "fast_kinematic_simulator_amd/environment.hpp"
#include "fast_kinematic_simulator_amd/fks_external_types.hpp"
#include "fast_kinematic_simulator_amd/tnuva_robot_models.hpp"
#include "fks_capi.h"

namespace simple_particle_contact_simulator {

/* SimulatorSolverParameters (SPCS:345-369) */
struct SimulatorSolverParameters {
    double forward_simulation_time;
    double simulation_shortcut_distance;
    double environment_collision_check_tolerance;
    double resolve_correction_step_scaling_decay_rate;
    double resolve_correction_initial_step_size;
    double resolve_correction_min_step_scaling;
    uint32_t max_resolver_iterations;
    uint32_t resolve_correction_step_scaling_decay_iterations;
    bool failed_resolves_end_motion;

    SimulatorSolverParameters() {
        forward_simulation_time = 1.0;
        simulation_shortcut_distance = 0.0;
        environment_collision_check_tolerance = 0.001;
        resolve_correction_step_scaling_decay_rate = 0.5;
        resolve_correction_initial_step_size = 1.0;
        resolve_correction_min_step_scaling = 0.03125;
        max_resolver_iterations = 25;
        resolve_correction_step_scaling_decay_iterations = 5;
        failed_resolves_end_motion = true;
    }
    fks_solver_params ToFks() const {
        fks_solver_params p{};
        p.forward_simulation_time = forward_simulation_time;
        p.simulation_shortcut_distance = simulation_shortcut_distance;
        p.environment_collision_check_tolerance = environment_collision_check_tolerance;
        p.resolve_correction_step_scaling_decay_rate = resolve_correction_step_scaling_decay_rate;
        p.resolve_correction_initial_step_size = resolve_correction_initial_step_size;
        p.resolve_correction_min_step_scaling = resolve_correction_min_step_scaling;
        p.max_resolver_iterations = max_resolver_iterations;
        p.resolve_correction_step_scaling_decay_iterations = resolve_correction_step_scaling_decay_iterations;
        p.failed_resolves_end_motion = failed_resolves_end_motion ? 1u : 0u;
        return p;
    }
};

template <typename DerivedRobotType, typename Configuration, typename RNG, typename ConfigAlloc = std::allocator<Configuration>>
class HipParticleContactSimulator : public simple_simulator_interface::SimulatorInterface<Configuration, RNG, ConfigAlloc> {
  public:
    typedef simple_simulator_interface::SimulatorInterface<Configuration, RNG, ConfigAlloc> Base;
    typedef typename Base::BaseRobotType BaseRobotType;
    typedef typename Base::SimulationResult SimulationResult;
    typedef typename Base::ForwardSimulationStepTrace ForwardSimulationStepTrace;
    typedef typename Base::DisplayFn DisplayFn;
    typedef fks_planner_types::MarkerArray MarkerArray;
    typedef fks_planner_types::ColorRGBA ColorRGBA;

    /* SPCS:420-444.  `devices` lists the MI355X devices the simulator runs on (no reference
     * counterpart; the reference's batch loop runs over the host's cores, SPCS:795): a batch
     * is split into contiguous shards by global particle id over as many of the listed devices
     * as keep at least ShardThreshold() particles each (fks_create_multi), bit-identical to
     * one device; batches that keep one device and single-particle calls run on devices[0].
     * The same device may be listed more than once. */
    HipParticleContactSimulator(const sdf_tools::TaggedObjectCollisionMapGrid& environment,
                                const sdf_tools::SignedDistanceField& environment_sdf,
                                const SurfaceNormalGrid& surface_normals_grid, const SimulatorSolverParameters& solver_config,
                                const double simulation_controller_frequency, const bool simulate_with_individual_jacobians,
                                const uint64_t prng_seed, const int32_t debug_level, const std::vector<int32_t>& devices)
        : environment_(environment), environment_sdf_(environment_sdf), surface_normals_grid_(surface_normals_grid),
          solver_config_(solver_config), simulation_controller_frequency_(simulation_controller_frequency),
          dev_(MakeDevices(environment_, environment_sdf_, surface_normals_grid_, solver_config, simulation_controller_frequency, prng_seed,
                           debug_level, devices)) {
        ctx_ = dev_->primary();
        dev_->set_individual_jacobians(simulate_with_individual_jacobians);
        ResetGenerators(prng_seed);
    }
    /* one device (the constructor of the reference's parameter list plus `device`) */
    HipParticleContactSimulator(const sdf_tools::TaggedObjectCollisionMapGrid& environment,
                                const sdf_tools::SignedDistanceField& environment_sdf,
                                const SurfaceNormalGrid& surface_normals_grid, const SimulatorSolverParameters& solver_config,
                                const double simulation_controller_frequency, const bool simulate_with_individual_jacobians,
                                const uint64_t prng_seed, const int32_t debug_level, const int32_t device = 0)
        : HipParticleContactSimulator(environment, environment_sdf, surface_normals_grid, solver_config, simulation_controller_frequency,
                                      simulate_with_individual_jacobians, prng_seed, debug_level, std::vector<int32_t>{device}) {}

    /* ---- SimulatorInterface (SPCS:446-1416) ---- */
    int32_t GetDebugLevel() const override { return fks_get_debug_level(ctx_); }
    int32_t SetDebugLevel(const int32_t debug_level) override { return dev_->set_debug_level(debug_level); }
    /* SPCS:457-471: the host generator seeded as the reference seeds its thread 0 one; the
     * simulation's own noise is the counter RNG re-keyed by the same seed */
    void ResetGenerators(const uint64_t prng_seed) {
        RNG prng(prng_seed);
        std::uniform_int_distribution<uint64_t> seed_dist(0, std::numeric_limits<uint64_t>::max());
        rng_ = RNG(seed_dist(prng));
        dev_->reset_generators(prng_seed);
    }
    RNG& GetRandomGenerator() override { return rng_; }
    std::map<std::string, double> GetStatistics() const override {
        const fks_statistics s = dev_->statistics(); /* summed over the devices */
        return {{"successful_resolves", (double)s.successful_resolves},
                {"unsuccessful_resolves", (double)s.unsuccessful_resolves},
                {"free_resolves", (double)s.free_resolves},
                {"collision_resolves", (double)s.collision_resolves},
                {"fallback_resolves", (double)s.fallback_resolves},
                {"unsuccessful_self_collision_resolves", (double)s.unsuccessful_self_collision_resolves},
                {"unsuccessful_env_collision_resolves", (double)s.unsuccessful_env_collision_resolves},
                {"recovered_unsuccessful_resolves", (double)s.recovered_unsuccessful_resolves}};
    }
    void ResetStatistics() override { dev_->reset_statistics(); }
    std::string GetFrame() const override { return environment_.GetFrame(); }
    double GetResolution() const { return environment_.GetResolution(); }

    /* SPCS:559-586, reduced to the grids this repository holds: the filled cells of the
     * collision map and the SDF cells colored by sign (sdf_tools' component / convex-segment
     * exports have no counterpart) */
    MarkerArray MakeEnvironmentDisplayRep() const override {
        MarkerArray rep;
        const double res = environment_.GetResolution();
        fks_planner_types::Marker env_marker = MakeMarker("sim_environment", 1, fks_planner_types::Marker::CUBE_LIST, res,
                                                          Base::MakeColor(1.0f, 0.0f, 0.0f, 1.0f));
        fks_planner_types::Marker sdf_marker = MakeMarker("sim_environment_sdf", 1, fks_planner_types::Marker::CUBE_LIST, res,
                                                          Base::MakeColor(1.0f, 1.0f, 1.0f, 1.0f));
        const fks_grid_geometry G = fks_ext::grid_geometry(environment_);
        const double* O = G.origin;
        for (int64_t x = 0; x < environment_.GetNumXCells(); ++x)
            for (int64_t y = 0; y < environment_.GetNumYCells(); ++y)
                for (int64_t z = 0; z < environment_.GetNumZCells(); ++z) {
                    const double c[3] = {res * ((double)x + 0.5), res * ((double)y + 0.5), res * ((double)z + 0.5)};
                    fks_planner_types::Point p;
                    p.x = ((O[0] * c[0] + O[1] * c[1]) + O[2] * c[2]) + O[3];
                    p.y = ((O[4] * c[0] + O[5] * c[1]) + O[6] * c[2]) + O[7];
                    p.z = ((O[8] * c[0] + O[9] * c[1]) + O[10] * c[2]) + O[11];
                    if (environment_.GetImmutable(x, y, z).first.occupancy > 0.5f) env_marker.points.push_back(p);
                    sdf_marker.points.push_back(p);
                    sdf_marker.colors.push_back(environment_sdf_.GetImmutable(x, y, z).first < 0.0f
                                                    ? Base::MakeColor(1.0f, 0.0f, 0.0f, 1.0f)
                                                    : Base::MakeColor(0.0f, 0.0f, 1.0f, 1.0f));
                }
        rep.markers.push_back(env_marker);
        rep.markers.push_back(sdf_marker);
        return rep;
    }
    /* MakeConfigurationDisplayRep with POINTS geometries (SPCS:634-688, 695-717): every link point */
    MarkerArray MakeConfigurationDisplayRep(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& configuration,
                                            const ColorRGBA& color, const int32_t starting_index,
                                            const std::string& config_marker_ns) const override {
        const DerivedRobotType& robot = Derived(immutable_robot);
        const std::vector<double> pts = Kinematics(robot, FKS_KIN_POINTS, {robot.ToFlat(configuration)});
        const double res = GetResolution();
        fks_planner_types::Marker m = MakeMarker(config_marker_ns, starting_index, fks_planner_types::Marker::SPHERE_LIST, res, color);
        const std::vector<double>& local = robot.HipDescription().points;
        for (size_t i = 0; i < pts.size() / 3; ++i) {
            m.points.push_back(Point(pts.data() + 3 * i));
            const double* q = local.data() + 4 * i;
            const bool zero = (q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]) == 0.0;
            m.colors.push_back(zero ? Base::MakeColor(0.0f, 0.0f, 0.0f, 1.0f) : color);
        }
        MarkerArray rep;
        rep.markers.push_back(m);
        return rep;
    }
    /* SPCS:719-774: each point before and after the clean control input */
    MarkerArray MakeControlInputDisplayRep(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& configuration,
                                           const fks_planner_types::VectorXd& control_input, const ColorRGBA& color,
                                           const int32_t starting_index, const std::string& control_input_marker_ns) const override {
        const DerivedRobotType& robot = Derived(immutable_robot);
        const std::vector<double> start = robot.ToFlat(configuration);
        const std::vector<double> after = Kinematics(robot, FKS_KIN_APPLY_CONTROL_INPUT, {start}, {fks_ext::vecx_values(control_input)});
        const std::vector<double> pts = Kinematics(robot, FKS_KIN_POINTS, {start, after});
        const size_t P = pts.size() / 6;
        fks_planner_types::Marker m =
            MakeMarker(control_input_marker_ns, starting_index, fks_planner_types::Marker::LINE_LIST, GetResolution() * 0.5, color);
        for (size_t i = 0; i < P; ++i) {
            m.points.push_back(Point(pts.data() + 3 * i));
            m.points.push_back(Point(pts.data() + 3 * (P + i)));
            m.colors.push_back(color);
            m.colors.push_back(color);
        }
        MarkerArray rep;
        rep.markers.push_back(m);
        return rep;
    }
    /* SPCS:776-786: origin of the last geometry's link, w = 1 */
    fks_planner_types::Vector4d Get3dPointForConfig(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                    const Configuration& config) const override {
        const DerivedRobotType& robot = Derived(immutable_robot);
        const std::vector<double> T = Kinematics(robot, FKS_KIN_LINK_TRANSFORMS, {robot.ToFlat(config)});
        const size_t l = (size_t)robot.HipDescription().geometry_link.back();
        return fks_planner_types::Vector4d(T[12 * l + 3], T[12 * l + 7], T[12 * l + 11], 1.0);
    }

    /* SPCS:788-804 */
    std::vector<SimulationResult> ForwardSimulateRobots(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                        const std::vector<Configuration, ConfigAlloc>& start_positions,
                                                        const std::vector<Configuration, ConfigAlloc>& target_positions,
                                                        const bool allow_contacts, const DisplayFn& display_fn) override {
        (void)display_fn;
        return Batch(Derived(immutable_robot), start_positions, target_positions, allow_contacts, fks_forward_simulate);
    }
    /* SPCS:806-822: the same simulation (ReverseSimulateMutableRobot, SPCS:838-841) */
    std::vector<SimulationResult> ReverseSimulateRobots(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                                        const std::vector<Configuration, ConfigAlloc>& start_positions,
                                                        const std::vector<Configuration, ConfigAlloc>& target_positions,
                                                        const bool allow_contacts, const DisplayFn& display_fn) override {
        (void)display_fn;
        return Batch(Derived(immutable_robot), start_positions, target_positions, allow_contacts, fks_reverse_simulate);
    }
    /* SPCS:824-829: a clone reset to the start (controllers zeroed) */
    SimulationResult ForwardSimulateRobot(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& start_position,
                                          const Configuration& target_position, const bool allow_contacts,
                                          ForwardSimulationStepTrace& trace, const bool enable_tracing,
                                          const DisplayFn& display_fn) override {
        std::shared_ptr<BaseRobotType> robot(immutable_robot->Clone());
        static_cast<DerivedRobotType*>(robot.get())->ResetPosition(start_position);
        return ForwardSimulateMutableRobot(robot, target_position, allow_contacts, trace, enable_tracing, display_fn);
    }
    /* SPCS:831-836 */
    SimulationResult ReverseSimulateRobot(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& start_position,
                                          const Configuration& target_position, const bool allow_contacts,
                                          ForwardSimulationStepTrace& trace, const bool enable_tracing,
                                          const DisplayFn& display_fn) override {
        std::shared_ptr<BaseRobotType> robot(immutable_robot->Clone());
        static_cast<DerivedRobotType*>(robot.get())->ResetPosition(start_position);
        return ReverseSimulateMutableRobot(robot, target_position, allow_contacts, trace, enable_tracing, display_fn);
    }
    /* SPCS:838-841 */
    SimulationResult ReverseSimulateMutableRobot(const std::shared_ptr<BaseRobotType>& robot, const Configuration& target_position,
                                                 const bool allow_contacts, ForwardSimulationStepTrace& trace,
                                                 const bool enable_tracing, const DisplayFn& display_fn) override {
        return ForwardSimulateMutableRobot(robot, target_position, allow_contacts, trace, enable_tracing, display_fn);
    }
    /* SPCS:843-919: simulates from the robot's position with its controllers as they are,
     * then leaves the robot at the reached position with the controllers' new state */
    SimulationResult ForwardSimulateMutableRobot(const std::shared_ptr<BaseRobotType>& robot, const Configuration& target_position,
                                                 const bool allow_contacts, ForwardSimulationStepTrace& trace,
                                                 const bool enable_tracing, const DisplayFn& display_fn) override {
        (void)display_fn;
        DerivedRobotType& r = *static_cast<DerivedRobotType*>(robot.get());
        SetRobot(r);
        const std::vector<double> s = r.ToFlat(r.GetPosition()), t = r.ToFlat(target_position);
        const size_t W = s.size(), D = (size_t)r.HipDescription().NumDofs();
        std::vector<double> q(W), pid = r.ControllerState();
        uint8_t collided = 0;
        uint32_t micro = 0, resolver = 0, errors = 0;
        if (!enable_tracing) {
            Check(fks_forward_simulate_mutable(ctx_, s.data(), 1, t.data(), 1, allow_contacts ? 1 : 0, pid.data(), q.data(),
                                               &collided, &micro, &resolver, &errors),
                  ctx_, "ForwardSimulateMutableRobot");
        } else {
            /* the trace holds one step record per controller step and every pushed
             * configuration.  The capacity starts at TraceCapacityHint() configurations
             * (16384); a longer trace is re-run with the exact size, from the same RNG call
             * index and controller state (the simulation is deterministic, so the rerun
             * reproduces it), and the statistics and call totals the first run added are taken
             * back, so GetStatistics counts the particle once */
            const uint32_t steps = ForwardSteps();
            const uint64_t call = fks_get_call_index(ctx_);
            const std::vector<double> pid0 = pid;
            fks_statistics stats0{};
            fks_call_counters totals0{};
            Check(fks_get_statistics(ctx_, &stats0), ctx_, "fks_get_statistics");
            Check(fks_get_total_counters(ctx_, &totals0), ctx_, "fks_get_total_counters");
            uint32_t cap = trace_capacity_hint_;
            for (int attempt = 0;; ++attempt) {
                std::vector<double> inputs((size_t)steps * 2 * D), configs((size_t)cap * W);
                std::vector<uint32_t> step_micro(steps), tags((size_t)cap * 3);
                uint32_t num_steps = 0, num_configs = 0;
                fks_trace tr{steps, cap, inputs.data(), step_micro.data(), configs.data(), tags.data(), &num_steps, &num_configs};
                Check(fks_forward_simulate_traced_mutable(ctx_, s.data(), 1, t.data(), 1, allow_contacts ? 1 : 0, pid.data(),
                                                          q.data(), &collided, &micro, &resolver, &errors, &tr),
                      ctx_, "ForwardSimulateMutableRobot (traced)");
                if (num_steps <= steps && num_configs <= cap) {
                    AppendTrace(r, trace, inputs, num_steps, configs, tags, num_configs, D);
                    break;
                }
                if (attempt > 0 || num_steps > steps) throw std::runtime_error("trace capacity exceeded");
                cap = num_configs;
                pid = pid0;
                Check(fks_set_call_index(ctx_, call), ctx_, "fks_set_call_index");
                Check(fks_set_statistics(ctx_, &stats0), ctx_, "fks_set_statistics");
                Check(fks_set_total_counters(ctx_, &totals0), ctx_, "fks_set_total_counters");
                retried_traces_++;
            }
        }
        last_errors_.assign(1, errors);
        r.SetPosition(r.FromFlat(q.data()));
        r.SetControllerState(pid);
        return SimulationResult(r.GetPosition(), target_position, collided != 0, true); /* SPCS:918 */
    }
    /* SPCS:1398-1416 */
    bool CheckConfigCollision(const std::shared_ptr<BaseRobotType>& immutable_robot, const Configuration& config,
                              const double inflation_ratio) const override {
        const DerivedRobotType& robot = Derived(immutable_robot);
        SetRobot(robot);
        const std::vector<double> c = robot.ToFlat(config);
        uint8_t collided = 0;
        Check(fks_check_config_collision(ctx_, c.data(), 1, inflation_ratio, &collided, nullptr), ctx_,
              "CheckConfigCollision");
        return collided != 0;
    }

    /* ---- beyond the interface ---- */
    /* per-particle FKS_PARTICLE_ERR_* bits of the last batch (the reference asserts instead) */
    const std::vector<uint32_t>& LastParticleErrors() const { return last_errors_; }
    const std::vector<uint32_t>& LastMicrosteps() const { return last_micro_; }
    const std::vector<uint32_t>& LastResolverIterations() const { return last_resolver_; }
    /* the context of devices[0] (single-particle calls and batches that keep one device) */
    fks_context* Context() const { return ctx_; }
    const std::vector<int32_t>& Devices() const { return dev_->devices(); }
    /* the particles each listed device must get before a batch is sharded over it (0:
     * automatic = three times the resident waves of devices[0] for the current robot: a smaller shard
     * is bounded by its slowest particle's chain); 1 shards every batch over all
     * of Devices() */
    void SetShardThreshold(uint64_t particles_per_device) { dev_->set_shard_threshold(particles_per_device); }
    uint64_t ShardThreshold() const { return dev_->shard_threshold(); }
    /* whether the last batch call ran sharded, and over how many of Devices() */
    bool LastBatchSharded() const { return dev_->last_sharded(); }
    int32_t LastBatchDevices() const { return dev_->last_devices(); }
    /* batched CheckConfigCollision (SPCS:1398-1416, one configuration per call there),
     * sharded like the simulation batches */
    std::vector<uint8_t> CheckConfigCollisions(const std::shared_ptr<BaseRobotType>& immutable_robot,
                                               const std::vector<Configuration, ConfigAlloc>& configs, const double inflation_ratio) const {
        const DerivedRobotType& robot = Derived(immutable_robot);
        SetRobot(robot);
        std::vector<double> c;
        for (const auto& q : configs) {
            const std::vector<double> f = robot.ToFlat(q);
            c.insert(c.end(), f.begin(), f.end());
        }
        std::vector<uint8_t> collided(configs.size());
        dev_->check_configs(c.data(), configs.size(), inflation_ratio, collided.data(), nullptr, "CheckConfigCollisions");
        return collided;
    }
    /* Robot-shape specialisation (fks_set_specialization; no reference counterpart, results are
     * identical either way).  PrepareKernels builds `robot`'s kernel on every device now, so the
     * compile (2-20 s the first time on a machine, then from the disk cache) lands at setup and
     * not inside the first large ForwardSimulateRobots; SpecializationStatus reports whether the
     * calls run it, and the compiler log when its build failed (they then run the generic
     * kernel).  Neither throws on a failed build. */
    fks::SpecializationStatus PrepareKernels(const std::shared_ptr<BaseRobotType>& robot) {
        SetRobot(Derived(robot));
        return dev_->prepare_kernels(FKS_SPECIALIZE_ON);
    }
    fks::SpecializationStatus SpecializationStatus() const { return dev_->specialization_status(); }
    /* the configuration capacity a traced call starts with (a longer trace is re-run once with
     * the exact size); RetriedTraces() counts those re-runs */
    void SetTraceCapacityHint(uint32_t configs) { trace_capacity_hint_ = configs > 0 ? configs : 1; }
    uint32_t TraceCapacityHint() const { return trace_capacity_hint_; }
    uint64_t RetriedTraces() const { return retried_traces_; }

  private:
    static std::unique_ptr<fks::DeviceSet> MakeDevices(const sdf_tools::TaggedObjectCollisionMapGrid& environment,
                                                       const sdf_tools::SignedDistanceField& environment_sdf,
                                                       const SurfaceNormalGrid& surface_normals_grid,
                                                       const SimulatorSolverParameters& solver_config,
                                                       const double simulation_controller_frequency, const uint64_t prng_seed,
                                                       const int32_t debug_level, const std::vector<int32_t>& devices) {
        std::vector<float> sdf_storage; /* the values fks_create uploads (real sdf_tools only) */
        const fks_environment env =
            simulator_environment_builder::ToFksEnvironment(environment, environment_sdf, surface_normals_grid, sdf_storage);
        const fks_solver_params p = solver_config.ToFks();
        return std::unique_ptr<fks::DeviceSet>(
            new fks::DeviceSet(env, p, simulation_controller_frequency, prng_seed, debug_level, devices));
    }
    typedef fks_status (*BatchFn)(fks_context*, const double*, uint64_t, const double*, uint64_t, int32_t, double*, uint8_t*,
                                  uint32_t*, uint32_t*, uint32_t*);

    static void Check(fks_status st, const fks_context* ctx, const char* what) {
        if (st == FKS_OK) return;
        std::string msg = std::string(what) + ": " + fks_status_string(st);
        if (ctx) {
            const char* detail = fks_get_last_error(ctx);
            if (detail && detail[0]) msg += std::string(" (") + detail + ")";
        }
        throw fks::SimulatorError(st, msg);
    }
    static const DerivedRobotType& Derived(const std::shared_ptr<BaseRobotType>& robot) {
        if (!robot) throw std::invalid_argument("null robot");
        return *static_cast<const DerivedRobotType*>(robot.get()); /* SPCS:868 */
    }
    static fks_planner_types::Point Point(const double* p) {
        fks_planner_types::Point o;
        o.x = p[0];
        o.y = p[1];
        o.z = p[2];
        return o;
    }
    fks_planner_types::Marker MakeMarker(const std::string& ns, int32_t id, int32_t type, double scale, const ColorRGBA& color) const {
        fks_planner_types::Marker m;
        m.ns = ns;
        m.id = id;
        m.type = type;
        m.header.frame_id = GetFrame();
        m.scale.x = m.scale.y = m.scale.z = scale;
        m.color = color;
        return m;
    }
    uint32_t ForwardSteps() const {
        const double raw = solver_config_.forward_simulation_time * std::fabs(simulation_controller_frequency_);
        return raw >= 1.0 && raw < 4294967295.0 ? (uint32_t)raw : 1u; /* SPCS:856 */
    }
    /* the robot every particle clones: flattened once per description (clones share it).
     * The cache key owns the description, so a destroyed robot's address can never be
     * mistaken for a new robot's (the description is immutable once built). */
    void SetRobot(const DerivedRobotType& robot) const {
        const std::shared_ptr<const fks::RobotDescription>& d = robot.SharedHipDescription();
        if (d == robot_key_) return;
        robot_key_.reset();
        const fks_robot_desc v = d->View();
        dev_->set_robot(v);
        robot_key_ = d;
    }
    std::vector<double> Kinematics(const DerivedRobotType& robot, int32_t mode, const std::vector<std::vector<double>>& configs,
                                   const std::vector<std::vector<double>>& inputs = {}) const {
        SetRobot(robot);
        int32_t links = 0, points = 0, dofs = 0, width = 0;
        Check(fks_robot_sizes(ctx_, &links, &points, &dofs, &width), ctx_, "fks_robot_sizes");
        std::vector<double> c, u;
        for (const auto& q : configs) c.insert(c.end(), q.begin(), q.end());
        for (const auto& q : inputs) u.insert(u.end(), q.begin(), q.end());
        if (mode == FKS_KIN_APPLY_CONTROL_INPUT && u.size() != configs.size() * (size_t)dofs)
            throw std::invalid_argument("control input has the wrong width");
        const size_t per = mode == FKS_KIN_LINK_TRANSFORMS ? 12u * (size_t)links : (mode == FKS_KIN_POINTS ? 3u * (size_t)points : (size_t)width);
        std::vector<double> out(configs.size() * per);
        Check(fks_kinematics(ctx_, mode, c.data(), configs.size(), u.empty() ? nullptr : u.data(), out.data()), ctx_,
              "fks_kinematics");
        return out;
    }
    std::vector<SimulationResult> Batch(const DerivedRobotType& robot, const std::vector<Configuration, ConfigAlloc>& starts,
                                        const std::vector<Configuration, ConfigAlloc>& targets, bool allow_contacts, BatchFn fn) {
        if (!starts.empty() && targets.size() != 1 && targets.size() != starts.size())
            throw std::invalid_argument("target_positions must hold 1 or start_positions.size() configurations (SPCS:792)");
        SetRobot(robot);
        std::vector<double> s, t;
        for (const auto& c : starts) {
            const std::vector<double> f = robot.ToFlat(c);
            s.insert(s.end(), f.begin(), f.end());
        }
        for (const auto& c : targets) {
            const std::vector<double> f = robot.ToFlat(c);
            t.insert(t.end(), f.begin(), f.end());
        }
        const size_t n = starts.size(), W = n ? s.size() / n : 0;
        std::vector<double> q(n * W);
        std::vector<uint8_t> collided(n);
        last_micro_.assign(n, 0);
        last_resolver_.assign(n, 0);
        last_errors_.assign(n, 0);
        dev_->simulate(fn == fks_reverse_simulate, s.data(), n, t.data(), targets.size(), allow_contacts, q.data(), collided.data(),
                       last_micro_.data(), last_resolver_.data(), last_errors_.data(), "ForwardSimulateRobots");
        std::vector<SimulationResult> out;
        out.reserve(n);
        for (size_t i = 0; i < n; ++i) /* SimulationResult(reached, target, collided, true), SPCS:918 */
            out.emplace_back(robot.FromFlat(q.data() + i * W), targets.size() == n ? targets[i] : targets[0], collided[i] != 0, true);
        return out;
    }
    /* regroup the flat records into the reference's nesting: one resolver step per
     * controller step (SPCS:1583-1588), one contact-resolver step per (step, microstep)
     * (SPCS:1594), configurations in push order (SPCS:1617, 1703, 1714, 1778) */
    void AppendTrace(const DerivedRobotType& robot, ForwardSimulationStepTrace& trace, const std::vector<double>& inputs,
                     uint32_t num_steps, const std::vector<double>& configs, const std::vector<uint32_t>& tags, uint32_t num_configs,
                     size_t D) const {
        const size_t base = trace.resolver_steps.size(), W = configs.size() / (tags.size() / 3);
        for (uint32_t k = 0; k < num_steps; ++k) {
            typename decltype(trace.resolver_steps)::value_type rs;
            rs.control_input =
                fks_ext::vecx(std::vector<double>(inputs.begin() + (long)(k * 2 * D), inputs.begin() + (long)(k * 2 * D + D)));
            rs.control_input_step =
                fks_ext::vecx(std::vector<double>(inputs.begin() + (long)(k * 2 * D + D), inputs.begin() + (long)((k + 1) * 2 * D)));
            trace.resolver_steps.push_back(rs);
        }
        int64_t last_step = -1, last_micro = -1;
        for (uint32_t k = 0; k < num_configs; ++k) {
            const uint32_t st = tags[3 * k], mi = tags[3 * k + 1];
            auto& rs = trace.resolver_steps.at(base + st);
            if ((int64_t)st != last_step || (int64_t)mi != last_micro) rs.contact_resolver_steps.emplace_back();
            last_step = st;
            last_micro = mi;
            rs.contact_resolver_steps.back().contact_resolution_steps.push_back(robot.FromFlat(configs.data() + (size_t)k * W));
        }
    }

    sdf_tools::TaggedObjectCollisionMapGrid environment_;
    sdf_tools::SignedDistanceField environment_sdf_;
    SurfaceNormalGrid surface_normals_grid_;
    SimulatorSolverParameters solver_config_;
    double simulation_controller_frequency_;
    std::unique_ptr<fks::DeviceSet> dev_; /* the devices (DeviceSet: sharded batches, summed statistics) */
    fks_context* ctx_ = nullptr;          /* devices[0]: single-particle calls, small batches */
    mutable std::shared_ptr<const fks::RobotDescription> robot_key_;
    RNG rng_;
    std::vector<uint32_t> last_errors_, last_micro_, last_resolver_;
    uint32_t trace_capacity_hint_ = 16384;
    uint64_t retried_traces_ = 0;
};

}  // namespace simple_particle_contact_simulator

namespace fast_kinematic_simulator {

typedef simple_particle_contact_simulator::SimulatorSolverParameters SolverParameters;

/* FKS.hpp:13-16 */
inline SolverParameters GetDefaultSolverParameters() { return SolverParameters(); }

using fks::AllVisibleDevices;

/* FKS.hpp:18-22 / FKS.cpp:4-71: simulate_with_individual_jacobians = false.  The reference's
 * parameter list runs on every visible MI355X (batches sharded by particle, small batches on
 * the first); an extra `device` or `devices` argument selects them explicitly. */
#define FKS_DEFINE_FACTORY(NAME, PTR, ROBOT, CONFIG, ALLOC)                                                                          \
    inline uncertainty_planning_core::PTR NAME(                                                                                   \
        const sdf_tools::TaggedObjectCollisionMapGrid& environment, const sdf_tools::SignedDistanceField& environment_sdf,        \
        const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid, const SolverParameters& solver_config,  \
        const double simulation_controller_frequency, const uint64_t prng_seed, const int32_t debug_level,                        \
        const std::vector<int32_t>& devices) {                                                                                    \
        using namespace uncertainty_planning_core;                                                                                \
        return PTR(new simple_particle_contact_simulator::HipParticleContactSimulator<tnuva_robot_models::ROBOT<PRNG>, CONFIG, PRNG, \
                                                                                       ALLOC>(                                     \
            environment, environment_sdf, surface_normals_grid, solver_config, simulation_controller_frequency, false, prng_seed,  \
            debug_level, devices));                                                                                               \
    }                                                                                                                             \
    inline uncertainty_planning_core::PTR NAME(                                                                                   \
        const sdf_tools::TaggedObjectCollisionMapGrid& environment, const sdf_tools::SignedDistanceField& environment_sdf,        \
        const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid, const SolverParameters& solver_config,  \
        const double simulation_controller_frequency, const uint64_t prng_seed, const int32_t debug_level,                        \
        const int32_t device) {                                                                                                   \
        return NAME(environment, environment_sdf, surface_normals_grid, solver_config, simulation_controller_frequency, prng_seed, \
                    debug_level, std::vector<int32_t>{device});                                                                   \
    }                                                                                                                             \
    inline uncertainty_planning_core::PTR NAME(                                                                                   \
        const sdf_tools::TaggedObjectCollisionMapGrid& environment, const sdf_tools::SignedDistanceField& environment_sdf,        \
        const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid, const SolverParameters& solver_config,  \
        const double simulation_controller_frequency, const uint64_t prng_seed, const int32_t debug_level) {                     \
        return NAME(environment, environment_sdf, surface_normals_grid, solver_config, simulation_controller_frequency, prng_seed, \
                    debug_level, AllVisibleDevices());                                                                            \
    }

FKS_DEFINE_FACTORY(MakeSE2Simulator, SE2SimulatorPtr, TnuvaSE2Robot, SE2Config, SE2ConfigAlloc)
FKS_DEFINE_FACTORY(MakeSE3Simulator, SE3SimulatorPtr, TnuvaSE3Robot, SE3Config, SE3ConfigAlloc)
FKS_DEFINE_FACTORY(MakeLinkedSimulator, LinkedSimulatorPtr, TnuvaLinkedRobot, LinkedConfig, LinkedConfigAlloc)
#undef FKS_DEFINE_FACTORY

}  // namespace fast_kinematic_simulator

#endif
