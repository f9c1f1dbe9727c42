/*
 * Planner-side drop-in test: drives the HIP simulator only through
 * std::shared_ptr<simple_simulator_interface::SimulatorInterface<...>> as the
 * reference's planner does (FKS.hpp:18-22 factories, SPCS:446-1416 virtuals).
 *
 *   planner_interface_test <scene file> [--dump | --normals-out <file>]
 *
 * The scene (written by tests/test_planner_interface.py) gives the robot's constructor
 * arguments (TnuvaLinkedRobot TNUVA:486-517, TnuvaSE2Robot 109-132, TnuvaSE3Robot
 * 293-325), the obstacles for BuildCompleteEnvironment (SEB.cpp:470-476), the solver
 * parameters, starts and targets.  Every number is printed as a C99 hex float so the
 * Python side compares with the CPU oracle bit for bit.  Exit status 3 = no GPU.
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <cmath>
#include <iostream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/fast_kinematic_simulator.hpp"
/* the reference's two remaining public headers, by the include paths planner code uses */
#include <fast_kinematic_simulator/simple_pid_controller.hpp>
#include <fast_kinematic_simulator/simple_uncertainty_models.hpp>

namespace upc = uncertainty_planning_core;
using fks_planner_types::Isometry3d;
using fks_planner_types::Vector3d;
using fks_planner_types::Vector4d;
/* the point container PointSphereGeometry holds (EigenHelpers::VectorVector4d in a planner workspace) */
typedef std::remove_cv<std::remove_reference<decltype(*std::declval<simple_robot_models::PointSphereGeometry>().Geometry())>::type>::type Points;

struct Reader {
    std::ifstream in;
    explicit Reader(const char* path) : in(path) {
        if (!in) throw std::runtime_error("cannot open scene file");
    }
    std::string word() {
        std::string w;
        if (!(in >> w)) throw std::runtime_error("truncated scene file");
        return w;
    }
    double num() { return std::strtod(word().c_str(), nullptr); }
    int64_t integer() { return std::strtoll(word().c_str(), nullptr, 10); }
    void expect(const char* tag) {
        const std::string w = word();
        if (w != tag) throw std::runtime_error("scene file: expected " + std::string(tag) + ", got " + w);
    }
    Isometry3d iso() {
        double m[12];
        for (double& v : m) v = num();
        return fks_ext::iso_from_row_major34(m);
    }
    /* one value per call, in file order (function-argument evaluation order is unspecified) */
    Vector3d vec3() {
        const std::vector<double> v = nums(3);
        return Vector3d(v[0], v[1], v[2]);
    }
    Vector4d vec4() {
        const std::vector<double> v = nums(4);
        return Vector4d(v[0], v[1], v[2], v[3]);
    }
    std::vector<double> nums(size_t n) {
        std::vector<double> v(n);
        for (double& x : v) x = num();
        return v;
    }
};

static void hex(const double v) { std::printf(" %a", v); }

struct Scene {
    std::string family;
    double frequency = 0.0;
    uint64_t seed = 0;
    bool allow = true;
    fast_kinematic_simulator::SolverParameters solver;
    std::unique_ptr<simulator_environment_builder::EnvironmentComponents> env;
    std::vector<simulator_environment_builder::OBSTACLE_CONFIG> obstacles;
};

static Scene read_common(Reader& r) {
    Scene s;
    r.expect("family");
    s.family = r.word();
    r.expect("frequency");
    s.frequency = r.num();
    r.expect("seed");
    s.seed = (uint64_t)r.integer();
    r.expect("allow");
    s.allow = r.integer() != 0;
    r.expect("solver");
    s.solver.forward_simulation_time = r.num();
    s.solver.simulation_shortcut_distance = r.num();
    s.solver.environment_collision_check_tolerance = r.num();
    s.solver.resolve_correction_step_scaling_decay_rate = r.num();
    s.solver.resolve_correction_initial_step_size = r.num();
    s.solver.resolve_correction_min_step_scaling = r.num();
    s.solver.max_resolver_iterations = (uint32_t)r.integer();
    s.solver.resolve_correction_step_scaling_decay_iterations = (uint32_t)r.integer();
    s.solver.failed_resolves_end_motion = r.integer() != 0;
    r.expect("env");
    const double res = r.num();
    const std::vector<double> origin = r.nums(12);
    const int64_t cells[3] = {r.integer(), r.integer(), r.integer()};
    const int64_t nobs = r.integer();
    std::vector<simulator_environment_builder::OBSTACLE_CONFIG>& obstacles = s.obstacles;
    for (int64_t k = 0; k < nobs; ++k) {
        const Isometry3d pose = r.iso();
        const Vector3d ext = r.vec3();
        obstacles.emplace_back((uint32_t)r.integer(), pose, ext);
    }
    s.env.reset(new simulator_environment_builder::EnvironmentComponents(
        simulator_environment_builder::BuildCompleteEnvironment(obstacles, res, origin.data(), cells)));
    return s;
}

static simple_robot_models::PointSphereGeometry read_points(Reader& r) {
    const int64_t n = r.integer();
    auto pts = std::make_shared<Points>();
    for (int64_t i = 0; i < n; ++i) pts->push_back(r.vec4());
    return simple_robot_models::PointSphereGeometry(simple_robot_models::PointSphereGeometry::POINTS, pts);
}

/* --dump: the flattened robot the GPU receives and the flat starts / targets (no GPU needed) */
static bool g_dump = false;

/* the devices the simulators run on: FKS_TEST_DEVICES="0,0" (a list), "all" (every visible
 * device, the factories' default), unset = {0}; FKS_TEST_SHARD=<n> sets the shard threshold
 * (1: every batch is sharded over the list).  The printed results must not depend on either. */
static std::vector<int32_t> test_devices() {
    const char* e = std::getenv("FKS_TEST_DEVICES");
    if (!e || !e[0]) return {0};
    if (std::string(e) == "all") return fks::AllVisibleDevices();
    std::vector<int32_t> d;
    std::stringstream ss(e);
    std::string tok;
    while (std::getline(ss, tok, ',')) d.push_back((int32_t)std::stoi(tok));
    return d;
}
template <typename Hip>
static void apply_shard_threshold(Hip* hip) {
    const char* e = std::getenv("FKS_TEST_SHARD");
    if (hip && e && e[0]) hip->SetShardThreshold(std::strtoull(e, nullptr, 10));
}

/* FNV-1a of a byte range (environment fingerprints in --dump) */
static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

/* --dump, environment side (no GPU): the builder's public steps on the scene's obstacles */
static void dump_environment(const Scene& s, const std::vector<simulator_environment_builder::OBSTACLE_CONFIG>& obstacles) {
    namespace seb = simulator_environment_builder;
    const auto& E = *s.env;
    const auto& N = E.GetSurfaceNormalsGrid();
    const uint64_t cells = (uint64_t)N.GetNumXCells() * (uint64_t)N.GetNumYCells() * (uint64_t)N.GetNumZCells();
    const uint32_t* off = N.CsrOffsets();
    std::printf("env_normals %u %llx %llx\n", off[cells], (unsigned long long)fnv(off, 4 * (size_t)(cells + 1)),
                (unsigned long long)(off[cells] ? fnv(N.CsrEntries(), 48 * (size_t)off[cells]) : 0ull));
    /* BuildSurfaceNormalsGrid on the complete environment's SDF gives the same grid */
    const auto again = seb::BuildSurfaceNormalsGrid(obstacles, E.GetEnvironmentSDF());
    const uint32_t* off2 = again.CsrOffsets();
    std::printf("env_normals_again %u %llx %llx\n", off2[cells], (unsigned long long)fnv(off2, 4 * (size_t)(cells + 1)),
                (unsigned long long)(off2[cells] ? fnv(again.CsrEntries(), 48 * (size_t)off2[cells]) : 0ull));
    /* object ids of the collision map (SEB.cpp:151-155) */
    std::map<uint32_t, uint64_t> ids;
    const auto& G = E.GetEnvironment();
    for (int64_t x = 0; x < G.GetNumXCells(); ++x)
        for (int64_t y = 0; y < G.GetNumYCells(); ++y)
            for (int64_t z = 0; z < G.GetNumZCells(); ++z) {
                const auto c = G.GetImmutable(x, y, z).first;
                if (c.occupancy > 0.5f) ids[c.object_id]++;
            }
    std::printf("env_ids");
    for (const auto& kv : ids) std::printf(" %u:%llu", kv.first, (unsigned long long)kv.second);
    std::printf("\n");
    /* DiscretizeObstacle of the first obstacle, and OBSTACLE_CONFIG's quaternion constructor */
    const auto d = seb::DiscretizeObstacle(obstacles.front(), G.GetResolution());
    std::printf("env_discretize %zu %a %a %a %u\n", d.size(), d.front().first(0), d.front().first(1), d.front().first(2),
                d.front().second.object_id);
    const double h = 0.5 * std::sqrt(2.0);
    const seb::OBSTACLE_CONFIG q(7u, Vector3d(0.1, 0.2, 0.3), fks_planner_types::Quaterniond(h, 0.0, 0.0, h), Vector3d(0.1, 0.2, 0.3));
    std::printf("env_quat");
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) hex(q.pose.matrix()(r, c));
    std::printf("\n");
}
template <typename Configs, typename Robot>
static int dump(const Robot& robot, const Configs& starts, const Configs& targets) {
    const fks::RobotDescription& d = robot.HipDescription();
    std::printf("types %s\n", FKS_EXTERNAL_PLANNER_TYPES ? "workspace" : "standalone"); /* fks_external_types.hpp */
    std::printf("type %d links %d dofs %d\nbase", (int)d.type, d.num_links, d.num_dofs);
    for (double v : d.base_transform) hex(v);
    std::printf("\njoints");
    for (const auto& j : d.joints) {
        std::printf(" %d %d %d", j.parent_link, j.child_link, j.type);
        for (double v : j.origin) hex(v);
        for (double v : j.axis) hex(v);
        hex(j.limit_lower);
        hex(j.limit_upper);
    }
    std::printf("\ngeometry_link");
    for (int32_t v : d.geometry_link) std::printf(" %d", v);
    std::printf("\noffsets");
    for (uint32_t v : d.geometry_point_offset) std::printf(" %u", v);
    std::printf("\npoints");
    for (double v : d.points) hex(v);
    std::printf("\nallowed");
    for (int32_t v : d.allowed_pairs) std::printf(" %d", v);
    std::printf("\ncontrollers");
    for (const auto& c : d.controllers)
        for (double v : {c.kp, c.ki, c.kd, c.integral_clamp, c.velocity_limit, c.acceleration_limit, c.max_sensor_noise,
                         c.max_actuator_proportional_noise, c.max_actuator_minimum_noise})
            hex(v);
    std::printf("\nweights");
    for (double v : d.distance_weights) hex(v);
    std::printf("\nstarts");
    for (const auto& c : starts)
        for (double v : robot.ToFlat(c)) hex(v);
    std::printf("\ntargets");
    for (const auto& c : targets)
        for (double v : robot.ToFlat(c)) hex(v);
    std::printf("\n");
    return 0;
}

/* one robot stepped by hand through the TnuvaRobot interface (TNUVA:15-23), as execution
 * code does: GenerateControlAction, then ApplyControlInput(u) on even steps and
 * ApplyControlInput(u, rng) on odd ones (std::mt19937_64(seed + 77)); prints every control
 * and configuration, then the controllers' state */
template <typename Robot, typename Config>
static void step_by_hand(const Scene& s, const Robot& prototype, const Config& start, const Config& target) {
    std::unique_ptr<Robot> robot(static_cast<Robot*>(prototype.Clone()));
    robot->ResetPosition(start);
    upc::PRNG rng(s.seed + 77);
    for (int k = 0; k < 12; ++k) {
        const auto u = robot->GenerateControlAction(target, 1.0 / s.frequency);
        std::printf("hand_u %d", k);
        for (int64_t d = 0; d < (int64_t)u.size(); ++d) hex(u(d));
        std::printf("\n");
        if (k % 2 == 0)
            robot->ApplyControlInput(u);
        else
            robot->ApplyControlInput(u, rng);
        std::printf("hand_q %d", k);
        for (double v : robot->ToFlat(robot->GetPosition())) hex(v);
        std::printf("\n");
    }
    std::printf("hand_pid");
    for (double v : robot->ControllerState()) hex(v);
    std::printf("\n");
    robot->ResetControllers();
    std::printf("hand_reset %d\n", robot->ControllersAreZero() ? 1 : 0);
}

/* a surface-normal grid made through the SurfaceNormalGrid API (SPCS:138-343) and the
 * builder's public steps (SEB.hpp:61-70): the built grid's entries re-inserted cell by cell
 * with InsertSurfaceNormal, then AdjustSurfaceNormalGridForAllFlatSurfaces and one
 * UpdateSurfaceNormalGridCell; its CSR is written to `path` (offsets then entries, raw) for
 * the oracle, and a simulator made over it runs the batch (fresh simulator, call index 0) */
template <typename Robot, typename Configs>
static void custom_normals(const Scene& s, const std::shared_ptr<Robot>& robot, const Configs& starts, const Configs& targets,
                           const char* path) {
    namespace seb = simulator_environment_builder;
    const auto& E = *s.env;
    const simple_particle_contact_simulator::SurfaceNormalGrid& built = E.GetSurfaceNormalsGrid();
    const double res = built.GetResolution();
    simple_particle_contact_simulator::SurfaceNormalGrid grid(built.GetOriginTransform(), res, ((double)built.GetNumXCells() - 0.5) * res,
                                                              ((double)built.GetNumYCells() - 0.5) * res,
                                                              ((double)built.GetNumZCells() - 0.5) * res);
    std::printf("custom_init %d %d\n", simple_particle_contact_simulator::SurfaceNormalGrid().IsInitialized() ? 1 : 0,
                grid.IsInitialized() ? 1 : 0);
    size_t inserted = 0;
    for (int64_t x = 0; x < built.GetNumXCells(); ++x)
        for (int64_t y = 0; y < built.GetNumYCells(); ++y)
            for (int64_t z = 0; z < built.GetNumZCells(); ++z)
                for (const auto& e : built.GetCellEntries(x, y, z)) {
                    grid.InsertSurfaceNormal(x, y, z, e.second, Vector3d(e.first(0), e.first(1), e.first(2)));
                    inserted++;
                }
    seb::AdjustSurfaceNormalGridForAllFlatSurfaces(E.GetEnvironmentSDF(), grid);
    const Vector3d probe(0.3, 0.02, 0.5);
    seb::UpdateSurfaceNormalGridCell({seb::RawCellSurfaceNormal(Vector3d(0.0, 0.0, 1.0), Vector3d(0.0, 0.0, -1.0))},
                                     fks_planner_types::Isometry3d::Identity(), probe, E.GetEnvironmentSDF(), grid);
    const auto look = grid.LookupSurfaceNormal(probe, Vector3d(0.0, 0.0, -1.0));
    std::printf("custom_lookup %d %a %a %a %zu\n", look.second ? 1 : 0, look.first(0), look.first(1), look.first(2), inserted);
    const uint64_t cells = (uint64_t)grid.GetNumXCells() * (uint64_t)grid.GetNumYCells() * (uint64_t)grid.GetNumZCells();
    const uint32_t* off = grid.CsrOffsets();
    FILE* f = std::fopen(path, "wb");
    if (!f) throw std::runtime_error("cannot write the normals file");
    std::fwrite(off, sizeof(uint32_t), (size_t)cells + 1, f);
    if (off[cells]) std::fwrite(grid.CsrEntries(), sizeof(double), 6 * (size_t)off[cells], f);
    std::fclose(f);
    upc::LinkedSimulatorPtr sim = fast_kinematic_simulator::MakeLinkedSimulator(E.GetEnvironment(), E.GetEnvironmentSDF(), grid, s.solver,
                                                                                s.frequency, s.seed, 0, test_devices());
    apply_shard_threshold(dynamic_cast<simple_particle_contact_simulator::HipParticleContactSimulator<
                              tnuva_robot_models::TnuvaLinkedRobot<upc::PRNG>, upc::LinkedConfig, upc::PRNG, upc::LinkedConfigAlloc>*>(sim.get()));
    const auto res_c = sim->ForwardSimulateRobots(robot, starts, targets, s.allow, {});
    for (size_t i = 0; i < res_c.size(); ++i) {
        std::printf("custom %zu", i);
        for (double v : robot->ToFlat(res_c[i].result_config)) hex(v);
        std::printf(" %d\n", res_c[i].did_contact ? 1 : 0);
    }
}

/* `--pid-replay`: SimplePIDController (PID:55-136) over error sequences from stdin, lines
 * "kp ki kd iclamp n" then n lines "error timestep zero" (zero = 1: Zero() before the step);
 * prints one hex-float ComputeFeedbackTerm output per step */
static int pid_replay() {
    double kp, ki, kd, iclamp;
    long n = 0;
    while (std::scanf("%la %la %la %la %ld", &kp, &ki, &kd, &iclamp, &n) == 5) {
        simple_pid_controller::SimplePIDController pid(simple_pid_controller::PIDParams(kp, ki, kd, iclamp));
        if (!pid.IsInitialized()) return 1;
        for (long i = 0; i < n; ++i) {
            double e, dt;
            int zero = 0;
            if (std::scanf("%la %la %d", &e, &dt, &zero) != 3) return 1;
            if (zero) pid.Zero();
            std::printf("%a\n", pid.ComputeFeedbackTerm(e, dt));
        }
    }
    return 0;
}

/* `--sampled <csv>` (linked scenes): every dof's actuator a SampledUncertainVelocityActuator
 * whose model LoadModel (UNC:156-222) builds from the CSV (8 bins, 32 samples, seed = scene
 * seed + dof); the models go into the robot's description (SetSampledActuator) and the plain
 * C++ simulator runs the batch on the GPU.  Prints the bins (for the oracle) and the results. */
template <typename Robot, typename Configs>
static int sampled_actuators(const Scene& s, const Robot& robot, const Configs& starts, const Configs& targets, const char* csv) {
    namespace sum = simple_uncertainty_models;
    fks::RobotDescription desc = robot.HipDescription();
    for (int32_t k = 0; k < desc.NumDofs(); ++k) {
        const double vmax = std::abs(desc.controllers[(size_t)k].velocity_limit);
        const std::shared_ptr<sum::JointUncertaintySampleModel> model = sum::LoadModel(csv, vmax, 8, 32, s.seed + (uint64_t)k);
        /* the host actuator over the same model: clamp, then the picked sample */
        const sum::SampledUncertainVelocityActuator act(model, vmax);
        std::mt19937_64 rng(5);
        const double probe = act.GetControlValue(0.25 * vmax, rng), clamp = act.GetControlValue(3.0 * vmax);
        std::printf("host_sampled %d %a %a %d\n", k, probe, clamp, act.IsInitialized() ? 1 : 0);
        sum::SetSampledActuator(desc, k, *model);
        std::printf("bins %d", k);
        for (const auto& bin : *model) {
            hex(bin.first.first);
            hex(bin.first.second);
        }
        std::printf("\nsamples %d", k);
        for (const auto& bin : *model)
            for (double v : bin.second) hex(v);
        std::printf("\n");
    }
    std::vector<float> sdf_storage;
    const auto& E = *s.env;
    const fks_environment env =
        simulator_environment_builder::ToFksEnvironment(E.GetEnvironment(), E.GetEnvironmentSDF(), E.GetSurfaceNormalsGrid(), sdf_storage);
    fks::HipParticleContactSimulator sim(env, s.solver.ToFks(), s.frequency, s.seed, 0, test_devices());
    std::vector<std::vector<double>> st, tg;
    for (const auto& c : starts) st.push_back(robot.ToFlat(c));
    for (const auto& c : targets) tg.push_back(robot.ToFlat(c));
    const auto res = sim.ForwardSimulateRobots(desc, st, tg, s.allow);
    for (size_t i = 0; i < res.size(); ++i) {
        std::printf("sampled %zu", i);
        for (double v : res[i].result_config) hex(v);
        std::printf(" %d %u\n", res[i].did_contact ? 1 : 0, res[i].error_flags);
    }
    /* the truncated-normal models of the same header: sensor and velocity actuator */
    const sum::TruncatedNormalUncertainSensor sensor(-0.1, 0.1);
    const sum::TruncatedNormalUncertainVelocityActuator tn(1.0, 2.0, 0.5, 0.1, 0.5);
    std::mt19937_64 rng(11);
    double smin = 1e300, smax = -1e300, amin = 1e300, amax = -1e300;
    for (int i = 0; i < 4000; ++i) {
        const double v = sensor.GetSensorValue(1.0, rng) - 1.0;
        smin = std::min(smin, v);
        smax = std::max(smax, v);
        const double a = tn.GetControlValue(0.4, rng) - 0.4;
        amin = std::min(amin, a);
        amax = std::max(amax, a);
    }
    std::printf("tn_models %a %a %a %a %a %a %a\n", smin, smax, amin, amax, tn.GetControlValue(5.0), tn.GetMaxVelocityNoise(),
                tn.GetMaxVelocityNoise(-0.5));
    return 0;
}

/* the interface calls every family goes through; `to_flat` prints a configuration */
template <typename Config, typename Alloc, typename Robot>
static int exercise(const Scene& s, const std::shared_ptr<simple_simulator_interface::SimulatorInterface<Config, upc::PRNG, Alloc>>& sim,
                    const std::shared_ptr<Robot>& robot, const std::vector<Config, Alloc>& starts,
                    const std::vector<Config, Alloc>& targets) {
    typedef simple_simulator_interface::SimulatorInterface<Config, upc::PRNG, Alloc> Interface;
    const std::shared_ptr<typename Interface::BaseRobotType> base = robot;
    auto print = [&](const char* tag, size_t i, const typename Interface::SimulationResult& res) {
        std::printf("%s %zu", tag, i);
        for (double v : robot->ToFlat(res.result_config)) hex(v);
        std::printf(" %d %d\n", res.did_contact ? 1 : 0, res.outcome_is_valid ? 1 : 0);
    };
    auto* hip = dynamic_cast<simple_particle_contact_simulator::HipParticleContactSimulator<Robot, Config, upc::PRNG, Alloc>*>(sim.get());
    if (!hip) throw std::runtime_error("the factory did not return the HIP simulator");
    apply_shard_threshold(hip);
    /* the shape-specialised kernel built at setup, on every device (PrepareKernels), so the
     * first batch does not pay the compile; a failed build would only fall back (same bytes) */
    {
        const fks::SpecializationStatus st = hip->PrepareKernels(base);
        std::fprintf(stderr, "kernels %s active %d failed %d%s%s\n", st.shape.c_str(), st.active ? 1 : 0, st.failed ? 1 : 0,
                     st.failed ? ": " : "", st.message.c_str());
        if (st.per_device.size() != hip->Devices().size()) throw std::runtime_error("one specialisation status per device");
    }
    /* call index 0: ForwardSimulateRobots (SPCS:788) */
    const auto fwd = sim->ForwardSimulateRobots(base, starts, targets, s.allow, [](const fks_planner_types::MarkerArray&) {});
    std::fprintf(stderr, "devices %zu sharded %d over %d\n", hip->Devices().size(), hip->LastBatchSharded() ? 1 : 0,
                 hip->LastBatchDevices());
    for (size_t i = 0; i < fwd.size(); ++i) print("fwd", i, fwd[i]);
    for (const auto& kv : sim->GetStatistics()) std::printf("stat %s %.0f\n", kv.first.c_str(), kv.second);
    /* call index 1: ReverseSimulateRobots (SPCS:806) */
    const auto rev = sim->ReverseSimulateRobots(base, starts, targets, s.allow, {});
    for (size_t i = 0; i < rev.size(); ++i) print("rev", i, rev[i]);
    /* call index 2: ForwardSimulateRobot with tracing (SPCS:824) of particle 0, started with a
     * trace capacity of 8 configurations so the longer trace is re-run at its exact size; the
     * statistics must count the particle once (reset before, printed after) */
    typename Interface::ForwardSimulationStepTrace trace;
    hip->SetTraceCapacityHint(8);
    sim->ResetStatistics();
    const auto tr = sim->ForwardSimulateRobot(base, starts[0], targets[0], s.allow, trace, true, {});
    print("traced", 0, tr);
    std::printf("traced_retries %llu\n", (unsigned long long)hip->RetriedTraces());
    for (const auto& kv : sim->GetStatistics()) std::printf("stat_traced %s %.0f\n", kv.first.c_str(), kv.second);
    size_t configs = 0;
    for (const auto& rs : trace.resolver_steps)
        for (const auto& c : rs.contact_resolver_steps) configs += c.contact_resolution_steps.size();
    std::printf("trace %zu %zu", trace.resolver_steps.size(), configs);
    for (int64_t k = 0; k < trace.resolver_steps.front().control_input.size(); ++k) hex(trace.resolver_steps.front().control_input(k));
    std::printf("\n");
    /* CheckConfigCollision (SPCS:1398) of every reached configuration, inflation 0.5 */
    std::printf("check");
    for (const auto& r : fwd) std::printf(" %d", sim->CheckConfigCollision(base, r.result_config, 0.5) ? 1 : 0);
    std::printf("\n");
    /* the same configurations in one batched call (sharded like the simulation batches) */
    std::vector<Config, Alloc> reached;
    for (const auto& r : fwd) reached.push_back(r.result_config);
    std::printf("check_batch");
    for (uint8_t c : hip->CheckConfigCollisions(base, reached, 0.5)) std::printf(" %d", (int)c);
    std::printf("\n");
    /* call indices 3 and 4: ForwardSimulateMutableRobot (SPCS:843) twice on one robot, the
     * second continuing the first's controllers */
    std::shared_ptr<typename Interface::BaseRobotType> mutable_robot(base->Clone());
    static_cast<Robot*>(mutable_robot.get())->ResetPosition(starts[0]);
    typename Interface::ForwardSimulationStepTrace unused;
    const auto m1 = sim->ForwardSimulateMutableRobot(mutable_robot, targets[0], s.allow, unused, false, {});
    print("mut1", 0, m1);
    const auto m2 = sim->ReverseSimulateMutableRobot(mutable_robot, starts[0], s.allow, unused, false, {});
    print("mut2", 0, m2);
    std::printf("pid");
    for (double v : static_cast<Robot*>(mutable_robot.get())->ControllerState()) hex(v);
    std::printf("\n");
    /* display helpers through the interface */
    const Vector4d p = sim->Get3dPointForConfig(base, fwd[0].result_config);
    std::printf("point %a %a %a %a\n", p(0), p(1), p(2), p(3));
    const auto rep = sim->MakeConfigurationDisplayRep(base, fwd[0].result_config, Interface::MakeColor(0.f, 1.f, 0.f, 1.f), 3, "cfg");
    std::printf("markers %zu %zu %s\n", rep.markers.size(), rep.markers[0].points.size(), sim->GetFrame().c_str());
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <scene> [--dump]\n", argv[0]);
        return 2;
    }
    if (std::string(argv[1]) == "--pid-replay") return pid_replay();
    g_dump = argc > 2 && std::string(argv[2]) == "--dump";
    const char* sampled_csv = (argc > 3 && std::string(argv[2]) == "--sampled") ? argv[3] : nullptr;
    const bool hand_only = argc > 2 && std::string(argv[2]) == "--hand"; /* TnuvaRobot stepping only: no GPU */
    const char* normals_out = (argc > 3 && std::string(argv[2]) == "--normals-out") ? argv[3] : nullptr;
    try {
        Reader r(argv[1]);
        const Scene s = read_common(r);
        const auto& E = *s.env;
        if (s.family == "linked") {
            typedef tnuva_robot_models::TnuvaLinkedRobot<upc::PRNG> Robot;
            r.expect("base");
            const Isometry3d base = r.iso();
            r.expect("links");
            std::vector<simple_linked_robot_model::RobotLink> links((size_t)r.integer());
            for (size_t l = 0; l < links.size(); ++l) links[l].link_name = "link_" + std::to_string(l);
            r.expect("joints");
            const int64_t J = r.integer();
            std::vector<simple_linked_robot_model::RobotJoint> joints;
            upc::LinkedConfig initial;
            for (int64_t j = 0; j < J; ++j) {
                simple_linked_robot_model::RobotJoint jt;
                jt.parent_link_index = r.integer();
                jt.child_link_index = r.integer();
                const auto type = (simple_linked_robot_model::SimpleJointModel::JOINT_TYPE)r.integer();
                jt.joint_transform = r.iso();
                jt.joint_axis = r.vec3();
                const double lo = r.num(), hi = r.num();
                jt.joint_model = simple_linked_robot_model::SimpleJointModel({lo, hi}, 0.0, type);
                if (!jt.joint_model.IsFixed()) initial.push_back(jt.joint_model);
                joints.push_back(jt);
            }
            r.expect("geoms");
            const int64_t G = r.integer();
            std::vector<std::pair<std::string, simple_robot_models::PointSphereGeometry>> geoms;
            for (int64_t g = 0; g < G; ++g) {
                const int64_t link = r.integer();
                geoms.emplace_back(links[(size_t)link].link_name, read_points(r));
            }
            r.expect("allowed");
            std::vector<std::pair<size_t, size_t>> allowed((size_t)r.integer());
            for (auto& a : allowed) a = {(size_t)r.integer(), (size_t)r.integer()};
            r.expect("controllers");
            std::vector<Robot::LINKED_ROBOT_CONFIG> ctrl((size_t)r.integer());
            for (auto& c : ctrl) {
                const std::vector<double> v = r.nums(9);
                c = Robot::LINKED_ROBOT_CONFIG(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]);
            }
            r.expect("weights");
            const std::vector<double> weights = r.nums((size_t)r.integer());
            auto robot = std::make_shared<Robot>(base, links, joints, initial, weights, geoms, allowed, ctrl);
            auto read_configs = [&](const char* tag) {
                r.expect(tag);
                const int64_t n = r.integer();
                std::vector<upc::LinkedConfig> v;
                for (int64_t i = 0; i < n; ++i) {
                    const std::vector<double> f = r.nums(initial.size());
                    v.push_back(robot->FromFlat(f.data()));
                }
                return v;
            };
            const auto starts = read_configs("starts");
            const auto targets = read_configs("targets");
            if (g_dump) {
                dump_environment(s, s.obstacles);
                return dump(*robot, starts, targets);
            }
            if (hand_only) {
                step_by_hand(s, *robot, starts[0], targets[0]);
                return 0;
            }
            if (sampled_csv) return sampled_actuators(s, *robot, starts, targets, sampled_csv);
            upc::LinkedSimulatorPtr sim = fast_kinematic_simulator::MakeLinkedSimulator(
                E.GetEnvironment(), E.GetEnvironmentSDF(), E.GetSurfaceNormalsGrid(), s.solver, s.frequency, s.seed, 0, test_devices());
            const int rc = exercise<upc::LinkedConfig, upc::LinkedConfigAlloc>(s, sim, robot, starts, targets);
            if (rc != 0) return rc;
            step_by_hand(s, *robot, starts[0], targets[0]);
            if (normals_out) custom_normals(s, robot, starts, targets, normals_out);
            /* Two robots alternating on one simulator, each destroyed before the next is made
             * (call indices 5-8): "other" keeps only the first point of every geometry, "same"
             * is rebuilt from the scene's arguments and must reproduce the oracle's run of the
             * scene robot; a simulator that recognised robots by address could hand a new robot
             * a destroyed one's tables. */
            auto make_other = [&]() {
                std::vector<std::pair<std::string, simple_robot_models::PointSphereGeometry>> one;
                for (const auto& g : geoms) {
                    auto pts = std::make_shared<Points>(1, g.second.Geometry()->front());
                    one.emplace_back(g.first, simple_robot_models::PointSphereGeometry(simple_robot_models::PointSphereGeometry::POINTS, pts));
                }
                return std::make_shared<Robot>(base, links, joints, initial, weights, one, allowed, ctrl);
            };
            typedef simple_simulator_interface::SimulatorInterface<upc::LinkedConfig, upc::PRNG, upc::LinkedConfigAlloc> Interface;
            auto print_alt = [&](const char* tag, int call, const std::vector<Interface::SimulationResult>& res) {
                for (size_t i = 0; i < res.size(); ++i) {
                    std::printf("%s %d %zu", tag, call, i);
                    for (double v : robot->ToFlat(res[i].result_config)) hex(v);
                    std::printf(" %d\n", res[i].did_contact ? 1 : 0);
                }
            };
            for (int call = 5; call < 9; call += 2) {
                {
                    std::shared_ptr<Interface::BaseRobotType> other = make_other();
                    print_alt("alt_other", call, sim->ForwardSimulateRobots(other, starts, targets, s.allow, {}));
                }
                std::shared_ptr<Interface::BaseRobotType> same =
                    std::make_shared<Robot>(base, links, joints, initial, weights, geoms, allowed, ctrl);
                print_alt("alt_same", call + 1, sim->ForwardSimulateRobots(same, starts, targets, s.allow, {}));
            }
            return 0;
        }
        /* SE(2) / SE(3): pos weight, rot weight, points, the 18 gains of the config */
        const double pw = r.num(), rw = r.num();
        const simple_robot_models::PointSphereGeometry geometry = read_points(r);
        const std::vector<double> c = r.nums(18);
        const tnuva_robot_models::AXIS_ROBOT_CONFIG cfg(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8], c[9], c[10], c[11],
                                                        c[12], c[13], c[14], c[15], c[16], c[17]);
        if (s.family == "se2") {
            typedef tnuva_robot_models::TnuvaSE2Robot<upc::PRNG> Robot;
            auto robot = std::make_shared<Robot>(upc::SE2Config(0.0, 0.0, 0.0), pw, rw, "body", geometry, cfg);
            auto read_configs = [&](const char* tag) {
                r.expect(tag);
                const int64_t n = r.integer();
                std::vector<upc::SE2Config> v;
                for (int64_t i = 0; i < n; ++i) {
                    const std::vector<double> f = r.nums(3);
                    v.push_back(robot->FromFlat(f.data()));
                }
                return v;
            };
            const auto starts = read_configs("starts");
            const auto targets = read_configs("targets");
            if (g_dump) return dump(*robot, starts, targets);
            if (hand_only) {
                step_by_hand(s, *robot, starts[0], targets[0]);
                return 0;
            }
            upc::SE2SimulatorPtr sim = fast_kinematic_simulator::MakeSE2Simulator(
                E.GetEnvironment(), E.GetEnvironmentSDF(), E.GetSurfaceNormalsGrid(), s.solver, s.frequency, s.seed, 0, test_devices());
            const int rc = exercise<upc::SE2Config, upc::SE2ConfigAlloc>(s, sim, robot, starts, targets);
            if (rc == 0) step_by_hand(s, *robot, starts[0], targets[0]);
            return rc;
        }
        typedef tnuva_robot_models::TnuvaSE3Robot<upc::PRNG> Robot;
        auto robot = std::make_shared<Robot>(upc::SE3Config::Identity(), pw, rw, "body", geometry, cfg);
        auto read_configs = [&](const char* tag) {
            r.expect(tag);
            const int64_t n = r.integer();
            std::vector<upc::SE3Config, upc::SE3ConfigAlloc> v; /* Eigen::aligned_allocator in the planner (UPC.cpp:131) */
            for (int64_t i = 0; i < n; ++i) {
                const std::vector<double> f = r.nums(12);
                v.push_back(robot->FromFlat(f.data()));
            }
            return v;
        };
        const auto starts = read_configs("starts");
        const auto targets = read_configs("targets");
        if (g_dump) return dump(*robot, starts, targets);
        if (hand_only) {
            step_by_hand(s, *robot, starts[0], targets[0]);
            return 0;
        }
        upc::SE3SimulatorPtr sim = fast_kinematic_simulator::MakeSE3Simulator(
            E.GetEnvironment(), E.GetEnvironmentSDF(), E.GetSurfaceNormalsGrid(), s.solver, s.frequency, s.seed, 0, test_devices());
        const int rc = exercise<upc::SE3Config, upc::SE3ConfigAlloc>(s, sim, robot, starts, targets);
        if (rc == 0) step_by_hand(s, *robot, starts[0], targets[0]);
        return rc;
    } catch (const fks::SimulatorError& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return e.status() == FKS_ERR_NO_DEVICE ? 3 : 1;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
}
