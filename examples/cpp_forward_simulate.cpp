/*
 * C++ usage of the drop-in simulator (include/fast_kinematic_simulator_amd/
 * hip_particle_contact_simulator.hpp): a planar 3-link arm pushed into a box.
 *
 *   build:  python -c "from fast_kinematic_simulator_amd.build import build_example; build_example()"
 *   run:    build/cpp_forward_simulate [num_particles]
 *
 * Prints one line per particle: index, reached joint values (%.17g), collided,
 * microsteps, resolver iterations, error bits.  tests/test_cpp_interface.py builds
 * the same robot and scene through the Python mirror and checks that both paths
 * give identical results.  Exit status 3 = no GPU (fks_create reports
 * FKS_ERR_NO_DEVICE).
 */
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp"

static fks_dof_controller joint_controller() {
    fks_dof_controller c{};
    c.kp = 10.0;
    c.ki = 1.0;
    c.kd = 0.1;
    c.integral_clamp = 0.5;
    c.velocity_limit = 1.0;
    c.max_actuator_proportional_noise = 0.2;
    c.max_actuator_minimum_noise = 0.0002;
    return c;
}

/* three revolute joints about z, links of 0.3 m along x, 16 points per link */
static fks::RobotDescription planar_arm() {
    fks::RobotDescription r;
    r.type = FKS_ROBOT_LINKED;
    r.num_links = 4;
    r.num_dofs = 3;
    r.base_transform[11] = 0.05; /* base 5 cm above the grid floor */
    for (int j = 0; j < 3; ++j) {
        fks_joint_desc jd{};
        jd.parent_link = j;
        jd.child_link = j + 1;
        jd.type = FKS_JOINT_REVOLUTE;
        const double o[12] = {1, 0, 0, j == 0 ? 0.0 : 0.3, 0, 1, 0, 0, 0, 0, 1, 0};
        for (int k = 0; k < 12; ++k) jd.origin[k] = o[k];
        jd.axis[2] = 1.0;
        jd.limit_lower = -2.5;
        jd.limit_upper = 2.5;
        r.joints.push_back(jd);
        r.controllers.push_back(joint_controller());
        r.distance_weights.push_back(1.0);
    }
    for (int l = 1; l <= 3; ++l) {
        std::vector<double> pts;
        for (int i = 0; i < 16; ++i) {
            pts.push_back(0.3 * (i + 0.5) / 16.0);
            pts.push_back(0.0);
            pts.push_back(0.0);
            pts.push_back(1.0);
        }
        r.AddGeometry(l, pts);
    }
    r.AllowSelfCollision(0, 1);
    r.AllowSelfCollision(1, 2);
    return r;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 128;
    /* one box at (0.55, 0.35) in a 64 x 64 x 16 grid of 2 cm cells */
    fks_obstacle box{};
    const double pose[12] = {1, 0, 0, 0.55, 0, 1, 0, 0.35, 0, 0, 1, 0.1};
    for (int k = 0; k < 12; ++k) box.pose[k] = pose[k];
    box.extents[0] = 0.08;
    box.extents[1] = 0.08;
    box.extents[2] = 0.2;
    box.object_id = 1;
    const double origin[12] = {1, 0, 0, -0.64, 0, 1, 0, -0.64, 0, 0, 1, -0.1};
    const int64_t cells[3] = {64, 64, 16};
    fks_env_handle* env_handle = nullptr;
    fks::check(fks_env_build(&box, 1, 0.02, origin, cells, &env_handle), nullptr, "fks_env_build");
    fks_environment env;
    fks::check(fks_env_view(env_handle, &env), nullptr, "fks_env_view");

    const fks::RobotDescription robot = planar_arm();
    int status = 0;
    try {
        auto sim = fks::MakeLinkedSimulator(env, fks::GetDefaultSolverParameters(), 50.0, 42, 0);
        std::vector<fks::Configuration> starts, targets{{1.1, 0.2, -0.3}};
        for (int i = 0; i < n; ++i) {
            const double d = 0.01 * std::sin(0.37 * i);
            starts.push_back({0.1 + d, -0.2 - d, 0.3 + 0.5 * d});
        }
        const auto results = sim->ForwardSimulateRobots(robot, starts, targets, true);
        for (int i = 0; i < n; ++i) {
            const auto& r = results[i];
            std::printf("%d %.17g %.17g %.17g %d %u %u %u\n", i, r.result_config[0], r.result_config[1], r.result_config[2],
                        r.did_contact ? 1 : 0, r.microsteps, r.resolver_iterations, r.error_flags);
        }
        for (const auto& kv : sim->GetStatistics()) std::printf("# %s %.0f\n", kv.first.c_str(), kv.second);
        /* the planner's validity check (CheckConfigCollision) on every reached configuration */
        std::vector<fks::Configuration> reached;
        for (const auto& r : results) reached.push_back(r.result_config);
        const std::vector<bool> in_collision = sim->CheckConfigCollisions(robot, reached, 0.25);
        for (int i = 0; i < n; ++i) std::printf("#check %d %d\n", i, in_collision[i] ? 1 : 0);
        /* DemonstrateSimulator-style traced run of the particle that needed the most resolver iterations */
        int worst = 0;
        for (int i = 0; i < n; ++i)
            if (results[i].resolver_iterations > results[worst].resolver_iterations) worst = i;
        fks::ForwardSimulationStepTrace trace;
        const fks::SimulationResult tr = sim->ForwardSimulateRobot(robot, starts[worst], targets[0], true, trace, true);
        size_t configs = 0;
        for (const auto& rs : trace.resolver_steps)
            for (const auto& c : rs.contact_resolver_steps) configs += c.contact_resolution_steps.size();
        std::printf("#trace %d %zu %zu %.17g %.17g %.17g %u %u\n", worst, trace.resolver_steps.size(), configs,
                    tr.result_config[0], tr.result_config[1], tr.result_config[2], tr.microsteps, tr.resolver_iterations);
        /* host-side helpers of the interface */
        const std::array<double, 4> p3 = sim->Get3dPointForConfig(robot, results[worst].result_config);
        std::printf("#point %.17g %.17g %.17g\n", p3[0], p3[1], p3[2]);
        const auto markers = sim->MakeControlInputDisplayRep(robot, starts[0], {0.1, -0.2, 0.3}, {{0.f, 1.f, 0.f, 1.f}}, 7, "u");
        std::printf("#marker %s %zu\n", markers[0].type.c_str(), markers[0].points.size());
    } catch (const fks::SimulatorError& e) {
        std::fprintf(stderr, "%s\n", e.what());
        status = e.status() == FKS_ERR_NO_DEVICE ? 3 : 1;
    }
    fks_env_free(env_handle);
    return status;
}
