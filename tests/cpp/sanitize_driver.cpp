/*
 * TEST INFRASTRUCTURE ONLY — host code under AddressSanitizer + UndefinedBehaviorSanitizer.
 *
 * Built by `make -C oracle sanitize` (g++ -fsanitize=address,undefined, no GPU) from the
 * CPU oracle (oracle/*.cpp), the host environment builder of the product
 * (fks_env_builder.cpp: obstacles -> collision grid, exact EDT, surface-normal CSR) and
 * the host side of the planner-facing headers (robot flattening, configuration
 * conversion).  Runs a small linked scene (a continuous joint included) through the oracle's forward
 * simulation (both RNG modes, traced and untraced), the batched config check, the QR
 * solve on rank-deficient systems and the environment builder with auto and fixed
 * bounds; exits non-zero on any sanitizer report (halt_on_error) or wrong shape.
 * tests/test_sanitizers.py builds and runs it.
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "fast_kinematic_simulator_amd/tnuva_robot_models.hpp"
#include "fks_capi.h"

extern "C" {
int oracle_forward_simulate(const fks_environment* env, const fks_solver_params* params, double frequency, uint64_t seed,
                            uint64_t call_index, const fks_robot_desc* robot_desc, const double* starts, uint64_t n,
                            const double* targets, uint64_t num_targets, uint64_t first_particle_id, int32_t allow_contacts,
                            int32_t rng_mode, int32_t num_threads, double* out_positions, uint8_t* out_collided,
                            uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                            fks_statistics* out_stats, fks_call_counters* out_counters, int32_t individual_jacobians,
                            double* controller_state);
int oracle_forward_simulate_traced(const fks_environment* env, const fks_solver_params* params, double frequency, uint64_t seed,
                                   uint64_t call_index, const fks_robot_desc* robot_desc, const double* starts, uint64_t n,
                                   const double* targets, uint64_t num_targets, int32_t allow_contacts, int32_t num_threads,
                                   double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                   uint32_t* out_resolver_iterations, uint32_t* out_error_flags, const fks_trace* trace);
int oracle_check_config_collision(const fks_environment* env, const fks_solver_params* params, const fks_robot_desc* robot_desc,
                                  const double* configs, uint64_t n, double inflation_ratio, int32_t num_threads,
                                  uint8_t* out_collided, uint32_t* out_error_flags, uint64_t* out_sdf_bytes);
void oracle_qr_solve(const double* J, uint64_t R, uint64_t D, const double* b, double* x);
}

#define CHECK(cond)                                                          \
    do {                                                                     \
        if (!(cond)) {                                                       \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #cond, __LINE__); \
            return 1;                                                        \
        }                                                                    \
    } while (0)

static fks_obstacle box(uint32_t id, double x, double y, double z, double hx, double hy, double hz) {
    fks_obstacle o{};
    const double pose[12] = {1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z};
    std::memcpy(o.pose, pose, sizeof(pose));
    o.extents[0] = hx;
    o.extents[1] = hy;
    o.extents[2] = hz;
    o.object_id = id;
    return o;
}

static std::shared_ptr<const std::vector<fks_planner_types::Vector4d>> segment_points(double length, int n) {
    auto pts = std::make_shared<std::vector<fks_planner_types::Vector4d>>();
    for (int i = 0; i < n; ++i) {
        const double a = 0.7 * i;
        pts->push_back(fks_planner_types::Vector4d(0.02 * std::cos(a), 0.02 * std::sin(a), length * (i + 0.5) / n, 1.0));
    }
    return pts;
}

int main() {
    /* environment builder: fixed grid and auto-sized grid */
    const std::vector<fks_obstacle> obstacles = {box(1, 0.0, 0.0, -0.1, 0.5, 0.5, 0.05), box(2, 0.25, 0.1, 0.3, 0.05, 0.2, 0.05)};
    const double origin[12] = {1, 0, 0, -0.32, 0, 1, 0, -0.32, 0, 0, 1, -0.2};
    const int64_t cells[3] = {64, 64, 64};
    fks_env_handle* h = nullptr;
    CHECK(fks_env_build(obstacles.data(), (int32_t)obstacles.size(), 0.01, origin, cells, &h) == FKS_OK);
    fks_env_handle* h2 = nullptr;
    CHECK(fks_env_build(obstacles.data(), (int32_t)obstacles.size(), 0.02, nullptr, nullptr, &h2) == FKS_OK);
    fks_env_free(h2);
    CHECK(fks_env_build(obstacles.data(), 0, -1.0, nullptr, nullptr, &h2) == FKS_ERR_INVALID_ARGUMENT);
    fks_environment env;
    CHECK(fks_env_view(h, &env) == FKS_OK);
    std::vector<uint8_t> occ(64 * 64 * 64);
    CHECK(fks_env_occupancy(h, occ.data(), occ.size()) == FKS_OK);

    /* a 3-link arm built through the planner-facing TNUVA constructor (host flattening) */
    typedef tnuva_robot_models::TnuvaLinkedRobot<std::mt19937_64> Robot;
    std::vector<simple_linked_robot_model::RobotLink> links(4);
    std::vector<simple_linked_robot_model::RobotJoint> joints;
    simple_linked_robot_model::SimpleLinkedConfiguration initial;
    std::vector<std::pair<std::string, simple_robot_models::PointSphereGeometry>> geoms;
    for (int l = 0; l < 4; ++l) links[(size_t)l].link_name = "l" + std::to_string(l);
    for (int j = 0; j < 3; ++j) {
        simple_linked_robot_model::RobotJoint jt;
        jt.parent_link_index = j;
        jt.child_link_index = j + 1;
        const double o[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, j == 0 ? 0.05 : 0.2};
        jt.joint_transform = fks_ext::iso_from_row_major34(o);
        jt.joint_axis = fks_planner_types::Vector3d(0.0, 1.0, 0.0);
        jt.joint_model = simple_linked_robot_model::SimpleJointModel(
            {-2.5, 2.5}, 0.0, j == 2 ? simple_linked_robot_model::SimpleJointModel::CONTINUOUS : simple_linked_robot_model::SimpleJointModel::REVOLUTE);
        joints.push_back(jt);
        initial.push_back(jt.joint_model);
        geoms.emplace_back(links[(size_t)j + 1].link_name,
                           simple_robot_models::PointSphereGeometry(simple_robot_models::PointSphereGeometry::POINTS, segment_points(0.2, 40)));
    }
    std::vector<Robot::LINKED_ROBOT_CONFIG> ctrl(3, Robot::LINKED_ROBOT_CONFIG(8.0, 1.0, 0.1, 0.5, 1.0, 10.0, 0.0, 0.2, 0.001));
    Robot robot(fks_planner_types::Isometry3d::Identity(), links, joints, initial, {1.0, 1.0, 1.0}, geoms, {{0, 1}, {1, 2}}, ctrl);
    std::unique_ptr<simple_robot_model_interface::SimpleRobotModelInterface<simple_linked_robot_model::SimpleLinkedConfiguration>>
        clone(robot.Clone());
    CHECK(clone->GetPosition().size() == 3);
    const fks_robot_desc desc = robot.HipDescription().View();
    CHECK(desc.num_dofs == 3 && desc.num_geometries == 3);

    /* forward simulation: counter and reference RNG modes, traced, mutable controllers */
    fks_solver_params sp{};  /* SimulatorSolverParameters() defaults (SPCS:357-368) */
    sp.forward_simulation_time = 1.0;
    sp.environment_collision_check_tolerance = 0.001;
    sp.resolve_correction_step_scaling_decay_rate = 0.5;
    sp.resolve_correction_initial_step_size = 1.0;
    sp.resolve_correction_min_step_scaling = 0.03125;
    sp.max_resolver_iterations = 25;
    sp.resolve_correction_step_scaling_decay_iterations = 5;
    sp.failed_resolves_end_motion = 1;
    const int n = 6;
    std::vector<double> starts, targets = {1.2, 0.9, -2.8};
    for (int i = 0; i < n; ++i) starts.insert(starts.end(), {0.05 * i, 0.3, 2.9 - 0.01 * i});
    std::vector<double> out(3 * n), pid(6 * n, 0.01);
    std::vector<uint8_t> coll(n);
    std::vector<uint32_t> micro(n), res(n), err(n);
    fks_statistics st;
    fks_call_counters cc;
    for (int mode = 0; mode < 2; ++mode)
        CHECK(oracle_forward_simulate(&env, &sp, 50.0, 7, 0, &desc, starts.data(), n, targets.data(), 1, 0, 1, mode, 2, out.data(),
                                      coll.data(), micro.data(), res.data(), err.data(), &st, &cc, 0, nullptr) == 0);
    CHECK(oracle_forward_simulate(&env, &sp, 50.0, 7, 1, &desc, starts.data(), n, targets.data(), 1, 0, 1, 0, 2, out.data(),
                                  coll.data(), micro.data(), res.data(), err.data(), &st, &cc, 1, pid.data()) == 0);
    CHECK(cc.microsteps > 0);
    const uint32_t step_cap = 50, cfg_cap = 64;
    std::vector<double> tin((size_t)n * step_cap * 6), tcfg((size_t)n * cfg_cap * 3);
    std::vector<uint32_t> tmic((size_t)n * step_cap), ttag((size_t)n * cfg_cap * 3), ns(n), nc(n);
    fks_trace tr{step_cap, cfg_cap, tin.data(), tmic.data(), tcfg.data(), ttag.data(), ns.data(), nc.data()};
    CHECK(oracle_forward_simulate_traced(&env, &sp, 50.0, 7, 2, &desc, starts.data(), n, targets.data(), 1, 0, 2, out.data(),
                                         coll.data(), micro.data(), res.data(), err.data(), &tr) == 0);
    std::vector<uint8_t> cc_coll(n);
    std::vector<uint64_t> bytes(n);
    CHECK(oracle_check_config_collision(&env, &sp, &desc, starts.data(), n, 0.5, 2, cc_coll.data(), err.data(), bytes.data()) == 0);

    /* least squares on full-rank, rank-deficient and empty systems */
    const double J[12] = {1, 2, 3, 2, 4, 6, 0, 1, 1, 1, 0, 0};
    const double b[4] = {1, 2, 3, 4};
    double x[3];
    oracle_qr_solve(J, 4, 3, b, x);
    oracle_qr_solve(J, 2, 3, b, x);
    oracle_qr_solve(J, 1, 3, b, x);
    CHECK(std::isfinite(x[0]) && std::isfinite(x[1]) && std::isfinite(x[2]));
    fks_env_free(h);
    std::printf("sanitize driver ok: %llu microsteps, %llu resolver iterations\n", (unsigned long long)cc.microsteps,
                (unsigned long long)cc.resolver_iterations);
    return 0;
}
