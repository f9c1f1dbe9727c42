/*
 * fks_capi.h — C-ABI of the MI355X-native particle forward-simulation path.
 *
 * This is the drop-in boundary that replaces the OpenMP particle loop of
 * simple_particle_contact_simulator::SimpleParticleContactSimulator
 * (reference: include/fast_kinematic_simulator/simple_particle_contact_simulator.hpp,
 * abbreviated SPCS below).  Plain C types only: no C++, no torch, no HIP types
 * cross this header.  A C++ host wrapper that re-implements the
 * uncertainty_planning_core SimulatorInterface on top of these entry points is in
 * include/fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp and the
 * Python mirror is fast_kinematic_simulator_amd/simulator.py.
 *
 * Entry point  ->  reference interface it replaces
 *   fks_default_solver_params  -> fast_kinematic_simulator::GetDefaultSolverParameters   (FKS.hpp:13-16)
 *   fks_create + fks_set_robot -> fast_kinematic_simulator::Make{SE2,SE3,Linked}Simulator (FKS.cpp:4-71),
 *                                 SimpleParticleContactSimulator ctor (SPCS:420-444)
 *   fks_forward_simulate       -> SimpleParticleContactSimulator::ForwardSimulateRobots (SPCS:788-804)
 *   fks_reverse_simulate       -> SimpleParticleContactSimulator::ReverseSimulateRobots (SPCS:806-822)
 *   fks_forward_simulate_device-> same as fks_forward_simulate, inputs/outputs already in HBM
 *   fks_check_config_collision -> SimpleParticleContactSimulator::CheckConfigCollision   (SPCS:1398-1416),
 *                                 batched (one call per configuration in the reference)
 *   fks_get_statistics         -> SimpleParticleContactSimulator::GetStatistics          (SPCS:488-500)
 *   fks_reset_statistics       -> SimpleParticleContactSimulator::ResetStatistics        (SPCS:502-512)
 *   fks_reset_generators       -> SimpleParticleContactSimulator::ResetGenerators        (SPCS:457-471)
 *   fks_get/set_debug_level    -> Get/SetDebugLevel                                       (SPCS:446-455)
 *   fks_env_build              -> simulator_environment_builder::BuildCompleteEnvironment
 *                                 (src/.../simulator_environment_builder.cpp:470-476; CPU preprocessing)
 *
 * Errors: every call returns fks_status; fks_get_last_error() gives the text.
 * Nothing throws across the ABI.  Per-particle problems that the reference
 * handles with assert() (SPCS:1570-1575, 1882, GetBestSurfaceNormal SPCS:113-114)
 * are reported as FKS_PARTICLE_ERR_* bits and that particle stops simulating.
 *
 * Threading: a context is single-caller and stream-ordered (the reference's
 * simulator object is not safe for concurrent calls either, SPCS:846-850).
 */
#ifndef FKS_CAPI_H
#define FKS_CAPI_H

#if defined(__HIPCC_RTC__)
/* run-time compilation of shape-specialised kernels (fks_specialize): hiprtc's prelude
 * declares the fixed-width types in its own namespace and has no libc headers */
using __hip_internal::int16_t;
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::int8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::uint8_t;
#ifndef INT32_MIN
#define INT32_MIN (-2147483647 - 1)
#endif
#else
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* 5: the opt-in joint-space proof (ABI 4: fks_set_joint_proof, fks_call_counters.
 * proven_free_microsteps) removed: it broke even on the headline.
 * 6: host robot control (fks_robot_control_action, fks_robot_apply_control_input), the
 * environment builder's public steps (fks_env_discretize_obstacle, fks_env_build_normals,
 * fks_env_cell_objects), fks_set_statistics / fks_set_total_counters.
 * 7: fks_set_small_batch_kernel
 * 8: shape specialisation, launch info
 * 9: specialisation modes (FKS_SPECIALIZE_NO_PROOFS validation kernel), build failures in
 *    fks_specialization_info (failed, message), fks_multi_set_active_devices, pinned per-device
 *    staging in fks_multi_*
 * 10: cooperative small batches (fks_set_cooperative_waves, FKS_KERNEL_COOPERATIVE, launch
 *    info cooperative_*), the shape-specialised small-batch kernel (FKS_KERNEL_SHAPED_SMALL_BATCH),
 *    fks_set_segment_heavy_relative */
#define FKS_ABI_VERSION 10

typedef enum {
    FKS_OK = 0,
    FKS_ERR_INVALID_ARGUMENT = 1,
    FKS_ERR_HIP = 2,
    FKS_ERR_NO_ROBOT = 3,
    FKS_ERR_OUT_OF_MEMORY = 4,
    FKS_ERR_UNSUPPORTED = 5,
    FKS_ERR_NO_DEVICE = 6
} fks_status;

typedef enum { FKS_ROBOT_LINKED = 0, FKS_ROBOT_SE2 = 1, FKS_ROBOT_SE3 = 2 } fks_robot_type;

/* arc_utilities simple_linked_robot_model::SimpleJointModel::JOINT_TYPE values */
typedef enum {
    FKS_JOINT_FIXED = 0,
    FKS_JOINT_REVOLUTE = 1,
    FKS_JOINT_CONTINUOUS = 2,
    FKS_JOINT_PRISMATIC = 4
} fks_joint_type;

/* per-particle error bits (replace the reference's asserts) */
#define FKS_PARTICLE_ERR_MICROSTEP_MOTION 0x1u   /* SPCS:1570-1575 computed microstep motion > allowed  */
#define FKS_PARTICLE_ERR_NORMAL_OOB 0x2u         /* SPCS:1882 surface normal lookup out of bounds        */
#define FKS_PARTICLE_ERR_ZERO_DIRECTION 0x4u     /* SPCS:113-114 best-normal query with zero motion      */
#define FKS_PARTICLE_ERR_RNG_EXHAUSTED 0x8u      /* truncated-normal rejection exceeded its draw budget  */
#define FKS_PARTICLE_ERR_SELF_CAPACITY 0x10u     /* reserved: ABI <= 2 capped the self-collision impulse
                                                    solve; since ABI 3 it is unbounded (never raised)    */
#define FKS_PARTICLE_ERR_KEY_RANGE 0x20u         /* non-finite point in the self-collision grid          */
#define FKS_PARTICLE_ERR_MICROSTEP_CAP 0x40u     /* microsteps per controller step exceeded 2^20         */
#define FKS_PARTICLE_ERR_SELF_SINGULAR 0x80u     /* NaN self-collision correction (assert SPCS:1151-1153) */
#define FKS_PARTICLE_ERR_NO_NOISE_BIN 0x100u     /* sampled actuator: no bin holds the command (UNC:152-153) */

/* SimulatorSolverParameters (SPCS:345-369); booleans widened to uint32 */
typedef struct {
    double forward_simulation_time;
    double simulation_shortcut_distance;
    double environment_collision_check_tolerance;
    double resolve_correction_step_scaling_decay_rate;
    double resolve_correction_initial_step_size;
    double resolve_correction_min_step_scaling;
    uint32_t max_resolver_iterations;
    uint32_t resolve_correction_step_scaling_decay_iterations;
    uint32_t failed_resolves_end_motion;
    uint32_t reserved;
} fks_solver_params;

/* A VoxelGrid geometry (arc_utilities VoxelGrid): origin transform as a 3x4
 * row-major [R | t], cubic cells, cell counts; storage index
 * (x * ny + y) * nz + z (z fastest). */
typedef struct {
    double origin[12];
    double resolution;
    int64_t num_cells[3];
} fks_grid_geometry;

/* The three inputs the reference simulator copies at construction (SPCS:379-381):
 * environment_ (collision map: only its geometry is used on the path: GetResolution
 * SPCS:524-527 and GetInverseOriginTransform SPCS:1176), environment_sdf_
 * (float distance per cell, oob_value returned outside, SEB.cpp:473 uses +inf) and
 * surface_normals_grid_ (SPCS:44-343, stored as CSR: cell c owns entries
 * [normal_offsets[c], normal_offsets[c+1]); each entry is 6 doubles: the
 * SafeNormal'ed entry direction xyz (its w is always 0) then the SafeNormal'ed
 * normal xyz, in insertion order).  Arrays are read during fks_create/fks_env
 * upload only; the caller keeps ownership. */
typedef struct {
    fks_grid_geometry collision_map;
    fks_grid_geometry sdf;
    const float* sdf_values;
    float sdf_oob_value;
    uint32_t reserved;
    fks_grid_geometry normals;
    const uint32_t* normal_offsets; /* num_cells+1 entries */
    const double* normal_entries;   /* 6 * normal_offsets[num_cells] doubles */
} fks_environment;

/* TnuvaLinkedRobot::LINKED_ROBOT_CONFIG (TNUVA:420-457); SE2/SE3 use one per axis */
typedef struct {
    double kp;
    double ki;
    double kd;
    double integral_clamp;
    double velocity_limit;
    double acceleration_limit;
    double max_sensor_noise;
    double max_actuator_proportional_noise;
    double max_actuator_minimum_noise;
} fks_dof_controller;

/* SampledUncertainVelocityActuator (UNC:123-281): bins of observed velocity errors
 * keyed by commanded velocity (JointUncertaintySampleModel, UNC:123).  Bin k covers
 * [bin_bounds[2k], bin_bounds[2k+1]]; the first bin holding the clamped command
 * wins (GetMatchingBin, UNC:140-154) and one of its bin_elements samples, picked
 * uniformly, is added to it (GetNoiseValue, UNC:228-243).  num_bins == 0 keeps the
 * truncated-normal actuator of fks_dof_controller for that dof. */
typedef struct {
    uint32_t num_bins;
    uint32_t bin_elements;
    const double* bin_bounds;  /* num_bins x (lower, upper) */
    const double* bin_samples; /* num_bins x bin_elements */
} fks_sampled_actuator;

/* simple_linked_robot_model::RobotJoint */
typedef struct {
    int32_t parent_link;
    int32_t child_link;
    int32_t type; /* fks_joint_type */
    int32_t reserved;
    double origin[12]; /* parent link frame -> joint frame, 3x4 row-major */
    double axis[3];
    double limit_lower;
    double limit_upper;
} fks_joint_desc;

/* Flattened robot.  Geometries are the robot_link_geometries vector
 * (GetLinkGeometries): geometry g belongs to link geometry_link[g] and owns
 * points [geometry_point_offset[g], geometry_point_offset[g+1]) of `points`
 * (x, y, z, w per point: PointSphereGeometry POINTS with w = 1).  Allowed
 * self-collision pairs are given as geometry indices (the indices that
 * CheckIfSelfCollisionAllowed receives at SPCS:1008,1193).
 *  linked: num_dofs = number of non-fixed joints, configuration = joint values
 *  SE2:    num_dofs = 3, configuration = (x, y, theta), controllers = x, y, theta
 *  SE3:    num_dofs = 6, configuration = 3x4 row-major pose (12 doubles),
 *          controllers = x, y, z, rx, ry, rz (twist order, TNUVA:352-358)
 * distance_weights: linked -> one weight per dof; SE2/SE3 -> [position, rotation]. */
typedef struct {
    int32_t robot_type; /* fks_robot_type */
    int32_t num_links;
    int32_t num_joints;
    int32_t num_geometries;
    int32_t num_dofs;
    int32_t num_allowed_pairs;
    double base_transform[12];
    const fks_joint_desc* joints;
    const int32_t* geometry_link;
    const uint32_t* geometry_point_offset;
    const double* points;
    const int32_t* allowed_pairs;
    const fks_dof_controller* controllers;
    const double* distance_weights;
    /* NULL, or num_dofs entries: per-dof SampledUncertainVelocityActuator (ABI 2) */
    const fks_sampled_actuator* sampled_actuators;
} fks_robot_desc;

/* SimpleParticleContactSimulator statistics counters (SPCS:392-400, 488-500) */
typedef struct {
    uint64_t successful_resolves;
    uint64_t unsuccessful_resolves;
    uint64_t free_resolves;
    uint64_t collision_resolves;
    uint64_t fallback_resolves;
    uint64_t unsuccessful_env_collision_resolves;
    uint64_t unsuccessful_self_collision_resolves;
    uint64_t recovered_unsuccessful_resolves;
} fks_statistics;

/* Work/traffic counters of the last forward/reverse call (all particles). */
typedef struct {
    uint64_t particles;
    uint64_t controller_steps;
    uint64_t microsteps;          /* executions of the microstep loop body, SPCS:1590-1796 */
    uint64_t resolver_iterations; /* executions of the resolver loop body, SPCS:1625-1762 */
    uint64_t sdf_bytes;           /* algorithmic SDF/normal-grid bytes the reference would read */
    uint64_t error_particles;
    double kernel_ms;             /* device time of the simulation kernel (HIP events) */
    double call_ms;               /* host wall time of the whole call */
    uint64_t calls;               /* number of calls these counters cover */
    uint64_t least_squares_rows;  /* sum over resolver iterations of the stacked-Jacobian rows (3 x corrected points) */
    /* ABI 3: the self-collision branch of the resolver (SPCS:983-1275) */
    uint64_t self_collision_checks; /* CheckCollision calls (SPCS:1418-1436) whose self-collision map came back
                                       non-empty, i.e. ExtractSelfCollidingPoints produced corrections (SPCS:1264-1271) */
    uint64_t self_corrected_points; /* sum over resolver iterations of the points whose correction holds a
                                       self-collision term (SPCS:1846-1853, 1909-1916) */
    uint64_t reserved0;             /* ABI 4's proven_free_microsteps (removed in ABI 5); always 0 */
} fks_call_counters;

typedef struct fks_context fks_context;

int fks_abi_version(void);
const char* fks_status_string(fks_status status);

/* GetDefaultSolverParameters (FKS.hpp:13-16) */
fks_status fks_default_solver_params(fks_solver_params* out);

/* Make{SE2,SE3,Linked}Simulator (FKS.cpp:4-71): copies env to device `device`.
 * The stacked-Jacobian resolver is always used (FKS.cpp:22,45,68 pass false). */
fks_status fks_create(const fks_environment* env, const fks_solver_params* params,
                      double simulation_controller_frequency, uint64_t prng_seed,
                      int32_t debug_level, int32_t device, fks_context** out_ctx);
void fks_destroy(fks_context* ctx);
const char* fks_get_last_error(const fks_context* ctx);

/* Upload/replace the robot every particle is a clone of (the immutable_robot
 * argument of ForwardSimulateRobots, SPCS:788).  Cached until replaced. */
fks_status fks_set_robot(fks_context* ctx, const fks_robot_desc* robot);
/* configuration width in doubles for the current robot (linked D, SE2 3, SE3 12) */
int32_t fks_config_width(const fks_context* ctx);

/* ForwardSimulateRobots (SPCS:788): host buffers.  starts: n*W doubles;
 * targets: num_targets*W doubles with num_targets == 1 or n (SPCS:792).
 * Outputs (n entries each, any may be NULL except out_positions):
 * reached configuration, collided flag (SimulationResult), microsteps,
 * resolver iterations and FKS_PARTICLE_ERR_* bits per particle. */
fks_status fks_forward_simulate(fks_context* ctx, const double* starts, uint64_t n,
                                const double* targets, uint64_t num_targets,
                                int32_t allow_contacts, double* out_positions,
                                uint8_t* out_collided, uint32_t* out_microsteps,
                                uint32_t* out_resolver_iterations, uint32_t* out_error_flags);
/* ReverseSimulateRobots (SPCS:806): identical semantics (SPCS:838-841). */
fks_status fks_reverse_simulate(fks_context* ctx, const double* starts, uint64_t n,
                                const double* targets, uint64_t num_targets,
                                int32_t allow_contacts, double* out_positions,
                                uint8_t* out_collided, uint32_t* out_microsteps,
                                uint32_t* out_resolver_iterations, uint32_t* out_error_flags);

/* ForwardSimulateMutableRobot (SPCS:843-919) / ReverseSimulateMutableRobot (SPCS:838-841)
 * for a batch: particle i starts from starts[i] (SetPosition: joint limits / angle wrap)
 * with its PID controllers as the robot holds them, not zeroed as ResetPosition does
 * (TNUVA:524-536).  controller_state (n x 2D doubles, in/out): per dof the controller's
 * error integral, then per dof its last error (SimplePIDController PID:53-136; D = dofs, 3 for
 * SE(2), 6 for SE(3)); on return it holds each particle's controllers when it stopped.
 * All zeros gives fks_forward_simulate's results. */
fks_status fks_forward_simulate_mutable(fks_context* ctx, const double* starts, uint64_t n, const double* targets,
                                        uint64_t num_targets, int32_t allow_contacts, double* controller_state,
                                        double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                        uint32_t* out_resolver_iterations, uint32_t* out_error_flags);

/* Same call with every buffer already in device memory of the context's GPU.
 * first_particle_id: global id of particle 0 of this shard (the RNG stream is
 * keyed by global id, so sharding across GPUs does not change results).
 * stream: a hipStream_t (NULL = default stream); the call returns once the
 * work is enqueued unless `synchronize` is non-zero. */
fks_status fks_forward_simulate_device(fks_context* ctx, const double* d_starts, uint64_t n,
                                       const double* d_targets, uint64_t num_targets,
                                       uint64_t first_particle_id, int32_t allow_contacts,
                                       double* d_out_positions, uint8_t* d_out_collided,
                                       uint32_t* d_out_microsteps,
                                       uint32_t* d_out_resolver_iterations,
                                       uint32_t* d_out_error_flags, void* stream,
                                       int32_t synchronize);

/* CheckConfigCollision (SPCS:1398-1416) for a batch of n configurations (host
 * buffers): SetPosition(config), CheckEnvironmentCollision at threshold
 * inflation_ratio * res (SPCS:1403, 921-981) and CheckSelfCollisions at extended
 * cells of (inflation_ratio + 1) * res (SPCS:1404, 1324-1396).  out_collided[i] = 1
 * if configuration i collides; out_error_flags (may be NULL): FKS_PARTICLE_ERR_KEY_RANGE
 * for non-finite points.  The reference checks one configuration per call (the
 * planner's state-validity check); a batch of one is that call. */
fks_status fks_check_config_collision(fks_context* ctx, const double* configs, uint64_t n,
                                      double inflation_ratio, uint8_t* out_collided,
                                      uint32_t* out_error_flags);
/* Same with device buffers on the caller's stream (see fks_forward_simulate_device). */
fks_status fks_check_config_collision_device(fks_context* ctx, const double* d_configs, uint64_t n,
                                             double inflation_ratio, uint8_t* d_out_collided,
                                             uint32_t* d_out_error_flags, void* stream,
                                             int32_t synchronize);
/* counters of the last config-check call: particles = configurations, sdf_bytes,
 * kernel_ms, call_ms */
fks_status fks_get_last_check_counters(const fks_context* ctx, fks_call_counters* out);

/* ForwardSimulationStepTrace (simple_simulator_interface, filled at SPCS:1583-1595,
 * 1615-1618, 1701-1704, 1712-1715, 1776-1779) flattened per particle:
 *   resolver_steps[s].control_input / .control_input_step  -> step record s
 *   resolver_steps[s].contact_resolver_steps[m].contact_resolution_steps[k]
 *                                                          -> config records tagged (s, m, kind)
 * in the order the reference appends them.  Buffers are caller-owned, n particles x
 * capacity each; records beyond a capacity are counted but not stored. */
#define FKS_TRACE_POST_ACTION 0u    /* post_action_configuration of microstep m (SPCS:1617)          */
#define FKS_TRACE_RESOLVER_STEP 1u  /* active_configuration after a resolver iteration (SPCS:1703)  */
#define FKS_TRACE_RESOLVE_FAILED 2u /* previous_configuration, resolver gave up (SPCS:1714)         */
#define FKS_TRACE_CONTACT_STOP 3u   /* previous_configuration, contact with allow_contacts=false (SPCS:1778) */
typedef struct {
    uint32_t step_capacity;    /* step records per particle */
    uint32_t config_capacity;  /* configuration records per particle */
    double* step_inputs;       /* n * step_capacity * 2D: control_input (u * dt), control_input_step */
    uint32_t* step_microsteps; /* n * step_capacity: number of microsteps of the step */
    double* configs;           /* n * config_capacity * W */
    uint32_t* config_tags;     /* n * config_capacity * 3: controller step, microstep, FKS_TRACE_* kind */
    uint32_t* num_steps;       /* n: step records produced (may exceed step_capacity) */
    uint32_t* num_configs;     /* n: configuration records produced (may exceed config_capacity) */
} fks_trace;

/* ForwardSimulateRobot(..., trace, enable_tracing = true, ...) (SPCS:824-829) for a
 * batch: same results as fks_forward_simulate plus the trace of every particle
 * (host buffers; the traced kernel is a separate instantiation, the untraced path
 * does not pay for it). */
fks_status fks_forward_simulate_traced(fks_context* ctx, const double* starts, uint64_t n,
                                       const double* targets, uint64_t num_targets,
                                       int32_t allow_contacts, double* out_positions,
                                       uint8_t* out_collided, uint32_t* out_microsteps,
                                       uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                                       const fks_trace* trace);

/* ForwardSimulateMutableRobot(..., trace, enable_tracing = true, ...) (SPCS:843-919) for a
 * batch: fks_forward_simulate_mutable's controller state in/out plus the trace. */
fks_status fks_forward_simulate_traced_mutable(fks_context* ctx, const double* starts, uint64_t n, const double* targets,
                                               uint64_t num_targets, int32_t allow_contacts, double* controller_state,
                                               double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                               uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                                               const fks_trace* trace);

/* Kinematics of a batch of configurations (host buffers), the pieces the reference's
 * host-side helpers build on, computed with the simulation kernels' own FK:
 *   FKS_KIN_LINK_TRANSFORMS     out: n x num_links x 12 (3x4 row-major link transforms
 *                               after SetPosition; GetLinkTransform, used by
 *                               Get3dPointForConfig SPCS:776-786)
 *   FKS_KIN_POINTS              out: n x num_points x 3 (link points in the world frame,
 *                               geometry order; MakeConfigurationDisplayRep SPCS:634-688)
 *   FKS_KIN_APPLY_CONTROL_INPUT inputs: n x num_dofs; out: n x config width (the clean
 *                               ApplyControlInput of MakeControlInputDisplayRep,
 *                               SPCS:719-774, TNUVA:538-566) */
#define FKS_KIN_LINK_TRANSFORMS 0
#define FKS_KIN_POINTS 1
#define FKS_KIN_APPLY_CONTROL_INPUT 2
fks_status fks_kinematics(fks_context* ctx, int32_t mode, const double* configs, uint64_t n, const double* inputs,
                          double* out);
/* sizes of the robot set with fks_set_robot (any pointer may be NULL) */
fks_status fks_robot_sizes(const fks_context* ctx, int32_t* num_links, int32_t* num_points, int32_t* num_dofs,
                           int32_t* config_width);

/* Each forward/reverse call consumes one RNG "call index" (the reference's
 * per-thread std::mt19937_64 streams advance across calls, SPCS:850).  Ranks
 * that shard one logical call must use the same index: set it explicitly. */
fks_status fks_set_call_index(fks_context* ctx, uint64_t call_index);
uint64_t fks_get_call_index(const fks_context* ctx);

fks_status fks_get_statistics(const fks_context* ctx, fks_statistics* out);
fks_status fks_reset_statistics(fks_context* ctx);
/* overwrite the statistics (a caller that re-runs a call restores what it read before) */
fks_status fks_set_statistics(fks_context* ctx, const fks_statistics* stats);
fks_status fks_reset_generators(fks_context* ctx, uint64_t prng_seed);
int32_t fks_get_debug_level(const fks_context* ctx);
int32_t fks_set_debug_level(fks_context* ctx, int32_t debug_level);
fks_status fks_get_last_call_counters(const fks_context* ctx, fks_call_counters* out);
/* Kernel phase profile: shader-clock cycles (s_memtime) spent by all waves in each
 * phase of the hot path, summed over the particles of a call.  Diagnostic only;
 * the phases follow the reference's call structure (SPCS line ranges). */
#define FKS_NUM_PHASES 16
enum fks_phase {
    FKS_PHASE_PARTICLE = 0,        /* whole particle: ForwardSimulateMutableRobot SPCS:843-919 */
    FKS_PHASE_CONTROL = 1,         /* controller + sensor noise SPCS:861-876 */
    FKS_PHASE_STEP_SETUP = 2,      /* microstep count estimate SPCS:1549-1572 */
    FKS_PHASE_MICRO_INPUT = 3,     /* ApplyControlInput incl. actuator noise SPCS:1599, TNUVA:568-596 */
    FKS_PHASE_MICRO_FK = 4,        /* SetPosition (FK) of the post-action configuration SPCS:1600-1601 */
    FKS_PHASE_ENV_CHECK = 5,       /* CheckEnvironmentCollision SPCS:921-981 */
    FKS_PHASE_SELF_CHECK = 6,      /* CollectSelfCollisions SPCS:1183-1275 (+ ExtractSelfCollidingPoints 983-1171) */
    FKS_PHASE_CORRECTIONS = 7,     /* CollectPointCorrectionsAndJacobians SPCS:1818-1939 */
    FKS_PHASE_SOLVE = 8,           /* ComputeResolverCorrectionStep{StackedJacobian,IndividualJacobians} SPCS:1966-1998 */
    FKS_PHASE_RESOLVE_APPLY = 9,   /* correction step sizing / application SPCS:1630-1690 */
    FKS_PHASE_OUTPUT = 10,         /* reached configuration + counters */
    /* event counts (not cycles) of the profiling build */
    FKS_PHASE_ENV_ROUNDS_SKIPPED = 11,   /* 64-point rounds proven free (no SDF reads) */
    FKS_PHASE_ENV_ROUNDS_EVALUATED = 12, /* 64-point rounds read from the SDF */
    FKS_PHASE_CORR_ROUNDS_SKIPPED = 13,  /* correction rounds proven free */
    FKS_PHASE_CORR_ROUNDS_EVALUATED = 14,
    /* residency of the persistent waves: 100 MHz s_memrealtime ticks from a wave's
     * start to its exit (queue drained), summed over waves; with the kernel time it
     * gives the share of wave slots kept busy (the batch's tail) */
    FKS_PHASE_WAVE_RESIDENCY = 15
};
/* which: 0 = last call, 1 = sums since fks_create / fks_reset_total_counters */
fks_status fks_get_phase_cycles(const fks_context* ctx, int which, uint64_t* out /* FKS_NUM_PHASES */);
/* Launch geometry of the simulation kernel for the robot set last: resident waves of
 * the persistent grid (CUs x workgroups per CU x waves per workgroup, one particle
 * per wave at a time) and LDS bytes per workgroup.  Diagnostic (no reference
 * counterpart); with FKS_PHASE_WAVE_RESIDENCY it gives the busy share of the grid. */
fks_status fks_get_launch_geometry(const fks_context* ctx, uint32_t* resident_waves, uint64_t* lds_bytes_per_group);
/* which simulation kernel a call ran (fks_launch_info.last_kernel) */
typedef enum {
    FKS_KERNEL_NONE = 0,
    FKS_KERNEL_THROUGHPUT = 1,   /* fks_simulate_<family>[_lean] */
    FKS_KERNEL_SMALL_BATCH = 2,  /* fks_simulate_<family>_small (fks_set_small_batch_kernel) */
    FKS_KERNEL_SHAPED = 3,       /* the robot-shape-specialised kernel (fks_set_specialization) */
    FKS_KERNEL_TRACED = 4,       /* fks_simulate_<family>[_lean]_traced */
    FKS_KERNEL_INDIVIDUAL = 5,   /* fks_simulate_<family>[_lean]_indiv (fks_set_individual_jacobians) */
    FKS_KERNEL_COOPERATIVE = 6,  /* ABI 10: fks_simulate_<family>_coop (fks_set_cooperative_waves) */
    FKS_KERNEL_SHAPED_SMALL_BATCH = 7 /* ABI 10: the shape-specialised module's small-batch kernel
                                         (a small batch once the robot's module is built) */
} fks_kernel_kind;
/* The launch layout fks_set_robot chose (ABI 8; diagnostic, no reference counterpart). */
typedef struct fks_launch_info {
    uint32_t resident_waves;                 /* the persistent grid (fks_get_launch_geometry) */
    uint32_t waves_per_group;
    uint64_t lds_bytes_per_group;
    uint32_t small_batch_resident_waves;     /* the small-batch kernel's grid (0: not for this layout) */
    uint32_t standard_layout_resident_waves; /* what the non-lean LDS layout would hold */
    int32_t fk_pair;                         /* paired FK of free microsteps */
    int32_t lean;                            /* lean LDS block (skip-proof cache in scratch) */
    int32_t last_kernel;                     /* fks_kernel_kind of the last simulation call */
    int32_t last_check_kernel;               /* ABI 9: of the last batched CheckConfigCollision call
                                                (FKS_KERNEL_THROUGHPUT: generic, FKS_KERNEL_SHAPED) */
    uint32_t cooperative_resident_particles; /* ABI 10: the cooperative kernel's grid (0: not for this robot) */
    uint32_t cooperative_waves_per_particle; /* ABI 10: its waves per particle (workgroup) */
} fks_launch_info;
fks_status fks_get_launch_info(const fks_context* ctx, fks_launch_info* out);
/* Scheduling granularity of fks_forward_simulate*: when a batch holds more particles
 * than the grid has resident waves, each particle's controller steps are run in
 * segments of `controller_steps` (0 = automatic: 14 when the batch outnumbers the
 * resident waves, else whole; nonzero: always), handed out segment-major so
 * that every particle progresses from the start of the launch and contact-heavy
 * particles do not start last (the batch's tail).  Results are bit-identical for
 * every value (the resting state between segments is exact).  No reference
 * counterpart (SPCS:795 runs each particle whole on one OpenMP thread). */
fks_status fks_set_segment_steps(fks_context* ctx, uint32_t controller_steps);
/* Scheduling policy of segmented batches (ABI 3; no reference counterpart, results are
 * bit-identical for every value):
 *   heavy_resolver_per_step: a segment whose particle averaged at least this many
 *     resolver iterations per controller step is contact-heavy and its wave keeps the
 *     particle's next segment instead of returning it to the round-robin (0 = off;
 *     default 2; at most 65536);
 *   heavy_priority: issue priority (s_setprio 0..2) of a wave carrying a contact-heavy
 *     particle (1 = raised to 2 for heavy segments only; 0 = never raised; 2, the default
 *     since ABI 10 = also 1 for particles that fell behind the round-robin).
 * The priority is reset to 0 at the start of every segment a wave claims. */
fks_status fks_set_segment_policy(fks_context* ctx, uint32_t heavy_resolver_per_step, uint32_t heavy_priority);
/* ABI 10: once the batch's mean resolver iterations per finished segment reaches the absolute
 * threshold (a contact-heavy batch), a heavy segment must also have at least `times_mean` times
 * that mean (the kernel keeps the running sums; default 3, 0 = the absolute test alone, at most
 * 64; off for batches of 2^24 or more particle-segments).  Results are bit-identical for every
 * value. */
fks_status fks_set_segment_heavy_relative(fks_context* ctx, uint32_t times_mean);
/* Small batches (ABI 7; no reference counterpart, results are bit-identical either way):
 * with `enabled` (the default) a plain simulation call whose particles all fit the
 * resident waves of a low-occupancy instantiation (two waves per SIMD, no register
 * spills; not for lean LDS blocks, traced or individual-Jacobian calls, or explicit
 * segments) runs that kernel — a batch that small is the latency of its slowest particle
 * (a planner's typical call: cfg1, 32 particles, 10 % shorter).  0 = always the
 * throughput kernel. */
fks_status fks_set_small_batch_kernel(fks_context* ctx, int32_t enabled);
/* Cooperative small batches (ABI 10; no reference counterpart, results are bit-identical
 * either way; opt-in, default 0): with `enabled` a plain simulation call of at most
 * fks_launch_info.cooperative_resident_particles particles (one per workgroup slot: 256 CUs
 * x the kernel's occupancy; same exclusions as the small-batch kernel, robots of at most
 * 1024 points) runs each particle on a workgroup of cooperative_waves_per_particle waves: one
 * runs the particle, and every environment check and correction pass is shared out over all
 * of them, 64-point rounds each.  Takes precedence over the small-batch kernel;
 * fks_set_small_batch_kernel(ctx, 0) turns both off.  Measured on cfg3's heaviest particles
 * alone it is 5-10 % SLOWER than the small-batch kernel (about three rounds per check are left
 * after the skip proofs, too few to share), hence off by default. */
fks_status fks_set_cooperative_waves(fks_context* ctx, int32_t enabled);
/* SimpleParticleContactSimulator(..., simulate_with_individual_jacobians, ...) (SPCS:420-423,
 * 1629): 0 = ComputeResolverCorrectionStepStackedJacobian (SPCS:1990-1998; what the factories
 * FKS.cpp:22,45,68 hard-wire, the default), 1 = ComputeResolverCorrectionStepIndividualJacobians
 * (SPCS:1966-1988: one ColPivHouseholderQR solve per corrected point, summed in point order). */
fks_status fks_set_individual_jacobians(fks_context* ctx, int32_t simulate_with_individual_jacobians);
/* Robot-shape specialisation (ABI 8; no reference counterpart, results are bit-identical
 * either way).  While enabled (the default), the plain throughput simulation
 * (fks_forward_simulate*, not traced, individual-Jacobian or small-batch calls) runs a kernel
 * compiled at run time (hiprtc, in the helper process fks_shapec installed beside the
 * library) from the library's own kernel source with the robot's link / joint / dof /
 * geometry counts and LDS and scratch carve-outs as constants (cfg3: 10-13 % faster,
 * DESIGN.md §4.9).  A robot's kernel is built at the first call that runs it (a robot only
 * simulated in small batches never compiles) or at once by fks_set_specialization(ctx, 1);
 * the first robot of a shape on a machine costs one compile (2-20 s in the calling thread),
 * later ones come from the per-process cache or the disk cache (FKS_KERNEL_CACHE=<dir>,
 * default ~/.cache/fast_kinematic_simulator_amd; "off" disables it).  When the kernel cannot
 * be built the calls keep the generic kernel (same results), fks_get_specialization reports
 * failed = 1 with the compiler log in `message`, and so does fks_get_last_error;
 * fks_set_specialization(ctx, FKS_SPECIALIZE_ON) then returns FKS_ERR_UNSUPPORTED.
 * FKS_SPECIALIZE_OFF = generic kernels only (also the default when the environment variable
 * FKS_SPECIALIZE=0 is set at fks_create).  FKS_SPECIALIZE_NO_PROOFS (ABI 9, validation only)
 * builds the same shaped kernel with every skip proof compiled out (FKS_NO_SKIP_PROOFS: the
 * environment / correction round proofs, the motion-estimate pruning, the self-collision gap
 * proof and both lever-arm shortcuts): the results must not change, only the
 * time, which is what tests/test_proof_free.py checks on full batches. */
typedef enum {
    FKS_SPECIALIZE_OFF = 0,
    FKS_SPECIALIZE_ON = 1,
    FKS_SPECIALIZE_NO_PROOFS = 2
} fks_specialization_mode;
fks_status fks_set_specialization(fks_context* ctx, int32_t mode);
typedef struct fks_specialization_info {
    int32_t enabled;         /* fks_set_specialization's mode (fks_specialization_mode) */
    int32_t active;          /* the current robot's plain simulation calls run the shape-specialised kernel */
    int32_t from_cache;      /* its code object came from the process or disk cache */
    int32_t pending;         /* enabled, robot set, kernel to be built at the first call that runs it */
    double compile_seconds;  /* hiprtc time of that code object (0 when it came from a cache) */
    uint64_t launches;       /* launches of the specialised kernel since the robot was set */
    char shape[64];          /* the shape key, e.g. "t0-L8-J7-D7-W7-G8-P512-p1-l0" */
    int32_t failed;          /* ABI 9: the current robot's build failed; its calls run the generic kernel */
    int32_t reserved;
    char message[512];       /* ABI 9: why it failed (the start of the compiler log), else empty */
} fks_specialization_info;
fks_status fks_get_specialization(const fks_context* ctx, fks_specialization_info* out);

/* sums over every call since fks_create / fks_reset_total_counters */
fks_status fks_get_total_counters(const fks_context* ctx, fks_call_counters* out);
fks_status fks_reset_total_counters(fks_context* ctx);
fks_status fks_set_total_counters(fks_context* ctx, const fks_call_counters* totals);

/* One robot stepped by hand on the host (the TnuvaRobot control interface, TNUVA:15-23), the
 * same arithmetic as the simulation kernels:
 *   fks_robot_control_action       -> GenerateControlAction(target, controller_interval)
 *                                     (TNUVA:179-198, 384-412, 598-614); pid_state: the robot's
 *                                     controllers, 2 * num_dofs doubles (error integrals, then
 *                                     last errors), updated in place; out_control: num_dofs
 *   fks_robot_apply_control_input  -> ApplyControlInput(u) (TNUVA:152-163, 348-364, 538-566)
 *                                     with unit_noise NULL; ApplyControlInput(u, rng)
 *                                     (TNUVA:165-177, 366-382, 568-596) with one truncated-normal
 *                                     TN(0, 0.5) on [-1, 1] sample per dof drawn by the caller
 *                                     (UNC:77-90); out_config: the robot's config width */
fks_status fks_robot_control_action(const fks_robot_desc* robot, const double* config, const double* target,
                                    double controller_interval, double* pid_state, double* out_control);
fks_status fks_robot_apply_control_input(const fks_robot_desc* robot, const double* config, const double* input,
                                         const double* unit_noise, double* out_config);

/* ---- environment preprocessing (CPU; reference SEB.cpp:21-476) ---- */
/* OBSTACLE_CONFIG (SEB.hpp): pose as 3x4 row-major, half extents, object id > 0 */
typedef struct {
    double pose[12];
    double extents[3];
    uint32_t object_id;
    uint32_t reserved;
} fks_obstacle;

typedef struct fks_env_handle fks_env_handle;

/* BuildCompleteEnvironment(obstacles, resolution).  If `grid_origin` and
 * `num_cells` are non-NULL the grid is that box (a fixed-size grid, e.g. 256^3);
 * otherwise it is sized to the obstacles plus a 3-cell border (SEB.cpp:128-149). */
fks_status fks_env_build(const fks_obstacle* obstacles, int32_t num_obstacles,
                         double resolution, const double* grid_origin,
                         const int64_t* num_cells, fks_env_handle** out);
/* The same environment built on the GPU (obstacle rasterisation, exact squared EDT,
 * surface-normal CSR: fks_env_gpu.hip); bit-identical to fks_env_build.  The result
 * is copied back into a host handle (fks_env_view / fks_env_free as above).
 * stats (optional): sizes and the device time of the build. */
typedef struct {
    uint64_t cells;
    uint64_t obstacle_samples;
    uint64_t normal_entries;
    double gpu_ms;   /* device time: rasterise + EDT + SDF + CSR (HIP events) */
    double total_ms; /* host wall time of the call incl. allocation and copy-back */
} fks_env_build_stats;
fks_status fks_env_build_gpu(const fks_obstacle* obstacles, int32_t num_obstacles,
                             double resolution, const double* grid_origin,
                             const int64_t* num_cells, int32_t device, fks_env_handle** out,
                             fks_env_build_stats* stats);
/* The same GPU build kept in device memory, handed to a context without a trip
 * through the host (the simulation reads exactly these bytes). */
typedef struct fks_device_env fks_device_env;
fks_status fks_env_build_device(const fks_obstacle* obstacles, int32_t num_obstacles,
                                double resolution, const double* grid_origin,
                                const int64_t* num_cells, int32_t device, fks_device_env** out,
                                fks_env_build_stats* stats);
/* host copy of a device environment (then fks_env_view / fks_env_occupancy / fks_env_free) */
fks_status fks_device_env_download(const fks_device_env* env, fks_env_handle** out);
fks_status fks_device_env_geometry(const fks_device_env* env, fks_grid_geometry* out);
void fks_device_env_free(fks_device_env* env);
/* fks_create on the device environment's own device: the SDF and surface-normal CSR are
 * copied device to device; the context does not keep a reference to `env`. */
fks_status fks_create_from_device_env(const fks_device_env* env, const fks_solver_params* params,
                                      double simulation_controller_frequency, uint64_t prng_seed,
                                      int32_t debug_level, fks_context** out_ctx);
/* DiscretizeObstacle (SEB.cpp:21-46): *count = the obstacle's half-resolution samples; with
 * out_xyz (capacity >= *count triples) their positions relative to the obstacle (its frame: the
 * caller places them with obstacle.pose, as BuildEnvironment does, SEB.cpp:84-85), x then y
 * then z */
fks_status fks_env_discretize_obstacle(const fks_obstacle* obstacle, double resolution, double* out_xyz, uint64_t capacity,
                                       uint64_t* count);
/* BuildSurfaceNormalsGrid (SEB.cpp:258-468) on the caller's SDF (VoxelGrid order over
 * sdf_geometry, e.g. sdf_tools' ExtractSignedDistanceField result, SEB.cpp:473-475): a handle
 * with only the surface-normal CSR over that geometry (fks_env_view: sdf_values NULL) */
fks_status fks_env_build_normals(const fks_obstacle* obstacles, int32_t num_obstacles, const fks_grid_geometry* sdf_geometry,
                                 const float* sdf_values, fks_env_handle** out);
/* the object id of each cell of an fks_env_build collision map (BuildEnvironment's
 * SetValue(1.0, object_id) in obstacle order, the last write wins, SEB.cpp:151-155; 0 = free) */
fks_status fks_env_cell_objects(const fks_env_handle* env, uint32_t* out, uint64_t num_cells);

/* Fill a view whose pointers stay valid until fks_env_free. */
fks_status fks_env_view(const fks_env_handle* env, fks_environment* out);
/* The collision grid (1 = filled cell), z-fastest, num_cells = nx * ny * nz. */
fks_status fks_env_occupancy(const fks_env_handle* env, uint8_t* out, uint64_t num_cells);
void fks_env_free(fks_env_handle* env);

/* ---- several devices in one process (fks_multi.cpp) ----
 * The reference runs one simulator object over all host cores (`#pragma omp parallel for`
 * over particles, SPCS:795); a multi context runs one fks_context per listed device and
 * splits every batch into contiguous shards, particle i on the device whose
 * fks_shard_bounds range holds it, simulated with first_particle_id = the range start
 * (bit-identical results for any device list).  Each device has a host thread of its own for
 * the call: it stages its shard through pinned buffers of its own (H2D, kernel, D2H on the
 * device's stream, so no device's copies wait for another's), and copies its outcomes into
 * the caller's buffers at its offset; statistics and call counters are summed over the
 * devices (kernel_ms: the slowest).  The same device may be listed more than once. */
typedef struct fks_multi_context fks_multi_context;
/* [begin, end) of shard `shard` of n particles over ndev devices: balanced contiguous ranges,
 * the first n % ndev shards one particle longer */
fks_status fks_shard_bounds(uint64_t n, int32_t ndev, int32_t shard, uint64_t* begin, uint64_t* end);
fks_status fks_create_multi(const fks_environment* env, const fks_solver_params* params, double simulation_controller_frequency,
                            uint64_t prng_seed, int32_t debug_level, const int32_t* devices, int32_t ndev,
                            fks_multi_context** out);
void fks_destroy_multi(fks_multi_context* m);
const char* fks_multi_get_last_error(const fks_multi_context* m);
int32_t fks_multi_num_devices(const fks_multi_context* m);
/* the per-device context of shard `shard` (for per-device settings such as fks_set_segment_steps) */
fks_context* fks_multi_device_context(fks_multi_context* m, int32_t shard);
fks_status fks_multi_set_robot(fks_multi_context* m, const fks_robot_desc* robot);
/* ABI 9: the batches that follow are sharded over the first `count` listed devices only
 * (1 <= count <= fks_multi_num_devices; 0 = all).  A batch too small to keep every device
 * busy for longer than its slowest particle runs no faster on more devices, so
 * the planner-facing DeviceSet picks the count per batch from the particles per device. */
fks_status fks_multi_set_active_devices(fks_multi_context* m, int32_t count);
int32_t fks_multi_active_devices(const fks_multi_context* m);
/* ForwardSimulateRobots (SPCS:788-804) over the active devices; arguments as fks_forward_simulate */
fks_status fks_multi_forward_simulate(fks_multi_context* m, const double* starts, uint64_t n, const double* targets,
                                      uint64_t num_targets, int32_t allow_contacts, double* out_positions, uint8_t* out_collided,
                                      uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags);
fks_status fks_multi_get_statistics(const fks_multi_context* m, fks_statistics* out);
fks_status fks_multi_reset_statistics(fks_multi_context* m);
fks_status fks_multi_get_last_call_counters(const fks_multi_context* m, fks_call_counters* out);
fks_status fks_multi_set_call_index(fks_multi_context* m, uint64_t call_index);
/* Batched CheckConfigCollision (SPCS:1398-1416) over all devices: configuration i on the
 * device whose fks_shard_bounds range holds it; arguments as fks_check_config_collision. */
fks_status fks_multi_check_config_collision(fks_multi_context* m, const double* configs, uint64_t n, double inflation_ratio,
                                            uint8_t* out_collided, uint32_t* out_error_flags);
/* Number of MI355X devices visible to this process (HIP_VISIBLE_DEVICES applies); 0 when there
 * is none.  The planner-facing factories default to all of them (fast_kinematic_simulator.hpp). */
int32_t fks_device_count(void);

/* Device self-test of the portable libm against the host (bit equality). */
fks_status fks_selftest_math(int32_t device, uint64_t n, uint64_t* out_mismatches);

#ifdef __cplusplus
}
#endif

#endif /* FKS_CAPI_H */
