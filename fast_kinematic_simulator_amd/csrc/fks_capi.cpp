/*
 * fks_capi.cpp — host implementation of the C-ABI in include/fks_capi.h.
 *
 * A context mirrors one SimpleParticleContactSimulator (SPCS:371-1999): it owns
 * device copies of the SDF and the surface-normal grid (copied once, as the
 * reference copies them at construction SPCS:420), the flattened robot, the
 * solver parameters (SPCS:345-369) and the counter-based RNG stream state.
 * fks_forward_simulate replaces the OpenMP particle loop of
 * ForwardSimulateRobots (SPCS:788-804) with one launch of the persistent
 * simulation kernel.  No exceptions cross the ABI.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "fks_capi.h"
#include "fks_env_internal.h"
#include "fks_specialize.h"
#include "fks_device.h"
#include "fks_portable_math.h"

extern "C" __global__ void fks_simulate_linked(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se2(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se3(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_indiv(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se2_indiv(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se3_indiv(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_traced(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se2_traced(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se3_traced(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_small(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se2_small(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se3_small(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_coop(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se2_coop(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_se3_coop(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_lean(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_lean_indiv(const fksd::SimArgs* args);
extern "C" __global__ void fks_simulate_linked_lean_traced(const fksd::SimArgs* args);
extern "C" __global__ void fks_check_configs_linked(const fksd::SimArgs* args);
extern "C" __global__ void fks_check_configs_se2(const fksd::SimArgs* args);
extern "C" __global__ void fks_check_configs_se3(const fksd::SimArgs* args);
extern "C" __global__ void fks_kinematics_linked(const fksd::SimArgs* args);
extern "C" __global__ void fks_kinematics_se2(const fksd::SimArgs* args);
extern "C" __global__ void fks_kinematics_se3(const fksd::SimArgs* args);
extern "C" __global__ void fks_math_probe(const double* a, const double* b, double* out, uint64_t n);

namespace {

typedef void (*sim_kernel_t)(const fksd::SimArgs*);

/* the batched CheckConfigCollision kernel for one robot family */
sim_kernel_t check_kernel_for(int robot_type) {
    switch (robot_type) {
        case FKS_ROBOT_SE2: return fks_check_configs_se2;
        case FKS_ROBOT_SE3: return fks_check_configs_se3;
        default: return fks_check_configs_linked;
    }
}

/* the simulation kernel compiled for one robot family (FKS.cpp:4-71 factories) */
/* lean: the robot runs a lean LDS block (linked robots only, fks_set_robot) */
sim_kernel_t traced_kernel_for(int robot_type, bool lean = false) {
    switch (robot_type) {
        case FKS_ROBOT_SE2: return fks_simulate_se2_traced;
        case FKS_ROBOT_SE3: return fks_simulate_se3_traced;
        default: return lean ? fks_simulate_linked_lean_traced : fks_simulate_linked_traced;
    }
}

sim_kernel_t kernel_for(int robot_type, bool individual_jacobians = false, bool lean = false) {
    switch (robot_type) {
        case FKS_ROBOT_SE2: return individual_jacobians ? fks_simulate_se2_indiv : fks_simulate_se2;
        case FKS_ROBOT_SE3: return individual_jacobians ? fks_simulate_se3_indiv : fks_simulate_se3;
        default:
            if (lean) return individual_jacobians ? fks_simulate_linked_lean_indiv : fks_simulate_linked_lean;
            return individual_jacobians ? fks_simulate_linked_indiv : fks_simulate_linked;
    }
}

/* the low-occupancy instantiation for batches that fit its resident waves */
sim_kernel_t small_kernel_for(int robot_type) {
    switch (robot_type) {
        case FKS_ROBOT_SE2: return fks_simulate_se2_small;
        case FKS_ROBOT_SE3: return fks_simulate_se3_small;
        default: return fks_simulate_linked_small;
    }
}

/* the cooperative instantiation (one particle per workgroup) for batches of at most one
 * particle per resident workgroup */
sim_kernel_t coop_kernel_for(int robot_type) {
    switch (robot_type) {
        case FKS_ROBOT_SE2: return fks_simulate_se2_coop;
        case FKS_ROBOT_SE3: return fks_simulate_se3_coop;
        default: return fks_simulate_linked_coop;
    }
}

using fksd::GridDev;
/* controller steps per segment when a batch outnumbers the resident waves: short
 * enough that a contact-heavy particle progresses from the start of the launch, long
 * enough that the hand-over (resting state + one FK) costs < 1 % */
constexpr uint32_t kDefaultSegmentSteps = 14; /* re-swept in round 6: profiles/r06p_sched_ab_cfg*.json */
/* a segment averaging this many resolver iterations per controller step is
 * contact-heavy: its wave keeps the particle (the cfg3 batch averages 0.65) ... */
constexpr uint32_t kHeavyResolverPerStep = 2;
/* ... if it also has at least this many times the batch's mean resolver iterations per
 * segment so far: a batch where most segments resolve contacts (cfg5) carries only its
 * outliers */
constexpr uint32_t kHeavyRelative = 3;
using fksd::JointDev;
using fksd::RobotDev;

inline double dot3(double a0, double a1, double a2, double b0, double b1, double b2) { return (a0 * b0 + a1 * b1) + a2 * b2; }

void inverse34(const double* T, double* I) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) I[4 * i + j] = T[4 * j + i];
    for (int i = 0; i < 3; ++i) I[4 * i + 3] = -dot3(I[4 * i + 0], I[4 * i + 1], I[4 * i + 2], T[3], T[7], T[11]);
}

GridDev make_grid(const fks_grid_geometry& g) {
    GridDev d;
    std::memcpy(d.org, g.origin, sizeof(d.org));
    inverse34(d.org, d.inv);
    d.res = g.resolution;
    d.inv_res = 1.0 / g.resolution;
    for (int a = 0; a < 3; ++a) d.n[a] = g.num_cells[a];
    for (int w = 0; w < 3; ++w) d.inv_res_span[w] = 1.0 / (g.resolution * (double)w);
    for (int a = 0; a < 3; ++a) d.nb[a] = (uint32_t)((g.num_cells[a] + 3) >> fksd::kBrickShift);
    d.nb_pad = 0;
    return d;
}

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint32_t forward_steps(double time, double frequency) {
    const double raw = time * frequency;
    if (!(raw < 4294967295.0)) return 0xffffffffu;
    const uint32_t steps = (raw > 0.0) ? (uint32_t)raw : 0u;
    return steps > 1u ? steps : 1u;
}

template <typename T>
hipError_t dev_upload(T** dptr, const T* host, size_t count) {
    *dptr = nullptr;
    if (count == 0) return hipSuccess;
    hipError_t e = hipMalloc((void**)dptr, count * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpy(*dptr, host, count * sizeof(T), hipMemcpyHostToDevice);
}

bool valid_grid(const fks_grid_geometry& g) {
    if (!(g.resolution > 0.0) || !std::isfinite(g.resolution)) return false;
    for (int a = 0; a < 3; ++a)
        if (g.num_cells[a] < 2 || g.num_cells[a] > 65535) return false;
    const double cells = (double)g.num_cells[0] * (double)g.num_cells[1] * (double)g.num_cells[2];
    /* the kernels address cells of the 4x4x4-brick layout with 32-bit indices */
    const double padded = (double)((g.num_cells[0] + 3) & ~3ll) * (double)((g.num_cells[1] + 3) & ~3ll) *
                          (double)((g.num_cells[2] + 3) & ~3ll);
    return cells < 4294967295.0 && padded < 4294967295.0;
}

bool same_geometry(const fks_grid_geometry& a, const fks_grid_geometry& b) {
    return std::memcmp(a.origin, b.origin, sizeof(a.origin)) == 0 && a.resolution == b.resolution &&
           a.num_cells[0] == b.num_cells[0] && a.num_cells[1] == b.num_cells[1] && a.num_cells[2] == b.num_cells[2];
}

}  // namespace

/* Lipschitz-type constants of the SDF that make a round of points provably free of
 * contact: over axis-neighbour cell pairs, lplus = max |a - b| / res
 * where both values are positive, cmax = max a / res over positive cells with a
 * non-positive neighbour.  For an exact signed EDT both are 1.  Any non-finite value
 * disables skipping. */
static bool analyze_sdf(const float* v, int64_t nx, int64_t ny, int64_t nz, double res, double* lplus, double* cmax) {
    const int T = (int)std::max<unsigned>(1u, std::min<unsigned>(16u, std::thread::hardware_concurrency()));
    std::vector<double> lp(T, 0.0), cm(T, 0.0);
    std::vector<int> bad(T, 0);
    std::vector<std::thread> th;
    const double inv = 1.0 / res;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
            for (int64_t x = t; x < nx; x += T)
                for (int64_t y = 0; y < ny; ++y)
                    for (int64_t z = 0; z < nz; ++z) {
                        const size_t i = ((size_t)x * ny + y) * nz + z;
                        const double a = v[i];
                        if (!std::isfinite(a)) {
                            bad[t] = 1;
                            continue;
                        }
                        const size_t nb[3] = {x + 1 < nx ? i + (size_t)ny * nz : i, y + 1 < ny ? i + (size_t)nz : i,
                                              z + 1 < nz ? i + 1 : i};
                        for (int k = 0; k < 3; ++k) {
                            if (nb[k] == i) continue;
                            const double b = v[nb[k]];
                            if (!std::isfinite(b)) continue; /* flagged when visited */
                            if (a > 0.0 && b > 0.0) {
                                lp[t] = std::max(lp[t], std::fabs(a - b) * inv);
                            } else if (a > 0.0) {
                                cm[t] = std::max(cm[t], a * inv);
                            } else if (b > 0.0) {
                                cm[t] = std::max(cm[t], b * inv);
                            }
                        }
                    }
        });
    for (auto& h : th) h.join();
    *lplus = 0.0;
    *cmax = 0.0;
    for (int t = 0; t < T; ++t) {
        if (bad[t]) return false;
        *lplus = std::max(*lplus, lp[t]);
        *cmax = std::max(*cmax, cm[t]);
    }
    return *lplus > 0.0;
}

struct fks_context {
    int device = 0;
    std::string last_error;
    int32_t debug_level = 0;
    fks_solver_params params;
    double frequency = 1.0;
    uint64_t seed = 0;
    uint64_t call_index = 0;
    /* environment */
    float* d_sdf = nullptr;     /* bricked (fks_device.h brick_cell) */
    uint32_t* d_noff = nullptr; /* VoxelGrid-order CSR offsets, only until they are bricked */
    uint2* d_nrange = nullptr;  /* bricked [begin, end) per normal-grid cell */
    double* d_nent = nullptr;
    GridDev sdf_g, nrm_g, env_g;
    float oob = 0.0f;
    int32_t has_normals = 0;
    int32_t skip_enabled = 0;
    double skip_lplus = 0.0, skip_cmax = 0.0;
    /* robot */
    bool has_robot = false;
    RobotDev R;
    std::vector<void*> robot_allocs;
    /* launch resources */
    double* d_scratch = nullptr;
    size_t cap_scratch = 0; /* doubles allocated at d_scratch */
    uint64_t scratch_per_wave = 0;
    uint32_t grid_waves = 0;
    uint32_t waves_per_cu = 0;     /* resident waves per CU of the layout (LDS and registers) */
    uint32_t small_grid_waves = 0; /* resident waves of the small-batch kernel (0: none for this layout) */
    uint32_t coop_particles = 0;   /* resident workgroups (particles) of the cooperative kernel (0: none) */
    uint32_t coop_waves = 0;       /* its waves per workgroup */
    size_t coop_lds_bytes = 0;
    uint32_t grid_groups = 0;
    uint32_t waves_per_group = fksd::kWavesPerGroup;
    size_t lds_bytes = 0;
    unsigned long long* d_counters = nullptr; /* kNumCounters + queue + phase cycles */
    uint64_t phase_last[FKS_NUM_PHASES] = {};
    uint64_t phase_total[FKS_NUM_PHASES] = {};
    unsigned long long* h_counters = nullptr; /* pinned */
    fksd::SimArgs* d_args = nullptr;          /* kernel arguments, read through a pointer */
    fksd::SimArgs* h_args = nullptr;          /* pinned staging for d_args */
    bool pending = false;
    int pending_kind = 0; /* 0 = forward simulation, 1 = batched config check */
    hipStream_t pending_stream = nullptr;
    fks_call_counters check_last;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::chrono::steady_clock::time_point call_start;
    /* host-API staging */
    double* d_starts = nullptr;
    double* d_targets = nullptr;
    double* d_out = nullptr;
    uint8_t* d_coll = nullptr;
    uint32_t* d_micro = nullptr;
    uint32_t* d_res = nullptr;
    uint32_t* d_err = nullptr;
    double* d_pid = nullptr; /* fks_forward_simulate_mutable controller state */
    size_t cap_particles = 0, cap_targets = 0, cap_pid = 0;
    /* controller-step segments: resting particle state between segments */
    uint32_t segment_steps = 0; /* 0 = automatic (kDefaultSegmentSteps) */
    uint32_t heavy_per_step = kHeavyResolverPerStep; /* fks_set_segment_policy */
    uint32_t heavy_priority = 2; /* round 6: cfg5 -2 %, cfg3 / cfg4 equal (profiles/r06prio_*.json) */
    uint32_t heavy_relative = kHeavyRelative; /* fks_set_segment_heavy_relative */
    int32_t individual_jacobians = 0; /* fks_set_individual_jacobians (SPCS:420-423) */
    int32_t small_batch = 1;          /* fks_set_small_batch_kernel */
    int32_t cooperative = 0;          /* fks_set_cooperative_waves (opt-in: DESIGN.md §5.4) */
    bool fk_pair = false;             /* paired FK of free microsteps (fks_set_robot) */
    bool lean = false;                /* lean LDS block + lean kernels (fks_set_robot) */
    uint32_t standard_resident_waves = 0; /* resident waves of the non-lean layout (fks_get_launch_info) */
    int32_t last_kernel = FKS_KERNEL_NONE;       /* the simulation kernel of the last call */
    int32_t last_check_kernel = FKS_KERNEL_NONE; /* the configuration-check kernel of the last check */
    double* d_seg_state = nullptr;
    uint32_t* d_seg_done = nullptr;
    size_t cap_seg_state = 0, cap_seg_done = 0;
    fks_statistics stats;
    fks_call_counters last;
    fks_call_counters total;
    /* robot-shape specialisation (fks_set_specialization, fks_specialize.cpp) */
    int32_t specialize = 1;
    bool spec_pending = false; /* robot set, its kernel not built yet (built at the first launch that runs it) */
    hipModule_t spec_module = nullptr;
    hipFunction_t spec_fn = nullptr;       /* fks_simulate_shaped of the current robot's shape */
    hipFunction_t spec_check_fn = nullptr; /* fks_check_configs_shaped (same module) */
    hipFunction_t spec_small_fn = nullptr; /* fks_simulate_shaped_small (same module, non-lean shapes) */
    std::string spec_shape;
    double spec_seconds = 0.0;
    int32_t spec_from_cache = 0;
    uint64_t spec_launches = 0;
    bool spec_failed = false;  /* the current robot's build failed (its calls run the generic kernel) */
    std::string spec_message;  /* why (fks_specialization_info.message) */
};

template <typename T>
static hipError_t ensure(T** p, size_t count) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    return hipMalloc((void**)p, (count > 0 ? count : 1) * sizeof(T));
}

static fks_status fail(fks_context* ctx, fks_status st, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return st;
}
static fks_status hip_fail(fks_context* ctx, hipError_t e, const char* where) {
    return fail(ctx, FKS_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}
#define HIP_TRY(ctx, expr)                                       \
    do {                                                         \
        hipError_t _e = (expr);                                  \
        if (_e != hipSuccess) return hip_fail((ctx), _e, #expr); \
    } while (0)

static void spec_release(fks_context* ctx);

static void free_robot(fks_context* ctx) {
    spec_release(ctx); /* a specialised kernel belongs to one robot shape */
    for (void* p : ctx->robot_allocs) (void)hipFree(p);
    ctx->robot_allocs.clear();
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    ctx->d_scratch = nullptr;
    ctx->cap_scratch = 0;
    ctx->has_robot = false;
}

static void free_staging(fks_context* ctx) {
    void* ptrs[] = {ctx->d_starts, ctx->d_targets, ctx->d_out, ctx->d_coll, ctx->d_micro, ctx->d_res, ctx->d_err};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    ctx->d_starts = ctx->d_targets = ctx->d_out = nullptr;
    ctx->d_coll = nullptr;
    ctx->d_micro = ctx->d_res = ctx->d_err = nullptr;
    ctx->cap_particles = ctx->cap_targets = 0;
    if (ctx->d_pid) (void)hipFree(ctx->d_pid);
    ctx->d_pid = nullptr;
    ctx->cap_pid = 0;
    if (ctx->d_seg_state) (void)hipFree(ctx->d_seg_state);
    if (ctx->d_seg_done) (void)hipFree(ctx->d_seg_done);
    ctx->d_seg_state = nullptr;
    ctx->d_seg_done = nullptr;
    ctx->cap_seg_state = ctx->cap_seg_done = 0;
}

static void spec_release(fks_context* ctx) {
    if (ctx->spec_module) {
        (void)hipSetDevice(ctx->device);
        (void)hipModuleUnload(ctx->spec_module);
    }
    ctx->spec_module = nullptr;
    ctx->spec_fn = nullptr;
    ctx->spec_check_fn = nullptr;
    ctx->spec_small_fn = nullptr;
    ctx->spec_shape.clear();
    ctx->spec_seconds = 0.0;
    ctx->spec_from_cache = 0;
    ctx->spec_launches = 0;
    ctx->spec_failed = false;
    ctx->spec_message.clear();
}

static fks_status spec_build(fks_context* ctx);

/* the shape-specialised throughput kernel of the current robot: compiled (or taken from a
 * cache), loaded on the context's device, and used only if it keeps the generic kernel's
 * occupancy (the persistent grid is sized for that).  A failure leaves the generic kernel
 * in place and is recorded (fks_specialization_info.failed / message) */
static fks_status spec_prepare(fks_context* ctx) {
    spec_release(ctx);
    if (!ctx->specialize || !ctx->has_robot) return FKS_OK;
    const fks_status st = spec_build(ctx);
    if (st != FKS_OK) {
        ctx->spec_failed = true;
        ctx->spec_message = ctx->last_error;
        /* a failed module load can leave the runtime's per-thread error set; the generic
         * launch that follows checks hipGetLastError and must not pick it up */
        (void)hipGetLastError();
    }
    return st;
}

static fks_status spec_build(fks_context* ctx) {
    fks_spec::Shape sh;
    sh.type = ctx->R.type;
    sh.L = ctx->R.L;
    sh.J = ctx->R.J;
    sh.D = ctx->R.D;
    sh.W = ctx->R.W;
    sh.G = ctx->R.G;
    sh.P = ctx->R.P;
    sh.pair = ctx->fk_pair ? 1 : 0;
    sh.lean = ctx->lean ? 1 : 0;
    sh.no_proofs = ctx->specialize == FKS_SPECIALIZE_NO_PROOFS ? 1 : 0;
    /* the waves a SIMD holds at this layout (4 SIMDs per CU): when the LDS block keeps fewer
     * resident than the register budget allows (cfg5's lean blocks: 16 per CU), the
     * specialised kernel is compiled for that many and may use their registers */
    const int per_simd = (int)((ctx->waves_per_cu + 3) / 4);
    if (per_simd >= 1 && per_simd < fksd::kThroughputWavesPerEU) sh.waves_per_eu = per_simd;
    /* FKS_SPEC_WAVES_PER_EU=n (tuning and A/B runs): compile for n waves per SIMD instead
     * (n >= the layout's waves; 0 = the library's budget) */
    if (const char* e = std::getenv("FKS_SPEC_WAVES_PER_EU")) {
        const int n = std::atoi(e);
        if (n == 0 || n == fksd::kThroughputWavesPerEU) sh.waves_per_eu = 0;
        else if (n >= per_simd && n <= 8) sh.waves_per_eu = n;
    }
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    ctx->spec_shape = fks_spec::shape_key(sh); /* named in the report even when the build fails */
    std::string log;
    bool compiled = false;
    std::shared_ptr<const fks_spec::CodeObject> co = fks_spec::code_object(sh, &log, &compiled);
    if (!co) return fail(ctx, FKS_ERR_UNSUPPORTED, "shape specialisation: " + log);
    hipModule_t m = nullptr;
    hipFunction_t f = nullptr;
    hipError_t e = hipModuleLoadData(&m, co->bytes.data());
    if (e != hipSuccess && !compiled) {
        /* a cached code object the runtime refuses (truncated, or from another toolchain):
         * dropped from both caches and compiled afresh, once */
        (void)hipGetLastError();
        co = fks_spec::code_object(sh, &log, &compiled, /*refresh=*/true);
        if (!co) return fail(ctx, FKS_ERR_UNSUPPORTED, "shape specialisation (after an unloadable cached code object): " + log);
        e = hipModuleLoadData(&m, co->bytes.data());
    }
    if (e != hipSuccess) return hip_fail(ctx, e, "hipModuleLoadData (shape-specialised kernel)");
    e = hipModuleGetFunction(&f, m, "fks_simulate_shaped");
    if (e != hipSuccess) {
        (void)hipModuleUnload(m);
        return hip_fail(ctx, e, "hipModuleGetFunction(fks_simulate_shaped)");
    }
    /* the persistent grid is sized for the generic kernel's occupancy: the specialised kernel
     * (same launch bounds, same LDS block) is used only if it needs no more registers.  Its
     * count is read from the code object's metadata (the runtime's attribute query reports a
     * different quantity for module kernels than for the library's own) */
    const int shaped_vgpr = fks_spec::kernel_metadata_uint(co->bytes, "fks_simulate_shaped", ".vgpr_count") +
                            std::max(0, fks_spec::kernel_metadata_uint(co->bytes, "fks_simulate_shaped", ".agpr_count"));
    hipFuncAttributes gen{};
    if (hipFuncGetAttributes(&gen, reinterpret_cast<const void*>(kernel_for(ctx->R.type, false, ctx->lean))) != hipSuccess) gen.numRegs = 0;
    /* 512 VGPRs per SIMD lane, allocated in granules of 8 */
    const int budget = sh.waves_per_eu > 0 ? (512 / sh.waves_per_eu) & ~7 : gen.numRegs;
    if (shaped_vgpr <= 0 || shaped_vgpr > budget) {
        (void)hipModuleUnload(m);
        return fail(ctx, FKS_ERR_UNSUPPORTED,
                    "shape specialisation: the specialised kernel needs " + std::to_string(shaped_vgpr) + " VGPRs, the budget is " +
                        std::to_string(budget));
    }
    ctx->spec_module = m;
    ctx->spec_fn = f;
    /* the configuration check of the same shape, when the module carries it */
    hipFunction_t fc = nullptr;
    if (hipModuleGetFunction(&fc, m, "fks_check_configs_shaped") == hipSuccess) ctx->spec_check_fn = fc;
    /* ... and the small-batch kernel, used when it needs no more registers than two waves per
     * SIMD leave (the generic small-batch kernel's grid is the one launched) */
    hipFunction_t fs = nullptr;
    if (!ctx->lean && hipModuleGetFunction(&fs, m, "fks_simulate_shaped_small") == hipSuccess) {
        const int v = fks_spec::kernel_metadata_uint(co->bytes, "fks_simulate_shaped_small", ".vgpr_count") +
                      std::max(0, fks_spec::kernel_metadata_uint(co->bytes, "fks_simulate_shaped_small", ".agpr_count"));
        if (v > 0 && v <= 256) ctx->spec_small_fn = fs;
    }
    (void)hipGetLastError();
    ctx->spec_shape = fks_spec::shape_key(sh);
    ctx->spec_seconds = compiled ? co->compile_seconds : 0.0;
    ctx->spec_from_cache = compiled ? 0 : 1;
    return FKS_OK;
}

extern "C" {

int fks_abi_version(void) { return FKS_ABI_VERSION; }

const char* fks_status_string(fks_status status) {
    switch (status) {
        case FKS_OK: return "ok";
        case FKS_ERR_INVALID_ARGUMENT: return "invalid argument";
        case FKS_ERR_HIP: return "HIP runtime error";
        case FKS_ERR_NO_ROBOT: return "no robot set";
        case FKS_ERR_OUT_OF_MEMORY: return "out of memory";
        case FKS_ERR_UNSUPPORTED: return "unsupported";
        case FKS_ERR_NO_DEVICE: return "no HIP device";
        default: return "unknown status";
    }
}

fks_status fks_default_solver_params(fks_solver_params* out) {
    if (!out) return FKS_ERR_INVALID_ARGUMENT;
    /* SimulatorSolverParameters() defaults, SPCS:357-368 */
    out->forward_simulation_time = 1.0;
    out->simulation_shortcut_distance = 0.0;
    out->environment_collision_check_tolerance = 0.001;
    out->resolve_correction_step_scaling_decay_rate = 0.5;
    out->resolve_correction_initial_step_size = 1.0;
    out->resolve_correction_min_step_scaling = 0.03125;
    out->max_resolver_iterations = 25;
    out->resolve_correction_step_scaling_decay_iterations = 5;
    out->failed_resolves_end_motion = 1;
    out->reserved = 0;
    return FKS_OK;
}

/* fks_create / fks_create_from_device_env: the environment comes either from host
 * arrays (henv) or from a device-resident GPU build (denv) */
static fks_status create_impl(const fks_environment* henv, const fks_device_env* denv, const fks_solver_params* params,
                              double simulation_controller_frequency, uint64_t prng_seed, int32_t debug_level, int32_t device,
                              fks_context** out_ctx) {
    if (!out_ctx) return FKS_ERR_INVALID_ARGUMENT;
    *out_ctx = nullptr;
    if (!params || (!henv && !denv)) return FKS_ERR_INVALID_ARGUMENT;
    if (henv) {
        if (!henv->sdf_values) return FKS_ERR_INVALID_ARGUMENT;
        if (!valid_grid(henv->sdf) || !valid_grid(henv->collision_map) || !valid_grid(henv->normals)) return FKS_ERR_INVALID_ARGUMENT;
    } else if (!valid_grid(denv->geometry) || !denv->sdf || !denv->offsets) {
        return FKS_ERR_INVALID_ARGUMENT;
    }
    if (!(simulation_controller_frequency != 0.0) || !std::isfinite(simulation_controller_frequency)) return FKS_ERR_INVALID_ARGUMENT;
    if (params->resolve_correction_step_scaling_decay_iterations == 0) return FKS_ERR_INVALID_ARGUMENT;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return FKS_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return FKS_ERR_INVALID_ARGUMENT;
    fks_context* ctx = new (std::nothrow) fks_context();
    if (!ctx) return FKS_ERR_OUT_OF_MEMORY;
    ctx->device = device;
    ctx->params = *params;
    ctx->frequency = simulation_controller_frequency;
    ctx->seed = prng_seed;
    ctx->debug_level = debug_level;
    {
        const char* sp = std::getenv("FKS_SPECIALIZE");
        ctx->specialize = (sp && std::string(sp) == "0") ? 0 : 1;
    }
    std::memset(&ctx->stats, 0, sizeof(ctx->stats));
    std::memset(&ctx->last, 0, sizeof(ctx->last));
    std::memset(&ctx->total, 0, sizeof(ctx->total));
    auto bail = [&](hipError_t e, const char* where) {
        (void)where;
        (void)e;
        fks_destroy(ctx);
        return FKS_ERR_HIP;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bail(e, "hipSetDevice");
    double lp = 0.0, cm = 0.0;
    bool analyzed = false;
    if (henv) {
        ctx->sdf_g = make_grid(henv->sdf);
        ctx->nrm_g = make_grid(henv->normals);
        ctx->env_g = make_grid(henv->collision_map);
        ctx->oob = henv->sdf_oob_value;
        const size_t cells = (size_t)henv->sdf.num_cells[0] * (size_t)henv->sdf.num_cells[1] * (size_t)henv->sdf.num_cells[2];
        if ((e = dev_upload(&ctx->d_sdf, henv->sdf_values, cells)) != hipSuccess) return bail(e, "sdf upload");
        analyzed = analyze_sdf(henv->sdf_values, henv->sdf.num_cells[0], henv->sdf.num_cells[1], henv->sdf.num_cells[2],
                               henv->sdf.resolution, &lp, &cm);
        /* an initialized grid with no stored entries (every cell empty: a lookup in bounds finds
         * the zero normal, SPCS:219-222) has offsets and may have no entry array */
        if (henv->normal_offsets) {
            const size_t ncells =
                (size_t)henv->normals.num_cells[0] * (size_t)henv->normals.num_cells[1] * (size_t)henv->normals.num_cells[2];
            const size_t entries = henv->normal_offsets[ncells];
            if (entries > 0 && !henv->normal_entries) {
                fks_destroy(ctx);
                return FKS_ERR_INVALID_ARGUMENT;
            }
            if ((e = dev_upload(&ctx->d_noff, henv->normal_offsets, ncells + 1)) != hipSuccess)
                return bail(e, "normal offsets upload");
            if (entries > 0 && (e = dev_upload(&ctx->d_nent, henv->normal_entries, 6 * entries)) != hipSuccess)
                return bail(e, "normal entries upload");
            ctx->has_normals = 1;
        }
    } else {
        /* the GPU build's grids coincide (SEB.cpp builds all three on one grid); +inf out of bounds */
        ctx->sdf_g = make_grid(denv->geometry);
        ctx->nrm_g = ctx->sdf_g;
        ctx->env_g = ctx->sdf_g;
        ctx->oob = std::numeric_limits<float>::infinity();
        const size_t cells = (size_t)denv->cells;
        if ((e = hipMalloc((void**)&ctx->d_sdf, cells * sizeof(float))) != hipSuccess) return bail(e, "sdf");
        if ((e = hipMemcpy(ctx->d_sdf, denv->sdf, cells * sizeof(float), hipMemcpyDeviceToDevice)) != hipSuccess)
            return bail(e, "sdf copy");
        analyzed = fks_env::analyze_sdf_device(ctx->d_sdf, denv->geometry.num_cells[0], denv->geometry.num_cells[1],
                                               denv->geometry.num_cells[2], denv->geometry.resolution, &lp, &cm);
        if ((e = hipMalloc((void**)&ctx->d_noff, (cells + 1) * sizeof(uint32_t))) != hipSuccess) return bail(e, "offsets");
        if ((e = hipMemcpy(ctx->d_noff, denv->offsets, (cells + 1) * sizeof(uint32_t), hipMemcpyDeviceToDevice)) != hipSuccess)
            return bail(e, "offsets copy");
        if (denv->num_entries > 0) {
            const size_t bytes = 6 * (size_t)denv->num_entries * sizeof(double);
            if ((e = hipMalloc((void**)&ctx->d_nent, bytes)) != hipSuccess) return bail(e, "entries");
            if ((e = hipMemcpy(ctx->d_nent, denv->entries, bytes, hipMemcpyDeviceToDevice)) != hipSuccess)
                return bail(e, "entries copy");
        }
        ctx->has_normals = 1;
    }
    if (analyzed) {
        ctx->skip_enabled = 1;
        ctx->skip_lplus = lp * (1.0 + 1e-6) + 1e-6;
        ctx->skip_cmax = cm * (1.0 + 1e-6) + 1e-6;
    }
    /* the kernels' HBM layout: the SDF and the normal ranges in 4x4x4-cell bricks (the
     * analysis above read the VoxelGrid order) */
    {
        float* bricked = nullptr;
        if ((e = fks_env::brick_sdf_device(ctx->d_sdf, ctx->sdf_g.n, ctx->sdf_g.nb, &bricked)) != hipSuccess)
            return bail(e, "sdf bricks");
        (void)hipFree(ctx->d_sdf);
        ctx->d_sdf = bricked;
        if (ctx->d_noff) {
            if ((e = fks_env::brick_normal_ranges_device(ctx->d_noff, ctx->nrm_g.n, ctx->nrm_g.nb, &ctx->d_nrange)) != hipSuccess)
                return bail(e, "normal-range bricks");
            (void)hipFree(ctx->d_noff);
            ctx->d_noff = nullptr;
        }
    }
    if ((e = hipMalloc((void**)&ctx->d_counters, fksd::kCounterWords * sizeof(unsigned long long))) != hipSuccess)
        return bail(e, "counters");
    if ((e = hipHostMalloc((void**)&ctx->h_counters, fksd::kCounterWords * sizeof(unsigned long long), 0)) != hipSuccess)
        return bail(e, "pinned counters");
    if ((e = hipMalloc((void**)&ctx->d_args, sizeof(fksd::SimArgs))) != hipSuccess) return bail(e, "kernel arguments");
    if ((e = hipHostMalloc((void**)&ctx->h_args, sizeof(fksd::SimArgs), 0)) != hipSuccess) return bail(e, "kernel arguments");
    if ((e = hipEventCreate(&ctx->ev0)) != hipSuccess) return bail(e, "event");
    if ((e = hipEventCreate(&ctx->ev1)) != hipSuccess) return bail(e, "event");
    (void)same_geometry;
    *out_ctx = ctx;
    return FKS_OK;
}

fks_status fks_create(const fks_environment* env, const fks_solver_params* params, double simulation_controller_frequency,
                      uint64_t prng_seed, int32_t debug_level, int32_t device, fks_context** out_ctx) {
    if (!env) return FKS_ERR_INVALID_ARGUMENT;
    return create_impl(env, nullptr, params, simulation_controller_frequency, prng_seed, debug_level, device, out_ctx);
}

fks_status fks_create_from_device_env(const fks_device_env* env, const fks_solver_params* params,
                                      double simulation_controller_frequency, uint64_t prng_seed, int32_t debug_level,
                                      fks_context** out_ctx) {
    if (!env) return FKS_ERR_INVALID_ARGUMENT;
    return create_impl(nullptr, env, params, simulation_controller_frequency, prng_seed, debug_level, env->device, out_ctx);
}

void fks_destroy(fks_context* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->pending && ctx->pending_stream) (void)hipStreamSynchronize(ctx->pending_stream);
    (void)hipDeviceSynchronize();
    spec_release(ctx);
    free_robot(ctx);
    free_staging(ctx);
    if (ctx->d_sdf) (void)hipFree(ctx->d_sdf);
    if (ctx->d_noff) (void)hipFree(ctx->d_noff);
    if (ctx->d_nrange) (void)hipFree(ctx->d_nrange);
    if (ctx->d_nent) (void)hipFree(ctx->d_nent);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    if (ctx->h_counters) (void)hipHostFree(ctx->h_counters);
    if (ctx->d_args) (void)hipFree(ctx->d_args);
    if (ctx->h_args) (void)hipHostFree(ctx->h_args);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    delete ctx;
}

const char* fks_get_last_error(const fks_context* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int32_t fks_config_width(const fks_context* ctx) { return (ctx && ctx->has_robot) ? ctx->R.W : 0; }

/* Launch geometry of the current robot: the LDS layout (with the paired FK's second set
 * of joint motion matrices for linked chains of <= 32 joints when the occupancy it leaves
 * equals the plain layout's), workgroup size, resident workgroups per CU and the per-wave
 * workspace.  Computed into locals and committed to ctx only when all of it succeeds. */
static fks_status launch_layout(fks_context* ctx, const fksd::RobotDev& R) {
    const int P = R.P, G = R.G;
    /* resident waves per CU of a layout at the largest workgroup (<= wmax waves) whose
     * blocks fit the CU's 160 KiB */
    auto blocks = [&](const fksd::LdsLayout& l, uint32_t wmax, uint32_t* wpg, size_t* bytes) -> int {
        uint32_t w = wmax;
        size_t b = 0;
        for (;;) {
            b = ((size_t)l.shared_total + (size_t)w * l.total) * sizeof(double);
            if (b <= 160 * 1024 || w == 1) break;
            w /= 2;
        }
        *wpg = w;
        *bytes = b;
        if (b > 160 * 1024) return 0;
        /* every kernel launched with this layout (plain, individual-Jacobian and traced
         * simulation, configuration check, kinematics) must hold that many groups: the
         * smallest occupancy of them all */
        const bool lean_l = l.lean != 0;
        const sim_kernel_t kernels[] = {kernel_for(R.type, false, lean_l), kernel_for(R.type, true, lean_l),
                                        traced_kernel_for(R.type, lean_l), check_kernel_for(R.type),
                                        R.type == FKS_ROBOT_SE2 ? fks_kinematics_se2
                                                                : (R.type == FKS_ROBOT_SE3 ? fks_kinematics_se3 : fks_kinematics_linked)};
        int n = 1 << 30;
        for (sim_kernel_t k : kernels) {
            int nk = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nk, reinterpret_cast<const void*>(k), 64 * (int)w, b) != hipSuccess)
                return 0;
            n = std::min(n, nk);
        }
        return n * (int)w; /* resident waves per CU */
    };
    uint32_t wpg = 0;
    size_t bytes = 0;
    const bool linked_pairable = R.type == FKS_ROBOT_LINKED && R.J >= 1 && R.J <= 32;
    const int w0 = blocks(fksd::make_lds_layout(R.L, R.J, R.D, R.W, R.G, R.nrounds), fksd::kWavesPerGroup, &wpg, &bytes);
    bool pair = false;
    if (linked_pairable && w0 > 0) {
        uint32_t w = 0;
        size_t b = 0;
        pair = blocks(fksd::make_lds_layout(R.L, R.J, R.D, R.W, R.G, R.nrounds, true), fksd::kWavesPerGroup, &w, &b) >= w0;
    }
    int waves_per_cu = blocks(fksd::make_lds_layout(R.L, R.J, R.D, R.W, R.G, R.nrounds, pair), fksd::kWavesPerGroup, &wpg, &bytes);
    const int standard_waves_per_cu = waves_per_cu;
    /* a linked robot whose LDS block caps the resident waves below the register limit may run
     * lean blocks (the skip-proof cache in scratch) in workgroups of up to 8 waves, if that
     * keeps more waves resident (cfg5's 14-dof arm: 12 -> 16 per CU) */
    bool lean = false;
    if (R.type == FKS_ROBOT_LINKED) {
        for (uint32_t wmax : {(uint32_t)fksd::kMaxWavesPerGroup, (uint32_t)fksd::kWavesPerGroup}) {
            uint32_t w = 0;
            size_t b = 0;
            const int n = blocks(fksd::make_lds_layout(R.L, R.J, R.D, R.W, R.G, R.nrounds, false, true), wmax, &w, &b);
            if (n > waves_per_cu) {
                waves_per_cu = n;
                wpg = w;
                bytes = b;
                lean = true;
                pair = false;
            }
        }
    }
    if (waves_per_cu < 1)
        return fail(ctx, FKS_ERR_UNSUPPORTED,
                    "robot too large: one wave's LDS block (" + std::to_string(bytes) + " bytes) does not fit a CU");
    int cus = 0;
    HIP_TRY(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    uint32_t grid_groups = (uint32_t)(cus * (waves_per_cu / (int)wpg));
    const uint64_t scratch_per_wave = fksd::make_scratch_layout(3u * P, R.D, (int)P, G).total;
    /* the per-wave workspace grows with 3P x D (the stacked Jacobian) and the robot's
     * geometry count: for very large robots the persistent grid keeps only as many waves
     * as half the free HBM holds (the ticket queue hands out the work either way) */
    size_t free_b = 0, total_b = 0;
    HIP_TRY(ctx, hipMemGetInfo(&free_b, &total_b));
    free_b += ctx->cap_scratch * sizeof(double); /* the current workspace is given back below */
    const size_t per_group = (size_t)wpg * scratch_per_wave * sizeof(double);
    const size_t max_groups = std::max<size_t>(1, (free_b / 2) / std::max<size_t>(1, per_group));
    if ((size_t)grid_groups > max_groups) grid_groups = (uint32_t)max_groups;
    const size_t words = (size_t)grid_groups * wpg * scratch_per_wave;
    if (words > ctx->cap_scratch || !ctx->d_scratch) {
        if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
        ctx->d_scratch = nullptr;
        ctx->cap_scratch = 0;
        HIP_TRY(ctx, hipMalloc((void**)&ctx->d_scratch, words * sizeof(double)));
        ctx->cap_scratch = words;
    }
    ctx->fk_pair = pair;
    ctx->lean = lean;
    ctx->standard_resident_waves = (uint32_t)(cus * std::max(0, standard_waves_per_cu));
    ctx->waves_per_cu = (uint32_t)waves_per_cu;
    ctx->waves_per_group = wpg;
    ctx->lds_bytes = bytes;
    ctx->grid_groups = grid_groups;
    ctx->grid_waves = grid_groups * wpg;
    /* the small-batch kernel on the same layout (not for lean blocks) */
    ctx->small_grid_waves = 0;
    if (!lean) {
        int nk = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nk, reinterpret_cast<const void*>(small_kernel_for(R.type)), 64 * (int)wpg,
                                                         bytes) == hipSuccess &&
            nk > 0)
            ctx->small_grid_waves = std::min<uint32_t>((uint32_t)(cus * nk) * wpg, ctx->grid_waves);
    }
    /* the cooperative kernel: one wave's block plus the mailbox per workgroup, its workgroup
     * size from its launch bound (a build's FKS_COOP_WAVES); each workgroup uses one wave's
     * workspace, so at most grid_waves of them */
    ctx->coop_particles = 0;
    ctx->coop_waves = 0;
    ctx->coop_lds_bytes = 0;
    if (!lean && R.nrounds <= fksd::kCoopMaxRounds) {
        const fksd::LdsLayout l = fksd::make_lds_layout(R.L, R.J, R.D, R.W, R.G, R.nrounds, pair);
        const size_t cb = ((size_t)l.shared_total + l.total + fksd::kCoopBoxDoubles) * sizeof(double);
        hipFuncAttributes fa{};
        int nk = 0;
        if (cb <= 160 * 1024 && hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(coop_kernel_for(R.type))) == hipSuccess &&
            fa.maxThreadsPerBlock >= 128 &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&nk, reinterpret_cast<const void*>(coop_kernel_for(R.type)),
                                                         fa.maxThreadsPerBlock, cb) == hipSuccess &&
            nk > 0) {
            ctx->coop_waves = (uint32_t)fa.maxThreadsPerBlock / 64u;
            ctx->coop_lds_bytes = cb;
            ctx->coop_particles = std::min<uint32_t>((uint32_t)(cus * nk), ctx->grid_waves);
        }
    }
    (void)hipGetLastError();
    ctx->scratch_per_wave = scratch_per_wave;
    return FKS_OK;
}

fks_status fks_set_robot(fks_context* ctx, const fks_robot_desc* d) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!d) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null robot");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (ctx->pending && ctx->pending_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->pending_stream));
    const int G = d->num_geometries;
    if (G < 1 || G > fksd::kMaxGeoms || !d->geometry_link || !d->geometry_point_offset || !d->points || !d->controllers)
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "robot geometries/controllers missing or more than 64 geometries");
    const uint32_t P = d->geometry_point_offset[G];
    if (d->geometry_point_offset[0] != 0 || P < 1 || P > 65535)
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "robot needs 1..65535 points with offsets starting at 0");
    for (int g = 0; g < G; ++g)
        if (d->geometry_point_offset[g + 1] < d->geometry_point_offset[g])
            return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "geometry offsets must be non-decreasing");
    for (uint32_t i = 0; i < 4 * P; ++i)
        if (!std::isfinite(d->points[i])) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "non-finite robot point");
    RobotDev R;
    std::memset(&R, 0, sizeof(R));
    R.type = d->robot_type;
    R.G = G;
    R.P = (int32_t)P;
    std::vector<JointDev> joints;
    std::vector<int32_t> dof_joint;
    std::vector<int32_t> link_parent_joint;
    if (d->robot_type == FKS_ROBOT_LINKED) {
        const int L = d->num_links, J = d->num_joints;
        if (L < 1 || L > fksd::kMaxLinks || J < 0 || J > fksd::kMaxJoints || (J > 0 && !d->joints))
            return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "linked robot needs 1..64 links and 0..64 joints");
        std::vector<int> seen(L, 0);
        seen[0] = 1;
        link_parent_joint.assign(L, -1);
        for (int j = 0; j < J; ++j) {
            const fks_joint_desc& jd = d->joints[j];
            if (jd.parent_link < 0 || jd.parent_link >= L || jd.child_link <= 0 || jd.child_link >= L)
                return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "joint link index out of range");
            if (!seen[jd.parent_link] || seen[jd.child_link])
                return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "joints must be in topological order, one parent per link");
            seen[jd.child_link] = 1;
            link_parent_joint[jd.child_link] = j;
            if (jd.type != FKS_JOINT_FIXED && jd.type != FKS_JOINT_REVOLUTE && jd.type != FKS_JOINT_CONTINUOUS &&
                jd.type != FKS_JOINT_PRISMATIC)
                return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "unknown joint type");
            JointDev jv;
            std::memset(&jv, 0, sizeof(jv));
            jv.parent = jd.parent_link;
            jv.child = jd.child_link;
            jv.type = jd.type;
            jv.dof = -1;
            std::memcpy(jv.origin, jd.origin, sizeof(jv.origin));
            std::memcpy(jv.axis, jd.axis, sizeof(jv.axis));
            jv.lo = jd.limit_lower;
            jv.hi = jd.limit_upper;
            if (jd.type != FKS_JOINT_FIXED) {
                jv.dof = (int32_t)dof_joint.size();
                dof_joint.push_back(j);
            }
            joints.push_back(jv);
        }
        for (int l = 0; l < L; ++l)
            if (!seen[l]) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "every link must be reached by a joint");
        if ((int)dof_joint.size() != d->num_dofs || d->num_dofs < 1 || d->num_dofs > fksd::kMaxDofs)
            return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "num_dofs must equal the number of non-fixed joints (1..64)");
        for (int g = 0; g < G; ++g)
            if (d->geometry_link[g] < 0 || d->geometry_link[g] >= L)
                return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "geometry link index out of range");
        R.L = L;
        R.J = J;
        R.D = d->num_dofs;
        R.W = d->num_dofs;
    } else if (d->robot_type == FKS_ROBOT_SE2 || d->robot_type == FKS_ROBOT_SE3) {
        const int D = (d->robot_type == FKS_ROBOT_SE2) ? 3 : 6;
        if (d->num_dofs != D || G != 1 || d->geometry_link[0] != 0)
            return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "SE(2)/SE(3) robots have one geometry on link 0 and 3/6 dofs");
        R.L = 1;
        R.J = 0;
        R.D = D;
        R.W = (d->robot_type == FKS_ROBOT_SE2) ? 3 : 12;
    } else {
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "unknown robot type");
    }
    std::memcpy(R.base, d->base_transform, sizeof(R.base));
    /* allowed self-collision masks (CheckIfSelfCollisionAllowed, symmetric, self allowed) */
    std::vector<uint64_t> allowed(G, 0);
    for (int g = 0; g < G; ++g) allowed[g] |= 1ull << g;
    for (int k = 0; k < d->num_allowed_pairs; ++k) {
        const int a = d->allowed_pairs[2 * k], b = d->allowed_pairs[2 * k + 1];
        if (a < 0 || a >= G || b < 0 || b >= G) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "allowed pair out of range");
        allowed[a] |= 1ull << b;
        allowed[b] |= 1ull << a;
    }
    std::vector<int32_t> pairs;
    for (int a = 0; a < G; ++a)
        for (int b = a + 1; b < G; ++b)
            if (!((allowed[a] >> b) & 1ull)) {
                pairs.push_back(a);
                pairs.push_back(b);
            }
    R.npairs = (int32_t)(pairs.size() / 2);
    R.self_possible = !(G == 1 || (G == 2 && ((allowed[0] >> 1) & 1ull)));
    /* per point geometry, per geometry local boxes and link masses (SPCS:1244-1255) */
    std::vector<uint16_t> point_geom(P), point_link(P);
    std::vector<double> box(7 * (size_t)G), mass(G);
    for (int g = 0; g < G; ++g) {
        const uint32_t b0 = d->geometry_point_offset[g], b1 = d->geometry_point_offset[g + 1];
        double mn[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, mx[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        bool w_one = true;
        for (uint32_t i = b0; i < b1; ++i) {
            point_geom[i] = (uint16_t)g;
            point_link[i] = (uint16_t)d->geometry_link[g];
            for (int a = 0; a < 3; ++a) {
                mn[a] = std::fmin(mn[a], d->points[4 * i + a]);
                mx[a] = std::fmax(mx[a], d->points[4 * i + a]);
            }
            w_one = w_one && d->points[4 * i + 3] == 1.0;
        }
        if (b1 == b0) {
            for (int a = 0; a < 3; ++a) mn[a] = mx[a] = 0.0;
        }
        for (int a = 0; a < 3; ++a) {
            box[7 * g + a] = 0.5 * (mn[a] + mx[a]);
            box[7 * g + 3 + a] = 0.5 * (mx[a] - mn[a]);
        }
        box[7 * g + 6] = w_one ? 1.0 : 0.0;
    }
    /* 64-point rounds of the kernel's lane-strided loops */
    const int NR = ((int)P + 63) / 64;
    std::vector<fksd::RoundDev> rounds(NR > 0 ? NR : 1);
    for (int r = 0; r < NR; ++r) {
        fksd::RoundDev rd;
        rd.link = -1;
        rd.npts = std::min(64, (int)P - 64 * r);
        rd.radius = 0.0;
        bool uniform = true;
        for (int i = 64 * r; i < 64 * r + rd.npts; ++i) {
            const double* p = d->points + 4 * (size_t)i;
            uniform = uniform && point_link[i] == point_link[64 * r] && p[3] == 1.0;
            rd.radius = std::max(rd.radius, std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]));
        }
        if (uniform && std::isfinite(rd.radius)) rd.link = point_link[64 * r];
        rd.radius = rd.radius * (1.0 + 1e-9) + 1e-12;
        rounds[r] = rd;
    }
    R.nrounds = NR;
    double previous_link_masses = 0.0;
    for (int g = G - 1; g >= 0; --g) {
        const double link_mass = (double)(d->geometry_point_offset[g + 1] - d->geometry_point_offset[g]);
        mass[g] = link_mass + previous_link_masses;
        previous_link_masses += link_mass;
    }
    /* dofs moving each link: joints whose child is an ancestor-or-self of the link */
    std::vector<uint64_t> link_mask(R.L, 0);
    if (d->robot_type == FKS_ROBOT_LINKED) {
        for (int l = 0; l < R.L; ++l) {
            int cur = l;
            while (cur > 0) {
                const int j = link_parent_joint[cur];
                if (joints[j].dof >= 0) link_mask[l] |= 1ull << joints[j].dof;
                cur = joints[j].parent;
            }
        }
    }
    /* lever arm bound per dof: max over downstream points of (path reach from the
     * joint frame origin) + |p|; prismatic joints on the path add their largest stroke */
    std::vector<double> lever(std::max(1, R.D), HUGE_VAL);
    if (d->robot_type == FKS_ROBOT_LINKED) {
        bool w_one = true;
        for (uint32_t i = 0; i < P; ++i) w_one = w_one && d->points[4 * (size_t)i + 3] == 1.0;
        for (int k = 0; k < R.D && w_one; ++k) {
            const int jd = dof_joint[k];
            if (joints[jd].type == FKS_JOINT_PRISMATIC) {
                const double* ax = joints[jd].axis;
                lever[k] = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
                continue;
            }
            double worst = 0.0;
            for (int g = 0; g < G; ++g) {
                const int l = d->geometry_link[g];
                if (!((link_mask[l] >> k) & 1ull)) continue;
                /* reach from joint jd's frame origin (= its child link origin) down to link l */
                double reach = 0.0;
                for (int cur = l; cur != joints[jd].child;) {
                    const JointDev& jp = joints[link_parent_joint[cur]];
                    reach += std::sqrt(jp.origin[3] * jp.origin[3] + jp.origin[7] * jp.origin[7] + jp.origin[11] * jp.origin[11]);
                    if (jp.type == FKS_JOINT_PRISMATIC)
                        reach += std::max(std::fabs(jp.lo), std::fabs(jp.hi)) *
                                 std::sqrt(jp.axis[0] * jp.axis[0] + jp.axis[1] * jp.axis[1] + jp.axis[2] * jp.axis[2]);
                    cur = jp.parent;
                }
                for (uint32_t i = d->geometry_point_offset[g]; i < d->geometry_point_offset[g + 1]; ++i) {
                    const double* p = d->points + 4 * (size_t)i;
                    worst = std::max(worst, reach + std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]));
                }
            }
            const double* ax = joints[jd].axis;
            const double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
            /* AngleAxis with a non-unit axis is not a rotation: no bound */
            lever[k] = (std::fabs(an - 1.0) < 1e-12 && std::isfinite(worst)) ? worst * (1.0 + 1e-9) + 1e-12 : HUGE_VAL;
        }
    } else {
        /* SE(2) (x, y, theta, applied additively) and SE(3) (body twist v, w: P * exp(twist)):
         * a point p of the body moves by at most |dt| + |rotation angle| * |p|, the angle at most
         * the sum of the angular components' magnitudes and |V v| <= |v| (exp's V has operator
         * norm <= 1), so translation components get lever 1, rotation components max |p| */
        bool w_one = true;
        double rmax = 0.0;
        for (uint32_t i = 0; i < P; ++i) {
            const double* p = d->points + 4 * (size_t)i;
            w_one = w_one && p[3] == 1.0;
            rmax = std::max(rmax, std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]));
        }
        if (w_one && std::isfinite(rmax)) {
            const int nt = d->robot_type == FKS_ROBOT_SE2 ? 2 : 3; /* translation components first */
            for (int k = 0; k < R.D; ++k) lever[k] = (k < nt) ? 1.0 + 1e-9 : rmax * (1.0 + 1e-9) + 1e-12;
        }
    }
    /* the same bound over the geometries' local boxes (corner distance <= |centre| + |half
     * extents|): the self-collision boxes are built from them */
    std::vector<double> lever_box(std::max(1, R.D), HUGE_VAL);
    if (d->robot_type == FKS_ROBOT_LINKED) {
        for (int k = 0; k < R.D; ++k) {
            const int jd = dof_joint[k];
            if (joints[jd].type == FKS_JOINT_PRISMATIC) {
                lever_box[k] = lever[k];
                continue;
            }
            const double* ax = joints[jd].axis;
            const double an = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
            double worst = 0.0;
            bool ok = std::fabs(an - 1.0) < 1e-12;
            for (int g = 0; g < G && ok; ++g) {
                const int l = d->geometry_link[g];
                if (!((link_mask[l] >> k) & 1ull)) continue;
                const double* b = box.data() + 7 * (size_t)g;
                if (b[6] == 0.0) {
                    ok = false; /* no box (a point with w != 1): the box test never skips anyway */
                    break;
                }
                double reach = 0.0;
                for (int cur = l; cur != joints[jd].child;) {
                    const JointDev& jp = joints[link_parent_joint[cur]];
                    reach += std::sqrt(jp.origin[3] * jp.origin[3] + jp.origin[7] * jp.origin[7] + jp.origin[11] * jp.origin[11]);
                    if (jp.type == FKS_JOINT_PRISMATIC)
                        reach += std::max(std::fabs(jp.lo), std::fabs(jp.hi)) *
                                 std::sqrt(jp.axis[0] * jp.axis[0] + jp.axis[1] * jp.axis[1] + jp.axis[2] * jp.axis[2]);
                    cur = jp.parent;
                }
                worst = std::max(worst, reach + std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]) +
                                            std::sqrt(b[3] * b[3] + b[4] * b[4] + b[5] * b[5]));
            }
            lever_box[k] = (ok && std::isfinite(worst)) ? worst * (1.0 + 1e-9) + 1e-12 : HUGE_VAL;
        }
    }
    std::vector<double> weights;
    if (d->robot_type == FKS_ROBOT_LINKED) {
        for (int k = 0; k < R.D; ++k) weights.push_back(d->distance_weights ? d->distance_weights[k] : 1.0);
    } else {
        weights.push_back(d->distance_weights ? d->distance_weights[0] : 1.0);
        weights.push_back(d->distance_weights ? d->distance_weights[1] : 1.0);
    }
    /* SampledUncertainVelocityActuator tables (UNC:123-281), validated before the old robot goes */
    if (d->sampled_actuators) {
        for (int k = 0; k < R.D; ++k) {
            const fks_sampled_actuator& a = d->sampled_actuators[k];
            if (a.num_bins == 0) continue;
            if (a.bin_elements == 0 || !a.bin_bounds || !a.bin_samples)
                return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "sampled actuator needs bounds and >= 1 sample per bin");
            for (uint64_t i = 0; i < 2ull * a.num_bins; ++i)
                if (std::isnan(a.bin_bounds[i])) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "NaN sampled-actuator bin bound");
            for (uint64_t i = 0; i < (uint64_t)a.num_bins * a.bin_elements; ++i)
                if (!std::isfinite(a.bin_samples[i]))
                    return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "non-finite sampled-actuator sample");
        }
    }
    free_robot(ctx);
    auto up = [&](auto** dptr, const auto* host, size_t count) -> hipError_t {
        hipError_t e = dev_upload(dptr, host, count);
        if (*dptr) ctx->robot_allocs.push_back((void*)*dptr);
        return e;
    };
    JointDev* dj = nullptr;
    int32_t *dgl = nullptr, *ddj = nullptr, *dpairs = nullptr;
    uint32_t* dgo = nullptr;
    double *dpts = nullptr, *dbox = nullptr, *dmass = nullptr, *dw = nullptr;
    uint16_t *dpg = nullptr, *dpl = nullptr;
    uint64_t *dlm = nullptr, *dam = nullptr;
    fks_dof_controller* dctrl = nullptr;
    HIP_TRY(ctx, up(&dj, joints.data(), joints.size()));
    HIP_TRY(ctx, up(&dgl, d->geometry_link, (size_t)G));
    HIP_TRY(ctx, up(&dgo, d->geometry_point_offset, (size_t)G + 1));
    HIP_TRY(ctx, up(&dpts, d->points, 4 * (size_t)P));
    HIP_TRY(ctx, up(&dpg, point_geom.data(), (size_t)P));
    HIP_TRY(ctx, up(&dpl, point_link.data(), (size_t)P));
    HIP_TRY(ctx, up(&ddj, dof_joint.data(), dof_joint.size()));
    HIP_TRY(ctx, up(&dlm, link_mask.data(), link_mask.size()));
    HIP_TRY(ctx, up(&dpairs, pairs.data(), pairs.size()));
    HIP_TRY(ctx, up(&dam, allowed.data(), allowed.size()));
    HIP_TRY(ctx, up(&dbox, box.data(), box.size()));
    HIP_TRY(ctx, up(&dmass, mass.data(), mass.size()));
    HIP_TRY(ctx, up(&dctrl, d->controllers, (size_t)R.D));
    HIP_TRY(ctx, up(&dw, weights.data(), weights.size()));
    fksd::RoundDev* drounds = nullptr;
    HIP_TRY(ctx, up(&drounds, rounds.data(), rounds.size()));
    double* dlever = nullptr;
    HIP_TRY(ctx, up(&dlever, lever.data(), lever.size()));
    double* dlever_box = nullptr;
    HIP_TRY(ctx, up(&dlever_box, lever_box.data(), lever_box.size()));
    R.joints = dj;
    R.geom_link = dgl;
    R.geom_off = dgo;
    R.points = dpts;
    R.point_geom = dpg;
    R.point_link = dpl;
    R.dof_joint = ddj;
    R.link_dof_mask = dlm;
    R.pairs = dpairs;
    R.allowed_mask = dam;
    R.geom_box = dbox;
    R.geom_mass = dmass;
    R.ctrl = dctrl;
    R.weights = dw;
    R.rounds = drounds;
    R.dof_lever = dlever;
    R.dof_lever_box = dlever_box;
    R.sampled_mask = 0;
    R.sampled = nullptr;
    if (d->sampled_actuators) {
        std::vector<fksd::SampledDev> sd((size_t)R.D);
        for (int k = 0; k < R.D; ++k) {
            const fks_sampled_actuator& a = d->sampled_actuators[k];
            std::memset(&sd[k], 0, sizeof(sd[k]));
            if (a.num_bins == 0) continue;
            double *dbounds = nullptr, *dsamples = nullptr;
            HIP_TRY(ctx, up(&dbounds, a.bin_bounds, 2 * (size_t)a.num_bins));
            HIP_TRY(ctx, up(&dsamples, a.bin_samples, (size_t)a.num_bins * a.bin_elements));
            sd[k].nbins = a.num_bins;
            sd[k].elems = a.bin_elements;
            sd[k].bounds = dbounds;
            sd[k].samples = dsamples;
            R.sampled_mask |= 1ull << k;
        }
        fksd::SampledDev* dsd = nullptr;
        HIP_TRY(ctx, up(&dsd, sd.data(), sd.size()));
        R.sampled = dsd;
    }
    {
        const fks_status st = launch_layout(ctx, R);
        if (st != FKS_OK) return st; /* has_robot stays false (free_robot above) */
    }
    ctx->R = R;
    ctx->has_robot = true;
    /* the new robot's shape-specialised kernel is built at the first launch that runs it
     * (simulate_device), so robots only ever simulated in small batches cost no compile */
    spec_release(ctx);
    ctx->spec_pending = ctx->specialize != 0;
    return FKS_OK;
}

/* fold the counters of a finished launch into the statistics */
static fks_status settle(fks_context* ctx) {
    if (!ctx->pending) return FKS_OK;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->pending_stream));
    ctx->pending = false;
    const unsigned long long* c = ctx->h_counters;
    if (ctx->pending_kind == 1) {
        /* a config check: no simulator statistics, only its own counters */
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        ctx->check_last.sdf_bytes = c[fksd::kCntSdfBytes];
        ctx->check_last.kernel_ms = (double)ms;
        ctx->check_last.call_ms =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ctx->call_start).count();
        ctx->check_last.calls = 1;
        return FKS_OK;
    }
    ctx->stats.successful_resolves += c[fksd::kCntSuccessful];
    ctx->stats.unsuccessful_resolves += c[fksd::kCntUnsuccessful];
    ctx->stats.free_resolves += c[fksd::kCntFree];
    ctx->stats.collision_resolves += c[fksd::kCntCollision];
    ctx->stats.fallback_resolves += c[fksd::kCntFallback];
    ctx->stats.unsuccessful_env_collision_resolves += c[fksd::kCntUnsuccessfulEnv];
    ctx->stats.unsuccessful_self_collision_resolves += c[fksd::kCntUnsuccessfulSelf];
    ctx->stats.recovered_unsuccessful_resolves += c[fksd::kCntRecovered];
    ctx->last.controller_steps = c[fksd::kCntSteps];
    ctx->last.microsteps = c[fksd::kCntMicrosteps];
    ctx->last.resolver_iterations = c[fksd::kCntResolver];
    ctx->last.sdf_bytes = c[fksd::kCntSdfBytes];
    ctx->last.error_particles = c[fksd::kCntErrorParticles];
    ctx->last.least_squares_rows = c[fksd::kCntLsqRows];
    ctx->last.self_collision_checks = c[fksd::kCntSelfChecks];
    ctx->last.self_corrected_points = c[fksd::kCntSelfPoints];
    for (int k = 0; k < FKS_NUM_PHASES; ++k) {
        ctx->phase_last[k] = c[fksd::kPhaseBase + k];
        ctx->phase_total[k] += ctx->phase_last[k];
    }
    float ms = 0.0f;
    HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last.kernel_ms = (double)ms;
    ctx->last.call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ctx->call_start).count();
    ctx->last.calls = 1;
    ctx->total.particles += ctx->last.particles;
    ctx->total.controller_steps += ctx->last.controller_steps;
    ctx->total.microsteps += ctx->last.microsteps;
    ctx->total.resolver_iterations += ctx->last.resolver_iterations;
    ctx->total.sdf_bytes += ctx->last.sdf_bytes;
    ctx->total.error_particles += ctx->last.error_particles;
    ctx->total.least_squares_rows += ctx->last.least_squares_rows;
    ctx->total.self_collision_checks += ctx->last.self_collision_checks;
    ctx->total.self_corrected_points += ctx->last.self_corrected_points;
    ctx->total.kernel_ms += ctx->last.kernel_ms;
    ctx->total.call_ms += ctx->last.call_ms;
    ctx->total.calls += 1;
    return FKS_OK;
}

}  // extern "C"

/* device trace buffers of a traced launch (fks_forward_simulate_traced) */
struct TraceDev {
    double* inputs;
    uint32_t* micro;
    double* cfg;
    uint32_t* tags;
    uint32_t* nsteps;
    uint32_t* ncfg;
    uint32_t step_cap, cfg_cap;
};

static fks_status simulate_device(fks_context* ctx, const double* d_starts, uint64_t n, const double* d_targets,
                                  uint64_t num_targets, uint64_t first_particle_id, int32_t allow_contacts,
                                  double* d_out_positions, uint8_t* d_out_collided, uint32_t* d_out_microsteps,
                                  uint32_t* d_out_resolver_iterations, uint32_t* d_out_error_flags, void* stream,
                                  int32_t synchronize, const TraceDev* tr, double* d_pid_io = nullptr) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (n > 0 && (!d_starts || !d_targets || !d_out_positions))
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null device buffer");
    if (n > 0 && num_targets != 1 && num_targets != n)
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "targets must be 1 or n (SPCS:792)");
    if (n > 0xffffffffull) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "at most 2^32-1 particles per call");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ctx->call_start = std::chrono::steady_clock::now();
    const uint64_t key = splitmix64(ctx->seed ^ splitmix64(ctx->call_index));
    ctx->call_index++;
    std::memset(&ctx->last, 0, sizeof(ctx->last));
    ctx->last.particles = n;
    fksd::SimArgs a;
    std::memset(&a, 0, sizeof(a));
    a.sdf_g = ctx->sdf_g;
    a.nrm_g = ctx->nrm_g;
    a.env_g = ctx->env_g;
    a.sdf = ctx->d_sdf;
    a.nrange = ctx->d_nrange;
    a.nent = ctx->d_nent;
    a.oob = ctx->oob;
    a.has_normals = ctx->has_normals;
    a.skip_enabled = ctx->skip_enabled;
    a.skip_lplus = ctx->skip_lplus;
    a.skip_cmax = ctx->skip_cmax;
    a.R = ctx->R;
    a.S = ctx->params;
    a.dt = 1.0 / ctx->frequency;
    a.thr_env = 0.0 - (ctx->params.environment_collision_check_tolerance * ctx->sdf_g.res);
    a.target_micro = ctx->env_g.res * 0.125;
    a.allowed_micro = ctx->env_g.res * 1.0;
    a.time_multiplier = 1.0 / a.dt;
    a.T = forward_steps(ctx->params.forward_simulation_time, std::fabs(ctx->frequency));
    a.key0 = (uint32_t)key;
    a.key1 = (uint32_t)(key >> 32);
    a.starts = d_starts;
    a.targets = d_targets;
    a.num_targets = num_targets;
    a.n = n;
    a.first_pid = first_particle_id;
    a.allow_contacts = allow_contacts ? 1 : 0;
    a.individual_jacobians = ctx->individual_jacobians;
    a.out_q = d_out_positions;
    a.pid_io = d_pid_io;
    a.out_collided = d_out_collided;
    a.out_micro = d_out_microsteps;
    a.out_resolver = d_out_resolver_iterations;
    a.out_err = d_out_error_flags;
    a.counters = ctx->d_counters;
    a.queue = ctx->d_counters + fksd::kNumCounters;
    a.scratch = ctx->d_scratch;
    a.scratch_per_wave = ctx->scratch_per_wave;
    a.row_cap = 3u * (uint32_t)ctx->R.P;
    a.L = fksd::make_lds_layout(ctx->R.L, ctx->R.J, ctx->R.D, ctx->R.W, ctx->R.G, ctx->R.nrounds, ctx->fk_pair, ctx->lean);
    a.SL = fksd::make_scratch_layout(a.row_cap, ctx->R.D, ctx->R.P, ctx->R.G);
    /* controller-step segments: automatically only when the batch outnumbers the
     * resident waves (otherwise every particle has a wave from the start), always
     * when set explicitly (fks_set_segment_steps); traced calls run whole */
    a.seg_steps = a.T;
    a.nseg = 1;
    a.seg_stride = 2u * (uint32_t)ctx->R.D + 4u + (uint32_t)fksd::kRoundState * (uint32_t)std::min(ctx->R.nrounds, 64);
    if (!tr && n > 0 && (ctx->segment_steps != 0 || n > (uint64_t)ctx->grid_waves)) {
        uint32_t k = ctx->segment_steps ? ctx->segment_steps : kDefaultSegmentSteps;
        if (k > a.T) k = a.T;
        a.seg_steps = k;
        /* T >= 1 and k >= 1: ceil(T / k) without the uint32 wrap of (T + k - 1) / k */
        a.nseg = (uint32_t)(((uint64_t)a.T - 1u) / k + 1u);
        /* heavy_per_step <= 65536 (fks_set_segment_policy): the product fits in 64 bits,
         * and the kernel compares it with a per-segment count of at most 2^32 - 1 */
        const uint64_t heavy = (uint64_t)ctx->heavy_per_step * k;
        a.seg_heavy_resolver = (uint32_t)std::min<uint64_t>(heavy, 0xffffffffull);
        a.seg_heavy_prio = ctx->heavy_priority;
        /* the relative test's running sums pack 24 bits of segments: off for larger batches */
        a.seg_heavy_rel = ((uint64_t)n * a.nseg < (1ull << 24)) ? ctx->heavy_relative : 0u;
    }
    if (a.nseg > 1) {
        const size_t words = (size_t)n * a.seg_stride;
        if (words > ctx->cap_seg_state) {
            HIP_TRY(ctx, ensure(&ctx->d_seg_state, words));
            ctx->cap_seg_state = words;
        }
        if (n > ctx->cap_seg_done) {
            HIP_TRY(ctx, ensure(&ctx->d_seg_done, (size_t)n));
            ctx->cap_seg_done = (size_t)n;
        }
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_seg_done, 0, (size_t)n * sizeof(uint32_t), s));
        a.seg_state = ctx->d_seg_state;
        a.seg_done = ctx->d_seg_done;
    }
    if (tr) {
        a.tr_inputs = tr->inputs;
        a.tr_micro = tr->micro;
        a.tr_cfg = tr->cfg;
        a.tr_tags = tr->tags;
        a.tr_nsteps = tr->nsteps;
        a.tr_ncfg = tr->ncfg;
        a.tr_step_cap = tr->step_cap;
        a.tr_cfg_cap = tr->cfg_cap;
    }
    /* the previous call has settled, so the pinned staging copy is free */
    *ctx->h_args = a;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_args, ctx->h_args, sizeof(a), hipMemcpyHostToDevice, s));
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, fksd::kCounterWords * sizeof(unsigned long long), s));
    const uint64_t groups_needed = (n + ctx->waves_per_group - 1) / ctx->waves_per_group;
    const uint32_t grid = (uint32_t)((groups_needed < (uint64_t)ctx->grid_groups) ? (groups_needed > 0 ? groups_needed : 1)
                                                                                  : ctx->grid_groups);
    /* a batch that fits the small-batch kernel's resident waves, whole particles, plain
     * simulation: that kernel (every particle has its wave from the start either way) */
    const bool coop = ctx->small_batch && ctx->cooperative && !tr && !ctx->individual_jacobians && !ctx->lean && a.nseg == 1 && n > 0 &&
                      n <= (uint64_t)ctx->coop_particles;
    const bool small = !coop && ctx->small_batch && !tr && !ctx->individual_jacobians && !ctx->lean && a.nseg == 1 &&
                       n <= (uint64_t)ctx->small_grid_waves;
    /* the plain throughput path runs the robot's shape-specialised kernel: built (or fetched
     * from a cache) here at the first such launch; a failure keeps the generic kernel and is
     * reported by fks_get_specialization / fks_get_last_error, not by this call */
    if (ctx->spec_pending && !tr && !small && !coop && !ctx->individual_jacobians) {
        ctx->spec_pending = false;
        const std::string keep = ctx->last_error;
        if (spec_prepare(ctx) != FKS_OK) ctx->last_error = keep + (keep.empty() ? "" : "; ") + ctx->last_error;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
    }
    const bool shaped = ctx->spec_fn && !tr && !small && !coop && !ctx->individual_jacobians;
    /* a small batch runs the shape's small-batch kernel once the robot's module is built (it is
     * never built for a small batch: robots only ever simulated in small batches cost no compile) */
    const bool shaped_small = small && ctx->spec_fn && ctx->spec_small_fn;
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, s));
    ctx->last_kernel = tr ? FKS_KERNEL_TRACED
                          : (shaped ? FKS_KERNEL_SHAPED
                                    : shaped_small ? FKS_KERNEL_SHAPED_SMALL_BATCH
                                    : (coop ? FKS_KERNEL_COOPERATIVE
                                            : (small ? FKS_KERNEL_SMALL_BATCH
                                                     : (ctx->individual_jacobians ? FKS_KERNEL_INDIVIDUAL : FKS_KERNEL_THROUGHPUT))));
    if (shaped) {
        const fksd::SimArgs* argp = ctx->d_args;
        void* params[] = {&argp};
        HIP_TRY(ctx, hipModuleLaunchKernel(ctx->spec_fn, grid, 1, 1, 64 * ctx->waves_per_group, 1, 1, (unsigned)ctx->lds_bytes, s,
                                           params, nullptr));
        ctx->spec_launches++;
    } else if (shaped_small) {
        const fksd::SimArgs* argp = ctx->d_args;
        void* params[] = {&argp};
        HIP_TRY(ctx, hipModuleLaunchKernel(ctx->spec_small_fn, grid, 1, 1, 64 * ctx->waves_per_group, 1, 1, (unsigned)ctx->lds_bytes,
                                           s, params, nullptr));
        ctx->spec_launches++;
    } else if (coop) {
        hipLaunchKernelGGL(coop_kernel_for(ctx->R.type), dim3((uint32_t)n), dim3(64 * ctx->coop_waves), ctx->coop_lds_bytes, s,
                           static_cast<const fksd::SimArgs*>(ctx->d_args));
    } else {
        hipLaunchKernelGGL(tr ? traced_kernel_for(ctx->R.type, ctx->lean)
                              : (small ? small_kernel_for(ctx->R.type) : kernel_for(ctx->R.type, ctx->individual_jacobians != 0, ctx->lean)),
                           dim3(grid), dim3(64 * ctx->waves_per_group), ctx->lds_bytes, s, static_cast<const fksd::SimArgs*>(ctx->d_args));
    }
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, s));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_counters, ctx->d_counters, fksd::kCounterWords * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, s));
    ctx->pending = true;
    ctx->pending_kind = 0;
    ctx->pending_stream = s;
    if (synchronize) return settle(ctx);
    return FKS_OK;
}

extern "C" {

fks_status fks_forward_simulate_device(fks_context* ctx, const double* d_starts, uint64_t n, const double* d_targets,
                                       uint64_t num_targets, uint64_t first_particle_id, int32_t allow_contacts,
                                       double* d_out_positions, uint8_t* d_out_collided, uint32_t* d_out_microsteps,
                                       uint32_t* d_out_resolver_iterations, uint32_t* d_out_error_flags, void* stream,
                                       int32_t synchronize) {
    return simulate_device(ctx, d_starts, n, d_targets, num_targets, first_particle_id, allow_contacts, d_out_positions,
                           d_out_collided, d_out_microsteps, d_out_resolver_iterations, d_out_error_flags, stream,
                           synchronize, nullptr);
}

fks_status fks_check_config_collision_device(fks_context* ctx, const double* d_configs, uint64_t n, double inflation_ratio,
                                             uint8_t* d_out_collided, uint32_t* d_out_error_flags, void* stream,
                                             int32_t synchronize) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (n > 0 && (!d_configs || !d_out_collided)) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null device buffer");
    if (!(inflation_ratio == inflation_ratio)) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "inflation_ratio is NaN");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    ctx->call_start = std::chrono::steady_clock::now();
    std::memset(&ctx->check_last, 0, sizeof(ctx->check_last));
    ctx->check_last.particles = n;
    if (n == 0) return FKS_OK;
    fksd::SimArgs a;
    std::memset(&a, 0, sizeof(a));
    a.sdf_g = ctx->sdf_g;
    a.nrm_g = ctx->nrm_g;
    a.env_g = ctx->env_g;
    a.sdf = ctx->d_sdf;
    a.nrange = ctx->d_nrange;
    a.nent = ctx->d_nent;
    a.oob = ctx->oob;
    a.has_normals = ctx->has_normals;
    a.R = ctx->R;
    a.S = ctx->params;
    /* SPCS:1403-1404 thresholds, SPCS:923 tolerance */
    a.thr_env = (inflation_ratio * ctx->env_g.res) - (ctx->params.environment_collision_check_tolerance * ctx->sdf_g.res);
    a.self_res = (inflation_ratio + 1.0) * ctx->env_g.res;
    a.starts = d_configs;
    a.n = n;
    a.out_collided = d_out_collided;
    a.out_err = d_out_error_flags;
    a.counters = ctx->d_counters;
    a.queue = ctx->d_counters + fksd::kNumCounters;
    a.scratch = ctx->d_scratch;
    a.scratch_per_wave = ctx->scratch_per_wave;
    a.row_cap = 3u * (uint32_t)ctx->R.P;
    a.L = fksd::make_lds_layout(ctx->R.L, ctx->R.J, ctx->R.D, ctx->R.W, ctx->R.G, ctx->R.nrounds, ctx->fk_pair, ctx->lean);
    a.SL = fksd::make_scratch_layout(a.row_cap, ctx->R.D, ctx->R.P, ctx->R.G);
    *ctx->h_args = a;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_args, ctx->h_args, sizeof(a), hipMemcpyHostToDevice, s));
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, fksd::kCounterWords * sizeof(unsigned long long), s));
    const uint64_t groups_needed = (n + ctx->waves_per_group - 1) / ctx->waves_per_group;
    const uint32_t grid = (uint32_t)((groups_needed < (uint64_t)ctx->grid_groups) ? groups_needed : ctx->grid_groups);
    /* a batch larger than the resident grid runs the robot's shape-specialised check (built
     * here if the simulation has not built the module yet; a failure keeps the generic one) */
    if (ctx->spec_pending && n > (uint64_t)ctx->grid_waves) {
        ctx->spec_pending = false;
        const std::string keep = ctx->last_error;
        if (spec_prepare(ctx) != FKS_OK) ctx->last_error = keep + (keep.empty() ? "" : "; ") + ctx->last_error;
        HIP_TRY(ctx, hipSetDevice(ctx->device));
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev0, s));
    if (ctx->spec_check_fn) {
        const fksd::SimArgs* argp = ctx->d_args;
        void* params[] = {&argp};
        HIP_TRY(ctx, hipModuleLaunchKernel(ctx->spec_check_fn, grid, 1, 1, 64 * ctx->waves_per_group, 1, 1, (unsigned)ctx->lds_bytes,
                                           s, params, nullptr));
        ctx->last_check_kernel = FKS_KERNEL_SHAPED;
    } else {
        hipLaunchKernelGGL(check_kernel_for(ctx->R.type), dim3(grid), dim3(64 * ctx->waves_per_group), ctx->lds_bytes, s,
                           static_cast<const fksd::SimArgs*>(ctx->d_args));
        ctx->last_check_kernel = FKS_KERNEL_THROUGHPUT;
    }
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipEventRecord(ctx->ev1, s));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_counters, ctx->d_counters, fksd::kCounterWords * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, s));
    ctx->pending = true;
    ctx->pending_kind = 1;
    ctx->pending_stream = s;
    if (synchronize) return settle(ctx);
    return FKS_OK;
}

fks_status fks_check_config_collision(fks_context* ctx, const double* configs, uint64_t n, double inflation_ratio,
                                      uint8_t* out_collided, uint32_t* out_error_flags) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (n > 0 && (!configs || !out_collided)) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null host buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    const size_t W = (size_t)ctx->R.W;
    if (n > ctx->cap_particles) {
        HIP_TRY(ctx, ensure(&ctx->d_starts, n * W));
        HIP_TRY(ctx, ensure(&ctx->d_out, n * W));
        HIP_TRY(ctx, ensure(&ctx->d_coll, n));
        HIP_TRY(ctx, ensure(&ctx->d_micro, n));
        HIP_TRY(ctx, ensure(&ctx->d_res, n));
        HIP_TRY(ctx, ensure(&ctx->d_err, n));
        ctx->cap_particles = n;
    }
    if (n == 0) return fks_check_config_collision_device(ctx, nullptr, 0, inflation_ratio, nullptr, nullptr, nullptr, 1);
    HIP_TRY(ctx, hipMemcpy(ctx->d_starts, configs, n * W * sizeof(double), hipMemcpyHostToDevice));
    st = fks_check_config_collision_device(ctx, ctx->d_starts, n, inflation_ratio, ctx->d_coll, ctx->d_err, nullptr, 1);
    if (st != FKS_OK) return st;
    HIP_TRY(ctx, hipMemcpy(out_collided, ctx->d_coll, n, hipMemcpyDeviceToHost));
    if (out_error_flags) HIP_TRY(ctx, hipMemcpy(out_error_flags, ctx->d_err, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    ctx->check_last.call_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ctx->call_start).count();
    return FKS_OK;
}

fks_status fks_get_last_check_counters(const fks_context* ctx, fks_call_counters* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(const_cast<fks_context*>(ctx));
    if (st != FKS_OK) return st;
    *out = ctx->check_last;
    return FKS_OK;
}

static fks_status simulate_host(fks_context* ctx, const double* starts, uint64_t n, const double* targets, uint64_t num_targets,
                                int32_t allow_contacts, double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                uint32_t* out_resolver_iterations, uint32_t* out_error_flags, const TraceDev* tr = nullptr,
                                double* controller_state = nullptr) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (n > 0 && (!starts || !targets || !out_positions)) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null host buffer");
    if (n > 0 && num_targets != 1 && num_targets != n)
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "targets must be 1 or n (SPCS:792)");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    const size_t W = (size_t)ctx->R.W;
    if (n > ctx->cap_particles) {
        HIP_TRY(ctx, ensure(&ctx->d_starts, n * W));
        HIP_TRY(ctx, ensure(&ctx->d_out, n * W));
        HIP_TRY(ctx, ensure(&ctx->d_coll, n));
        HIP_TRY(ctx, ensure(&ctx->d_micro, n));
        HIP_TRY(ctx, ensure(&ctx->d_res, n));
        HIP_TRY(ctx, ensure(&ctx->d_err, n));
        ctx->cap_particles = n;
    }
    const uint64_t nt = (n > 0) ? num_targets : 0;
    if (nt > ctx->cap_targets || !ctx->d_targets) {
        HIP_TRY(ctx, ensure(&ctx->d_targets, (nt > 0 ? nt : 1) * W));
        ctx->cap_targets = nt > 0 ? nt : 1;
    }
    if (n == 0) {
        ctx->call_index++;
        std::memset(&ctx->last, 0, sizeof(ctx->last));
        return FKS_OK;
    }
    HIP_TRY(ctx, hipMemcpy(ctx->d_starts, starts, n * W * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_targets, targets, nt * W * sizeof(double), hipMemcpyHostToDevice));
    const size_t pid_words = (size_t)n * 2u * (size_t)ctx->R.D;
    if (controller_state) {
        if (pid_words > ctx->cap_pid) {
            HIP_TRY(ctx, ensure(&ctx->d_pid, pid_words));
            ctx->cap_pid = pid_words;
        }
        HIP_TRY(ctx, hipMemcpy(ctx->d_pid, controller_state, pid_words * sizeof(double), hipMemcpyHostToDevice));
    }
    st = simulate_device(ctx, ctx->d_starts, n, ctx->d_targets, nt, 0, allow_contacts, ctx->d_out, ctx->d_coll, ctx->d_micro,
                         ctx->d_res, ctx->d_err, nullptr, 1, tr, controller_state ? ctx->d_pid : nullptr);
    if (st != FKS_OK) return st;
    if (controller_state)
        HIP_TRY(ctx, hipMemcpy(controller_state, ctx->d_pid, pid_words * sizeof(double), hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(out_positions, ctx->d_out, n * W * sizeof(double), hipMemcpyDeviceToHost));
    if (out_collided) HIP_TRY(ctx, hipMemcpy(out_collided, ctx->d_coll, n, hipMemcpyDeviceToHost));
    if (out_microsteps) HIP_TRY(ctx, hipMemcpy(out_microsteps, ctx->d_micro, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (out_resolver_iterations)
        HIP_TRY(ctx, hipMemcpy(out_resolver_iterations, ctx->d_res, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (out_error_flags) HIP_TRY(ctx, hipMemcpy(out_error_flags, ctx->d_err, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    ctx->last.call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ctx->call_start).count();
    return FKS_OK;
}

fks_status fks_forward_simulate(fks_context* ctx, const double* starts, uint64_t n, const double* targets, uint64_t num_targets,
                                int32_t allow_contacts, double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                uint32_t* out_resolver_iterations, uint32_t* out_error_flags) {
    return simulate_host(ctx, starts, n, targets, num_targets, allow_contacts, out_positions, out_collided, out_microsteps,
                         out_resolver_iterations, out_error_flags);
}

/* ReverseSimulateRobots: ReverseSimulateMutableRobot == ForwardSimulateMutableRobot (SPCS:838-841) */
fks_status fks_reverse_simulate(fks_context* ctx, const double* starts, uint64_t n, const double* targets, uint64_t num_targets,
                                int32_t allow_contacts, double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                uint32_t* out_resolver_iterations, uint32_t* out_error_flags) {
    return simulate_host(ctx, starts, n, targets, num_targets, allow_contacts, out_positions, out_collided, out_microsteps,
                         out_resolver_iterations, out_error_flags);
}

/* ForwardSimulateMutableRobot (SPCS:843-919) over a batch of robots that keep their controllers */
fks_status fks_forward_simulate_mutable(fks_context* ctx, const double* starts, uint64_t n, const double* targets,
                                        uint64_t num_targets, int32_t allow_contacts, double* controller_state,
                                        double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                        uint32_t* out_resolver_iterations, uint32_t* out_error_flags) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (n > 0 && !controller_state) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null controller state");
    return simulate_host(ctx, starts, n, targets, num_targets, allow_contacts, out_positions, out_collided, out_microsteps,
                         out_resolver_iterations, out_error_flags, nullptr, controller_state);
}

}  // extern "C"

/* the traced calls: device trace buffers around simulate_host, copied to the caller's */
static fks_status simulate_traced(fks_context* ctx, const double* starts, uint64_t n, const double* targets, uint64_t num_targets,
                                  int32_t allow_contacts, double* controller_state, double* out_positions, uint8_t* out_collided,
                                  uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                                  const fks_trace* trace) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (!trace || !trace->num_steps || !trace->num_configs ||
        (trace->step_capacity > 0 && (!trace->step_inputs || !trace->step_microsteps)) ||
        (trace->config_capacity > 0 && (!trace->configs || !trace->config_tags)))
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "incomplete fks_trace");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t D = (size_t)ctx->R.D, W = (size_t)ctx->R.W;
    const size_t ns = (size_t)n * trace->step_capacity, nc = (size_t)n * trace->config_capacity;
    TraceDev tr{};
    tr.step_cap = trace->step_capacity;
    tr.cfg_cap = trace->config_capacity;
    std::vector<void*> allocs;
    auto alloc = [&](void** p, size_t bytes) {
        hipError_t e = hipMalloc(p, bytes > 0 ? bytes : 8);
        if (e == hipSuccess) allocs.push_back(*p);
        /* records past a particle's count stay zero, as in the caller's view */
        if (e == hipSuccess) e = hipMemset(*p, 0, bytes > 0 ? bytes : 8);
        return e;
    };
    auto release = [&]() {
        for (void* p : allocs) (void)hipFree(p);
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = alloc((void**)&tr.inputs, ns * 2 * D * sizeof(double));
    if (e == hipSuccess) e = alloc((void**)&tr.micro, ns * sizeof(uint32_t));
    if (e == hipSuccess) e = alloc((void**)&tr.cfg, nc * W * sizeof(double));
    if (e == hipSuccess) e = alloc((void**)&tr.tags, nc * 3 * sizeof(uint32_t));
    if (e == hipSuccess) e = alloc((void**)&tr.nsteps, (size_t)n * sizeof(uint32_t));
    if (e == hipSuccess) e = alloc((void**)&tr.ncfg, (size_t)n * sizeof(uint32_t));
    if (e != hipSuccess) {
        release();
        return hip_fail(ctx, e, "trace buffers");
    }
    fks_status st = simulate_host(ctx, starts, n, targets, num_targets, allow_contacts, out_positions, out_collided,
                                  out_microsteps, out_resolver_iterations, out_error_flags, &tr, controller_state);
    if (st == FKS_OK && n > 0) {
        struct Copy {
            void* dst;
            const void* src;
            size_t bytes;
        } copies[] = {{trace->step_inputs, tr.inputs, ns * 2 * D * sizeof(double)},
                      {trace->step_microsteps, tr.micro, ns * sizeof(uint32_t)},
                      {trace->configs, tr.cfg, nc * W * sizeof(double)},
                      {trace->config_tags, tr.tags, nc * 3 * sizeof(uint32_t)},
                      {trace->num_steps, tr.nsteps, (size_t)n * sizeof(uint32_t)},
                      {trace->num_configs, tr.ncfg, (size_t)n * sizeof(uint32_t)}};
        for (const Copy& c : copies) {
            if (c.bytes == 0) continue;
            e = hipMemcpy(c.dst, c.src, c.bytes, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                st = hip_fail(ctx, e, "trace copy");
                break;
            }
        }
    }
    release();
    return st;
}

extern "C" {

/* ForwardSimulateRobot with enable_tracing = true (SPCS:824-829), batched */
fks_status fks_forward_simulate_traced(fks_context* ctx, const double* starts, uint64_t n, const double* targets,
                                       uint64_t num_targets, int32_t allow_contacts, double* out_positions,
                                       uint8_t* out_collided, uint32_t* out_microsteps, uint32_t* out_resolver_iterations,
                                       uint32_t* out_error_flags, const fks_trace* trace) {
    return simulate_traced(ctx, starts, n, targets, num_targets, allow_contacts, nullptr, out_positions, out_collided,
                           out_microsteps, out_resolver_iterations, out_error_flags, trace);
}

/* ForwardSimulateMutableRobot with enable_tracing = true (SPCS:843-919) */
fks_status fks_forward_simulate_traced_mutable(fks_context* ctx, const double* starts, uint64_t n, const double* targets,
                                               uint64_t num_targets, int32_t allow_contacts, double* controller_state,
                                               double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                               uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                                               const fks_trace* trace) {
    if (ctx && n > 0 && !controller_state) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null controller state");
    return simulate_traced(ctx, starts, n, targets, num_targets, allow_contacts, controller_state, out_positions, out_collided,
                           out_microsteps, out_resolver_iterations, out_error_flags, trace);
}

fks_status fks_robot_sizes(const fks_context* ctx, int32_t* num_links, int32_t* num_points, int32_t* num_dofs,
                           int32_t* config_width) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return FKS_ERR_NO_ROBOT;
    if (num_links) *num_links = ctx->R.L;
    if (num_points) *num_points = ctx->R.P;
    if (num_dofs) *num_dofs = ctx->R.D;
    if (config_width) *config_width = ctx->R.W;
    return FKS_OK;
}

/* FK / world points / clean control input of a batch (include/fks_capi.h) */
fks_status fks_kinematics(fks_context* ctx, int32_t mode, const double* configs, uint64_t n, const double* inputs,
                          double* out) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return fail(ctx, FKS_ERR_NO_ROBOT, "fks_set_robot has not been called");
    if (mode != FKS_KIN_LINK_TRANSFORMS && mode != FKS_KIN_POINTS && mode != FKS_KIN_APPLY_CONTROL_INPUT)
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "unknown kinematics mode");
    if (n > 0 && (!configs || !out || (mode == FKS_KIN_APPLY_CONTROL_INPUT && !inputs)))
        return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "null host buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    if (n == 0) return FKS_OK;
    const size_t W = (size_t)ctx->R.W, D = (size_t)ctx->R.D;
    const size_t per_out = (mode == FKS_KIN_LINK_TRANSFORMS) ? 12 * (size_t)ctx->R.L
                                                             : (mode == FKS_KIN_POINTS ? 3 * (size_t)ctx->R.P : W);
    double *d_cfg = nullptr, *d_in = nullptr, *d_out = nullptr;
    auto release = [&]() {
        if (d_cfg) (void)hipFree(d_cfg);
        if (d_in) (void)hipFree(d_in);
        if (d_out) (void)hipFree(d_out);
    };
    hipError_t e = dev_upload(&d_cfg, configs, (size_t)n * W);
    if (e == hipSuccess && mode == FKS_KIN_APPLY_CONTROL_INPUT) e = dev_upload(&d_in, inputs, (size_t)n * D);
    if (e == hipSuccess) e = hipMalloc((void**)&d_out, (size_t)n * per_out * sizeof(double));
    if (e != hipSuccess) {
        release();
        return hip_fail(ctx, e, "kinematics buffers");
    }
    fksd::SimArgs a;
    std::memset(&a, 0, sizeof(a));
    a.sdf_g = ctx->sdf_g;
    a.nrm_g = ctx->nrm_g;
    a.env_g = ctx->env_g;
    a.R = ctx->R;
    a.S = ctx->params;
    a.starts = d_cfg;
    a.targets = d_in;
    a.n = n;
    a.scratch = ctx->d_scratch;
    a.scratch_per_wave = ctx->scratch_per_wave;
    a.row_cap = 3u * (uint32_t)ctx->R.P;
    a.L = fksd::make_lds_layout(ctx->R.L, ctx->R.J, ctx->R.D, ctx->R.W, ctx->R.G, ctx->R.nrounds, ctx->fk_pair, ctx->lean);
    a.SL = fksd::make_scratch_layout(a.row_cap, ctx->R.D, ctx->R.P, ctx->R.G);
    a.kin_mode = mode;
    a.kin_out = d_out;
    *ctx->h_args = a;
    e = hipMemcpy(ctx->d_args, ctx->h_args, sizeof(a), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        const uint64_t groups_needed = (n + ctx->waves_per_group - 1) / ctx->waves_per_group;
        const uint32_t grid = (uint32_t)((groups_needed < (uint64_t)ctx->grid_groups) ? groups_needed : ctx->grid_groups);
        sim_kernel_t k = (ctx->R.type == FKS_ROBOT_SE2) ? fks_kinematics_se2
                                                        : (ctx->R.type == FKS_ROBOT_SE3 ? fks_kinematics_se3 : fks_kinematics_linked);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64 * ctx->waves_per_group), ctx->lds_bytes, nullptr,
                           static_cast<const fksd::SimArgs*>(ctx->d_args));
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, (size_t)n * per_out * sizeof(double), hipMemcpyDeviceToHost);
    release();
    if (e != hipSuccess) return hip_fail(ctx, e, "fks_kinematics");
    return FKS_OK;
}

fks_status fks_set_call_index(fks_context* ctx, uint64_t call_index) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->call_index = call_index;
    return FKS_OK;
}
uint64_t fks_get_call_index(const fks_context* ctx) { return ctx ? ctx->call_index : 0; }

fks_status fks_get_statistics(const fks_context* ctx, fks_statistics* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(const_cast<fks_context*>(ctx));
    if (st != FKS_OK) return st;
    *out = ctx->stats;
    return FKS_OK;
}
fks_status fks_reset_statistics(fks_context* ctx) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    std::memset(&ctx->stats, 0, sizeof(ctx->stats));
    return FKS_OK;
}
fks_status fks_set_statistics(fks_context* ctx, const fks_statistics* stats) {
    if (!ctx || !stats) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    ctx->stats = *stats;
    return FKS_OK;
}
fks_status fks_reset_generators(fks_context* ctx, uint64_t prng_seed) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->seed = prng_seed;
    ctx->call_index = 0;
    return FKS_OK;
}
int32_t fks_get_debug_level(const fks_context* ctx) { return ctx ? ctx->debug_level : 0; }
int32_t fks_set_debug_level(fks_context* ctx, int32_t debug_level) {
    if (!ctx) return 0;
    ctx->debug_level = debug_level;
    return ctx->debug_level;
}
fks_status fks_get_last_call_counters(const fks_context* ctx, fks_call_counters* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(const_cast<fks_context*>(ctx));
    if (st != FKS_OK) return st;
    *out = ctx->last;
    return FKS_OK;
}

fks_status fks_get_total_counters(const fks_context* ctx, fks_call_counters* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(const_cast<fks_context*>(ctx));
    if (st != FKS_OK) return st;
    *out = ctx->total;
    return FKS_OK;
}
fks_status fks_set_total_counters(fks_context* ctx, const fks_call_counters* totals) {
    if (!ctx || !totals) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    ctx->total = *totals;
    return FKS_OK;
}
fks_status fks_reset_total_counters(fks_context* ctx) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    std::memset(&ctx->total, 0, sizeof(ctx->total));
    std::memset(ctx->phase_total, 0, sizeof(ctx->phase_total));
    return FKS_OK;
}

fks_status fks_get_phase_cycles(const fks_context* ctx, int which, uint64_t* out) {
    if (!ctx || !out || (which != 0 && which != 1)) return FKS_ERR_INVALID_ARGUMENT;
    fks_status st = settle(const_cast<fks_context*>(ctx));
    if (st != FKS_OK) return st;
    std::memcpy(out, which ? ctx->phase_total : ctx->phase_last, sizeof(ctx->phase_last));
    return FKS_OK;
}

fks_status fks_set_segment_steps(fks_context* ctx, uint32_t controller_steps) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->segment_steps = controller_steps;
    return FKS_OK;
}

fks_status fks_set_small_batch_kernel(fks_context* ctx, int32_t enabled) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->small_batch = enabled ? 1 : 0;
    return FKS_OK;
}

fks_status fks_set_cooperative_waves(fks_context* ctx, int32_t enabled) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->cooperative = enabled ? 1 : 0;
    return FKS_OK;
}

fks_status fks_set_segment_heavy_relative(fks_context* ctx, uint32_t times_mean) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (times_mean > 64u) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "times_mean must be at most 64");
    ctx->heavy_relative = times_mean;
    return FKS_OK;
}

fks_status fks_set_segment_policy(fks_context* ctx, uint32_t heavy_resolver_per_step, uint32_t heavy_priority) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    if (heavy_resolver_per_step > 65536u) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "heavy_resolver_per_step > 65536");
    if (heavy_priority > 2u) return fail(ctx, FKS_ERR_INVALID_ARGUMENT, "heavy_priority must be 0, 1 or 2");
    ctx->heavy_per_step = heavy_resolver_per_step;
    ctx->heavy_priority = heavy_priority;
    return FKS_OK;
}

fks_status fks_set_individual_jacobians(fks_context* ctx, int32_t simulate_with_individual_jacobians) {
    if (!ctx) return FKS_ERR_INVALID_ARGUMENT;
    ctx->individual_jacobians = simulate_with_individual_jacobians ? 1 : 0;
    return FKS_OK;
}

fks_status fks_set_specialization(fks_context* ctx, int32_t mode) {
    if (!ctx || mode < FKS_SPECIALIZE_OFF || mode > FKS_SPECIALIZE_NO_PROOFS) return FKS_ERR_INVALID_ARGUMENT;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    fks_status st = settle(ctx);
    if (st != FKS_OK) return st;
    ctx->specialize = mode;
    ctx->spec_pending = false;
    return spec_prepare(ctx); /* now, for the current robot (releases it when disabled) */
}

fks_status fks_get_specialization(const fks_context* ctx, fks_specialization_info* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    out->enabled = ctx->specialize;
    out->active = ctx->spec_fn ? 1 : 0;
    out->pending = ctx->spec_pending ? 1 : 0;
    out->from_cache = ctx->spec_from_cache;
    out->compile_seconds = ctx->spec_seconds;
    out->launches = ctx->spec_launches;
    std::snprintf(out->shape, sizeof(out->shape), "%s", ctx->spec_shape.c_str());
    out->failed = ctx->spec_failed ? 1 : 0;
    std::snprintf(out->message, sizeof(out->message), "%s", ctx->spec_message.c_str());
    return FKS_OK;
}

fks_status fks_get_launch_geometry(const fks_context* ctx, uint32_t* resident_waves, uint64_t* lds_bytes_per_group) {
    if (!ctx || !resident_waves || !lds_bytes_per_group) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return FKS_ERR_NO_ROBOT;
    *resident_waves = ctx->grid_waves;
    *lds_bytes_per_group = (uint64_t)ctx->lds_bytes;
    return FKS_OK;
}

fks_status fks_get_launch_info(const fks_context* ctx, fks_launch_info* out) {
    if (!ctx || !out) return FKS_ERR_INVALID_ARGUMENT;
    if (!ctx->has_robot) return FKS_ERR_NO_ROBOT;
    std::memset(out, 0, sizeof(*out));
    out->resident_waves = ctx->grid_waves;
    out->waves_per_group = ctx->waves_per_group;
    out->lds_bytes_per_group = (uint64_t)ctx->lds_bytes;
    out->small_batch_resident_waves = ctx->small_grid_waves;
    out->standard_layout_resident_waves = ctx->standard_resident_waves;
    out->fk_pair = ctx->fk_pair ? 1 : 0;
    out->lean = ctx->lean ? 1 : 0;
    out->last_kernel = ctx->last_kernel;
    out->last_check_kernel = ctx->last_check_kernel;
    out->cooperative_resident_particles = ctx->coop_particles;
    out->cooperative_waves_per_particle = ctx->coop_waves;
    return FKS_OK;
}

fks_status fks_selftest_math(int32_t device, uint64_t n, uint64_t* out_mismatches) {
    if (!out_mismatches || n == 0 || n > (1ull << 26)) return FKS_ERR_INVALID_ARGUMENT;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return FKS_ERR_NO_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return FKS_ERR_HIP;
    std::vector<double> a(n), b(n), host(8 * n), dev(8 * n);
    uint64_t st = 0x1234567ull;
    for (uint64_t i = 0; i < n; ++i) {
        st = splitmix64(st);
        a[i] = ((double)(st >> 11) * (1.0 / 9007199254740992.0) - 0.5) * 40.0;
        st = splitmix64(st);
        b[i] = ((double)(st >> 11) * (1.0 / 9007199254740992.0) - 0.5) * std::pow(10.0, (double)((st & 15) - 6));
    }
    for (uint64_t i = 0; i < n; ++i) {
        const double x = a[i], y = b[i];
        host[8 * i + 0] = fks_math::sin(x);
        host[8 * i + 1] = fks_math::cos(x);
        host[8 * i + 2] = fks_math::log(fks_math::dabs(y) + 1e-300);
        host[8 * i + 3] = fks_math::atan2(x, y);
        host[8 * i + 4] = fks_math::dsqrt(fks_math::dabs(y));
        host[8 * i + 5] = x / y;
        host[8 * i + 6] = fks_math::enforce_continuous_revolute_bounds(x / y); /* glibc fmod vs the kernel's wrap */
        host[8 * i + 7] = (x * y + x) * y - x * x;
    }
    double *da = nullptr, *db = nullptr, *dout = nullptr;
    if (dev_upload(&da, a.data(), n) != hipSuccess || dev_upload(&db, b.data(), n) != hipSuccess ||
        hipMalloc((void**)&dout, 8 * n * sizeof(double)) != hipSuccess)
        return FKS_ERR_HIP;
    hipLaunchKernelGGL(fks_math_probe, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, da, db, dout, n);
    hipError_t e = hipMemcpy(dev.data(), dout, 8 * n * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    if (e != hipSuccess) return FKS_ERR_HIP;
    uint64_t mism = 0;
    for (uint64_t i = 0; i < 8 * n; ++i)
        if (std::memcmp(&host[i], &dev[i], sizeof(double)) != 0) mism++;
    *out_mismatches = mism;
    return FKS_OK;
}

}  // extern "C"
