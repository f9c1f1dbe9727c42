/*
 * Device-side data layout of the particle forward-simulation kernel (shared by
 * the host launcher fks_capi.cpp and the kernels in fks_kernels.hip).
 *
 * HBM layout (all resident for the life of a context / robot):
 *   SDF            float per cell in 4x4x4-cell bricks (brick_cell below): a cell's
 *                  7-point EstimateDistance4d stencil and the neighbouring points of a
 *                  link fall in one or two 128-B lines instead of the five or more of
 *                  the VoxelGrid's linear order (x neighbours nx*ny*4 bytes apart)
 *   normal grid    per cell (in the same bricks) the (begin, end) range of its entries,
 *                  6 doubles per entry in VoxelGrid cell order (the CSR of fks_environment)
 *   robot          JointDev[J], per-geometry tables, points as double4 (x,y,z,w)
 *                  in geometry-major order (the order of robot_link_geometries)
 *   per-wave scratch  least-squares matrix (column-major, 3P rows x (D+1) cols),
 *                  self-collision keys / corrections / flags
 * LDS layout (one wavefront per workgroup): see LdsLayout below.
 * The kernel reads SimArgs through a pointer to a device copy (scalar loads),
 * never from a private copy of the kernel argument.
 */
#ifndef FKS_DEVICE_H
#define FKS_DEVICE_H

#if !defined(__HIPCC_RTC__)
#include <stdint.h>
#endif

#include "fks_capi.h"
#include "fks_portable_math.h"

namespace fksd {

/* 4x4x4-cell bricks, bricks in VoxelGrid order (z fastest), cells inside a brick x-major
 * and z-fastest; nb = bricks per axis (ceil(n / 4)).  256 B of floats per brick (two
 * 128-B lines); cells past the grid's edge in the last bricks are padding, never read. */
constexpr int kBrickShift = 2;
constexpr int kBrickCells = 64;
FKS_HD inline uint32_t brick_cell(const uint32_t nb[3], uint32_t i, uint32_t j, uint32_t k) {
    const uint32_t brick = ((i >> kBrickShift) * nb[1] + (j >> kBrickShift)) * nb[2] + (k >> kBrickShift);
    return (brick << 6) | ((i & 3u) << 4) | ((j & 3u) << 2) | (k & 3u);
}
FKS_HD inline uint64_t brick_total(const uint32_t nb[3]) { return (uint64_t)nb[0] * nb[1] * nb[2] * kBrickCells; }

constexpr int kWave = 64;
constexpr int kMaxLinks = 64;
constexpr int kMaxDofs = 64;
constexpr int kMaxGeoms = 64;
constexpr int kMaxJoints = 64;

struct GridDev {
    double org[12]; /* origin transform, 3x4 row-major */
    double inv[12]; /* inverse origin */
    double res, inv_res;
    int64_t n[3];
    /* 1 / (res * d) for the gradient stencil widths d = 0, 1, 2 of EstimateDistance4d
     * (the same correctly rounded division, done once on the host) */
    double inv_res_span[3];
    uint32_t nb[3]; /* bricks per axis (brick_cell) */
    uint32_t nb_pad;
};

struct JointDev {
    int32_t parent, child, type, dof;
    double origin[12];
    double axis[3];
    double lo, hi;
};
constexpr int kJointWords = (int)(sizeof(JointDev) / 8); /* 19 */
static_assert(sizeof(JointDev) % 8 == 0, "JointDev is copied to LDS as 64-bit words");
constexpr int kCtrlWords = (int)(sizeof(fks_dof_controller) / 8); /* 9 */

/* a 64-point round of the lane-strided point loops: the link of all its points
 * (-1 if mixed or any w != 1: such rounds are never skipped), point count and the
 * largest |p_xyz| (link frame) for motion bounds */
struct RoundDev {
    int32_t link;
    int32_t npts;
    double radius;
};
/* per round in LDS: reference transform (12), min SDF value, min grid-bounds margin
 * (cells), min distance to a cell face (cells), spare */
constexpr int kRoundState = 16;
constexpr int kLdsPairs = 128; /* disallowed geometry pairs cached in LDS (the rest are read from HBM) */

/* one dof's SampledUncertainVelocityActuator tables (fks_sampled_actuator) */
struct SampledDev {
    uint32_t nbins, elems;
    const double* bounds;  /* 2 per bin */
    const double* samples; /* elems per bin */
};

struct RobotDev {
    int32_t type, L, J, G, D, P, W, npairs;
    int32_t self_possible;
    int32_t nrounds;
    double base[12];
    const JointDev* joints;
    const int32_t* geom_link;
    const uint32_t* geom_off;
    const double* points;      /* 4 per point */
    const uint16_t* point_geom;
    const uint16_t* point_link; /* link of each point's geometry (one load instead of two) */
    const int32_t* dof_joint;   /* linked: joint index of dof d */
    const uint64_t* link_dof_mask; /* per link: dofs whose joint child is an ancestor-or-self */
    const int32_t* pairs;       /* disallowed geometry pairs, 2 per pair (a < b) */
    const uint64_t* allowed_mask; /* per geometry: bit b set if self-collision with b allowed */
    const double* geom_box;     /* per geometry: local centre xyz, half extent xyz, all_w_one */
    const double* geom_mass;    /* per geometry: link mass + masses of all later geometries */
    const fks_dof_controller* ctrl;
    const double* weights;
    const RoundDev* rounds;
    /* per dof: a configuration-independent bound on how far any point moves per
     * unit of joint motion (distance to the joint axis; 1 for prismatic), +inf if
     * unknown.  Lets the microstep-motion check of SPCS:1570-1575 be proven instead
     * of recomputed. */
    const double* dof_lever;
    /* the same for every point of the geometries' local boxes (their corners reach past the
     * points): bounds how far a self-collision box moves (the self-collision skip proof) */
    const double* dof_lever_box;
    /* dofs whose actuator is a SampledUncertainVelocityActuator (bit d), their tables */
    uint64_t sampled_mask;
    const SampledDev* sampled;
};

/* LDS carve-out (in doubles), identical on host and device.  A workgroup holds
 * kWavesPerGroup waves, one particle each (2 or 1 for robots whose blocks do not fit
 * four times in the 160 KiB of a CU, fks_set_robot).  The robot tables (joints ... gpairs) are
 * one shared copy at the start of the workgroup's LDS (offsets relative to it,
 * `shared_total` doubles); every other offset is relative to the wave's own block of
 * `total` doubles that follows. */
constexpr int kWavesPerGroup = 4;
/* an LDS-bound robot may run a lean block (its round skip-proof cache in the wave's scratch,
 * fks_simulate_*_lean kernels) at up to 8 waves per workgroup */
constexpr int kMaxWavesPerGroup = 8;
/* the throughput kernels' register budget: amdgpu_waves_per_eu(FKS_WAVES_PER_EU) in
 * fks_kernels.hip, 5 waves per SIMD = 96 VGPRs */
constexpr int kThroughputWavesPerEU = 5;
/* cooperative small batches (fks_simulate_<family>_coop, fks_set_cooperative_waves): one
 * particle per workgroup of kCoopWaves waves that share its point loops through a CoopBox
 * behind the leader's LDS block; robots of up to kCoopMaxRounds 64-point rounds */
constexpr int kCoopWaves = 8;
constexpr int kMaxCoopWaves = 8;
constexpr int kCoopMaxRounds = 16;
struct CoopBox {
    uint32_t cmd;
    uint32_t self_nonempty;
    uint32_t tc_off, tp_off, cfg_off; /* offsets (doubles) into the leader's LDS block */
    uint32_t pad;
    uint64_t work;                    /* the rounds handed out (bit r), taken in rank order */
    uint64_t skip;                    /* corrections: the proven rounds (collect_corrections' skip mask) */
    uint64_t cmask;                   /* environment: the rounds holding a colliding point */
    uint32_t cnt[kCoopMaxRounds];     /* environment: a round's bytes as the sequential loop counts them;
                                         corrections: its row count */
    uint32_t err[kMaxCoopWaves];      /* corrections: each helper's error bits */
    uint64_t selfk[kMaxCoopWaves];    /* corrections: each helper's self-corrected points */
};
constexpr uint32_t kCoopBoxDoubles = (uint32_t)((sizeof(CoopBox) + 7) / 8);
struct LdsLayout {
    uint32_t joints, ctrl, base, dofj, gbox, gpairs, rounds, shared_total;
    uint32_t rstate, noise, noise_err, Tcur, Tprev, Ttmp, jm, cfg, cfg_work, cfg_res, cfg_prev, cfg_tmp, cfg_act, tgt, u,
        ustep, x, real, axis_w, orig_w, colsq, hcoef, box, misc, ints, selfref, jm2, total;
    uint32_t fk_pair; /* 1: the free-motion microsteps pair their FK chains (jm2 allocated) */
    uint32_t lean;    /* 1: no rstate here: the skip-proof cache is ScratchLayout.rstate (lean kernels) */
};

constexpr inline
#if defined(__HIPCC__)
    __host__ __device__
#endif
    LdsLayout make_lds_layout(int L, int J, int D, int W, int G, int NR, bool fk_pair = false, bool lean = false) {
    LdsLayout l{};
    uint32_t o = 0;
    /* shared: the robot tables the hot loops read (filled once per workgroup) */
    l.joints = o;
    o += (uint32_t)kJointWords * (J > 0 ? J : 1);
    l.ctrl = o;
    o += (uint32_t)kCtrlWords * (D > 0 ? D : 1);
    l.base = o;
    o += 12;
    l.dofj = o; /* int32 per dof */
    o += (uint32_t)(D + 1) / 2;
    l.gbox = o; /* per geometry: local box (7) + link */
    o += 8u * (G > 0 ? G : 1);
    l.gpairs = o; /* first kLdsPairs disallowed pairs, a | b << 16 */
    o += (uint32_t)kLdsPairs / 2;
    o = (o + 1u) & ~1u;
    l.rounds = o; /* per 64-point round r < 64: (double)link, radius (RoundDev) */
    o += 2u * (uint32_t)(NR < 1 ? 1 : (NR > 64 ? 64 : NR));
    l.shared_total = o;
    /* per wave */
    o = 0;
    /* kRoundState per round r < 64 (the 64-bit skip masks), persists across the wave's
     * particles; a lean block keeps it in the wave's scratch instead (ScratchLayout.rstate) */
    l.lean = lean ? 1u : 0u;
    l.rstate = o;
    if (!lean) o += (uint32_t)kRoundState * (uint32_t)(NR < 1 ? 1 : (NR > 64 ? 64 : NR));
    l.noise = o; /* actuator noise samples of the next floor(64/D) microsteps, [micro][dof] */
    o += 64;
    l.noise_err = o; /* their error bits, 64 x u32 */
    o += 32;
    l.Tcur = o;
    o += 12u * L;
    l.Tprev = o;
    o += 12u * L;
    l.Ttmp = o;
    o += 12u * L;
    /* one region, two lifetimes: the joint motion matrices live only inside fk(); the
     * world joint frames (Jacobian), QR column norms / Householder coefficients and the
     * self-collision boxes only between fk() calls */
    {
        const uint32_t motion = 12u * (uint32_t)(J > 0 ? J : 1);
        const uint32_t boxes = 6u * (uint32_t)(G > 0 ? G : 1);
        const uint32_t others = 8u * (uint32_t)D + boxes;
        l.jm = o;
        l.axis_w = o;
        l.orig_w = o + 3u * D;
        l.colsq = o + 6u * D;
        l.hcoef = o + 7u * D;
        l.box = o + 8u * D;
        o += (motion > others) ? motion : others;
    }
    l.cfg = o;
    o += W;
    l.cfg_work = o;
    o += W;
    l.cfg_res = o;
    o += W;
    l.tgt = o;
    o += W;
    l.cfg_prev = o;
    o += W;
    l.cfg_tmp = o;
    o += W;
    l.cfg_act = o;
    o += W;
    l.u = o;
    o += D;
    l.ustep = o;
    o += D;
    l.x = o;
    o += D;
    l.real = o;
    o += D;
    l.misc = o; /* tw[6], phase sums, stats, self counters, hand-over words, wave totals */
    o += 40;
    l.ints = o; /* int32 region: perm[64], transpositions[64], 16 spare words */
    o += (2 * kMaxDofs + 16) / 2;
    /* the self-collision skip proof's reference: the configuration of the last full box
     * evaluation [D] and the boxes' smallest gap then (cells) [D]; a lean block keeps it in
     * the wave's scratch (ScratchLayout.selfref) */
    l.selfref = o;
    if (!lean) o += (uint32_t)(D + 2) & ~1u;
    /* the second FK chain's joint motion matrices (paired FK of the next free microstep) */
    l.fk_pair = fk_pair ? 1u : 0u;
    l.jm2 = o;
    if (fk_pair) o += 12u * (uint32_t)(J > 0 ? J : 1);
    o = (o + 1u) & ~1u; /* 16-byte alignment */
    l.total = o;
    return l;
}

/* dense workspace (doubles) of the self-collision impulse solve of one cell
 * (ExtractSelfCollidingPoints SPCS:1054-1150) when a link may touch up to n = G - 1
 * others: C, N, M, V, N^T, C^T, M^-1, two products, the Gauss-Jordan tableau (2 rows^2),
 * A^-1, impulses and dv, rows = 3 (n + 1).  The reference's maps are unbounded; so is
 * this (it is sized by the robot, not capped). */
constexpr inline
#if defined(__HIPCC__)
    __host__ __device__
#endif
    uint64_t self_dense_words(int G) {
    const uint64_t n = (uint64_t)(G > 1 ? G - 1 : 1), rows = 3 * (n + 1), cc = 3 * n;
    return 2 * rows * cc + 2 * cc * n + 6 * rows * rows + 2 * rows + n * n + n + 64;
}

/* per-wave scratch layout (doubles) */
struct ScratchLayout {
    uint64_t J, b, keys, corr, flag, cand, list, cellw, dense, rstate, pid, selfref, total;
};
constexpr inline
#if defined(__HIPCC__)
    __host__ __device__
#endif
    ScratchLayout make_scratch_layout(uint32_t row_cap, int D, int P, int G) {
    ScratchLayout l{};
    uint64_t o = 0;
    l.J = o;
    o += (uint64_t)row_cap * (uint64_t)(D > 0 ? D : 1);
    l.b = o;
    o += row_cap;
    l.keys = o;
    o += 3ull * (uint64_t)P;
    l.corr = o;
    o += 3ull * (uint64_t)P;
    l.flag = o;
    o += (uint64_t)P;
    l.cand = o;
    o += (uint64_t)P;
    l.list = o;
    o += (uint64_t)P;
    l.cellw = o; /* ExtractSelfCollidingPoints tables: 4 x kMaxGeoms int32, kMaxGeoms momenta (D4) */
    o += 2u * kMaxGeoms + 4u * kMaxGeoms;
    l.dense = o;
    o += (G > 1) ? self_dense_words(G) : 8;
    l.rstate = o; /* the round skip-proof cache of a lean LDS block (kRoundState per round r < 64) */
    o += (uint64_t)kRoundState * 64u;
    l.pid = o; /* the particle's controller state: error integral [dof], last error [64 + dof] */
    o += 2u * 64u;
    l.selfref = o; /* a lean block's self-collision proof reference (LdsLayout.selfref) */
    o += 66u;
    l.total = (o + 7) & ~7ull;
    return l;
}

struct SimArgs {
    GridDev sdf_g, nrm_g, env_g;
    const float* sdf;     /* bricked (brick_cell over sdf_g) */
    const uint2* nrange;  /* bricked (brick_cell over nrm_g): [begin, end) of the cell's entries */
    const double* nent;
    float oob;
    int32_t has_normals;
    /* provably-free rounds may skip their SDF reads when the SDF
     * satisfies: axis neighbours with positive values differ by <= lplus*res, and
     * positive cells next to a non-positive one are <= cmax*res */
    int32_t skip_enabled;
    int32_t skip_pad;
    double skip_lplus, skip_cmax;
    RobotDev R;
    fks_solver_params S;
    double dt;               /* simulation_controller_interval_ = 1/frequency  (SPCS:427)   */
    double thr_env;          /* 0 - tolerance * sdf resolution (SPCS:923, threshold 0 SPCS:424) */
    double target_micro;     /* GetResolution() * 0.125 (SPCS:1560) */
    double allowed_micro;    /* GetResolution() * 1.0   (SPCS:1561) */
    double time_multiplier;  /* 1.0 / time_interval     (SPCS:1027) */
    uint32_t T;              /* forward simulation steps (SPCS:856) */
    uint32_t key0, key1;
    uint32_t pad0;
    const double* starts;
    const double* targets;
    uint64_t num_targets;
    uint64_t n;
    uint64_t first_pid;
    int32_t allow_contacts;
    int32_t individual_jacobians; /* ComputeResolverCorrectionStepIndividualJacobians (SPCS:1966-1988) */
    double* out_q;
    /* ForwardSimulateMutableRobot (fks_forward_simulate_mutable): per particle 2D doubles,
     * the PID error integrals then last errors the particle starts with, overwritten
     * with its controllers' state when it stops; NULL = ResetPosition (zeroed PIDs) */
    double* pid_io;
    uint8_t* out_collided;
    uint32_t* out_micro;
    uint32_t* out_resolver;
    uint32_t* out_err;
    unsigned long long* counters; /* kCounter* */
    unsigned long long* queue;     /* ticket counter: ticket t = segment t / n of particle t % n */
    /* controller-step segments (processor sharing across the persistent grid): a
     * particle's steps [k*seg_steps, (k+1)*seg_steps) form segment k; between
     * segments its state rests in seg_state (PID integral / last error per DOF,
     * flags, per-particle counters, its round skip-proof cache; the configuration
     * in out_q) and seg_done[p]
     * counts its finished segments (nseg once the particle has ended; the top bit
     * marks a segment claimed by a wave) */
    double* seg_state;
    uint32_t* seg_done;
    uint32_t seg_steps, nseg;
    uint32_t seg_stride;          /* doubles per particle in seg_state */
    uint32_t seg_heavy_resolver;  /* resolver iterations that mark a segment contact-heavy (0: off) */
    uint32_t seg_heavy_prio;      /* waves carrying a heavy particle raise their issue priority */
    uint32_t seg_heavy_rel;       /* ... and, when nonzero, at least this many times the batch's mean resolver
                                   * iterations per segment so far (the running sums in counters[kSchedWord]:
                                   * 40 bits of iterations over 24 bits of segments) */
    double* scratch;
    uint64_t scratch_per_wave; /* doubles */
    uint32_t row_cap;          /* 3 * P */
    uint32_t pad2;
    LdsLayout L;               /* per-wave LDS carve-out */
    ScratchLayout SL;          /* per-wave scratch carve-out */
    double self_res;           /* batched CheckConfigCollision: extended-cell size (SPCS:1404) */
    /* ForwardSimulationStepTrace buffers of the traced kernels (fks_trace) */
    double* tr_inputs;
    uint32_t* tr_micro;
    double* tr_cfg;
    uint32_t* tr_tags;
    uint32_t* tr_nsteps;
    uint32_t* tr_ncfg;
    uint32_t tr_step_cap, tr_cfg_cap;
    /* fks_kinematics: FKS_KIN_* mode, per-configuration inputs (targets) and output */
    int32_t kin_mode;
    int32_t kin_pad;
    double* kin_out;
};

enum {
    kCntSuccessful = 0,
    kCntUnsuccessful,
    kCntFree,
    kCntCollision,
    kCntFallback,
    kCntUnsuccessfulEnv,
    kCntUnsuccessfulSelf,
    kCntRecovered,
    kCntSteps,
    kCntMicrosteps,
    kCntResolver,
    kCntSdfBytes,
    kCntErrorParticles,
    kCntLsqRows,
    kCntSelfChecks,
    kCntSelfPoints,
    kNumCounters = 16
};

/* per-phase s_memtime cycle sums (lane 0 of every wave), after the counters and the
 * particle queue in the counter buffer; order = FKS_PHASE_* in fks_capi.h */
enum {
    kPhaseBase = kNumCounters + 2,
    /* the running sums of the relative heavy-segment test (SimArgs.seg_heavy_rel), on a cache line
     * of their own (not the ticket counter's) */
    kSchedWord = ((kPhaseBase + FKS_NUM_PHASES + 15) / 16) * 16,
    kCounterWords = kSchedWord + 1
};

}  // namespace fksd

#endif
