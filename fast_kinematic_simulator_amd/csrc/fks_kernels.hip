/*
 * fks_kernels.hip — the particle forward-simulation hot path on CDNA4 (gfx950).
 *
 * One 64-lane wavefront simulates one particle at a time (workgroup = 1 wave,
 * persistent grid, atomic particle queue for load balance across contact-heavy
 * and free particles).  Inside a wave:
 *   - DOF lanes (lane d < D): PID state, actuator clamp, truncated-normal
 *     actuation noise (Philox4x32-10 counter RNG), joint-limit enforcement
 *     (TNUVA:538-614, PID:122-135, UNC:70-90);
 *   - FK: lane j < J builds joint j's motion matrix; the chain
 *     T_child = (T_parent * origin_j) * motion_j is composed by 12 lanes, one
 *     3x4 element each, link transforms kept in LDS (UpdateTransforms of the
 *     arc_utilities linked model);
 *   - link points are lane-strided (point i -> lane i % 64) for the SDF
 *     collision check (SPCS:921-981), workspace-motion maxima (SPCS:1492-1544),
 *     the per-point Jacobians / corrections (SPCS:1818-1939);
 *   - the stacked least-squares solve (Eigen ColPivHouseholderQR, SPCS:1990-1998)
 *     keeps rows lane-strided and reduces with a 64-lane xor butterfly — the
 *     canonical summation order the CPU oracle reproduces bit for bit;
 *   - self-collision (SPCS:1183-1275): per-geometry conservative cell-key boxes
 *     (one lane per geometry) reject disallowed pairs; only overlapping pairs run
 *     the exact key comparison, and true self-contacts run the impulse solve
 *     (SPCS:983-1171) on one lane;
 * All double arithmetic is IEEE (no contraction: built with -ffp-contract=off),
 * transcendentals come from include/fks_portable_math.h, so results are
 * bit-identical to the CPU oracle on the same inputs.
 */
#if !defined(__HIPCC_RTC__) /* hiprtc (fks_specialize) brings the HIP device API and the integer types itself */
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "fks_capi.h"
#include "fks_control.h"
#include "fks_device.h"
#include "fks_portable_math.h"
#include "fks_se3.h"

namespace fksd {

using fks_math::clamp;
using fks_math::dabs;
using fks_math::dmax;
using fks_math::dmin;
using fks_math::dsqrt;

/* ---------------- robot shape ----------------
 * The generic kernels read the robot's dimensions and the LDS / scratch carve-outs from
 * SimArgs at run time.  A shape-specialised build (FKS_SHAPE_L defined: fks_specialize.cpp
 * compiles this file at run time for one robot shape) fixes the carve-outs and the link,
 * joint, dof, width and geometry counts at compile time: every carve-out offset becomes an
 * instruction immediate, every per-dof / per-joint loop a fixed trip count, and the kernel
 * keeps far fewer wave-uniform values live in SGPRs (the SGPR spills of the generic kernel
 * cost one VALU lane read each).  The point, round and pair counts stay run-time values:
 * unrolling the point loops made the kernel larger and slower.  Same expression trees,
 * same results, bit for bit. */
#if defined(FKS_SHAPE_L)
struct RobotShape {
    int L, J, D, W, G;
};
constexpr RobotShape kShape{FKS_SHAPE_L, FKS_SHAPE_J, FKS_SHAPE_D, FKS_SHAPE_W, FKS_SHAPE_G};
constexpr LdsLayout kShapeLayout = make_lds_layout(FKS_SHAPE_L, FKS_SHAPE_J, FKS_SHAPE_D, FKS_SHAPE_W, FKS_SHAPE_G,
                                                   (FKS_SHAPE_P + 63) / 64, FKS_SHAPE_PAIR != 0, FKS_SHAPE_LEAN != 0);
constexpr ScratchLayout kShapeScratch = make_scratch_layout(3u * FKS_SHAPE_P, FKS_SHAPE_D, FKS_SHAPE_P, FKS_SHAPE_G);
#define RDIM(r, f) FKS_RDIM_##f(r)
#define FKS_RDIM_L(r) (::fksd::kShape.L)
#define FKS_RDIM_J(r) (::fksd::kShape.J)
#define FKS_RDIM_D(r) (::fksd::kShape.D)
#define FKS_RDIM_W(r) (::fksd::kShape.W)
#define FKS_RDIM_G(r) (::fksd::kShape.G)
#define FKS_RDIM_P(r) ((r).P)
#define FKS_RDIM_nrounds(r) ((r).nrounds)
#define FKS_RDIM_npairs(r) ((r).npairs)
#define FKS_RDIM_self_possible(r) ((r).self_possible)
#define LAY(a) (::fksd::kShapeLayout)
#define SLAY(a) (::fksd::kShapeScratch)
#define ROWCAP(a) (3u * (uint32_t)FKS_SHAPE_P)
/* with the per-dof / per-joint loops unrolled, the functions that take the wave's Sim state
 * grow past the inliner's threshold; an out-of-line one would put Sim in memory and turn
 * every LDS access into a flat one and every argument read into a vector load */
#define FKS_SHAPE_INLINE __forceinline__
#else
#define FKS_SHAPE_INLINE
#define RDIM(r, f) ((r).f)
#define LAY(a) ((a).L)
#define SLAY(a) ((a).SL)
#define ROWCAP(a) ((a).row_cap)
#endif

struct D3 {
    double x, y, z;
};
struct D4 {
    double x, y, z, w;
};

/* ---------------- geometry (same evaluation order as oracle_geometry.h) ---------------- */
__device__ __forceinline__ double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
    return (a0 * b0 + a1 * b1) + a2 * b2;
}
__device__ __forceinline__ D4 xform4(const double* T, const D4& p) {
    D4 o;
    o.x = dot3(T[0], T[1], T[2], p.x, p.y, p.z) + T[3] * p.w;
    o.y = dot3(T[4], T[5], T[6], p.x, p.y, p.z) + T[7] * p.w;
    o.z = dot3(T[8], T[9], T[10], p.x, p.y, p.z) + T[11] * p.w;
    o.w = p.w;
    return o;
}
__device__ __forceinline__ D3 xform3(const double* T, const D3& p) {
    D3 o;
    o.x = dot3(T[0], T[1], T[2], p.x, p.y, p.z) + T[3];
    o.y = dot3(T[4], T[5], T[6], p.x, p.y, p.z) + T[7];
    o.z = dot3(T[8], T[9], T[10], p.x, p.y, p.z) + T[11];
    return o;
}
__device__ __forceinline__ D3 rotate(const double* T, const D3& v) {
    D3 o;
    o.x = dot3(T[0], T[1], T[2], v.x, v.y, v.z);
    o.y = dot3(T[4], T[5], T[6], v.x, v.y, v.z);
    o.z = dot3(T[8], T[9], T[10], v.x, v.y, v.z);
    return o;
}
__device__ __forceinline__ D3 cross(const D3& a, const D3& b) {
    D3 c;
    c.x = a.y * b.z - a.z * b.y;
    c.y = a.z * b.x - a.x * b.z;
    c.z = a.x * b.y - a.y * b.x;
    return c;
}
/* Eigen Vector4d squaredNorm / norm / dot reduce two-lane packets: (x + z) + (y + w)
 * (SSE2 Packet2d, the reference's -O3 x86-64 build).  Vector3d
 * reductions are sequential. */
__device__ __forceinline__ double sqnorm4(const D4& v) { return (v.x * v.x + v.z * v.z) + (v.y * v.y + v.w * v.w); }
__device__ __forceinline__ double sqnorm3(const D3& v) { return (v.x * v.x + v.y * v.y) + v.z * v.z; }
__device__ __forceinline__ D4 safe_normal4(const D4& v) {
    const double n = dsqrt(sqnorm4(v));
    if (n > 2.220446049250313e-16) return D4{v.x / n, v.y / n, v.z / n, v.w / n};
    return v;
}
__device__ __forceinline__ D3 safe_normal3(const D3& v) {
    const double n = dsqrt(sqnorm3(v));
    if (n > 2.220446049250313e-16) return D3{v.x / n, v.y / n, v.z / n};
    return v;
}
/* Eigen::AngleAxisd::toRotationMatrix into a 3x4 (translation untouched) */
__device__ __forceinline__ void angle_axis34(double angle, double a0, double a1, double a2, double* M) {
    double s, c;
    fks_math::sincos(angle, &s, &c);
    const double sa0 = s * a0, sa1 = s * a1, sa2 = s * a2;
    const double omc = 1.0 - c;
    const double c1a0 = omc * a0, c1a1 = omc * a1, c1a2 = omc * a2;
    double tmp = c1a0 * a1;
    M[1] = tmp - sa2;
    M[4] = tmp + sa2;
    tmp = c1a0 * a2;
    M[2] = tmp + sa1;
    M[8] = tmp - sa1;
    tmp = c1a1 * a2;
    M[6] = tmp - sa0;
    M[9] = tmp + sa0;
    M[0] = c1a0 * a0 + c;
    M[5] = c1a1 * a1 + c;
    M[10] = c1a2 * a2 + c;
}

/* SE(3) exp/log of body twists, 3x4 composition and inverse: fks_se3.h (shared with the
 * host-side robot control, fks_robot_control.cpp) */
using fks_se3::compose34;
using fks_se3::exp_twist34;
using fks_se3::inverse34;
using fks_se3::log_twist34;

/* ---------------- wave primitives ---------------- */
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }

/* global-memory view of a pointer read out of SimArgs: the loads become global_load
 * (SGPR base + offset addressing, vmcnt only) instead of flat loads, which also count
 * against lgkmcnt and so serialise against every LDS wait */
#define FKS_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const FKS_GLOBAL T* gp(const T* p) {
    return (const FKS_GLOBAL T*)p;
}
template <typename T>
__device__ __forceinline__ FKS_GLOBAL T* gpw(T* p) {
    return (FKS_GLOBAL T*)p;
}
__device__ __forceinline__ RoundDev load_round(const RoundDev* p, int r) {
    const FKS_GLOBAL RoundDev* g = gp(p) + r;
    RoundDev o;
    o.link = g->link;
    o.npts = g->npts;
    o.radius = g->radius;
    return o;
}
__device__ __forceinline__ SampledDev load_sampled(const SampledDev* p, int d) {
    const FKS_GLOBAL SampledDev* g = gp(p) + d;
    SampledDev o;
    o.nbins = g->nbins;
    o.elems = g->elems;
    o.bounds = g->bounds;
    o.samples = g->samples;
    return o;
}
/* 64-bit lane moves: DPP within rows of 16, readlane across rows.  Every control used
 * (quad_perm, row_mirror, row_half_mirror) reads a valid lane for every lane, so the
 * "old" operand is never selected and needs no zero-initialised register. */
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    static_assert(CTRL <= 0xFF || CTRL == 0x140 || CTRL == 0x141, "full-permutation DPP controls only");
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ int readlane_i32(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
constexpr int kDppXor1 = 0xB1;       /* quad_perm [1,0,3,2] */
constexpr int kDppXor2 = 0x4E;       /* quad_perm [2,3,0,1] */
constexpr int kDppHalfMirror = 0x141; /* lane 7-i within 8: xor 4 once quads are uniform */
constexpr int kDppMirror = 0x140;     /* lane 15-i within 16: xor 8 once 8-groups are uniform */
constexpr int kDppQuadBcast0 = 0x00;  /* quad_perm [0,0,0,0] */
constexpr int kDppQuadBcast1 = 0x55;  /* quad_perm [1,1,1,1] */
constexpr int kDppQuadBcast2 = 0xAA;  /* quad_perm [2,2,2,2] */
constexpr int kDppQuadBcast3 = 0xFF;  /* quad_perm [3,3,3,3] */

/* The cross-row steps of a wave reduction once every row of 16 lanes holds its row's
 * value: v_permlane16_swap / v_permlane32_swap (gfx950) give every lane the value of the
 * lower and of the upper row (half) of its pair, so the combine runs in all lanes in the
 * order the scalar tree (r0 . r1) . (r2 . r3) uses, with no v_readlane per row; the result
 * is then read once from lane 0 (wave-uniform, so branches on it stay scalar). */
#ifndef FKS_PERMLANE_REDUCE
#define FKS_PERMLANE_REDUCE 1
#endif
template <bool HALVES>
__device__ __forceinline__ void row_pair_f64(double v, double* lower, double* upper) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    const auto l = HALVES ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = HALVES ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    *lower = __longlong_as_double((long long)(((uint64_t)h[0] << 32) | l[0]));
    *upper = __longlong_as_double((long long)(((uint64_t)h[1] << 32) | l[1]));
}
__device__ __forceinline__ double readfirstlane_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
/* canonical 64-lane sum (oracle canon_sum): xor butterfly with offsets 1, 2, 4,
 * 8, 16, 32; every lane gets the same value.  Call with all 64 lanes active. */
__device__ __forceinline__ double bfly_sum(double v) {
    v = v + dpp_f64<kDppXor1>(v);
    v = v + dpp_f64<kDppXor2>(v);
    v = v + dpp_f64<kDppHalfMirror>(v);
    v = v + dpp_f64<kDppMirror>(v);
#if FKS_PERMLANE_REDUCE
    double a, b;
    row_pair_f64<false>(v, &a, &b);
    row_pair_f64<true>(a + b, &a, &b); /* r0 + r1, r2 + r3 */
    return readfirstlane_f64(a + b);
#else
    const double r0 = readlane_f64(v, 0), r1 = readlane_f64(v, 16), r2 = readlane_f64(v, 32), r3 = readlane_f64(v, 48);
    return (r0 + r1) + (r2 + r3);
#endif
}
/* max over lanes of non-negative values (order-insensitive) */
__device__ __forceinline__ double wave_max_nonneg(double v) {
    double o = dpp_f64<kDppXor1>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppXor2>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppHalfMirror>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppMirror>(v);
    v = (o > v) ? o : v;
#if FKS_PERMLANE_REDUCE
    double a, b;
    row_pair_f64<false>(v, &a, &b);
    row_pair_f64<true>((b > a) ? b : a, &a, &b);
    return readfirstlane_f64((b > a) ? b : a);
#else
    const double r0 = readlane_f64(v, 0), r1 = readlane_f64(v, 16), r2 = readlane_f64(v, 32), r3 = readlane_f64(v, 48);
    const double a = (r1 > r0) ? r1 : r0, b = (r3 > r2) ? r3 : r2;
    return (b > a) ? b : a;
#endif
}
/* OR over the wave's lanes.  Error bits are rare: one ballot answers the common
 * all-zero case without the six dependent LDS-crossbar shuffles. */
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    if (__ballot(v != 0u) == 0ull) return 0u;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v |= (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += (uint64_t)__shfl_xor((long long)v, off, 64);
    return v;
}
__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }
/* LDS / scratch hand-off between the lanes of the wave (one wave per workgroup):
 * a wavefront-scope fence orders the wave's own memory operations without waiting
 * for outstanding global loads, unlike a workgroup barrier */
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* ---------------- RNG (same spec as oracle_rng.h) ---------------- */
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
        const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0;
        c[1] = lo1;
        c[2] = n2;
        c[3] = lo0;
        k0 += W0;
        k1 += W1;
    }
}
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    const uint64_t bits = (((uint64_t)a << 32) | (uint64_t)b) >> 11;
    return (double)bits * (1.0 / 9007199254740992.0);
}
/* truncated normal TN(0, 0.5) on [-1, 1]: TYPE_1 accept-reject over polar normals.
 * The attempts are those of the oracle (counter_truncated_normal) in the same order;
 * the loop is split so that a wave first advances every lane to its next attempt
 * inside the unit disc (Philox only) and then takes the logarithm once for all
 * lanes, instead of once per attempt that any lane is still rejecting. */
__device__ double tn_sample(uint32_t k0, uint32_t k1, uint64_t particle, uint32_t step, uint32_t micro, uint32_t dof,
                            uint32_t* err) {
    const double mean = 0.0, stddev = 0.5, lo = -2.0, hi = 2.0;
    uint32_t attempt = 0;
    while (attempt < 64u) {
        double x, y, r2;
        for (;;) {
            uint32_t c[4] = {(uint32_t)particle, step, micro,
                             ((uint32_t)(particle >> 32) << 16) | ((dof & 0xffu) << 8) | attempt};
            philox4x32_10(c, k0, k1);
            x = 2.0 * u53(c[0], c[1]) - 1.0;
            y = 2.0 * u53(c[2], c[3]) - 1.0;
            r2 = x * x + y * y;
            if (!(r2 > 1.0 || r2 == 0.0)) break;
            if (++attempt >= 64u) {
                *err |= FKS_PARTICLE_ERR_RNG_EXHAUSTED;
                return 0.0;
            }
        }
        const double mult = dsqrt(-2.0 * fks_math::log(r2) / r2);
        const double n1 = (y * mult) * 1.0 + 0.0;
        const double n2 = (x * mult) * 1.0 + 0.0;
        if ((n1 <= hi) && (n1 >= lo)) return mean + stddev * n1;
        if ((n2 <= hi) && (n2 >= lo)) return mean + stddev * n2;
        ++attempt;
    }
    *err |= FKS_PARTICLE_ERR_RNG_EXHAUSTED;
    return 0.0;
}

/* SampledUncertainVelocityActuator pick (UNC:236-237): uniform index into a bin of
 * `elems` samples from the first Philox block of the (particle, step, micro, dof)
 * counter; which bin it indexes depends on the clamped command (apply_input). */
__device__ double sampled_pick(uint32_t k0, uint32_t k1, uint64_t particle, uint32_t step, uint32_t micro, uint32_t dof,
                               uint32_t elems) {
    uint32_t c[4] = {(uint32_t)particle, step, micro, ((uint32_t)(particle >> 32) << 16) | ((dof & 0xffu) << 8)};
    philox4x32_10(c, k0, k1);
    uint32_t pick = (uint32_t)(u53(c[0], c[1]) * (double)elems);
    if (pick >= elems) pick = elems - 1u;
    return (double)pick;
}

/* Actuator noise does not depend on the particle state, so the samples of the next
 * floor(64 / D) microsteps are drawn at once, one lane per (microstep, dof), into LDS;
 * noise_sample() consumes them (and their error bits) in the DOF lanes. */
struct Sim;
__device__ FKS_SHAPE_INLINE void refill_noise(Sim& s, uint32_t micro0, uint32_t M);
__device__ __forceinline__ double noise_sample(Sim& s, uint32_t micro);

/* ---------------- grids ---------------- */
/* VoxelGrid LocationToGridIndex4d + IndexInBounds: trunc toward zero of
 * (inverse_origin * p) * (1/res); indices beyond int32 are out of bounds anyway */
__device__ __forceinline__ bool grid_index(const GridDev& g, const D4& p, int32_t idx[3]) {
    const D4 q = xform4(g.inv, p);
    const double v[3] = {q.x * g.inv_res, q.y * g.inv_res, q.z * g.inv_res};
    bool ok = true;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const bool fin = (v[a] > -2147483648.0) && (v[a] < 2147483647.0);
        idx[a] = fin ? (int32_t)v[a] : -1;
        ok = ok && fin && idx[a] >= 0 && (int64_t)idx[a] < g.n[a];
    }
    return ok;
}
/* the SDF's and normal ranges' HBM position of in-bounds cell (i, j, k) (fks_device.h) */
__device__ __forceinline__ uint32_t grid_brick(const GridDev& g, int32_t i, int32_t j, int32_t k) {
    return brick_cell(g.nb, (uint32_t)i, (uint32_t)j, (uint32_t)k);
}

/* The wave's state.  Wave-uniform values live in SGPRs, which the hot loops run short of
 * (every value live across the microstep loop that does not fit is spilled to a VGPR lane
 * and costs a v_writelane / v_readlane per use): the LDS tables' addresses are therefore
 * derived from the two block bases at each use (constant offsets in shape builds), the
 * per-segment counters are 32-bit, and wave totals, timestamps and the particle id are not
 * kept live across the particle loop (simulate_particles). */
/* a linked robot's shape build carries no register copy of the controller state (Sim::pid_state) */
/* Where the lane index lives (Sim::lane).  Register allocation at the 96-VGPR budget is
 * chaotic, and the two choices measured best on different robots: the lean-block kernels
 * (LDS-bound robots with long chains, cfg5) run 3.4 % faster reading the index from the
 * hardware at each use, which keeps it from being spilled and reloaded across the microstep
 * loop; the others keep it in a VGPR (cfg3 2.7 % faster that way) */
#ifndef FKS_ASM_LANE
#if defined(FKS_SHAPE_LEAN) && FKS_SHAPE_LEAN
#define FKS_ASM_LANE 1
#else
#define FKS_ASM_LANE 0
#endif
#endif
#if defined(FKS_SHAPE_TYPE) && FKS_SHAPE_TYPE == 0
#define FKS_PID_REGS 0
#else
#define FKS_PID_REGS 1
#endif
#ifndef FKS_PAR_PROOF
#define FKS_PAR_PROOF 1
#endif
/* FKS_NO_SKIP_PROOFS (validation builds only: fks_set_specialization(ctx,
 * FKS_SPECIALIZE_NO_PROOFS), tests/test_proof_free.py): every shortcut that rests on a cached
 * state and a floating-point margin is compiled out, so each check is evaluated as the
 * reference evaluates it — the environment / correction round proofs (skippable_rounds), the
 * motion estimate's round pruning (max_point_motion), the self-collision gap proof
 * (self_collisions) and the two lever-arm shortcuts of the resolver (resolve_step).  The
 * product's results must equal this build's on every particle, byte for byte. */
#ifndef FKS_NO_SKIP_PROOFS
#define FKS_NO_SKIP_PROOFS 0
#endif
/* the dynamic LDS of every kernel here: the workgroup's robot tables at offset 0, then one
 * block per wave (LdsLayout) */
extern __shared__ __attribute__((aligned(16))) double fks_lds[];

struct Sim {
    const SimArgs* A;
    double* lds_block; /* this wave's LDS block (a pointer: cfg5 ran 3-7 % slower with it formed from an offset at each use) */
    double* scratch;
    int lane_v; /* the lane index (FKS_ASM_LANE 0) */
    /* the lane index.  FKS_ASM_LANE: read from the hardware at each use (two VALU
     * instructions in a volatile asm the optimiser can neither hoist nor share), so no lane
     * index stays live across the loops to be spilled and reloaded */
    __device__ __forceinline__ int lane() const {
#if FKS_ASM_LANE
        int ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
        return ln;
#else
        return lane_v;
#endif
    }
    uint32_t step;
    uint32_t err;          /* per-lane error bits, OR-reduced at decision points */
    uint64_t lane_bytes;   /* per-lane algorithmic SDF bytes */
    uint64_t local;        /* particle index within the call (global id: pid()) */
    uint32_t micro_count, resolver_count, step_count, lsq_rows; /* this segment's */
    __device__ __forceinline__ double* lds() const { return lds_block; }
    __device__ __forceinline__ double* shared() const { return fks_lds; }         /* the workgroup's robot tables */
    __device__ __forceinline__ uint64_t pid() const { return A->first_pid + local; }
    __device__ __forceinline__ uint32_t* stats() const { return reinterpret_cast<uint32_t*>(lds() + LAY(*A).misc + 24); } /* 8 x u32, lane 0 */
    __device__ __forceinline__ uint64_t* phase() const { return reinterpret_cast<uint64_t*>(lds() + LAY(*A).misc + 8); } /* FKS_NUM_PHASES x u64, lane 0 */
    __device__ __forceinline__ uint64_t* totals() const { return reinterpret_cast<uint64_t*>(lds() + LAY(*A).misc + 32); } /* kWaveTotals x u64, lane 0 */
    __device__ __forceinline__ const JointDev* joints() const { return reinterpret_cast<const JointDev*>(shared() + LAY(*A).joints); }
    __device__ __forceinline__ const fks_dof_controller* ctrl() const {
        return reinterpret_cast<const fks_dof_controller*>(shared() + LAY(*A).ctrl);
    }
    __device__ __forceinline__ const int32_t* dofj() const { return reinterpret_cast<const int32_t*>(shared() + LAY(*A).dofj); }
    __device__ __forceinline__ const double* base() const { return shared() + LAY(*A).base; }
    /* the particle's controller state (lane d < D: error integral [d], last error [kWave + d]).
     * Linked robots keep it in the wave's workspace rather than in two VGPR pairs live across
     * the whole step loop (it is read and written once per controller step; cfg3's and cfg5's
     * microstep loops lose most of their spill reloads); SE(2) / SE(3) robots keep the registers
     * (the workspace copy moved cfg4's allocation the other way) */
    __device__ __forceinline__ double* pid_state() const { return scratch + SLAY(*A).pid; }
#if FKS_PID_REGS
    double pid_integral, pid_last; /* DOF lanes, SE(2) / SE(3) */
#endif
    double* rstate;  /* the round skip-proof cache: LDS block, or scratch in the lean kernels */
    double* selfref; /* the self-collision proof's reference (LdsLayout / ScratchLayout selfref) */
    bool self_nonempty;
    bool tcur_valid; /* Tcur == FK(particle configuration) from the end of the last step */
    uint32_t tr_steps, tr_cfgs; /* trace records produced so far (traced kernels) */
};
template <int RT>
__device__ __forceinline__ void pid_get(const Sim& s, int ln, double* integral, double* last) {
    if constexpr (RT == FKS_ROBOT_LINKED) {
        *integral = s.pid_state()[ln];
        *last = s.pid_state()[kWave + ln];
    } else {
#if FKS_PID_REGS
        *integral = s.pid_integral;
        *last = s.pid_last;
#endif
    }
}
template <int RT>
__device__ __forceinline__ void pid_set(Sim& s, int ln, double integral, double last) {
    if constexpr (RT == FKS_ROBOT_LINKED) {
        s.pid_state()[ln] = integral;
        s.pid_state()[kWave + ln] = last;
    } else {
#if FKS_PID_REGS
        s.pid_integral = integral;
        s.pid_last = last;
#endif
    }
}
/* the wave's call totals in LDS (Sim::totals), flushed once when the queue is drained */
enum { kTotSteps = 0, kTotMicro, kTotResolver, kTotLsq, kTotErrors, kWaveTotals };

/* The lane index made opaque to the optimiser at the head of the microstep and
 * resolver loops: the per-lane LDS / workspace addresses derived from it are then
 * recomputed inside the loop instead of being hoisted out of it into VGPRs that stay
 * live across the whole loop nest. */
__device__ __forceinline__ int opaque_lane(int ln) {
    asm volatile("" : "+v"(ln));
    return ln;
}

/* wave totals of the self-collision branch (kCntSelfChecks, kCntSelfPoints), kept in the
 * wave's LDS block (misc + 28, + 29) rather than in registers: the branch is rare */
__device__ __forceinline__ uint64_t* self_counters(const Sim& s) { return reinterpret_cast<uint64_t*>(s.lds() + LAY(*s.A).misc + 28); }

/* ForwardSimulationStepTrace records (traced kernel instantiations only) */
template <bool TR>
__device__ __forceinline__ void trace_config(Sim& s, const double* cfg, uint32_t micro, uint32_t kind) {
    if constexpr (TR) {
        const SimArgs& A = *s.A;
        const uint32_t k = s.tr_cfgs++;
        if (k < A.tr_cfg_cap) {
            const uint64_t rec = s.local * (uint64_t)A.tr_cfg_cap + k;
            if (s.lane() < RDIM(A.R, W)) A.tr_cfg[rec * (uint64_t)RDIM(A.R, W) + s.lane()] = cfg[s.lane()];
            if (s.lane() == 0) {
                A.tr_tags[3 * rec] = s.step;
                A.tr_tags[3 * rec + 1] = micro;
                A.tr_tags[3 * rec + 2] = kind;
            }
        }
    }
}
template <bool TR>
__device__ __forceinline__ void trace_step(Sim& s, const double* u, const double* ustep, uint32_t M) {
    if constexpr (TR) {
        const SimArgs& A = *s.A;
        const uint32_t k = s.tr_steps++;
        if (k < A.tr_step_cap) {
            const int D = RDIM(A.R, D);
            const uint64_t rec = s.local * (uint64_t)A.tr_step_cap + k;
            if (s.lane() < D) {
                A.tr_inputs[rec * 2ull * (uint64_t)D + s.lane()] = u[s.lane()];
                A.tr_inputs[rec * 2ull * (uint64_t)D + D + s.lane()] = ustep[s.lane()];
            }
            if (s.lane() == 0) A.tr_micro[rec] = M;
        }
    }
}

/* per-phase timers (fks_get_phase_cycles) cost ~10% of wave cycles, so they are
 * compiled in only for profiling builds (-DFKS_PHASE_TIMERS=1); the per-particle
 * total is always kept */
#ifndef FKS_PHASE_TIMERS
#define FKS_PHASE_TIMERS 0
#endif
__device__ __forceinline__ uint64_t tick() {
    if constexpr (FKS_PHASE_TIMERS) return __builtin_amdgcn_s_memtime();
    return 0;
}
__device__ __forceinline__ void tock(Sim& s, int phase, uint64_t t0) {
    if constexpr (FKS_PHASE_TIMERS)
        if (s.lane() == 0) s.phase()[phase] += tick() - t0;
}
__device__ __forceinline__ void count_event(Sim& s, int slot, uint64_t n) {
    if constexpr (FKS_PHASE_TIMERS)
        if (s.lane() == 0) s.phase()[slot] += n;
}

__device__ __noinline__ void refill_noise_lanes(const SimArgs* __restrict__ Ap, double* lds, int ln, uint64_t pid, uint32_t step,
                                                uint32_t micro0, uint32_t M) {
    const SimArgs& A = *Ap;
    const int D = RDIM(A.R, D);
    const int per = kWave / D;
    double* nz = lds + LAY(A).noise;
    uint32_t* ne = reinterpret_cast<uint32_t*>(lds + LAY(A).noise_err);
    if (ln < per * D) {
        const uint32_t m = micro0 + (uint32_t)(ln / D);
        if (m < M) {
            uint32_t e = 0;
            const uint32_t dof = (uint32_t)(ln % D);
            if ((A.R.sampled_mask >> dof) & 1ull)
                nz[ln] = sampled_pick(A.key0, A.key1, pid, step, m, dof, load_sampled(A.R.sampled, (int)dof).elems);
            else
                nz[ln] = tn_sample(A.key0, A.key1, pid, step, m, dof, &e);
            ne[ln] = e;
        }
    }
    wsync();
}
__device__ FKS_SHAPE_INLINE void refill_noise(Sim& s, uint32_t micro0, uint32_t M) {
    refill_noise_lanes(s.A, s.lds(), s.lane(), s.pid(), s.step, micro0, M);
}
__device__ __forceinline__ double noise_sample(Sim& s, uint32_t micro) {
    const SimArgs& A = *s.A;
    const int D = RDIM(A.R, D);
    const int slot = (int)(micro % (uint32_t)(kWave / D)) * D + s.lane();
    s.err |= reinterpret_cast<const uint32_t*>(s.lds() + LAY(A).noise_err)[slot];
    return s.lds()[LAY(A).noise + slot];
}

/* sdf_tools EstimateDistance4d (same spec as oracle SDF::EstimateDistance4d) */
__device__ double estimate_distance(const SimArgs& A, const D4& p, bool* inb, uint64_t* bytes) {
    int32_t idx[3];
    if (!grid_index(A.sdf_g, p, idx)) {
        *inb = false;
        return (double)A.oob;
    }
    *inb = true;
    *bytes += 28;
    const GridDev& g = A.sdf_g;
    double grad[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        int32_t lo[3] = {idx[0], idx[1], idx[2]}, hi[3] = {idx[0], idx[1], idx[2]};
        lo[a] = (idx[a] - 1 > 0) ? idx[a] - 1 : 0;
        hi[a] = ((int64_t)idx[a] + 1 < g.n[a] - 1) ? idx[a] + 1 : (int32_t)(g.n[a] - 1);
        const double inv = g.inv_res_span[hi[a] - lo[a]]; /* 1.0 / (g.res * (hi - lo)), hi - lo in {0, 1, 2} */
        const float diff = gp(A.sdf)[grid_brick(g, hi[0], hi[1], hi[2])] - gp(A.sdf)[grid_brick(g, lo[0], lo[1], lo[2])];
        grad[a] = (double)diff * inv;
    }
    const D3 c = xform3(g.org, D3{g.res * ((double)idx[0] + 0.5), g.res * ((double)idx[1] + 0.5), g.res * ((double)idx[2] + 0.5)});
    const double dx = p.x - c.x, dy = p.y - c.y, dz = p.z - c.z;
    const double nominal = (double)gp(A.sdf)[grid_brick(g, idx[0], idx[1], idx[2])];
    const double corrected = (nominal >= 0.0) ? nominal - (g.res * 0.5) : nominal + (g.res * 0.5);
    const double adjustment = (dx * grad[0] + dy * grad[1]) + dz * grad[2];
    const double estimate = corrected + adjustment;
    if ((corrected >= 0.0) == (estimate >= 0.0)) return estimate;
    if (corrected >= 0.0) return g.res * 0.0625;
    return g.res * -0.0625;
}

/* SurfaceNormalGrid::LookupSurfaceNormal(Vector4d, Vector4d) + GetBestSurfaceNormal */
__device__ bool lookup_normal(const SimArgs& A, const D4& loc, const D4& dir, D3* out, uint32_t* err, uint64_t* bytes) {
    *out = D3{0.0, 0.0, 0.0};
    int32_t idx[3];
    if (!A.has_normals || !grid_index(A.nrm_g, loc, idx)) return false;
    /* one 8-byte load: begin in the low word, end in the high word (uint2 x, y) */
    const uint64_t range = gp(reinterpret_cast<const uint64_t*>(A.nrange))[grid_brick(A.nrm_g, idx[0], idx[1], idx[2])];
    const uint32_t begin = (uint32_t)range, end = (uint32_t)(range >> 32);
    /* 4 B for the cell, 56 B per entry examined (Vector4d + Vector3d, SPCS:52-53) */
    *bytes += 4;
    if (begin == end) return true;
    *bytes += 56ull * (uint64_t)(end - begin);
    const double direction_norm = dsqrt(sqnorm4(dir));
    if (!(direction_norm > 0.0)) {
        *err |= FKS_PARTICLE_ERR_ZERO_DIRECTION;
        return true;
    }
    const double ux = dir.x / direction_norm, uy = dir.y / direction_norm, uz = dir.z / direction_norm;
    /* the first entry is read whole (direction and normal in one round trip): nearly every
     * surface cell has exactly one, whose normal is then the answer without a second load */
    const FKS_GLOBAL double* e0 = gp(A.nent) + 6ull * begin;
    const double n0 = e0[3], n1 = e0[4], n2 = e0[5];
    int64_t best = -1;
    double best_dot = -__builtin_huge_val();
    for (uint32_t e = begin; e < end; ++e) {
        const FKS_GLOBAL double* ent = gp(A.nent) + 6ull * e;
        /* EntryDirection4d().dot(unit_direction), packet order; both w terms are +0 */
        const double dot = (ent[0] * ux + ent[2] * uz) + ent[1] * uy;
        if (dot > best_dot) {
            best_dot = dot;
            best = (int64_t)e;
        }
    }
    if (best < 0) {
        *err |= FKS_PARTICLE_ERR_ZERO_DIRECTION;
        return true;
    }
    if (best == (int64_t)begin) {
        *out = D3{n0, n1, n2};
    } else {
        const FKS_GLOBAL double* ent = gp(A.nent) + 6ull * (uint64_t)best;
        *out = D3{ent[3], ent[4], ent[5]};
    }
    return true;
}

__device__ __forceinline__ D4 load_point(const RobotDev& R, int i) {
    typedef double f64x2 __attribute__((ext_vector_type(2)));
    const FKS_GLOBAL f64x2* p2 = gp(reinterpret_cast<const f64x2*>(R.points + 4ull * (uint64_t)i));
    const f64x2 a = p2[0], b = p2[1];
    return D4{a.x, a.y, b.x, b.y};
}

/* ---------------- forward kinematics: cfg (LDS) -> link transforms T (LDS) ---------------- */
template <int RT>
__device__ FKS_SHAPE_INLINE void fk(Sim& s, const double* cfg, double* T) {
    const RobotDev& R = s.A->R;
    const int ln = s.lane();
    if constexpr (RT == FKS_ROBOT_LINKED) {
        double* jm = s.lds() + LAY(*s.A).jm;
        const JointDev* JD = s.joints();
        if (ln < RDIM(R, J)) {
            const JointDev& jd = JD[ln];
            if (jd.type == FKS_JOINT_REVOLUTE || jd.type == FKS_JOINT_CONTINUOUS) {
                double M[12];
                angle_axis34(cfg[jd.dof], jd.axis[0], jd.axis[1], jd.axis[2], M);
                M[3] = 0.0;
                M[7] = 0.0;
                M[11] = 0.0;
                for (int e = 0; e < 12; ++e) jm[12 * ln + e] = M[e];
            } else if (jd.type == FKS_JOINT_PRISMATIC) {
                const double v = cfg[jd.dof];
                const double M[12] = {1.0, 0.0, 0.0, jd.axis[0] * v, 0.0, 1.0, 0.0, jd.axis[1] * v, 0.0, 0.0, 1.0, jd.axis[2] * v};
                for (int e = 0; e < 12; ++e) jm[12 * ln + e] = M[e];
            }
        }
        wsync();
        /* 12-lane chain: lane 4r+c owns element (r, c) of the running transform; the
         * row a lane needs is broadcast inside its quad (DPP), so the chain never
         * goes through memory.  T_child = (T_parent * origin) * motion, each element
         * the same dot3 as the oracle. */
        const int r = ln >> 2, c = ln & 3;
        const bool act = ln < 12;
        double own = act ? s.base()[4 * r + c] : 0.0;
        if (act) T[4 * r + c] = own;
        double p0 = dpp_f64<kDppQuadBcast0>(own), p1 = dpp_f64<kDppQuadBcast1>(own), p2 = dpp_f64<kDppQuadBcast2>(own),
               p3 = dpp_f64<kDppQuadBcast3>(own);
        int last = 0;
        const int J = RDIM(R, J);
        /* the joint's origin / motion columns are read at the top of its iteration (no
         * prefetch registers to rotate: the other waves of the SIMD hide the LDS latency) */
        for (int j = 0; j < J; ++j) {
            const int parent = __builtin_amdgcn_readfirstlane(JD[j].parent);
            const int child = __builtin_amdgcn_readfirstlane(JD[j].child);
            const int type = __builtin_amdgcn_readfirstlane(JD[j].type);
            const double co0 = JD[j].origin[c], co1 = JD[j].origin[4 + c], co2 = JD[j].origin[8 + c];
            const double cm0 = jm[12 * j + c], cm1 = jm[12 * j + 4 + c], cm2 = jm[12 * j + 8 + c];
            if (parent != last) {
                const double* Tp = T + 12 * parent + 4 * (act ? r : 0);
                p0 = Tp[0];
                p1 = Tp[1];
                p2 = Tp[2];
                p3 = Tp[3];
            }
            double a = dot3(p0, p1, p2, co0, co1, co2);
            if (c == 3) a = a + p3;
            double out = a;
            if (type != FKS_JOINT_FIXED) {
                const double a0 = dpp_f64<kDppQuadBcast0>(a), a1 = dpp_f64<kDppQuadBcast1>(a),
                             a2 = dpp_f64<kDppQuadBcast2>(a), a3 = dpp_f64<kDppQuadBcast3>(a);
                out = dot3(a0, a1, a2, cm0, cm1, cm2);
                if (c == 3) out = out + a3;
            }
            if (act) T[12 * child + 4 * r + c] = out;
            p0 = dpp_f64<kDppQuadBcast0>(out);
            p1 = dpp_f64<kDppQuadBcast1>(out);
            p2 = dpp_f64<kDppQuadBcast2>(out);
            p3 = dpp_f64<kDppQuadBcast3>(out);
            last = child;
        }
        wsync();
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        double M[12];
        angle_axis34(cfg[2], 0.0, 0.0, 1.0, M);
        M[3] = cfg[0];
        M[7] = cfg[1];
        M[11] = 0.0;
        if (ln == 0)
#pragma unroll
            for (int e = 0; e < 12; ++e) T[e] = M[e]; /* not M[ln]: a lane-indexed private array lives in scratch */
        wsync();
    } else {
        if (ln < 12) T[ln] = cfg[ln];
        wsync();
    }
}

/* FK of two configurations of a linked robot in one pass (J <= 32): the chain of cfgA
 * runs on lanes 0-11 and the chain of cfgB on lanes 16-27 (quads 0-2 and 4-6), their
 * joint motion matrices on lanes j and 32 + j.  Every instruction of the chain serves
 * both, so the pair costs about one FK; each chain is the same arithmetic as fk(). */
__device__ FKS_SHAPE_INLINE void fk_pair(Sim& s, const double* cfgA, double* TA, const double* cfgB, double* TB) {
    const RobotDev& R = s.A->R;
    const int ln = s.lane();
    double* jmA = s.lds() + LAY(*s.A).jm;
    double* jmB = s.lds() + LAY(*s.A).jm2;
    const JointDev* JD = s.joints();
    {
        const int j = ln & 31;
        const bool second = ln >= 32;
        if (j < RDIM(R, J)) {
            const JointDev& jd = JD[j];
            const double* cfg = second ? cfgB : cfgA;
            double* jm = second ? jmB : jmA;
            if (jd.type == FKS_JOINT_REVOLUTE || jd.type == FKS_JOINT_CONTINUOUS) {
                double M[12];
                angle_axis34(cfg[jd.dof], jd.axis[0], jd.axis[1], jd.axis[2], M);
                M[3] = 0.0;
                M[7] = 0.0;
                M[11] = 0.0;
                for (int e = 0; e < 12; ++e) jm[12 * j + e] = M[e];
            } else if (jd.type == FKS_JOINT_PRISMATIC) {
                const double v = cfg[jd.dof];
                const double M[12] = {1.0, 0.0, 0.0, jd.axis[0] * v, 0.0, 1.0, 0.0, jd.axis[1] * v, 0.0, 0.0, 1.0, jd.axis[2] * v};
                for (int e = 0; e < 12; ++e) jm[12 * j + e] = M[e];
            }
        }
    }
    wsync();
    const int local = ln & 15;
    const bool chainB = (ln & 16) != 0;
    const int r = local >> 2, c = local & 3;
    const bool act = local < 12 && ln < 32;
    double* T = chainB ? TB : TA;
    const double* jm = chainB ? jmB : jmA;
    double own = act ? s.base()[4 * r + c] : 0.0;
    if (act) T[4 * r + c] = own;
    double p0 = dpp_f64<kDppQuadBcast0>(own), p1 = dpp_f64<kDppQuadBcast1>(own), p2 = dpp_f64<kDppQuadBcast2>(own),
           p3 = dpp_f64<kDppQuadBcast3>(own);
    int last = 0;
    const int J = RDIM(R, J);
    for (int j = 0; j < J; ++j) {
        const int parent = __builtin_amdgcn_readfirstlane(JD[j].parent);
        const int child = __builtin_amdgcn_readfirstlane(JD[j].child);
        const int type = __builtin_amdgcn_readfirstlane(JD[j].type);
        const double co0 = JD[j].origin[c], co1 = JD[j].origin[4 + c], co2 = JD[j].origin[8 + c];
        const double cm0 = jm[12 * j + c], cm1 = jm[12 * j + 4 + c], cm2 = jm[12 * j + 8 + c];
        if (parent != last) {
            const double* Tp = T + 12 * parent + 4 * (act ? r : 0);
            p0 = Tp[0];
            p1 = Tp[1];
            p2 = Tp[2];
            p3 = Tp[3];
        }
        double a = dot3(p0, p1, p2, co0, co1, co2);
        if (c == 3) a = a + p3;
        double out = a;
        if (type != FKS_JOINT_FIXED) {
            const double a0 = dpp_f64<kDppQuadBcast0>(a), a1 = dpp_f64<kDppQuadBcast1>(a),
                         a2 = dpp_f64<kDppQuadBcast2>(a), a3 = dpp_f64<kDppQuadBcast3>(a);
            out = dot3(a0, a1, a2, cm0, cm1, cm2);
            if (c == 3) out = out + a3;
        }
        if (act) T[12 * child + 4 * r + c] = out;
        p0 = dpp_f64<kDppQuadBcast0>(out);
        p1 = dpp_f64<kDppQuadBcast1>(out);
        p2 = dpp_f64<kDppQuadBcast2>(out);
        p3 = dpp_f64<kDppQuadBcast3>(out);
        last = child;
    }
    wsync();
}

/* noisy actuator of dof `dof` on its clamped command `real` (TNUVA:568-596):
 * TruncatedNormalUncertainVelocityActuator (UNC:77-90), or the sampled one
 * (UNC:270-279: first matching bin, then the picked sample) */
__device__ __forceinline__ double actuator_noisy(Sim& s, const fks_dof_controller& ct, int dof, double real, uint32_t micro) {
    const double ns = noise_sample(s, micro);
    const RobotDev& R = s.A->R;
    if ((R.sampled_mask >> dof) & 1ull) {
        const SampledDev sd = load_sampled(R.sampled, dof);
        for (uint32_t b = 0; b < sd.nbins; ++b)
            if (real >= gp(sd.bounds)[2 * b] && real <= gp(sd.bounds)[2 * b + 1])
                return real + gp(sd.samples)[(uint64_t)b * sd.elems + (uint32_t)ns];
        s.err |= FKS_PARTICLE_ERR_NO_NOISE_BIN;
        return real + 0.0;
    }
    const double bound = fks_control::actuator_noise_bound(real, dabs(ct.max_actuator_proportional_noise),
                                                           dabs(ct.max_actuator_minimum_noise), dabs(ct.velocity_limit));
    return real + ns * bound;
}

/* ---------------- robot control-input application (TNUVA ApplyControlInput) ----------------
 * cfg_out = apply(cfg_in, input) with clamp (+ noise if noisy).  Lane d < D owns dof d. */
template <int RT>
__device__ FKS_SHAPE_INLINE void apply_input(Sim& s, const double* cfg_in, const double* input, double* cfg_out, bool noisy, uint32_t micro) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    if constexpr (RT == FKS_ROBOT_LINKED) {
        if (ln < RDIM(R, D)) {
            const fks_dof_controller& ct = s.ctrl()[ln];
            const double vmax = dabs(ct.velocity_limit);
            double real = clamp(input[ln], -vmax, vmax);
            if (noisy) real = actuator_noisy(s, ct, ln, real, micro);
            const JointDev& jd = s.joints()[s.dofj()[ln]];
            const double raw = cfg_in[ln] + real;
            double v;
            if (jd.type == FKS_JOINT_CONTINUOUS) {
                v = fks_math::wrap_revolute(raw);
                v = fks_math::wrap_revolute(v);
            } else {
                v = clamp(raw, jd.lo, jd.hi);
                v = clamp(v, jd.lo, jd.hi);
            }
            cfg_out[ln] = v;
        }
        wsync();
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        if (ln < 3) {
            const fks_dof_controller& ct = s.ctrl()[ln];
            const double vmax = dabs(ct.velocity_limit);
            double real = clamp(input[ln], -vmax, vmax);
            if (noisy) real = actuator_noisy(s, ct, ln, real, micro);
            double v = cfg_in[ln] + real;
            if (ln == 2) v = fks_math::wrap_revolute(v);
            cfg_out[ln] = v;
        }
        wsync();
    } else {
        double* tw = s.lds() + LAY(*s.A).misc; /* 6 doubles */
        if (ln < 6) {
            const fks_dof_controller& ct = s.ctrl()[ln];
            const double vmax = dabs(ct.velocity_limit);
            double real = clamp(input[ln], -vmax, vmax);
            if (noisy) real = actuator_noisy(s, ct, ln, real, micro);
            tw[ln] = real;
        }
        wsync();
        double M[12], twr[6], P[12];
        for (int k = 0; k < 6; ++k) twr[k] = tw[k];
        for (int k = 0; k < 12; ++k) P[k] = cfg_in[k];
        exp_twist34(twr, M);
        double C[12];
        compose34(P, M, C);
        wsync();
        /* lane 0 stores all twelve: indexing the private array by lane would put it in scratch */
        if (ln == 0)
#pragma unroll
            for (int e = 0; e < 12; ++e) cfg_out[e] = C[e];
        wsync();
    }
}

/* GenerateControlAction (TNUVA:179-198, 384-412, 598-614): lane d < D returns u_d */
template <int RT>
__device__ FKS_SHAPE_INLINE double control_action(Sim& s, const double* cfg, const double* target) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    double err = 0.0;
    if constexpr (RT == FKS_ROBOT_LINKED) {
        if (ln < RDIM(R, D)) {
            const JointDev& jd = s.joints()[s.dofj()[ln]];
            if (jd.type == FKS_JOINT_CONTINUOUS)
                err = fks_math::wrap_revolute(target[ln] - cfg[ln]);
            else
                err = target[ln] - cfg[ln];
        }
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        if (ln < 2) err = target[ln] - cfg[ln];
        if (ln == 2) err = fks_math::wrap_revolute(target[2] - cfg[2]);
    } else {
        double P[12], Pi[12], Tg[12], Dm[12], tw[6];
        for (int k = 0; k < 12; ++k) {
            P[k] = cfg[k];
            Tg[k] = target[k];
        }
        inverse34(P, Pi);
        compose34(Pi, Tg, Dm);
        log_twist34(Dm, tw);
        double e = tw[0];
        for (int k = 1; k < 6; ++k)
            if (ln == k) e = tw[k];
        if (ln < 6) err = e;
    }
    double u = 0.0;
    if (ln < RDIM(R, D)) {
        const fks_dof_controller& ct = s.ctrl()[ln];
        /* SimplePIDController::ComputeFeedbackTerm (PID:122-135), gains made positive (PID:104-113),
         * then the actuator's clamp (UNC:70-75) */
        double integral, last;
        pid_get<RT>(s, ln, &integral, &last);
        const double term = fks_control::pid_feedback_term(dabs(ct.kp), dabs(ct.ki), dabs(ct.kd), dabs(ct.integral_clamp),
                                                           &integral, &last, err, A.dt);
        pid_set<RT>(s, ln, integral, last);
        u = fks_control::actuator_clamp(term, dabs(ct.velocity_limit));
    }
    return u;
}

/* configuration distance for the simulation shortcut (SPCS:898) */
template <int RT>
__device__ FKS_SHAPE_INLINE double config_distance(Sim& s, const double* cfg, const double* target) {
    const RobotDev& R = s.A->R;
    if constexpr (RT == FKS_ROBOT_LINKED) {
        double sum = 0.0;
        for (int k = 0; k < RDIM(R, D); ++k) {
            const JointDev& jd = s.joints()[s.dofj()[k]];
            const double sd = (jd.type == FKS_JOINT_CONTINUOUS) ? fks_math::wrap_revolute(target[k] - cfg[k])
                                                                : target[k] - cfg[k];
            const double d = gp(R.weights)[k] * dabs(sd);
            sum = sum + d * d;
        }
        return dsqrt(sum);
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        const double dx = target[0] - cfg[0];
        const double dy = target[1] - cfg[1];
        const double dr = fks_math::wrap_revolute(target[2] - cfg[2]);
        return gp(R.weights)[0] * dsqrt(dx * dx + dy * dy) + gp(R.weights)[1] * dabs(dr);
    } else {
        double P[12], Pi[12], Tg[12], Dm[12], tw[6];
        for (int k = 0; k < 12; ++k) {
            P[k] = cfg[k];
            Tg[k] = target[k];
        }
        const double dx = Tg[3] - P[3], dy = Tg[7] - P[7], dz = Tg[11] - P[11];
        inverse34(P, Pi);
        compose34(Pi, Tg, Dm);
        log_twist34(Dm, tw);
        const double angle = dsqrt((tw[3] * tw[3] + tw[4] * tw[4]) + tw[5] * tw[5]);
        return gp(R.weights)[0] * dsqrt((dx * dx + dy * dy) + dz * dz) + gp(R.weights)[1] * angle;
    }
}

/* ---------------- provably-free rounds ----------------
 * Every 64-point round whose points share one link (and have w = 1) keeps, in LDS,
 * the link transform at which it was last evaluated in full, the smallest nearest-
 * cell SDF value of its points there and their smallest margin to the grid
 * boundary (in cells).  A rigid motion moves each point by at most
 * b = |dt| + ||dR||_F * radius, i.e. by at most K = sqrt(3)*b/res + 3 axis steps
 * of cells; with the SDF constants of fks_create (positive neighbours differ by
 * <= lplus cells, positive cells next to a non-positive one are <= cmax) a round
 * whose cached minimum keeps every cell within K steps positive cannot collide, and
 * one that keeps them above 0.5 + 1.5*lplus cannot produce a correction.  Skipped
 * points are still counted in the algorithmic bytes the reference reads (their
 * grid margin guarantees they are in bounds). */
/* an upper bound of sqrt(x) for the proofs (never for results): the hardware v_sqrt_f64 is
 * within 2^29 ulp (2^-23 relative) of the root, so one instruction scaled by 1 + 2^-20
 * replaces the correctly rounded sequence (a dozen dependent instructions) */
__device__ __forceinline__ double sqrt_upper(double x) { return __builtin_amdgcn_sqrt(x) * (1.0 + 0x1p-20); }
__device__ __forceinline__ double rigid_motion_bound(const double* T, const double* Tref, double radius) {
    const double dt0 = T[3] - Tref[3], dt1 = T[7] - Tref[7], dt2 = T[11] - Tref[11];
    double f = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const double d = T[4 * r + c] - Tref[4 * r + c];
            f = f + d * d;
        }
    const double b = sqrt_upper((dt0 * dt0 + dt1 * dt1) + dt2 * dt2) + sqrt_upper(f) * radius;
    return b * (1.0 + 1e-9) + 1e-12;
}
__device__ __forceinline__ double wave_min(double v) {
    double o = dpp_f64<kDppXor1>(v);
    v = (o < v) ? o : v;
    o = dpp_f64<kDppXor2>(v);
    v = (o < v) ? o : v;
    o = dpp_f64<kDppHalfMirror>(v);
    v = (o < v) ? o : v;
    o = dpp_f64<kDppMirror>(v);
    v = (o < v) ? o : v;
#if FKS_PERMLANE_REDUCE
    double a, b;
    row_pair_f64<false>(v, &a, &b);
    row_pair_f64<true>((b < a) ? b : a, &a, &b);
    return readfirstlane_f64((b < a) ? b : a);
#else
    const double r0 = readlane_f64(v, 0), r1 = readlane_f64(v, 16), r2 = readlane_f64(v, 32), r3 = readlane_f64(v, 48);
    const double a = (r1 < r0) ? r1 : r0, b = (r3 < r2) ? r3 : r2;
    return (b < a) ? b : a;
#endif
}
constexpr double kInvalidRound = -1.0e308;
constexpr uint64_t kNoTicket = ~0ull;
/* particle hand-over between waves (possibly on different XCDs, each with its own L2):
 * the resting state moves through agent-scope atomic loads and stores, which gfx942 /
 * gfx950 issue with sc1 (coherent across XCDs at the memory side), so no L2 write-back
 * or invalidate is needed.  Between the state and the seg_done flag that publishes it,
 * publish_fence() is a workgroup-scope release fence: a compiler barrier for every
 * memory operation plus s_waitcnt vmcnt(0), i.e. the state stores have completed at the
 * coherence point before the flag store issues; claim_fence() is the matching acquire
 * after the claimant's CAS.  Formally the HIP model would want agent-scope
 * release/acquire (buffer_wbl2 / buffer_inv on these targets, measured 10-20 % slower);
 * the workgroup-scope fences are exact only because every access on both sides is an
 * sc1 atomic, which is why other targets refuse to compile this file (below). */
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "the segment hand-over relies on the gfx942/gfx950 memory model (sc1 atomics, see above)"
#endif
__device__ __forceinline__ void store_coherent(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_coherent(const double* p) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void store_coherent_u64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_coherent_u64(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish_fence() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
__device__ __forceinline__ void claim_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); }
constexpr uint32_t kSegClaimed = 0x80000000u; /* seg_done[p]: segment v is being run */
enum { kSkipCheck = 1, kSkipCorrections = 2 };

/* (link, radius) of round r < 64 from the workgroup's LDS copy of R.rounds */
__device__ __forceinline__ RoundDev lds_round(const Sim& s, int r) {
    RoundDev o;
    o.link = (int32_t)s.shared()[LAY(*s.A).rounds + 2 * r];
    o.npts = 0;
    o.radius = s.shared()[LAY(*s.A).rounds + 2 * r + 1];
    return o;
}

/* the proof's verdict for one round from its motion bound bm (meters) and cached state st */
__device__ __forceinline__ bool round_proof(const SimArgs& A, const double* st, double bm, bool still_if_floor, int what) {
    const double b = bm * A.sdf_g.inv_res; /* cells */
    const double K = 1.7320508075688773 * b + 3.0;
    const double Sr = st[12] * A.sdf_g.inv_res;
    const double lp = A.skip_lplus;
    const bool inb = st[13] - b > 1e-6;
    const bool same_cell = (b < st[14] - 1e-9) || (bm <= 1e-12 && still_if_floor);
    if (what == kSkipCheck) return (inb && (Sr - A.skip_cmax) > (K - 1.0) * lp + 1e-9) || (same_cell && st[12] >= A.thr_env);
    return (inb && (Sr - A.skip_cmax) > K * lp + 1e-9 && (Sr - K * lp) > 0.5 + 1.5 * lp + 1e-6) ||
           (same_cell && Sr > A.skip_cmax + 1e-9 && Sr > 0.5 + 1.5 * lp + 1e-6);
}

/* skippable_rounds for robots of at most 8 rounds: eight lanes per round, each taking one or
 * two of the twelve transform differences, summed inside the group by DPP (the same bound as
 * rigid_motion_bound, in another order: a bound either way), so a round's proof costs a few
 * instructions instead of the serial 3x4 difference on one lane */
__device__ __forceinline__ uint64_t skippable_rounds8(Sim& s, const double* T, int what) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    const int r = ln >> 3, e = ln & 7;
    const bool valid_r = r < RDIM(R, nrounds);
    const RoundDev rd = lds_round(s, valid_r ? r : 0);
    const double* st = s.rstate + kRoundState * (valid_r ? r : 0);
    const bool usable = valid_r && rd.link >= 0 && st[12] > kInvalidRound;
    const double* Tl = T + 12 * (rd.link >= 0 ? rd.link : 0);
    /* lane e: rotation entry kRot[e] (lane 0 also the ninth), translation entry e < 3 */
    const int ia = (e < 3) ? e : (e < 6 ? e + 1 : e + 2); /* 0 1 2 4 5 6 8 9 */
    const double da = Tl[ia] - st[ia];
    const double d9 = Tl[10] - st[10];
    const int it = 4 * (e < 3 ? e : 0) + 3;
    const double dt = Tl[it] - st[it];
    double f = da * da;
    if (e == 0) f = f + d9 * d9;
    double t = (e < 3) ? dt * dt : 0.0;
    f = f + dpp_f64<kDppXor1>(f);
    t = t + dpp_f64<kDppXor1>(t);
    f = f + dpp_f64<kDppXor2>(f);
    t = t + dpp_f64<kDppXor2>(t);
    f = f + dpp_f64<kDppHalfMirror>(f);
    t = t + dpp_f64<kDppHalfMirror>(t);
    const double bm = (sqrt_upper(t) + sqrt_upper(f) * rd.radius) * (1.0 + 1e-9) + 1e-12;
    /* an unmoved link: every difference exactly zero in the group (only looked at when the
     * bound is at its floor) */
    const bool eq = (da == 0.0) && (e != 0 || d9 == 0.0) && (e >= 3 || dt == 0.0);
    const uint64_t neq = __ballot(!eq);
    const bool still = ((neq >> (8 * r)) & 0xffull) == 0ull;
    const bool sk = usable && round_proof(A, st, bm, still, what);
    const uint64_t m = __ballot(sk && e == 0) & 0x0101010101010101ull;
    return (m * 0x0102040810204080ull) >> 56;
}

/* which rounds (bit r, r < 64) may skip the env check / the correction estimate at
 * transforms T; lane r evaluates round r */
__device__ __forceinline__ uint64_t skippable_rounds(Sim& s, const double* T, int what) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    if (FKS_NO_SKIP_PROOFS || !A.skip_enabled) return 0ull;
#if FKS_PAR_PROOF && defined(FKS_SHAPE_P) && FKS_SHAPE_TYPE == 0
    /* linked-robot shape builds of at most 8 rounds (cfg3: wave time -2.4 %; the SE(3) shape of
     * cfg4 ran 1.4 % slower with it, and generic builds keep one proof for every robot) */
    if constexpr ((FKS_SHAPE_P + kWave - 1) / kWave <= 8) return skippable_rounds8(s, T, what);
#endif
    bool sk = false;
    const int ln = s.lane();
    if (ln < RDIM(R, nrounds)) {
        const RoundDev rd = lds_round(s, ln);
        const double* st = s.rstate + kRoundState * ln;
        if (rd.link >= 0 && st[12] > kInvalidRound) {
            const double bm = rigid_motion_bound(T + 12 * rd.link, st, rd.radius);
            const double b = bm * A.sdf_g.inv_res; /* cells */
            const double K = 1.7320508075688773 * b + 3.0;
            const double Sr = st[12] * A.sdf_g.inv_res;
            const double lp = A.skip_lplus;
            const bool inb = st[13] - b > 1e-6;
            /* every point still in the cell it was evaluated in: nearest values unchanged.  The
             * bound says so unless a point sits within 1e-9 cells of a face; then only a link
             * that has not moved at all (e.g. a fixed base) keeps it there — which needs every
             * difference zero, so the bound is at its floor (1e-12) and only then is compared */
            bool same_cell = b < st[14] - 1e-9;
            if (!same_cell && bm <= 1e-12) {
                const double* Tl = T + 12 * rd.link;
                bool still = true;
#pragma unroll
                for (int e = 0; e < 12; ++e) still = still && (Tl[e] == st[e]);
                same_cell = still;
            }
            if (what == kSkipCheck)
                sk = (inb && (Sr - A.skip_cmax) > (K - 1.0) * lp + 1e-9) || (same_cell && st[12] >= A.thr_env);
            else
                sk = (inb && (Sr - A.skip_cmax) > K * lp + 1e-9 && (Sr - K * lp) > 0.5 + 1.5 * lp + 1e-6) ||
                     (same_cell && Sr > A.skip_cmax + 1e-9 && Sr > 0.5 + 1.5 * lp + 1e-6);
        }
    }
    return __ballot(sk);
}

/* minimum over the wave of a float (all 64 lanes active): DPP steps inside rows of 16 (folded
 * into v_min_f32), then the row pairs by v_permlane16/32_swap, read once from lane 0 */
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_min_f32(float v) {
    v = fminf(v, dpp_f32<kDppXor1>(v));
    v = fminf(v, dpp_f32<kDppXor2>(v));
    v = fminf(v, dpp_f32<kDppHalfMirror>(v));
    v = fminf(v, dpp_f32<kDppMirror>(v));
    const uint32_t b = (uint32_t)__float_as_int(v);
    const auto p16 = __builtin_amdgcn_permlane16_swap(b, b, false, false);
    v = fminf(__int_as_float((int)p16[0]), __int_as_float((int)p16[1]));
    const uint32_t c = (uint32_t)__float_as_int(v);
    const auto p32 = __builtin_amdgcn_permlane32_swap(c, c, false, false);
    v = fminf(__int_as_float((int)p32[0]), __int_as_float((int)p32[1]));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
/* a float no larger than x (x finite >= kInvalidRound, or +inf): the proofs use the cached
 * margins as lower bounds, so they are rounded down (by far more than the conversion's error) */
__device__ __forceinline__ float lower_f32(double x) {
    return (x < 3.0e38) ? (float)(x - (dabs(x) * 0x1p-20 + 0x1p-20)) : (float)x;
}

/* cache the state of round r after a full evaluation at T (uniform call).  The three minima
 * are taken in single precision: S is a float SDF value (exact; kInvalidRound becomes -inf,
 * which the validity tests treat alike), G and C are rounded down first.  Only skip decisions
 * read them, and those never change a result or a byte count (parity tests, counters). */
__device__ __forceinline__ void round_update(Sim& s, int r, const double* T, double S, double G, double C) {
    const SimArgs& A = *s.A;
    if (!A.skip_enabled || r >= kWave || r >= RDIM(A.R, nrounds)) return;
    const RoundDev rd = lds_round(s, r);
    if (rd.link < 0) return;
    const double smin = (double)wave_min_f32((float)S), gmin = (double)wave_min_f32(lower_f32(G)),
                 cmin = (double)wave_min_f32(lower_f32(C));
    double* st = s.rstate + kRoundState * r;
    if (s.lane() < 12) st[s.lane()] = T[12 * rd.link + s.lane()];
    if (s.lane() == 0) {
        st[12] = smin;
        st[13] = gmin;
        st[14] = cmin;
    }
}

/* EstimateMaxControlInputWorkspaceMotion over two transform sets (SPCS:1492-1527).
 * The result is the exact max over all points; rounds whose rigid-motion bound
 * cannot reach the max of the round with the largest bound are not evaluated. */
__device__ __forceinline__ double round_max_motion(const RobotDev& R, const double* TA, const double* TB, int r, int ln) {
    const int i = kWave * r + ln;
    if (i >= RDIM(R, P)) return 0.0;
    const D4 p = load_point(R, i);
    const int link = gp(R.point_link)[i];
    const D4 a = xform4(TA + 12 * link, p), b = xform4(TB + 12 * link, p);
    return sqnorm4(D4{b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w});
}
__device__ FKS_SHAPE_INLINE double max_point_motion(Sim& s, const double* TA, const double* TB) {
    const RobotDev& R = s.A->R;
    const int ln = s.lane();
    const int nr = RDIM(R, nrounds);
    double m = 0.0;
    if (FKS_NO_SKIP_PROOFS || nr <= 2 || nr > kWave) {
#pragma unroll 2
        for (int r = 0; r < nr; ++r) {
            const double sq = round_max_motion(R, TA, TB, r, ln);
            if (sq > m) m = sq;
        }
        return dsqrt(wave_max_nonneg(m));
    }
    double ub = 0.0;
    if (ln < nr) {
        const RoundDev rd = lds_round(s, ln);
        ub = (rd.link >= 0) ? rigid_motion_bound(TB + 12 * rd.link, TA + 12 * rd.link, rd.radius) : __builtin_huge_val();
    }
    const double top = wave_max_nonneg(ub);
    int rtop = __ffsll((unsigned long long)__ballot(ln < nr && ub == top)) - 1;
    if (rtop < 0) rtop = 0; /* non-finite transforms: evaluate every round */
    m = round_max_motion(R, TA, TB, rtop, ln);
    const double lower = wave_max_nonneg(m);
    uint64_t rest = __ballot(ln < nr && ln != rtop && !(ub * ub * (1.0 + 1e-9) < lower));
    while (rest) {
        const int r = __ffsll((unsigned long long)rest) - 1;
        rest &= rest - 1ull;
        const double sq = round_max_motion(R, TA, TB, r, ln);
        if (sq > m) m = sq;
    }
    return dsqrt(wave_max_nonneg(m));
}

/* one point of CheckEnvironmentCollision: nearest-cell read, then EstimateDistance4d
 * only where the nearest value cannot decide (SPCS:921-981, threshold 0).  Also
 * returns the nearest value S (-inf out of bounds) and the grid margin G in cells. */
__device__ __forceinline__ bool env_point(const SimArgs& A, const double* T, int i, uint64_t* b, double* S, double* G,
                                          double* C) {
    const RobotDev& R = A.R;
    if (i >= RDIM(R, P)) return false;
    const D4 p = load_point(R, i);
    const int link = gp(R.point_link)[i];
    const D4 x = xform4(T + 12 * link, p);
    const GridDev& g = A.sdf_g;
    const D4 q = xform4(g.inv, x);
    const double v[3] = {q.x * g.inv_res, q.y * g.inv_res, q.z * g.inv_res};
    int32_t idx[3];
    bool ok = true;
    double margin = __builtin_huge_val(), face = __builtin_huge_val();
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const bool fin = (v[a] > -2147483648.0) && (v[a] < 2147483647.0);
        idx[a] = fin ? (int32_t)v[a] : -1;
        ok = ok && fin && idx[a] >= 0 && (int64_t)idx[a] < g.n[a];
        margin = dmin(margin, dmin(v[a] + 1.0, (double)g.n[a] - v[a]));
        const double fr = v[a] - (double)idx[a];
        face = dmin(face, (v[a] >= 0.0) ? dmin(fr, 1.0 - fr) : 0.0);
    }
    float d = A.oob;
    if (ok) {
        d = gp(A.sdf)[grid_brick(g, idx[0], idx[1], idx[2])];
        *b += 4;
        *S = (double)d;
        *G = margin;
        *C = face;
    } else {
        *S = kInvalidRound;
        *G = kInvalidRound;
        *C = kInvalidRound;
    }
    const double thr = A.thr_env;
    if ((double)d < thr) {
        if ((double)d < thr - A.sdf_g.res) return true;
        bool inb;
        const double est = estimate_distance(A, x, &inb, b);
        if (est < thr) return true;
    }
    return false;
}

/* CheckEnvironmentCollision (SPCS:921-981) with threshold 0: two 64-point rounds are
 * evaluated together (their loads overlap), stopping after the pair holding the first
 * colliding point; algorithmic bytes are counted up to that point, as the reference
 * reads them (its loop returns at the first colliding point).  Provably-free rounds
 * are not read but still counted (4 B per point, all in bounds). */
template <bool GIVEN = false>
__device__ FKS_SHAPE_INLINE bool env_collision(Sim& s, const double* T, const uint64_t given = 0) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
#if defined(FKS_PROBE_PROOF_TWICE)
    /* A/B probe only: the proof evaluated twice (same answer), to measure what one costs */
    uint64_t skip = skippable_rounds(s, T, kSkipCheck);
    asm volatile("" ::: "memory");
    skip &= skippable_rounds(s, T, kSkipCheck) | skip;
#else
    const uint64_t skip = GIVEN ? given : skippable_rounds(s, T, kSkipCheck); /* GIVEN: the caller's proof */
#endif
    /* every round proven free (the common microstep): the reference reads 4 bytes per
     * point and finds nothing; account those reads without walking the rounds */
    if (RDIM(R, nrounds) <= kWave) {
        const uint64_t all = (RDIM(R, nrounds) == kWave) ? ~0ull : ((1ull << RDIM(R, nrounds)) - 1ull);
        if ((skip & all) == all) {
            if (s.lane() < RDIM(R, P)) s.lane_bytes += 4ull * (uint64_t)((RDIM(R, P) - s.lane() + kWave - 1) / kWave);
            count_event(s, FKS_PHASE_ENV_ROUNDS_SKIPPED, (uint64_t)RDIM(R, nrounds));
            return false;
        }
    }
    for (int base = 0, r = 0; base < RDIM(R, P); base += 2 * kWave, r += 2) {
        const bool sk0 = r < kWave && ((skip >> r) & 1ull);
        const bool sk1 = r + 1 < kWave && ((skip >> (r + 1)) & 1ull);
        uint64_t b0 = 0, b1 = 0;
        double S0 = __builtin_huge_val(), S1 = __builtin_huge_val(), G0 = __builtin_huge_val(), G1 = __builtin_huge_val();
        double C0 = __builtin_huge_val(), C1 = __builtin_huge_val();
        bool c0 = false, c1 = false;
        const int i0 = base + s.lane(), i1 = base + kWave + s.lane();
        if (sk0)
            b0 = (i0 < RDIM(R, P)) ? 4 : 0;
        else
            c0 = env_point(A, T, i0, &b0, &S0, &G0, &C0);
        if (sk1)
            b1 = (i1 < RDIM(R, P)) ? 4 : 0;
        else
            c1 = env_point(A, T, i1, &b1, &S1, &G1, &C1);
        if (!sk0) round_update(s, r, T, S0, G0, C0);
        if (!sk1 && base + kWave < RDIM(R, P)) round_update(s, r + 1, T, S1, G1, C1);
        count_event(s, FKS_PHASE_ENV_ROUNDS_SKIPPED, (sk0 ? 1 : 0) + ((sk1 && base + kWave < RDIM(R, P)) ? 1 : 0));
        count_event(s, FKS_PHASE_ENV_ROUNDS_EVALUATED, (sk0 ? 0 : 1) + ((!sk1 && base + kWave < RDIM(R, P)) ? 1 : 0));
        const uint64_t m0 = __ballot(c0);
        const uint64_t m1 = __ballot(c1);
        if (m0) {
            const int first = __ffsll((unsigned long long)m0) - 1;
            if (s.lane() <= first) s.lane_bytes += b0;
            return true;
        }
        s.lane_bytes += b0;
        if (m1) {
            const int first = __ffsll((unsigned long long)m1) - 1;
            if (s.lane() <= first) s.lane_bytes += b1;
            return true;
        }
        s.lane_bytes += b1;
    }
    return false;
}

/* ---- cooperative small batches (COOP waves per particle) ----
 * A batch far smaller than the resident grid is the latency of its slowest particle, a chain
 * of dependent memory round trips that one wave runs alone.  The cooperative kernels give each
 * particle a workgroup of COOP waves: wave 0 (the leader) runs the particle as every other
 * kernel does; where an environment check or a correction pass has two or more rounds left
 * after the skip proofs, it hands them out, one per wave, through a mailbox (CoopBox) behind its
 * LDS block, with a workgroup barrier to start them and one to collect them (a check with one
 * round left runs as in the other kernels).  Results are the sequential loop's bit for bit:
 * each round is evaluated by the same code, the first colliding point and the byte count of an
 * environment check are resolved in round order by the leader, and correction rows are placed
 * by a prefix sum of the rounds' row counts, in the sequential order. */
#ifndef FKS_COOP_WAVES
#define FKS_COOP_WAVES 8 /* fksd::kCoopWaves (the host reads a build's value from the kernel's launch bound) */
#endif
static_assert(FKS_COOP_WAVES >= 2 && FKS_COOP_WAVES <= kMaxCoopWaves, "cooperative workgroups hold 2..8 waves");
enum { kCoopExit = 0, kCoopEnv = 1, kCoopCorr = 2 };
__device__ __forceinline__ CoopBox* coop_box(const Sim& s) {
    return reinterpret_cast<CoopBox*>(s.lds() + LAY(*s.A).total); /* behind the leader's block */
}
__device__ __forceinline__ void coop_sync() { __syncthreads(); }
/* the k-th set bit of m (-1 if fewer) */
__device__ __forceinline__ int nth_bit(uint64_t m, int k) {
    for (int j = 0; j < k && m; ++j) m &= m - 1ull;
    return m ? __ffsll((unsigned long long)m) - 1 : -1;
}
/* points of 64-point round r */
__device__ __forceinline__ uint32_t round_points(int P, int r) {
    const int left = P - r * kWave;
    return (uint32_t)(left < kWave ? left : kWave);
}

/* wave w's share of a cooperative environment check: the work rounds of rank w, w + COOP, ... */
template <int COOP>
__device__ __forceinline__ void env_coop_share(Sim& s, CoopBox* box, int w) {
    const SimArgs& A = *s.A;
    const int ln = s.lane();
    const double* T = s.lds() + box->tc_off;
    const uint64_t work = box->work;
    for (int k = w;; k += COOP) {
        const int r = nth_bit(work, k);
        if (r < 0) break;
        uint64_t b = 0;
        double S = __builtin_huge_val(), G = __builtin_huge_val(), C = __builtin_huge_val();
        const bool c = env_point(A, T, r * kWave + ln, &b, &S, &G, &C);
        round_update(s, r, T, S, G, C);
        const uint64_t m = __ballot(c);
        const int first = m ? __ffsll((unsigned long long)m) - 1 : kWave;
        const uint64_t bytes = wave_sum_u64((ln <= first) ? b : 0ull);
        if (ln == 0) {
            box->cnt[r] = (uint32_t)bytes;
            if (m) __hip_atomic_fetch_or(&box->cmask, 1ull << r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

/* CheckEnvironmentCollision (SPCS:921-981) over the particle's COOP waves (leader side): the
 * verdict and the bytes of env_collision, the first colliding point in point order deciding
 * both (its bytes go to lane 0: only their sum over the wave is ever read) */
template <int COOP>
__device__ FKS_SHAPE_INLINE bool env_collision_coop(Sim& s, const double* T) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int nr = RDIM(R, nrounds);
    const uint64_t skip = skippable_rounds(s, T, kSkipCheck);
    const uint64_t all = (nr == kWave) ? ~0ull : ((1ull << nr) - 1ull);
    const uint64_t work = all & ~skip;
    if (__popcll(work) < 2) return env_collision<true>(s, T, skip);
    CoopBox* box = coop_box(s);
    if (s.lane() == 0) {
        box->cmd = kCoopEnv;
        box->tc_off = (uint32_t)(T - s.lds());
        box->work = work;
        box->cmask = 0;
    }
    coop_sync();
    env_coop_share<COOP>(s, box, 0);
    coop_sync();
    const uint64_t cm = box->cmask;
    const int rc = cm ? __ffsll((unsigned long long)cm) - 1 : nr - 1; /* the last round counted */
    const uint64_t upto = (rc >= 63) ? ~0ull : ((2ull << rc) - 1ull);
    /* proven rounds: 4 bytes per point (in bounds, as env_collision counts them) */
    const uint64_t proven = all & skip & upto;
    uint64_t bytes = 4ull * (uint64_t)__popcll(proven) * kWave;
    if ((proven >> (nr - 1)) & 1ull) bytes -= 4ull * (uint64_t)(kWave - round_points(RDIM(R, P), nr - 1));
    for (uint64_t m = work & upto; m; m &= m - 1ull) bytes += box->cnt[__ffsll((unsigned long long)m) - 1];
    if (s.lane() == 0) s.lane_bytes += bytes;
    count_event(s, FKS_PHASE_ENV_ROUNDS_SKIPPED, (uint64_t)__popcll(proven));
    count_event(s, FKS_PHASE_ENV_ROUNDS_EVALUATED, (uint64_t)__popcll(work & upto));
    return cm != 0ull;
}

/* ---------------- self-collision (SPCS:983-1275) ---------------- */
/* dense helpers on one lane (oracle Dense matmul / Gauss-Jordan inverse) */
__device__ void dense_matmul(const double* A, int ar, int ac, const double* B, int bc, double* C) {
    for (int i = 0; i < ar; ++i)
        for (int j = 0; j < bc; ++j) {
            double acc = 0.0;
            for (int k = 0; k < ac; ++k) acc = acc + A[i * ac + k] * B[k * bc + j];
            C[i * bc + j] = acc;
        }
}
__device__ void dense_transpose(const double* A, int r, int c, double* T) {
    for (int i = 0; i < r; ++i)
        for (int j = 0; j < c; ++j) T[j * r + i] = A[i * c + j];
}
__device__ void dense_inverse(const double* A, int n, double* aug, double* inv) {
    const int w = 2 * n;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < w; ++j) aug[i * w + j] = (j < n) ? A[i * n + j] : ((j - n == i) ? 1.0 : 0.0);
    for (int c = 0; c < n; ++c) {
        int p = c;
        double best = dabs(aug[c * w + c]);
        for (int r = c + 1; r < n; ++r)
            if (dabs(aug[r * w + c]) > best) {
                best = dabs(aug[r * w + c]);
                p = r;
            }
        if (p != c)
            for (int j = 0; j < w; ++j) {
                const double t = aug[c * w + j];
                aug[c * w + j] = aug[p * w + j];
                aug[p * w + j] = t;
            }
        const double piv = aug[c * w + c];
        for (int j = 0; j < w; ++j) aug[c * w + j] = aug[c * w + j] / piv;
        for (int r = 0; r < n; ++r) {
            if (r == c) continue;
            const double f = aug[r * w + c];
            for (int j = 0; j < w; ++j) aug[r * w + j] = aug[r * w + j] - f * aug[c * w + j];
        }
    }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) inv[i * n + j] = aug[i * w + n + j];
}

/* ExtractSelfCollidingPoints for one cell on lane 0.  members: point indices of
 * the cell in ascending order.  Writes corrections + flags into scratch; returns
 * true if the cell is a colliding cell (link_collisions.size() >= 2). */
__device__ __noinline__ uint32_t extract_cell(const SimArgs* __restrict__ Ap, double* scratch, const double* Tp, const double* Tc,
                                              const int32_t* members, int nm, uint32_t* cells) {
    const SimArgs& A = *Ap;
    uint32_t err = 0;
    const RobotDev& R = A.R;
    const ScratchLayout& SL = A.SL;
    double* corr = scratch + SL.corr;
    double* flag = scratch + SL.flag;
    double* dense = scratch + SL.dense;
    if (nm <= 1) return 0;
    /* by_link: geometries present (ascending), ranges into members.  The per-cell tables
     * live in the wave's global workspace, not in private arrays: private arrays become
     * per-lane scratch of the whole kernel, and scratch size limits the waves in flight */
    int32_t* geo = reinterpret_cast<int32_t*>(scratch + SL.cellw);
    int32_t* gbeg = geo + kMaxGeoms;
    int32_t* gend = gbeg + kMaxGeoms;
    int32_t* others = gend + kMaxGeoms;
    D4* mom = reinterpret_cast<D4*>(scratch + SL.cellw + 2 * kMaxGeoms);
    int ng = 0;
    for (int m = 0; m < nm; ++m) {
        const int g = gp(R.point_geom)[members[m]];
        if (ng == 0 || geo[ng - 1] != g) {
            if (ng == kMaxGeoms) break;
            geo[ng] = g;
            gbeg[ng] = m;
            ng++;
        }
        gend[ng - 1] = m + 1;
    }
    if (ng < 2) return 0;
    /* link_collisions: for each present geometry, the present geometries it may not touch */
    uint64_t present = 0;
    for (int a = 0; a < ng; ++a) present |= 1ull << geo[a];
    int ncollide_links = 0;
    for (int a = 0; a < ng; ++a) {
        const uint64_t disallowed = present & ~gp(R.allowed_mask)[geo[a]] & ~(1ull << geo[a]);
        if (disallowed) ncollide_links++;
    }
    if (ncollide_links < 2) return 0;
    (*cells)++;
    const double tm = A.time_multiplier;
    for (int a = 0; a < ng; ++a) {
        const uint64_t disallowed = present & ~gp(R.allowed_mask)[geo[a]] & ~(1ull << geo[a]);
        mom[a] = D4{0.0, 0.0, 0.0, 0.0};
        if (!disallowed) continue;
        const int link = gp(R.geom_link)[geo[a]];
        for (int m = gbeg[a]; m < gend[a]; ++m) {
            const D4 p = load_point(R, members[m]);
            const D4 pv = xform4(Tp + 12 * link, p), cv = xform4(Tc + 12 * link, p);
            const D4 vel{(cv.x - pv.x) * tm, (cv.y - pv.y) * tm, (cv.z - pv.z) * tm, (cv.w - pv.w) * tm};
            mom[a] = D4{mom[a].x + vel.x, mom[a].y + vel.y, mom[a].z + vel.z, mom[a].w + vel.w};
        }
    }
    for (int a = 0; a < ng; ++a) {
        const uint64_t disallowed = present & ~gp(R.allowed_mask)[geo[a]] & ~(1ull << geo[a]);
        if (!disallowed) continue;
        int n = 0;
        for (int b = 0; b < ng; ++b)
            if ((disallowed >> geo[b]) & 1ull) others[n++] = b;
        const int link = gp(R.geom_link)[geo[a]];
        const D4 link_loc = xform4(Tp + 12 * link, load_point(R, members[gbeg[a]]));
        const double cnt = (double)(gend[a] - gbeg[a]);
        const D4 link_vel{mom[a].x / cnt, mom[a].y / cnt, mom[a].z / cnt, mom[a].w / cnt};
        const int rows = (n + 1) * 3, ccols = n * 3;
        double* C = dense;                     /* rows x ccols */
        double* N = C + rows * ccols;          /* ccols x n */
        double* M = N + ccols * n;             /* rows x rows */
        double* V = M + rows * rows;           /* rows */
        double* Nt = V + rows;                 /* n x ccols */
        double* Ct = Nt + n * ccols;           /* ccols x rows */
        double* Minv = Ct + ccols * rows;      /* rows x rows */
        double* T1 = Minv + rows * rows;       /* work */
        double* T2 = T1 + rows * rows;
        double* aug = T2 + rows * rows;
        for (int k = 0; k < rows * ccols; ++k) C[k] = 0.0;
        for (int l = 1; l <= n; ++l)
            for (int d = 0; d < 3; ++d) {
                C[d * ccols + (l - 1) * 3 + d] = -1.0;
                C[(l * 3 + d) * ccols + (l - 1) * 3 + d] = 1.0;
            }
        for (int k = 0; k < ccols * n; ++k) N[k] = 0.0;
        for (int c = 0; c < n; ++c) {
            const int ob = others[c];
            const int olink = gp(R.geom_link)[geo[ob]];
            const D4 oloc = xform4(Tp + 12 * olink, load_point(R, members[gbeg[ob]]));
            const D4 cn = safe_normal4(D4{oloc.x - link_loc.x, oloc.y - link_loc.y, oloc.z - link_loc.z, oloc.w - link_loc.w});
            N[(c * 3 + 0) * n + c] = cn.x;
            N[(c * 3 + 1) * n + c] = cn.y;
            N[(c * 3 + 2) * n + c] = cn.z;
        }
        for (int k = 0; k < rows * rows; ++k) M[k] = 0.0;
        const double lm = gp(R.geom_mass)[geo[a]];
        for (int d = 0; d < 3; ++d) M[d * rows + d] = lm;
        for (int l = 1; l <= n; ++l) {
            const double om = gp(R.geom_mass)[geo[others[l - 1]]];
            for (int d = 0; d < 3; ++d) M[(l * 3 + d) * rows + (l * 3 + d)] = om;
        }
        V[0] = link_vel.x;
        V[1] = link_vel.y;
        V[2] = link_vel.z;
        for (int l = 1; l <= n; ++l) {
            const int ob = others[l - 1];
            const double oc = (double)(gend[ob] - gbeg[ob]);
            V[l * 3 + 0] = mom[ob].x / oc;
            V[l * 3 + 1] = mom[ob].y / oc;
            V[l * 3 + 2] = mom[ob].z / oc;
        }
        dense_transpose(N, ccols, n, Nt);
        dense_transpose(C, rows, ccols, Ct);
        dense_inverse(M, rows, aug, Minv);
        /* A = Nt*Ct*Minv*C*N (left to right) */
        dense_matmul(Nt, n, ccols, Ct, rows, T1);     /* n x rows */
        dense_matmul(T1, n, rows, Minv, rows, T2);    /* n x rows */
        dense_matmul(T2, n, rows, C, ccols, T1);      /* n x ccols */
        dense_matmul(T1, n, ccols, N, n, T2);         /* n x n */
        double* Ainv = T1 + rows * rows;              /* beyond T1 usage: reuse aug tail */
        Ainv = aug + 2 * rows * rows;
        dense_inverse(T2, n, aug, Ainv);
        /* impulses = Ainv*Nt*Ct*V */
        dense_matmul(Ainv, n, n, Nt, ccols, T1);      /* n x ccols */
        dense_matmul(T1, n, ccols, Ct, rows, T2);     /* n x rows */
        double* imp = Ainv + n * n;
        dense_matmul(T2, n, rows, V, 1, imp);         /* n x 1 */
        /* dv = (Minv*C*N*imp) * -1 */
        dense_matmul(Minv, rows, rows, C, ccols, T1); /* rows x ccols */
        dense_matmul(T1, rows, ccols, N, n, T2);      /* rows x n */
        double* dv = imp + n;
        dense_matmul(T2, rows, n, imp, 1, dv);        /* rows x 1 */
        const D3 corr3{dv[0] * -1.0, dv[1] * -1.0, dv[2] * -1.0};
        const double np = cnt;
        for (int m = gbeg[a]; m < gend[a]; ++m) {
            const D3 pc{corr3.x / np, corr3.y / np, corr3.z / np};
            if (pc.x != pc.x || pc.y != pc.y || pc.z != pc.z) err |= FKS_PARTICLE_ERR_SELF_SINGULAR;
            const int pi = members[m];
            corr[3 * pi + 0] = pc.x;
            corr[3 * pi + 1] = pc.y;
            corr[3 * pi + 2] = pc.z;
            flag[pi] = 1.0;
        }
    }
    return err;
}

__device__ __noinline__ uint32_t self_collisions_exact(const SimArgs* __restrict__ Ap, double* lds, double* scratch, int ln,
                                                       uint32_t err, const double* Tp, const double* Tc);

/* CollectSelfCollisions: returns whether the self-collision map is non-empty */
__device__ FKS_SHAPE_INLINE bool self_collisions(Sim& s, const double* Tp, const double* Tc, const double* q) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    if (!RDIM(R, self_possible)) return false;
#if defined(FKS_PROBE_NO_SELF)
    return false; /* A/B probe only: what the self-collision check costs (results may change) */
#endif
    /* Skip proof (a cheaper route to the fast path's "no box pair overlaps").  At the last full
     * evaluation, with configuration qref, every disallowed pair was separated along some axis
     * by gap >= 1 cells.  Since then every point of every geometry's local box has moved by at
     * most mu = sum_d |q_d - qref_d| * lever_box_d (joint motion along the straight path in
     * joint space; wrapping and clamping only shorten it); the world AABB of a moved box lies in
     * the old one grown by mu per side, the grid transform is rigid, and truncation moves each
     * integer bound by at most mu / res + 2 cells.  So gap - 2 mu / res - 4 >= 1 keeps every
     * pair apart: the fast path's answer (no self-collision) without building the boxes. */
    double* ref = s.selfref;
    const int D = RDIM(R, D);
    const double gap = readfirstlane_f64(ref[D]);
    if (!FKS_NO_SKIP_PROOFS && gap >= 6.0) {
        const double term = (ln < D) ? dabs(q[ln] - ref[ln]) * gp(R.dof_lever_box)[ln] : 0.0;
        const double mu = bfly_sum(0.0 + term) * (1.0 + 1e-6) + 1e-12;
        if (2.0 * mu * A.env_g.inv_res + 5.0 <= gap) return false;
    }
    double* box = s.lds() + LAY(*s.A).box;
    bool bad = false;
    if (ln < RDIM(R, G)) {
        const double* gb = s.shared() + LAY(A).gbox + 8 * ln;
        const int link = (int)gb[7];
        const double* T = Tc + 12 * link;
        double lo[3], hi[3];
        if (gb[6] != 0.0) {
            const D3 wc = xform3(T, D3{gb[0], gb[1], gb[2]});
            double wh[3];
            for (int i = 0; i < 3; ++i)
                wh[i] = (dabs(T[4 * i]) * gb[3] + dabs(T[4 * i + 1]) * gb[4]) + dabs(T[4 * i + 2]) * gb[5];
            const D3 gc = xform3(A.env_g.inv, wc);
            const double gcv[3] = {gc.x, gc.y, gc.z};
            for (int i = 0; i < 3; ++i) {
                const double* Ir = A.env_g.inv + 4 * i;
                const double gh = (dabs(Ir[0]) * wh[0] + dabs(Ir[1]) * wh[1]) + dabs(Ir[2]) * wh[2];
                /* conservative box: the margin (>= 1e-6 m) dwarfs the rounding of a
                 * multiplication by 1/res instead of the exact pass's division */
                const double margin = 1e-6 + 1e-9 * (dabs(gcv[i]) + gh);
                const double l = (gcv[i] - gh - margin) * A.env_g.inv_res;
                const double h = (gcv[i] + gh + margin) * A.env_g.inv_res;
                if (!(l > -1e18 && l < 1e18 && h > -1e18 && h < 1e18)) bad = true;
                lo[i] = __builtin_trunc(l);
                hi[i] = __builtin_trunc(h);
            }
        } else {
            bad = true;
        }
        if (bad) {
            for (int i = 0; i < 3; ++i) {
                lo[i] = -__builtin_huge_val();
                hi[i] = __builtin_huge_val();
            }
        }
        for (int i = 0; i < 3; ++i) {
            box[6 * ln + i] = lo[i];
            box[6 * ln + 3 + i] = hi[i];
        }
    }
    wsync();
    bool any = false;
    double gmin = __builtin_huge_val();
    const uint32_t* lpairs = reinterpret_cast<const uint32_t*>(s.shared() + LAY(A).gpairs);
    for (int k = ln; k < RDIM(R, npairs); k += kWave) {
        int a, b;
        if (k < kLdsPairs) {
            const uint32_t ab = lpairs[k];
            a = (int)(ab & 0xffffu);
            b = (int)(ab >> 16);
        } else {
            a = gp(R.pairs)[2 * k];
            b = gp(R.pairs)[2 * k + 1];
        }
        bool ov = true;
        double sep = -__builtin_huge_val(); /* the pair's largest separation over the axes (cells) */
        for (int i = 0; i < 3; ++i) {
            const double la = box[6 * a + i], ha = box[6 * a + 3 + i], lb = box[6 * b + i], hb = box[6 * b + 3 + i];
            ov = ov && (la <= hb) && (lb <= ha);
            sep = dmax(sep, dmax(lb - ha, la - hb));
        }
        any = any || ov;
        gmin = dmin(gmin, sep);
    }
    /* the new reference: this configuration and the smallest separation (-inf if a box was not
     * finite: no proof until the next full evaluation) */
    const float gw = wave_min_f32(wave_any(bad) ? -__builtin_inff() : lower_f32(gmin));
    if (ln < D) ref[ln] = q[ln];
    if (ln == 0) ref[D] = (double)gw;
    wsync();
    if (!wave_any(any || bad)) return false;
    const uint32_t r = self_collisions_exact(s.A, s.lds(), s.scratch, ln, s.err, Tp, Tc);
    s.err = r >> 1;
    return (r & 1u) != 0u;
}

/* exact extended-cell comparison for geometry pairs whose boxes overlap, then the
 * impulse solve of every colliding cell (out of line: rare) */
__device__ __noinline__ uint32_t self_collisions_exact(const SimArgs* __restrict__ Ap, double* lds, double* scratch, int ln,
                                                       uint32_t err, const double* Tp, const double* Tc) {
    const SimArgs& A = *Ap;
    const RobotDev& R = A.R;
    const double* box = lds + LAY(A).box;
    /* exact path: extended cell keys (SPCS:1173-1181: division, trunc).  The keys are
     * needed for the points of the geometries in a box-overlapping pair; every other
     * point's key only matters once some cell is shared, so it is computed then. */
    const ScratchLayout& SL = A.SL;
    int64_t* keys = reinterpret_cast<int64_t*>(scratch + SL.keys);
    double* flag = scratch + SL.flag;
    double* cand = scratch + SL.cand;
    int32_t* list = reinterpret_cast<int32_t*>(scratch + SL.list);
    int32_t* listb = list + RDIM(R, P); /* second half of the list region: one pair's b points */
    auto key_point = [&](int i) {
        const D4 p = load_point(R, i);
        const int link = gp(R.point_link)[i];
        const D4 x = xform4(Tc + 12 * link, p);
        const D4 g = xform4(A.env_g.inv, x);
        const double q[3] = {g.x / A.env_g.res, g.y / A.env_g.res, g.z / A.env_g.res};
        for (int a = 0; a < 3; ++a) {
            int64_t k;
            if (q[a] != q[a] || q[a] == __builtin_huge_val() || q[a] == -__builtin_huge_val()) {
                err |= FKS_PARTICLE_ERR_KEY_RANGE;
                k = 0;
            } else if (q[a] >= 9.0e18) {
                k = (int64_t)9000000000000000000ll;
            } else if (q[a] <= -9.0e18) {
                k = -(int64_t)9000000000000000000ll;
            } else {
                k = (int64_t)q[a];
            }
            keys[3 * i + a] = k;
        }
        flag[i] = 0.0;
        cand[i] = 0.0;
    };
    /* a point's key lies in geometry g's conservative cell box (self_collisions) */
    auto in_box = [&](int i, int g) {
        bool in = true;
        for (int a = 0; a < 3; ++a) {
            const double k = (double)keys[3 * i + a];
            in = in && box[6 * g + a] <= k && k <= box[6 * g + 3 + a];
        }
        return in;
    };
    auto overlap = [&](int a, int b) {
        bool ov = true;
        for (int i = 0; i < 3; ++i) ov = ov && (box[6 * a + i] <= box[6 * b + 3 + i]) && (box[6 * b + i] <= box[6 * a + 3 + i]);
        return ov;
    };
    /* geometries of the overlapping pairs; every geometry when a box is not finite (the
     * key-range error is then raised exactly as a pass over all points would) */
    const bool unbounded = wave_any(ln < RDIM(R, G) && !(box[6 * ln] > -__builtin_huge_val()));
    uint64_t need = 0ull;
    for (int k0 = 0; k0 < RDIM(R, npairs); k0 += kWave) {
        const int k = k0 + ln;
        int a = 0, b = 0;
        bool ov = false;
        if (k < RDIM(R, npairs)) {
            a = gp(R.pairs)[2 * k];
            b = gp(R.pairs)[2 * k + 1];
            ov = overlap(a, b);
        }
        uint64_t m = __ballot(ov);
        while (m) {
            const int bit = __ffsll((unsigned long long)m) - 1;
            m &= m - 1ull;
            need |= (1ull << readlane_i32(a, bit)) | (1ull << readlane_i32(b, bit));
        }
    }
    uint64_t done = 0ull;
    for (int g = 0; g < RDIM(R, G); ++g) {
        if (!unbounded && !((need >> g) & 1ull)) continue;
        done |= 1ull << g;
        for (int i = (int)gp(R.geom_off)[g] + ln; i < (int)gp(R.geom_off)[g + 1]; i += kWave) key_point(i);
    }
    wsync();
    /* exact candidate marking over pairs whose boxes overlap: a point of a can share a
     * cell only with the points of b whose keys lie in a's box (and only if its own key
     * lies in b's box), so b's points are first compacted to that list */
    bool any_cand = false;
    for (int k = 0; k < RDIM(R, npairs); ++k) {
        const int a = gp(R.pairs)[2 * k], b = gp(R.pairs)[2 * k + 1];
        if (!overlap(a, b)) continue;
        const int a0 = (int)gp(R.geom_off)[a], a1 = (int)gp(R.geom_off)[a + 1];
        const int b0 = (int)gp(R.geom_off)[b], b1 = (int)gp(R.geom_off)[b + 1];
        int nb = 0;
        for (int j0 = b0; j0 < b1; j0 += kWave) {
            const int j = j0 + ln;
            const bool in = j < b1 && in_box(j, a);
            const uint64_t mm = __ballot(in);
            if (in) listb[nb + __popcll(mm & ((1ull << ln) - 1ull))] = j;
            nb += __popcll(mm);
        }
        if (nb == 0) continue;
        wsync();
        for (int i = a0 + ln; i < a1; i += kWave) {
            if (!in_box(i, b)) continue;
            const int64_t kx = keys[3 * i], ky = keys[3 * i + 1], kz = keys[3 * i + 2];
            bool hit = false;
            for (int t = 0; t < nb && !hit; ++t) {
                const int j = listb[t];
                hit = (keys[3 * j] == kx) && (keys[3 * j + 1] == ky) && (keys[3 * j + 2] == kz);
            }
            if (hit) {
                cand[i] = 1.0;
                any_cand = true;
            }
        }
        wsync();
    }
    if (!wave_any(any_cand)) {
        err = wave_or(err);
        return err << 1;
    }
    /* some cell is shared: the cell members below come from every point */
    for (int g = 0; g < RDIM(R, G); ++g) {
        if ((done >> g) & 1ull) continue;
        for (int i = (int)gp(R.geom_off)[g] + ln; i < (int)gp(R.geom_off)[g + 1]; i += kWave) key_point(i);
    }
    wsync();
    /* process each candidate cell once */
    uint32_t* ui = reinterpret_cast<uint32_t*>(reinterpret_cast<int32_t*>(lds + LAY(A).ints) + 2 * kMaxDofs); /* spare int words */
    if (ln == 0) {
        ui[0] = 0; /* colliding cells */
        ui[1] = 0; /* any corrected point */
    }
    wsync();
    for (int base = 0; base < RDIM(R, P); base += kWave) {
        const int i0 = base + ln;
        uint64_t m = __ballot(i0 < RDIM(R, P) && cand[i0] != 0.0);
        while (m) {
            const int bit = __ffsll((unsigned long long)m) - 1;
            m &= m - 1ull;
            const int ci = base + bit;
            if (cand[ci] == 0.0) continue; /* already consumed by an earlier cell (uniform read) */
            const int64_t kx = keys[3 * ci], ky = keys[3 * ci + 1], kz = keys[3 * ci + 2];
            /* members of the cell in point order */
            int count = 0;
            for (int b2 = 0; b2 < RDIM(R, P); b2 += kWave) {
                const int j = b2 + ln;
                const bool in = j < RDIM(R, P) && keys[3 * j] == kx && keys[3 * j + 1] == ky && keys[3 * j + 2] == kz;
                const uint64_t mm = __ballot(in);
                if (in) {
                    const int rank = __popcll(mm & ((1ull << ln) - 1ull));
                    list[count + rank] = j;
                    cand[j] = 0.0;
                }
                count += __popcll(mm);
            }
            wsync();
            if (ln == 0) {
                err |= extract_cell(Ap, scratch, Tp, Tc, list, count, ui);
            }
            wsync();
        }
    }
    bool nonempty = false;
    for (int i = ln; i < RDIM(R, P); i += kWave) nonempty = nonempty || (flag[i] != 0.0);
    err = wave_or(err);
    return (err << 1) | (wave_any(nonempty) ? 1u : 0u);
}

/* CheckCollision (SPCS:1418-1436) */
template <int RT, int COOP = 0>
__device__ FKS_SHAPE_INLINE bool check_collision(Sim& s, const double* Tp, const double* Tc, const double* q) {
    uint64_t t0 = tick();
    bool env;
    if constexpr (COOP > 0)
        env = env_collision_coop<COOP>(s, Tc);
    else
        env = env_collision(s, Tc);
    tock(s, FKS_PHASE_ENV_CHECK, t0);
    bool self = false;
    if constexpr (RT == FKS_ROBOT_LINKED) {
        t0 = tick();
        self = self_collisions(s, Tp, Tc, q);
        tock(s, FKS_PHASE_SELF_CHECK, t0);
    }
    s.self_nonempty = self;
    if (self && s.lane() == 0) self_counters(s)[0]++;
    return env || self;
}

/* world joint axes/origins per dof for the Jacobian (linked robots) */
template <int RT>
__device__ FKS_SHAPE_INLINE void joint_frames(Sim& s, const double* Tc) {
    const RobotDev& R = s.A->R;
    const int ln = s.lane();
    if (RT == FKS_ROBOT_LINKED && ln < RDIM(R, D)) {
        const JointDev& jd = s.joints()[s.dofj()[ln]];
        const double* Tch = Tc + 12 * jd.child;
        const D3 aw = rotate(Tch, D3{jd.axis[0], jd.axis[1], jd.axis[2]});
        double* axw = s.lds() + LAY(*s.A).axis_w;
        double* orw = s.lds() + LAY(*s.A).orig_w;
        axw[3 * ln + 0] = aw.x;
        axw[3 * ln + 1] = aw.y;
        axw[3 * ln + 2] = aw.z;
        orw[3 * ln + 0] = Tch[3];
        orw[3 * ln + 1] = Tch[7];
        orw[3 * ln + 2] = Tch[11];
    }
    wsync();
}

/* CollectPointCorrectionsAndJacobians (SPCS:1818-1939): rows written to scratch, returns R
 * (GIVEN: the caller has put the joint frames in LDS and proven the rounds in `given`) */
template <int RT, bool GIVEN = false>
__device__ FKS_SHAPE_INLINE uint32_t collect_corrections(Sim& s, const double* Tp, const double* Tc, const double* cfg,
                                                         const uint64_t given = 0) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    const int D = RDIM(R, D);
    const ScratchLayout& SL = A.SL;
    FKS_GLOBAL double* J = gpw(s.scratch) + SL.J;
    FKS_GLOBAL double* bv = gpw(s.scratch) + SL.b;
    const FKS_GLOBAL double* corr = gp(s.scratch) + SL.corr;
    const FKS_GLOBAL double* flag = gp(s.scratch) + SL.flag;
    const uint32_t rc = ROWCAP(A);
    if constexpr (!GIVEN) joint_frames<RT>(s, Tc);
    const double* axw = s.lds() + LAY(*s.A).axis_w;
    const double* orw = s.lds() + LAY(*s.A).orig_w;
    uint32_t rows = 0;
    /* rounds that provably hold no corrected point: their EstimateDistance reads are
     * counted (28 B per point, in bounds) but not made */
    const uint64_t skip = GIVEN ? given : skippable_rounds(s, Tc, kSkipCorrections);
    for (int base = 0; base < RDIM(R, P); base += kWave) {
        const int i = base + ln;
        const int r = base / kWave;
        const bool skr = r < kWave && ((skip >> r) & 1ull);
        count_event(s, skr ? FKS_PHASE_CORR_ROUNDS_SKIPPED : FKS_PHASE_CORR_ROUNDS_EVALUATED, 1);
        if (skr && !s.self_nonempty) {
            if (i < RDIM(R, P)) s.lane_bytes += 28;
            continue;
        }
        bool has = false;
        D3 pcorr{0.0, 0.0, 0.0};
        D4 xc{0.0, 0.0, 0.0, 0.0};
        int link = 0;
        if (i < RDIM(R, P)) {
            const D4 p = load_point(R, i);
            link = gp(R.point_link)[i];
            xc = xform4(Tc + 12 * link, p);
            const bool has_self = s.self_nonempty && flag[i] != 0.0;
            bool inb = false;
            double est = 0.0;
            if (skr)
                s.lane_bytes += 28;
            else
                est = estimate_distance(A, xc, &inb, &s.lane_bytes);
            const bool has_env = (est < 0.0) && inb;
            D3 ecorr{0.0, 0.0, 0.0};
            if (has_env) {
                const D4 xp = xform4(Tp + 12 * link, p);
                const D4 motion{xc.x - xp.x, xc.y - xp.y, xc.z - xp.z, xc.w - xp.w};
                const D4 nm = safe_normal4(motion);
                D3 raw;
                const bool ok = lookup_normal(A, xc, nm, &raw, &s.err, &s.lane_bytes);
                if (!ok) s.err |= FKS_PARTICLE_ERR_NORMAL_OOB;
                const D3 g = safe_normal3(raw);
                const double pen = dabs(0.0 - est);
                ecorr = D3{g.x * pen, g.y * pen, g.z * pen};
            }
            has = has_self || has_env;
            if (has_self) pcorr = D3{pcorr.x + corr[3 * i], pcorr.y + corr[3 * i + 1], pcorr.z + corr[3 * i + 2]};
            if (has_env) pcorr = D3{pcorr.x + ecorr.x, pcorr.y + ecorr.y, pcorr.z + ecorr.z};
        }
        const uint64_t m = __ballot(has);
        if (s.self_nonempty) {
            const uint64_t k = (uint64_t)__popcll(__ballot(has && flag[i] != 0.0));
            if (ln == 0) self_counters(s)[1] += k;
        }
        if (has) {
            const uint32_t row = (rows + (uint32_t)__popcll(m & ((1ull << ln) - 1ull))) * 3u;
            bv[row + 0] = pcorr.x;
            bv[row + 1] = pcorr.y;
            bv[row + 2] = pcorr.z;
            if constexpr (RT == FKS_ROBOT_LINKED) {
                const uint64_t mask = gp(R.link_dof_mask)[link];
                for (int d = 0; d < D; ++d) {
                    D3 col{0.0, 0.0, 0.0};
                    if ((mask >> d) & 1ull) {
                        const D3 aw{axw[3 * d], axw[3 * d + 1], axw[3 * d + 2]};
                        const int jt = s.joints()[s.dofj()[d]].type;
                        if (jt == FKS_JOINT_PRISMATIC) {
                            col = aw;
                        } else {
                            col = cross(aw, D3{xc.x - orw[3 * d], xc.y - orw[3 * d + 1], xc.z - orw[3 * d + 2]});
                        }
                        col = D3{0.0 + col.x, 0.0 + col.y, 0.0 + col.z};
                    }
                    J[(uint64_t)d * rc + row + 0] = col.x;
                    J[(uint64_t)d * rc + row + 1] = col.y;
                    J[(uint64_t)d * rc + row + 2] = col.z;
                }
            } else if constexpr (RT == FKS_ROBOT_SE2) {
                J[0 * rc + row + 0] = 0.0 + 1.0;
                J[0 * rc + row + 1] = 0.0;
                J[0 * rc + row + 2] = 0.0;
                J[1 * rc + row + 0] = 0.0;
                J[1 * rc + row + 1] = 0.0 + 1.0;
                J[1 * rc + row + 2] = 0.0;
                const D3 c2 = cross(D3{0.0, 0.0, 1.0}, D3{xc.x - cfg[0], xc.y - cfg[1], xc.z - 0.0});
                J[2 * rc + row + 0] = 0.0 + c2.x;
                J[2 * rc + row + 1] = 0.0 + c2.y;
                J[2 * rc + row + 2] = 0.0 + c2.z;
            } else {
                const D3 d{xc.x - cfg[3], xc.y - cfg[7], xc.z - cfg[11]};
                for (int a = 0; a < 3; ++a) {
                    const D3 axis{cfg[a], cfg[4 + a], cfg[8 + a]};
                    J[(uint64_t)a * rc + row + 0] = 0.0 + axis.x;
                    J[(uint64_t)a * rc + row + 1] = 0.0 + axis.y;
                    J[(uint64_t)a * rc + row + 2] = 0.0 + axis.z;
                    const D3 c = cross(axis, d);
                    J[(uint64_t)(3 + a) * rc + row + 0] = 0.0 + c.x;
                    J[(uint64_t)(3 + a) * rc + row + 1] = 0.0 + c.y;
                    J[(uint64_t)(3 + a) * rc + row + 2] = 0.0 + c.z;
                }
            }
        }
        rows += (uint32_t)__popcll(m);
    }
    wsync();
    return rows * 3u;
}

/* one round of CollectPointCorrectionsAndJacobians (SPCS:1818-1939) for the cooperative
 * pass: whether this lane's point gets a row, its correction and world position */
template <int RT>
__device__ __forceinline__ bool corr_coop_round(Sim& s, const double* Tp, const double* Tc, uint64_t skip, int r, D3* pc, D4* xc,
                                                int* link, uint64_t* selfk) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    const int i = r * kWave + ln;
    const bool skr = (skip >> r) & 1ull;
    const FKS_GLOBAL double* corr = gp(s.scratch) + A.SL.corr;
    const FKS_GLOBAL double* flag = gp(s.scratch) + A.SL.flag;
    bool has = false;
    *pc = D3{0.0, 0.0, 0.0};
    *xc = D4{0.0, 0.0, 0.0, 0.0};
    *link = 0;
    if (skr && !s.self_nonempty) {
        if (i < RDIM(R, P)) s.lane_bytes += 28;
        return false;
    }
    if (i < RDIM(R, P)) {
        const D4 p = load_point(R, i);
        *link = gp(R.point_link)[i];
        *xc = xform4(Tc + 12 * *link, p);
        const bool has_self = s.self_nonempty && flag[i] != 0.0;
        bool inb = false;
        double est = 0.0;
        if (skr)
            s.lane_bytes += 28;
        else
            est = estimate_distance(A, *xc, &inb, &s.lane_bytes);
        const bool has_env = (est < 0.0) && inb;
        D3 ecorr{0.0, 0.0, 0.0};
        if (has_env) {
            const D4 xp = xform4(Tp + 12 * *link, p);
            const D4 motion{xc->x - xp.x, xc->y - xp.y, xc->z - xp.z, xc->w - xp.w};
            const D4 nm = safe_normal4(motion);
            D3 raw;
            const bool ok = lookup_normal(A, *xc, nm, &raw, &s.err, &s.lane_bytes);
            if (!ok) s.err |= FKS_PARTICLE_ERR_NORMAL_OOB;
            const D3 g = safe_normal3(raw);
            const double pen = dabs(0.0 - est);
            ecorr = D3{g.x * pen, g.y * pen, g.z * pen};
        }
        has = has_self || has_env;
        if (has_self) *pc = D3{pc->x + corr[3 * i], pc->y + corr[3 * i + 1], pc->z + corr[3 * i + 2]};
        if (has_env) *pc = D3{pc->x + ecorr.x, pc->y + ecorr.y, pc->z + ecorr.z};
    }
    if (s.self_nonempty) *selfk += (uint64_t)__popcll(__ballot(has && flag[i] != 0.0));
    return has;
}

/* the row (3 values of b, 3 x D of J) of one corrected point at row index `row` (x 3) */
template <int RT>
__device__ __forceinline__ void corr_coop_row(Sim& s, const double* cfg, uint32_t row, const D3& pc, const D4& xc, int link) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int D = RDIM(R, D);
    const uint32_t rc = ROWCAP(A);
    FKS_GLOBAL double* J = gpw(s.scratch) + A.SL.J;
    FKS_GLOBAL double* bv = gpw(s.scratch) + A.SL.b;
    bv[row + 0] = pc.x;
    bv[row + 1] = pc.y;
    bv[row + 2] = pc.z;
    if constexpr (RT == FKS_ROBOT_LINKED) {
        const double* axw = s.lds() + LAY(A).axis_w;
        const double* orw = s.lds() + LAY(A).orig_w;
        const uint64_t mask = gp(R.link_dof_mask)[link];
        for (int d = 0; d < D; ++d) {
            D3 col{0.0, 0.0, 0.0};
            if ((mask >> d) & 1ull) {
                const D3 aw{axw[3 * d], axw[3 * d + 1], axw[3 * d + 2]};
                const int jt = s.joints()[s.dofj()[d]].type;
                if (jt == FKS_JOINT_PRISMATIC) {
                    col = aw;
                } else {
                    col = cross(aw, D3{xc.x - orw[3 * d], xc.y - orw[3 * d + 1], xc.z - orw[3 * d + 2]});
                }
                col = D3{0.0 + col.x, 0.0 + col.y, 0.0 + col.z};
            }
            J[(uint64_t)d * rc + row + 0] = col.x;
            J[(uint64_t)d * rc + row + 1] = col.y;
            J[(uint64_t)d * rc + row + 2] = col.z;
        }
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        J[0 * rc + row + 0] = 0.0 + 1.0;
        J[0 * rc + row + 1] = 0.0;
        J[0 * rc + row + 2] = 0.0;
        J[1 * rc + row + 0] = 0.0;
        J[1 * rc + row + 1] = 0.0 + 1.0;
        J[1 * rc + row + 2] = 0.0;
        const D3 c2 = cross(D3{0.0, 0.0, 1.0}, D3{xc.x - cfg[0], xc.y - cfg[1], xc.z - 0.0});
        J[2 * rc + row + 0] = 0.0 + c2.x;
        J[2 * rc + row + 1] = 0.0 + c2.y;
        J[2 * rc + row + 2] = 0.0 + c2.z;
    } else {
        const D3 d{xc.x - cfg[3], xc.y - cfg[7], xc.z - cfg[11]};
        for (int a = 0; a < 3; ++a) {
            const D3 axis{cfg[a], cfg[4 + a], cfg[8 + a]};
            J[(uint64_t)a * rc + row + 0] = 0.0 + axis.x;
            J[(uint64_t)a * rc + row + 1] = 0.0 + axis.y;
            J[(uint64_t)a * rc + row + 2] = 0.0 + axis.z;
            const D3 c = cross(axis, d);
            J[(uint64_t)(3 + a) * rc + row + 0] = 0.0 + c.x;
            J[(uint64_t)(3 + a) * rc + row + 1] = 0.0 + c.y;
            J[(uint64_t)(3 + a) * rc + row + 2] = 0.0 + c.z;
        }
    }
}

/* wave w's share of a cooperative correction pass: the work rounds of rank w, w + COOP, ...
 * (at most two each, the pass's rounds beyond 2 x COOP are not handed out): their row counts
 * are published, and after the barrier their rows written at the prefix sum of the counts of
 * the work rounds before them; returns the total row count (the same in every wave) */
template <int RT, int COOP>
__device__ __forceinline__ uint32_t corr_coop_share(Sim& s, CoopBox* box, int w, uint64_t* selfk) {
    const int ln = s.lane();
    const double* Tc = s.lds() + box->tc_off;
    const double* Tp = s.lds() + box->tp_off;
    const double* cfg = s.lds() + box->cfg_off;
    const uint64_t skip = box->skip;
    const uint64_t work = box->work;
    const int r0 = nth_bit(work, w), r1 = nth_bit(work, w + COOP);
    D3 pc0, pc1;
    D4 xc0, xc1;
    int l0 = 0, l1 = 0;
    bool h0 = false, h1 = false;
    if (r0 >= 0) h0 = corr_coop_round<RT>(s, Tp, Tc, skip, r0, &pc0, &xc0, &l0, selfk);
    if (r1 >= 0) h1 = corr_coop_round<RT>(s, Tp, Tc, skip, r1, &pc1, &xc1, &l1, selfk);
    const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
    if (ln == 0) {
        if (r0 >= 0) box->cnt[r0] = (uint32_t)__popcll(m0);
        if (r1 >= 0) box->cnt[r1] = (uint32_t)__popcll(m1);
    }
    coop_sync();
    uint32_t before0 = 0, before1 = 0, total = 0;
    for (uint64_t m = work; m; m &= m - 1ull) {
        const int r = __ffsll((unsigned long long)m) - 1;
        const uint32_t c = box->cnt[r];
        if (r < r0) before0 += c;
        if (r < r1) before1 += c;
        total += c;
    }
    const uint64_t below = (1ull << ln) - 1ull;
    if (h0) corr_coop_row<RT>(s, cfg, (before0 + (uint32_t)__popcll(m0 & below)) * 3u, pc0, xc0, l0);
    if (h1) corr_coop_row<RT>(s, cfg, (before1 + (uint32_t)__popcll(m1 & below)) * 3u, pc1, xc1, l1);
    return total;
}

/* CollectPointCorrectionsAndJacobians (SPCS:1818-1939) over the particle's COOP waves
 * (leader side): the rows collect_corrections writes, in its order; returns R.  The work
 * rounds are those collect_corrections evaluates (a proven round is still read for its
 * self-collision flags); a pass with fewer than two, or more than 2 x COOP, runs as there. */
template <int RT, int COOP>
__device__ FKS_SHAPE_INLINE uint32_t collect_corrections_coop(Sim& s, const double* Tp, const double* Tc, const double* cfg) {
    const int nr = RDIM(s.A->R, nrounds);
    const uint64_t all = (nr == kWave) ? ~0ull : ((1ull << nr) - 1ull);
    joint_frames<RT>(s, Tc);
    const uint64_t skip = skippable_rounds(s, Tc, kSkipCorrections);
    const uint64_t work = s.self_nonempty ? all : (all & ~skip);
    const int nw = __popcll(work);
    if (nw < 2 || nw > 2 * COOP) return collect_corrections<RT, true>(s, Tp, Tc, cfg, skip);
    count_event(s, FKS_PHASE_CORR_ROUNDS_SKIPPED, (uint64_t)__popcll(skip & all));
    count_event(s, FKS_PHASE_CORR_ROUNDS_EVALUATED, (uint64_t)(nr - __popcll(skip & all)));
    /* the rounds nobody evaluates: 28 bytes per point, as collect_corrections counts them */
    const uint64_t idle = all & ~work;
    uint64_t bytes = 28ull * (uint64_t)__popcll(idle) * kWave;
    if ((idle >> (nr - 1)) & 1ull) bytes -= 28ull * (uint64_t)(kWave - round_points(RDIM(s.A->R, P), nr - 1));
    if (s.lane() == 0) s.lane_bytes += bytes;
    CoopBox* box = coop_box(s);
    if (s.lane() == 0) {
        box->cmd = kCoopCorr;
        box->tc_off = (uint32_t)(Tc - s.lds());
        box->tp_off = (uint32_t)(Tp - s.lds());
        box->cfg_off = (uint32_t)(cfg - s.lds());
        box->work = work;
        box->skip = skip;
        box->self_nonempty = s.self_nonempty ? 1u : 0u;
    }
    coop_sync();
    uint64_t selfk = 0;
    const uint32_t rows = corr_coop_share<RT, COOP>(s, box, 0, &selfk);
    coop_sync();
    uint32_t e = 0;
#pragma unroll
    for (int w = 1; w < COOP; ++w) {
        e |= box->err[w];
        selfk += box->selfk[w];
    }
    s.err |= e;
    if (s.self_nonempty && s.lane() == 0) self_counters(s)[1] += selfk;
    return rows * 3u;
}

/* the helper waves of a cooperative workgroup: the leader's share of each loop it hands out,
 * until it posts kCoopExit; their byte counts go to the call's counters at the end */
template <int RT, int COOP>
__device__ __noinline__ void coop_helper(const SimArgs* __restrict__ args, double* lds_mem, int w) {
    const SimArgs& A = *args;
    Sim s;
    s.A = args;
    s.lds_block = lds_mem + LAY(A).shared_total;
    s.scratch = A.scratch + (uint64_t)blockIdx.x * A.scratch_per_wave;
    s.lane_v = lane_id();
    s.rstate = s.lds() + LAY(A).rstate;
    s.selfref = s.lds() + LAY(A).selfref;
    s.lane_bytes = 0;
    s.err = 0;
    s.self_nonempty = false;
    CoopBox* box = coop_box(s);
    for (;;) {
        coop_sync();
        const uint32_t cmd = box->cmd;
        if (cmd == kCoopExit) break;
        if (cmd == kCoopEnv) {
            env_coop_share<COOP>(s, box, w);
        } else {
            s.err = 0;
            s.self_nonempty = box->self_nonempty != 0u;
            uint64_t selfk = 0;
            (void)corr_coop_share<RT, COOP>(s, box, w, &selfk);
            const uint32_t e = wave_or(s.err);
            if (s.lane() == 0) {
                box->err[w] = e;
                box->selfk[w] = selfk;
            }
        }
        coop_sync();
    }
    const uint64_t bytes = wave_sum_u64(s.lane_bytes);
    if (s.lane() == 0 && bytes) atomicAdd(A.counters + kCntSdfBytes, (unsigned long long)bytes);
}

/* value of column `k` (wave-uniform, runtime) of this lane's register row */
template <int DM>
__device__ __forceinline__ double col_sel(const double (&a)[DM], int k) {
    double v = a[0];
#pragma unroll
    for (int c = 1; c < DM; ++c)
        if (c == k) v = a[c];
    return v;
}

/* ColPivHouseholderQR::solve for Rn <= 64 rows and D <= DM columns with the matrix
 * in registers: lane r holds row r (the lane-strided layout of the general solver
 * with one row per lane), so every long sum is the same canonical reduction and the
 * results equal qr_solve's bit for bit, without touching scratch memory. */
template <int DM>
__device__ __noinline__ void qr_solve_regs(const SimArgs* __restrict__ Ap, double* lds, const double* scratch, int ln,
                                           uint32_t Rn, double* x) {
    const SimArgs& A = *Ap;
    const int D = RDIM(A.R, D);
    const uint32_t rc = ROWCAP(A);
    const FKS_GLOBAL double* Jm = gp(scratch) + SLAY(A).J;
    const FKS_GLOBAL double* bv = gp(scratch) + SLAY(A).b;
    double* colsq = lds + LAY(A).colsq;
    double* hco = lds + LAY(A).hcoef;
    int32_t* perm = reinterpret_cast<int32_t*>(lds + LAY(A).ints);
    int32_t* transp = perm + kMaxDofs;
    const bool has = (uint32_t)ln < Rn;
    double a[DM];
#pragma unroll
    for (int c = 0; c < DM; ++c) a[c] = (has && c < D) ? Jm[(uint64_t)c * rc + ln] : 0.0;
    double bb = has ? bv[ln] : 0.0;
    if (ln < D) x[ln] = 0.0;
    if (D == 0) {
        wsync();
        return;
    }
    {
        double cs[DM];
#pragma unroll
        for (int c = 0; c < DM; ++c) cs[c] = bfly_sum(has ? 0.0 + a[c] * a[c] : 0.0);
        if (ln == 0) {
#pragma unroll
            for (int c = 0; c < DM; ++c)
                if (c < D) colsq[c] = cs[c];
        }
    }
    wsync();
    double maxsq = colsq[0];
    for (int k = 1; k < D; ++k)
        if (colsq[k] > maxsq) maxsq = colsq[k];
    const double eps = 2.220446049250313e-16;
    const double threshold_helper = maxsq * (eps * eps) / (double)Rn;
    const int size = ((int)Rn < D) ? (int)Rn : D;
    int nz = size;
    for (int k = 0; k < size; ++k) {
        int biggest = k;
        double bsq = colsq[k];
        for (int c2 = k + 1; c2 < D; ++c2)
            if (colsq[c2] > bsq) {
                bsq = colsq[c2];
                biggest = c2;
            }
        {
            const double vb = col_sel(a, biggest);
            bsq = bfly_sum((has && ln >= k) ? 0.0 + vb * vb : 0.0);
        }
        if (nz == size && bsq < threshold_helper * (double)(Rn - (uint32_t)k)) nz = k;
        wsync();
        if (ln == 0) {
            colsq[biggest] = bsq;
            transp[k] = biggest;
        }
        if (k != biggest) {
            const double vk = col_sel(a, k), vb = col_sel(a, biggest);
#pragma unroll
            for (int c = 0; c < DM; ++c) a[c] = (c == k) ? vb : ((c == biggest) ? vk : a[c]);
            if (ln == 0) {
                const double t = colsq[k];
                colsq[k] = colsq[biggest];
                colsq[biggest] = t;
            }
        }
        wsync();
        const double colk = col_sel(a, k);
        const double c0 = readlane_f64(colk, k);
        const bool below = has && ln > k;
        const double tail = (Rn - (uint32_t)k == 1u) ? 0.0 : bfly_sum(below ? 0.0 + colk * colk : 0.0);
        double tau, beta, v;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0.0;
            beta = c0;
            v = below ? 0.0 : colk;
        } else {
            beta = dsqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double denom = c0 - beta;
            v = below ? colk / denom : colk;
            tau = (beta - c0) / beta;
        }
        if (ln == k) v = beta;
#pragma unroll
        for (int c = 0; c < DM; ++c)
            if (c == k) a[c] = v;
        if (ln == 0) hco[k] = tau;
        if (Rn - (uint32_t)k == 1u) {
            if (ln == k) {
#pragma unroll
                for (int c = 0; c < DM; ++c)
                    if (c > k && c < D) a[c] = a[c] * (1.0 - tau);
            }
        } else if (tau != 0.0) {
            double tmp[DM];
#pragma unroll
            for (int c = 0; c < DM; ++c) tmp[c] = (c > k && c < D) ? bfly_sum(below ? 0.0 + v * a[c] : 0.0) : 0.0;
#pragma unroll
            for (int c = 0; c < DM; ++c) {
                if (c > k && c < D) {
                    const double t = tmp[c] + readlane_f64(a[c], k);
                    if (ln == k) a[c] = a[c] - tau * t;
                    if (below) a[c] = a[c] - (tau * v) * t;
                }
            }
        }
        {
            /* colsq downdate with the updated row k (held by lane k) */
            double rk[DM];
#pragma unroll
            for (int c = 0; c < DM; ++c) rk[c] = (c > k && c < D) ? readlane_f64(a[c], k) : 0.0;
            if (ln == 0) {
#pragma unroll
                for (int c = 0; c < DM; ++c)
                    if (c > k && c < D) colsq[c] = colsq[c] - rk[c] * rk[c];
            }
        }
        wsync();
    }
    if (ln == 0) {
        for (int i = 0; i < D; ++i) perm[i] = i;
        for (int k = 0; k < size; ++k) {
            const int t = perm[k];
            perm[k] = perm[transp[k]];
            perm[transp[k]] = t;
        }
    }
    wsync();
    if (nz == 0) return;
    /* Q^T b */
    for (int k = 0; k < nz; ++k) {
        const double tau = hco[k];
        if (Rn - (uint32_t)k == 1u) {
            if (ln == k) bb = bb * (1.0 - tau);
        } else if (tau != 0.0) {
            const double vk = col_sel(a, k);
            const bool below = has && ln > k;
            const double t = bfly_sum(below ? 0.0 + vk * bb : 0.0) + readlane_f64(bb, k);
            if (ln == k) bb = bb - tau * t;
            if (below) bb = bb - (tau * vk) * t;
        }
    }
    /* column-oriented back substitution on the nz x nz upper triangle */
    for (int ii = nz - 1; ii >= 0; --ii) {
        const double ci = readlane_f64(bb, ii);
        if (ci != 0.0) {
            const double cii = col_sel(a, ii);
            const double v = ci / readlane_f64(cii, ii);
            if (ln == ii) bb = v;
            if (ln < ii) bb = bb - v * cii;
        }
    }
    if (ln < nz) x[perm[ln]] = bb;
    wsync();
}

/* canonical 64-lane sum (bfly_sum) of partials that only rows r < RM can hold, all
 * in one lane: the butterfly is the perfect binary tree over the lanes in index
 * order, and the lanes >= RM contribute +0.0 (the last "+ 0.0" is the (r0 + r1) +
 * (r2 + r3) of bfly_sum with r1 = r2 = r3 = +0.0) */
template <int RM>
__device__ __forceinline__ double lane_tree_sum(const double (&p)[RM]) {
    static_assert(RM == 4 || RM == 8 || RM == 16, "tree over 4, 8 or 16 rows");
    double l1[RM / 2];
#pragma unroll
    for (int i = 0; i < RM / 2; ++i) l1[i] = p[2 * i] + p[2 * i + 1];
    double l2[RM / 4];
#pragma unroll
    for (int i = 0; i < RM / 4; ++i) l2[i] = l1[2 * i] + l1[2 * i + 1];
    /* 4 rows: the 8-row tree's other half is (+0 + +0) + (+0 + +0) = +0, and
     * (x + +0) + +0 == x + +0 for every x, so the last "+ 0.0" alone keeps the bits */
    if constexpr (RM == 4) return l2[0] + 0.0;
    double t = (l2[0] + l2[1]);
    if constexpr (RM == 16) t = t + ((l2[2] + l2[3]));
    return t + 0.0;
}

/* max over the wave of v (pass -inf for lanes that do not take part) */
__device__ __forceinline__ double wave_max_any(double v) {
    double o = dpp_f64<kDppXor1>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppXor2>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppHalfMirror>(v);
    v = (o > v) ? o : v;
    o = dpp_f64<kDppMirror>(v);
    v = (o > v) ? o : v;
#if FKS_PERMLANE_REDUCE
    double a, b;
    row_pair_f64<false>(v, &a, &b);
    row_pair_f64<true>((b > a) ? b : a, &a, &b);
    return readfirstlane_f64((b > a) ? b : a);
#else
    const double r0 = readlane_f64(v, 0), r1 = readlane_f64(v, 16), r2 = readlane_f64(v, 32), r3 = readlane_f64(v, 48);
    const double a = (r1 > r0) ? r1 : r0, b = (r3 > r2) ? r3 : r2;
    return (b > a) ? b : a;
#endif
}
/* the serial scan "best = first; for i > first: if (val[i] > best) take i" over the
 * lanes first..last-1 (lane i holds val[i]), as one wave reduction: the first lane
 * holding the maximum of the non-NaN values, or `first` when val[first] is NaN or
 * already the maximum */
__device__ __forceinline__ int wave_first_argmax(double val, int ln, int first, int last) {
    const double vf = readlane_f64(val, first);
    const bool part = ln > first && ln < last && !__builtin_isnan(val);
    const double m = wave_max_any(part ? val : -__builtin_huge_val());
    if (__builtin_isnan(vf) || !(m > vf)) return first;
    return __ffsll((unsigned long long)__ballot(part && val == m)) - 1;
}

/* ---------------- ColPivHouseholderQR on a lane tile ----------------
 * Small stacked systems (<= 16 rows; the right-hand side as column D) with one element per
 * lane: CW = 8 columns (D <= 7: every linked arm of <= 7 dofs, SE(2), SE(3)) of RB = 8 rows,
 * or CW = 16 columns (D <= 15) of RB = 4 rows; lane RB*c + r holds row RB*q + r of column c
 * in register q (NQ register blocks).  A reduction over the rows of a column is then two or
 * three in-register DPP steps inside the column's RB lanes plus a tree over the NQ blocks,
 * which together are exactly the canonical tree of lane_tree_sum (xor 1: rows (0,1), (2,3)
 * ...; xor 2: pairs of pairs; row_half_mirror: halves of 8), so the arithmetic is that of
 * qr_solve_cols bit for bit; an update of every column is one instruction per block instead
 * of one per row, and a Householder step costs about a third of the column-per-lane one. */
template <int RB>
__device__ __forceinline__ double col_tree(double v) {
    v = v + dpp_f64<kDppXor1>(v);
    v = v + dpp_f64<kDppXor2>(v);
    if constexpr (RB == 8) v = v + dpp_f64<kDppHalfMirror>(v);
    return v;
}
/* lane_tree_sum<RB * NQ> over the rows of the lane's column (in every lane of the column) */
template <int RB, int NQ>
__device__ __forceinline__ double col_sum(const double (&p)[NQ]) {
    static_assert(NQ == 1 || NQ == 2 || NQ == 4, "1, 2 or 4 row blocks");
    if constexpr (NQ == 1) {
        return col_tree<RB>(p[0]) + 0.0;
    } else if constexpr (NQ == 2) {
        return (col_tree<RB>(p[0]) + col_tree<RB>(p[1])) + 0.0;
    } else {
        return ((col_tree<RB>(p[0]) + col_tree<RB>(p[1])) + (col_tree<RB>(p[2]) + col_tree<RB>(p[3]))) + 0.0;
    }
}
__device__ __forceinline__ double shfl_f64(double v, int src) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)b, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(b >> 32), src, 64);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <int CW, int NQ>
__device__ __forceinline__ void qr_solve_tile(const FKS_GLOBAL double* Jm, const FKS_GLOBAL double* bv, int32_t* perm, int D, uint32_t rc,
                                              int ln, uint32_t Rn, double* x) {
    constexpr int RB = kWave / CW; /* rows per register block */
    constexpr int RM = RB * NQ;    /* rows held */
    int32_t* transp = perm + kMaxDofs;
    const int c = ln / RB, r = ln % RB;
    const bool isc = c < D, isb = c == D;
    double a[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const uint32_t row = (uint32_t)(RB * q + r);
        a[q] = (row < Rn) ? (isc ? Jm[(uint64_t)c * rc + row] : (isb ? bv[row] : 0.0)) : 0.0;
    }
    if (ln < D) x[ln] = 0.0;
    if (D == 0) {
        wsync();
        return;
    }
    /* squared column norms (every lane of column c holds column c's) */
    double cs;
    {
        double p[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) p[q] = ((uint32_t)(RB * q + r) < Rn) ? 0.0 + a[q] * a[q] : 0.0;
        cs = col_sum<RB, NQ>(p);
    }
    /* maxsq = colsq[0]; for k: if (colsq[k] > maxsq) maxsq = colsq[k] (sums of squares have no
     * -0, so the maximum of the non-NaN values does not depend on the order it is taken in) */
    double maxsq;
    {
        const double c0 = readlane_f64(cs, 0);
        double m = -__builtin_huge_val();
        for (int cc = 1; cc < D; ++cc) {
            const double v = readlane_f64(cs, RB * cc);
            if (!__builtin_isnan(v) && v > m) m = v;
        }
        maxsq = (__builtin_isnan(c0) || !(m > c0)) ? c0 : m;
    }
    const double eps = 2.220446049250313e-16;
    const double threshold_helper = maxsq * (eps * eps) / (double)Rn;
    const int size = ((int)Rn < D) ? (int)Rn : D;
    int nz = size;
#pragma unroll
    for (int k = 0; k < RM; ++k) {
        if (k >= size) break;
        const int kq = k / RB, kr = k % RB;
        /* wave_first_argmax over columns k..D-1: the first column holding the maximum of the
         * non-NaN norms right of k, or k if its own is NaN or already the maximum */
        int biggest = k;
        {
            const double vf = readlane_f64(cs, RB * k);
            double m = -__builtin_huge_val();
            int at = k;
            for (int cc = k + 1; cc < D; ++cc) {
                const double v = readlane_f64(cs, RB * cc);
                if (!__builtin_isnan(v) && v > m) {
                    m = v;
                    at = cc;
                }
            }
            if (!(__builtin_isnan(vf) || !(m > vf))) biggest = at;
        }
        double bsq;
        {
            double p[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int row = RB * q + r;
                p[q] = ((uint32_t)row < Rn && row >= k) ? 0.0 + a[q] * a[q] : 0.0;
            }
            bsq = readlane_f64(col_sum<RB, NQ>(p), RB * biggest);
        }
        if (nz == size && bsq < threshold_helper * (double)(Rn - (uint32_t)k)) nz = k;
        if (ln == 0) transp[k] = biggest;
        if (c == biggest) cs = bsq;
        if (k != biggest) {
            /* columns k and biggest trade places (with their squared norms) */
            const int src = RB * ((c == k) ? biggest : ((c == biggest) ? k : c)) + r;
#pragma unroll
            for (int q = 0; q < NQ; ++q) a[q] = shfl_f64(a[q], src);
            cs = shfl_f64(cs, src);
        }
        /* Householder vector of column k */
        const double c0 = readlane_f64(a[kq], RB * k + kr);
        double tail = 0.0;
        if (Rn - (uint32_t)k != 1u) {
            double p[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int row = RB * q + r;
                p[q] = ((uint32_t)row < Rn && row > k) ? 0.0 + a[q] * a[q] : 0.0;
            }
            tail = readlane_f64(col_sum<RB, NQ>(p), RB * k);
        }
        double tau, beta;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0.0;
            beta = c0;
            if (c == k) {
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    if (RB * q + r > k) a[q] = 0.0;
            }
        } else {
            beta = dsqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double denom = c0 - beta;
            if (c == k) {
#pragma unroll
                for (int q = 0; q < NQ; ++q)
                    if (RB * q + r > k && (uint32_t)(RB * q + r) < Rn) a[q] = a[q] / denom;
            }
            tau = (beta - c0) / beta;
        }
        if (c == k && r == kr) a[kq] = beta;
        /* the reflector (rows k+1..Rn-1 of column k), along every row */
        double v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int row = RB * q + r;
            const double vk = shfl_f64(a[q], RB * k + r);
            v[q] = (row > k && (uint32_t)row < Rn) ? vk : 0.0;
        }
        /* apply H_k to the columns right of k (and, while the rank holds, to the rhs) */
        const bool upd = (isc && c > k) || (isb && k < nz);
        double akk = shfl_f64(a[kq], RB * c + kr); /* row k of the lane's column */
        if (Rn - (uint32_t)k == 1u) {
            akk = akk * (1.0 - tau);
        } else if (tau != 0.0) {
            double p[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int row = RB * q + r;
                p[q] = (row > k && (uint32_t)row < Rn) ? 0.0 + v[q] * a[q] : 0.0;
            }
            const double t = col_sum<RB, NQ>(p) + akk;
            akk = akk - tau * t;
            if (upd) {
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int row = RB * q + r;
                    if (row > k && (uint32_t)row < Rn) a[q] = a[q] - (tau * v[q]) * t;
                }
            }
        }
        if (upd) {
            if (r == kr) a[kq] = akk;
            /* colsq downdate with the updated row k */
            if (isc) cs = cs - akk * akk;
        }
    }
    if (ln == 0) {
        for (int i = 0; i < D; ++i) perm[i] = i;
        for (int k = 0; k < size; ++k) {
            const int t = perm[k];
            perm[k] = perm[transp[k]];
            perm[transp[k]] = t;
        }
    }
    wsync();
    if (nz == 0) return;
    /* column-oriented back substitution on the nz x nz upper triangle (uniform values) */
    double bu[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) bu[i] = ((uint32_t)i < Rn) ? readlane_f64(a[i / RB], RB * D + i % RB) : 0.0;
#pragma unroll
    for (int ii = RM - 1; ii >= 0; --ii) {
        if (ii >= nz) continue;
        const double ci = bu[ii];
        if (ci != 0.0) {
            const double vq = ci / readlane_f64(a[ii / RB], RB * ii + ii % RB);
            bu[ii] = vq;
#pragma unroll
            for (int i = 0; i < ii; ++i) bu[i] = bu[i] - vq * readlane_f64(a[i / RB], RB * ii + i % RB);
        }
    }
    double mine = 0.0;
#pragma unroll
    for (int i = 0; i < RM; ++i)
        if (i == ln) mine = bu[i];
    if (ln < nz) x[perm[ln]] = mine;
    wsync();
}

/* ColPivHouseholderQR::solve for Rn <= RM rows with one COLUMN per lane (lane c < D
 * holds column c, lane D the right-hand side): every reduction over rows is then a
 * short in-lane tree (lane_tree_sum, the same canonical order as bfly_sum) instead
 * of a wave butterfly, and the D - k - 1 column updates of step k run side by side
 * in their lanes.  Same arithmetic as qr_solve_regs / qr_solve, bit for bit. */
template <int RM>
__device__ __forceinline__ void qr_solve_cols_body(const SimArgs* __restrict__ Ap, double* lds, const double* scratch, int ln,
                                                   uint32_t Rn, double* x, uint32_t row0) {
    const SimArgs& A = *Ap;
    const int D = RDIM(A.R, D);
    const uint32_t rc = ROWCAP(A);
    const FKS_GLOBAL double* Jm = gp(scratch) + SLAY(A).J + row0; /* rows [row0, row0 + Rn) */
    const FKS_GLOBAL double* bv = gp(scratch) + SLAY(A).b + row0;
    int32_t* perm = reinterpret_cast<int32_t*>(lds + LAY(A).ints);
    int32_t* transp = perm + kMaxDofs;
    const bool isc = ln < D, isb = ln == D;
    double a[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r)
        a[r] = ((uint32_t)r < Rn) ? (isc ? Jm[(uint64_t)ln * rc + r] : (isb ? bv[r] : 0.0)) : 0.0;
    if (ln < D) x[ln] = 0.0;
    if (D == 0) {
        wsync();
        return;
    }
    /* squared column norms, one per column lane (the colsq vector of the solvers above) */
    double cs;
    {
        double p[RM];
#pragma unroll
        for (int r = 0; r < RM; ++r) p[r] = ((uint32_t)r < Rn) ? 0.0 + a[r] * a[r] : 0.0;
        cs = lane_tree_sum<RM>(p);
    }
    /* maxsq = colsq[0]; for k: if (colsq[k] > maxsq) maxsq = colsq[k] */
    double maxsq;
    {
        const double c0 = readlane_f64(cs, 0);
        const double m = wave_max_any((isc && ln > 0 && !__builtin_isnan(cs)) ? cs : -__builtin_huge_val());
        maxsq = (__builtin_isnan(c0) || !(m > c0)) ? c0 : m;
    }
    const double eps = 2.220446049250313e-16;
    const double threshold_helper = maxsq * (eps * eps) / (double)Rn;
    const int size = ((int)Rn < D) ? (int)Rn : D;
    int nz = size;
    /* k is a compile-time constant in every unrolled step: the row selections below
     * fold to plain register reads instead of RM-way selects */
#pragma unroll
    for (int k = 0; k < RM; ++k) {
        if (k >= size) break;
        const int biggest = wave_first_argmax(cs, ln, k, D);
        double bsq;
        {
            double p[RM];
#pragma unroll
            for (int r = 0; r < RM; ++r) p[r] = ((uint32_t)r < Rn && r >= k) ? 0.0 + a[r] * a[r] : 0.0;
            bsq = readlane_f64(lane_tree_sum<RM>(p), biggest);
        }
        if (nz == size && bsq < threshold_helper * (double)(Rn - (uint32_t)k)) nz = k;
        if (ln == 0) transp[k] = biggest;
        if (ln == biggest) cs = bsq;
        if (k != biggest) {
            /* lanes k and biggest trade columns (and their squared norms) */
            const int src = (ln == k) ? biggest : ((ln == biggest) ? k : ln);
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if ((uint32_t)r < Rn) a[r] = __shfl(a[r], src, 64);
            cs = __shfl(cs, src, 64);
        }
        /* Householder vector of column k, computed in lane k and broadcast */
        double tau, beta;
        {
            double c0 = 0.0;
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if (r == k) c0 = a[r];
            double p[RM];
#pragma unroll
            for (int r = 0; r < RM; ++r) p[r] = ((uint32_t)r < Rn && r > k) ? 0.0 + a[r] * a[r] : 0.0;
            const double tail = (Rn - (uint32_t)k == 1u) ? 0.0 : lane_tree_sum<RM>(p);
            if (tail <= 2.2250738585072014e-308) {
                tau = 0.0;
                beta = c0;
                if (ln == k) {
#pragma unroll
                    for (int r = 0; r < RM; ++r)
                        if (r > k) a[r] = 0.0;
                }
            } else {
                beta = dsqrt(c0 * c0 + tail);
                if (c0 >= 0.0) beta = -beta;
                const double denom = c0 - beta;
                if (ln == k) {
#pragma unroll
                    for (int r = 0; r < RM; ++r)
                        if (r > k && (uint32_t)r < Rn) a[r] = a[r] / denom;
                }
                tau = (beta - c0) / beta;
            }
            if (ln == k) {
#pragma unroll
                for (int r = 0; r < RM; ++r)
                    if (r == k) a[r] = beta;
            }
            tau = readlane_f64(tau, k);
        }
        double v[RM];
#pragma unroll
        for (int r = 0; r < RM; ++r) v[r] = (r > k && (uint32_t)r < Rn) ? readlane_f64(a[r], k) : 0.0;
        /* apply H_k to the columns right of k (and, while the rank holds, to the rhs) */
        const bool upd = (isc && ln > k) || (isb && k < nz);
        if (upd) {
            double akk = 0.0;
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if (r == k) akk = a[r];
            if (Rn - (uint32_t)k == 1u) {
                akk = akk * (1.0 - tau);
            } else if (tau != 0.0) {
                double p[RM];
#pragma unroll
                for (int r = 0; r < RM; ++r) p[r] = (r > k && (uint32_t)r < Rn) ? 0.0 + v[r] * a[r] : 0.0;
                const double t = lane_tree_sum<RM>(p) + akk;
                akk = akk - tau * t;
#pragma unroll
                for (int r = 0; r < RM; ++r)
                    if (r > k && (uint32_t)r < Rn) a[r] = a[r] - (tau * v[r]) * t;
            }
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if (r == k) a[r] = akk;
            /* colsq downdate with the updated row k */
            if (isc) cs = cs - akk * akk;
        }
    }
    if (ln == 0) {
        for (int i = 0; i < D; ++i) perm[i] = i;
        for (int k = 0; k < size; ++k) {
            const int t = perm[k];
            perm[k] = perm[transp[k]];
            perm[transp[k]] = t;
        }
    }
    wsync();
    if (nz == 0) return;
    /* column-oriented back substitution on the nz x nz upper triangle (uniform values) */
    double bu[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r) bu[r] = ((uint32_t)r < Rn) ? readlane_f64(a[r], D) : 0.0;
#pragma unroll
    for (int ii = RM - 1; ii >= 0; --ii) {
        if (ii >= nz) continue;
        double ci = 0.0;
#pragma unroll
        for (int r = 0; r < RM; ++r)
            if (r == ii) ci = bu[r];
        if (ci != 0.0) {
            double rii = 0.0;
#pragma unroll
            for (int r = 0; r < RM; ++r)
                if (r == ii) rii = readlane_f64(a[r], ii);
            const double vq = ci / rii;
#pragma unroll
            for (int r = 0; r < RM; ++r) {
                if (r == ii) bu[r] = vq;
                if (r < ii) bu[r] = bu[r] - vq * readlane_f64(a[r], ii);
            }
        }
    }
    double mine = 0.0;
#pragma unroll
    for (int r = 0; r < RM; ++r)
        if (r == ln) mine = bu[r];
    if (ln < nz) x[perm[ln]] = mine;
    wsync();
}

/* the out-of-line entry (one call site per row bound in the resolver): a single corrected
 * point (3 rows) runs the 4-row body, same arithmetic (lane_tree_sum<4>) with half the
 * unrolled rows of the 8-row one */
template <int RM>
__device__ __noinline__ void qr_solve_cols(const SimArgs* __restrict__ Ap, double* lds, const double* scratch, int ln,
                                           uint32_t Rn, double* x, uint32_t row0 = 0) {
    if (RDIM(Ap->R, D) <= 7) {
        /* <= 7 columns: the 8 x 8 tile (qr_solve_tile), same arithmetic */
        const FKS_GLOBAL double* Jm = gp(scratch) + SLAY(*Ap).J + row0;
        const FKS_GLOBAL double* bv = gp(scratch) + SLAY(*Ap).b + row0;
        int32_t* perm = reinterpret_cast<int32_t*>(lds + LAY(*Ap).ints);
        if constexpr (RM <= 8)
            qr_solve_tile<8, 1>(Jm, bv, perm, RDIM(Ap->R, D), ROWCAP(*Ap), ln, Rn, x);
        else
            qr_solve_tile<8, 2>(Jm, bv, perm, RDIM(Ap->R, D), ROWCAP(*Ap), ln, Rn, x);
        return;
    }
    /* (16 columns of 4-row blocks for 8-15 dofs measured 2-3 % slower on cfg5, 14 dofs, than
     * the column-per-lane body below: profiles/r03h_ab_cfg5.log) */
    if constexpr (RM == 8) {
        if (Rn <= 4u) {
            qr_solve_cols_body<4>(Ap, lds, scratch, ln, Rn, x, row0);
            return;
        }
    }
    qr_solve_cols_body<RM>(Ap, lds, scratch, ln, Rn, x, row0);
}

/* ColPivHouseholderQR::solve (Eigen 3.2 / 3.3-beta1), rows lane-strided; x -> LDS.
 * Works in place on rows [row0, row0 + Rn) of the stacked system in scratch. */
__device__ __noinline__ void qr_solve(const SimArgs* __restrict__ Ap, double* lds, double* scratch, int ln, uint32_t Rn, double* x,
                                      uint32_t row0 = 0) {
    const SimArgs& A = *Ap;
    const int D = RDIM(A.R, D);
    const uint32_t rc = ROWCAP(A);
    const ScratchLayout& SL = A.SL;
    double* Jm = scratch + SL.J + row0;
    double* c = scratch + SL.b + row0;
    double* colsq = lds + LAY(A).colsq;
    double* hco = lds + LAY(A).hcoef;
    int32_t* perm = reinterpret_cast<int32_t*>(lds + LAY(A).ints);
    int32_t* transp = perm + kMaxDofs;
    auto col = [&](int k) { return Jm + (uint64_t)k * rc; };
    /* canonical tail squared norm of column k over rows [begin, Rn) */
    auto tail_sq = [&](int k, uint32_t begin) {
        double acc = 0.0;
        const double* ck = col(k);
        for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave)
            if (r >= begin) acc = acc + ck[r] * ck[r];
        return bfly_sum(acc);
    };
    if (ln < D) x[ln] = 0.0;
    if (D == 0) {
        wsync();
        return;
    }
    for (int k = 0; k < D; ++k) {
        const double v = tail_sq(k, 0);
        if (ln == 0) colsq[k] = v;
    }
    wsync();
    double maxsq = colsq[0];
    for (int k = 1; k < D; ++k)
        if (colsq[k] > maxsq) maxsq = colsq[k];
    const double eps = 2.220446049250313e-16;
    const double threshold_helper = maxsq * (eps * eps) / (double)Rn;
    const int size = ((int)Rn < D) ? (int)Rn : D;
    int nz = size;
    for (int k = 0; k < size; ++k) {
        int biggest = k;
        double bsq = colsq[k];
        for (int c2 = k + 1; c2 < D; ++c2)
            if (colsq[c2] > bsq) {
                bsq = colsq[c2];
                biggest = c2;
            }
        bsq = tail_sq(biggest, (uint32_t)k);
        if (nz == size && bsq < threshold_helper * (double)(Rn - (uint32_t)k)) nz = k;
        wsync();
        if (ln == 0) {
            colsq[biggest] = bsq;
            transp[k] = biggest;
        }
        if (k != biggest) {
            double* ck = col(k);
            double* cb = col(biggest);
            for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave) {
                const double t = ck[r];
                ck[r] = cb[r];
                cb[r] = t;
            }
            if (ln == 0) {
                const double t = colsq[k];
                colsq[k] = colsq[biggest];
                colsq[biggest] = t;
            }
        }
        wsync();
        double* ck = col(k);
        const double c0 = ck[k];
        const double tail = (Rn - (uint32_t)k == 1u) ? 0.0 : tail_sq(k, (uint32_t)k + 1u);
        double tau, beta;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0.0;
            beta = c0;
            for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave)
                if (r > (uint32_t)k) ck[r] = 0.0;
        } else {
            beta = dsqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double denom = c0 - beta;
            for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave)
                if (r > (uint32_t)k) ck[r] = ck[r] / denom;
            tau = (beta - c0) / beta;
        }
        wsync();
        if (ln == 0) {
            hco[k] = tau;
            ck[k] = beta;
        }
        wsync();
        if (Rn - (uint32_t)k == 1u) {
            if (ln == 0)
                for (int j = k + 1; j < D; ++j) col(j)[k] = col(j)[k] * (1.0 - tau);
        } else if (tau != 0.0) {
            /* columns are independent: four Householder applications at a time so their
             * reductions overlap (same per-column arithmetic) */
            for (int j0 = k + 1; j0 < D; j0 += 4) {
                double acc[4] = {0.0, 0.0, 0.0, 0.0};
                for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave) {
                    if (r > (uint32_t)k) {
                        const double v = ck[r];
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (j0 + q < D) acc[q] = acc[q] + v * col(j0 + q)[r];
                    }
                }
                double tmp[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) tmp[q] = bfly_sum(acc[q]);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (j0 + q < D) tmp[q] = tmp[q] + col(j0 + q)[k];
                wsync();
                if (ln == 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (j0 + q < D) col(j0 + q)[k] = col(j0 + q)[k] - tau * tmp[q];
                }
                for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave) {
                    if (r > (uint32_t)k) {
                        const double tk = tau * ck[r];
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (j0 + q < D) col(j0 + q)[r] = col(j0 + q)[r] - tk * tmp[q];
                    }
                }
                wsync();
            }
        }
        wsync();
        if (ln == 0)
            for (int j = k + 1; j < D; ++j) colsq[j] = colsq[j] - col(j)[k] * col(j)[k];
        wsync();
    }
    if (ln == 0) {
        for (int i = 0; i < D; ++i) perm[i] = i;
        for (int k = 0; k < size; ++k) {
            const int t = perm[k];
            perm[k] = perm[transp[k]];
            perm[transp[k]] = t;
        }
    }
    wsync();
    if (nz == 0) return;
    for (int k = 0; k < nz; ++k) {
        const double tau = hco[k];
        const double* ck = col(k);
        if (Rn - (uint32_t)k == 1u) {
            wsync();
            if (ln == 0) c[k] = c[k] * (1.0 - tau);
            wsync();
        } else if (tau != 0.0) {
            double acc = 0.0;
            for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave)
                if (r > (uint32_t)k) acc = acc + ck[r] * c[r];
            double tmp = bfly_sum(acc);
            tmp = tmp + c[k];
            wsync();
            if (ln == 0) c[k] = c[k] - tau * tmp;
            for (uint32_t r = (uint32_t)ln; r < Rn; r += kWave)
                if (r > (uint32_t)k) c[r] = c[r] - (tau * ck[r]) * tmp;
            wsync();
        }
    }
    /* column-oriented back substitution on the nz x nz upper triangle */
    for (int ii = nz - 1; ii >= 0; --ii) {
        const double ci = c[ii];
        if (ci != 0.0) {
            const double* cc = col(ii);
            const double v = ci / cc[ii];
            wsync();
            if (ln == 0) c[ii] = v;
            if (ln < ii) c[ln] = c[ln] - v * cc[ln];
            wsync();
        }
    }
    if (ln < nz) x[perm[ln]] = c[ln];
    wsync();
}

/* ComputeResolverCorrectionStepIndividualJacobians (SPCS:1966-1988): one
 * ColPivHouseholderQR solve per corrected point (its 3 x D block of the stacked
 * system), the steps summed in point order (the first assigned, then raw + step).
 * No corrected point: the zero step (as the stacked solve of an empty system). */
__device__ __noinline__ void individual_jacobians_solve(Sim& s, uint32_t Rn, double* x) {
    const int ln = s.lane();
    const int D = RDIM(s.A->R, D);
    double* acc = s.lds() + LAY(*s.A).real;
    for (uint32_t r0 = 0; r0 < Rn; r0 += 3u) {
        if (D < kWave)
            qr_solve_cols<8>(s.A, s.lds(), s.scratch, ln, 3u, x, r0);
        else
            qr_solve(s.A, s.lds(), s.scratch, ln, 3u, x, r0);
        if (ln < D) acc[ln] = (r0 == 0u) ? x[ln] : acc[ln] + x[ln];
        wsync();
    }
    if (ln < D) x[ln] = (Rn == 0u) ? 0.0 : acc[ln];
    wsync();
}

/* one controller step: ResolveForwardSimulation (SPCS:1546-1816).
 * returns 0 ok, 1 error; sets collided/failed; result config in res_cfg.
 * IND: the individual-Jacobian solve (SPCS:1966-1988) is compiled into a kernel of its
 * own, so the default stacked-Jacobian kernel does not carry it; the traced kernels
 * (not on the hot path) read the choice at run time. */
template <int RT, bool TR, bool IND, int COOP = 0>
__device__ FKS_SHAPE_INLINE int resolve_step(Sim& s, const double* particle_cfg, double* res_cfg, bool allow_contacts, bool* out_collided,
                            bool* out_failed, double*& Tcur, double*& Tprev) {
    const SimArgs& A = *s.A;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    const int W = RDIM(R, W), D = RDIM(R, D);
    double* u = s.lds() + LAY(*s.A).u;
    double* ustep = s.lds() + LAY(*s.A).ustep;
    double* cfg_tmp = s.lds() + LAY(*s.A).cfg_tmp;
    double* cfg_prev = s.lds() + LAY(*s.A).cfg_prev;
    double* cfg_act = s.lds() + LAY(*s.A).cfg_act;
    double* x = s.lds() + LAY(*s.A).x;
    double* real = s.lds() + LAY(*s.A).real;
    /* the trial transforms live in whichever of the three transform buffers is neither
     * Tcur nor Tprev (the paired FK below rotates all three) */
    double* Ttmp;
    {
        double* b0 = s.lds() + LAY(*s.A).Tcur;
        double* b1 = s.lds() + LAY(*s.A).Tprev;
        double* b2 = s.lds() + LAY(*s.A).Ttmp;
        Ttmp = (b0 != Tcur && b0 != Tprev) ? b0 : ((b1 != Tcur && b1 != Tprev) ? b1 : b2);
    }
    double* cfg = s.lds() + LAY(*s.A).cfg_work; /* robot(immutable_robot->Clone()) SPCS:1548 */
    *out_collided = false;
    *out_failed = false;
    uint64_t t0 = tick();
    if (ln < W) cfg[ln] = particle_cfg[ln];
    wsync();
    /* real_control_input = u * dt (SPCS:1549), already in u.  FK of the start
     * configuration is still in Tcur when the previous step ended normally */
    if (!s.tcur_valid) fk<RT>(s, cfg, Tcur);
    apply_input<RT>(s, cfg, u, cfg_tmp, false, 0);
    fk<RT>(s, cfg_tmp, Ttmp);
    s.tcur_valid = false;
    const double computed_step_motion = max_point_motion(s, Tcur, Ttmp);
    const double raw_steps = __builtin_ceil(computed_step_motion / A.target_micro);
    if (!(raw_steps <= 1048576.0)) {
        s.err |= FKS_PARTICLE_ERR_MICROSTEP_CAP;
        return 1;
    }
    uint32_t M = (uint32_t)raw_steps;
    if (M < 1u) M = 1u;
    if (ln < D) ustep[ln] = u[ln] / (double)M;
    wsync();
    /* SPCS:1563-1575: the motion of one clean microstep must not exceed the allowed
     * distance.  sum_d |u_d / M| * lever_d bounds it (clamping only shortens the
     * motion), so the check is evaluated only when the bound does not already prove it. */
    bool proven = false;
    {
        /* per-dof lever arms (fks_set_robot): linked joints' reach, SE(2) / SE(3) 1 for
         * translation and max |p| for rotation components; +inf where no bound holds */
        const double term = (ln < D) ? dabs(ustep[ln]) * gp(R.dof_lever)[ln] : 0.0;
        const double bound = bfly_sum(0.0 + term);
        proven = !FKS_NO_SKIP_PROOFS && bound * (1.0 + 1e-6) + 1e-12 < A.allowed_micro;
    }
    if (!proven) {
        apply_input<RT>(s, cfg, ustep, cfg_tmp, false, 0);
        fk<RT>(s, cfg_tmp, Ttmp);
        const double micro_motion = max_point_motion(s, Tcur, Ttmp);
        if (micro_motion > A.allowed_micro) {
            s.err |= FKS_PARTICLE_ERR_MICROSTEP_MOTION;
            return 1;
        }
    }
    tock(s, FKS_PHASE_STEP_SETUP, t0);
    trace_step<TR>(s, u, ustep, M);
    bool collided = false;
    /* Paired FK (linked robots, LAY(A).fk_pair): while a microstep runs its FK, the chain's
     * idle lanes compute the FK of the NEXT microstep's configuration as it will be if
     * this one ends without contact (apply_input with the next noise sample, already in
     * the noise buffer).  If this microstep ends without contact, the next one's
     * apply_input would see exactly those inputs, so it takes that configuration, its
     * actuator error bits and those transforms instead of recomputing them; after a
     * contact the prediction is dropped (the resolver reuses cfg_tmp / Ttmp).  Results are
     * unchanged; free microsteps pay about half an FK and half an apply_input each. */
    const uint32_t noise_per = (uint32_t)(kWave / RDIM(R, D));
    bool pair_ready = false; /* Ttmp holds FK(cfg_tmp), cfg_tmp = the predicted configuration */
    uint32_t pair_err = 0;   /* the predicted configuration's actuator error bits (per lane) */
    for (uint32_t micro = 0; micro < M; ++micro) {
        s.lane_v = opaque_lane(s.lane_v);
        const int ln = s.lane();
        s.micro_count++;
        if (ln < W) cfg_prev[ln] = cfg[ln];
        wsync();
        t0 = tick();
        /* a predicted microstep (the previous one ended free of contact) takes the
         * configuration apply_input produced for it then: the same inputs, so the same bits */
        const bool predicted = pair_ready;
        if (predicted) {
            if (ln < W) cfg[ln] = cfg_tmp[ln];
            s.err |= pair_err;
            wsync();
        } else {
            if (micro % (uint32_t)(kWave / RDIM(R, D)) == 0u)
                refill_noise(s, micro, M);
            apply_input<RT>(s, cfg_prev, ustep, cfg, true, micro);
        }
        s.err = wave_or(s.err);
        tock(s, FKS_PHASE_MICRO_INPUT, t0);
        if (s.err) {
            if (ln < W) res_cfg[ln] = cfg_prev[ln];
            wsync();
            return 1;
        }
        t0 = tick();
        if (predicted) {
            /* this microstep's transforms were computed with the previous one's */
            double* t = Tprev;
            Tprev = Tcur;
            Tcur = Ttmp;
            Ttmp = t;
            pair_ready = false;
        } else {
            {
                double* t = Tprev;
                Tprev = Tcur;
                Tcur = t;
            }
            pair_ready = false;
            bool pair = false;
            if constexpr (RT == FKS_ROBOT_LINKED) {
                pair = LAY(A).fk_pair && micro + 1u < M && ((micro + 1u) % noise_per) != 0u;
                if (pair) {
                    /* the next microstep's configuration if this one ends free of contact;
                     * its error bits are the next microstep's, not this one's */
                    const uint32_t err_keep = s.err;
                    apply_input<RT>(s, cfg, ustep, cfg_tmp, true, micro + 1u);
                    pair_err = s.err; /* err_keep is 0 here: errors end the step above */
                    s.err = err_keep;
                    fk_pair(s, cfg, Tcur, cfg_tmp, Ttmp);
                    pair_ready = true;
                }
            }
            if (!pair)
                fk<RT>(s, cfg, Tcur);
        }
        tock(s, FKS_PHASE_MICRO_FK, t0);
        bool in_collision = check_collision<RT, COOP>(s, Tprev, Tcur, cfg);
        if (s.err) return 1;
        if (in_collision) pair_ready = false; /* the resolver reuses cfg_tmp / Ttmp */
        trace_config<TR>(s, cfg, micro, FKS_TRACE_POST_ACTION);
        if (in_collision) collided = true;
        if (in_collision && allow_contacts) {
            if (ln < W) cfg_act[ln] = cfg[ln];
            wsync();
            uint32_t iters = 0;
            /* the correction step scaling: a linked robot keeps it in the wave's LDS block
             * (misc + 38), one uniform double fewer live across the resolver loop (fewer spill
             * reloads on cfg3 / cfg5); SE(2) / SE(3) keep the register (cfg4's allocation
             * went the other way) */
            constexpr bool kScalingLds = RT == FKS_ROBOT_LINKED;
            double* scaling_p = s.lds() + LAY(*s.A).misc + 38;
            double scaling_reg = A.S.resolve_correction_initial_step_size;
            if (kScalingLds) {
                if (ln == 0) *scaling_p = scaling_reg;
                wsync();
            }
            while (in_collision) {
                s.lane_v = opaque_lane(s.lane_v);
                const int ln = s.lane();
                s.resolver_count++;
                t0 = tick();
                uint32_t Rn;
                if constexpr (COOP > 0)
                    Rn = collect_corrections_coop<RT, COOP>(s, Tprev, Tcur, cfg_act);
                else
                    Rn = collect_corrections<RT>(s, Tprev, Tcur, cfg_act);
                s.lsq_rows += Rn;
                s.err = wave_or(s.err);
                tock(s, FKS_PHASE_CORRECTIONS, t0);
                if (s.err) return 1;
                t0 = tick();
                if (IND || (TR && A.individual_jacobians)) {
                    individual_jacobians_solve(s, Rn, x);
                } else if (Rn <= 8u && RDIM(R, D) < kWave)
                    qr_solve_cols<8>(s.A, s.lds(), s.scratch, ln, Rn, x);
                else if (Rn <= 16u && RDIM(R, D) < kWave)
                    qr_solve_cols<16>(s.A, s.lds(), s.scratch, ln, Rn, x);
                else if (Rn <= (uint32_t)kWave && RDIM(R, D) <= 8)
                    qr_solve_regs<8>(s.A, s.lds(), s.scratch, ln, Rn, x);
                else if (RT == FKS_ROBOT_LINKED && Rn <= (uint32_t)kWave && RDIM(R, D) <= 16)
                    qr_solve_regs<RT == FKS_ROBOT_LINKED ? 16 : 8>(s.A, s.lds(), s.scratch, ln, Rn, x);
                else
                    qr_solve(s.A, s.lds(), s.scratch, ln, Rn, x);
                tock(s, FKS_PHASE_SOLVE, t0);
                t0 = tick();
                /* SPCS:1663-1682: the correction's workspace motion est decides
                 * step_fraction = max(est / allowed, 1).  The lever-arm bound
                 * sum_d |x_d| * lever_d (clamping and wrapping only shorten the motion; SE(2) /
                 * SE(3) levers in fks_set_robot) often proves est <= allowed, i.e.
                 * step_fraction == 1 exactly; the
                 * trial FK and the motion estimate are then not needed and the real step
                 * (x / 1) * |scaling| == x * |scaling| is applied directly */
                bool fraction_one;
                {
                    const double term = (ln < D) ? dabs(x[ln]) * gp(R.dof_lever)[ln] : 0.0;
                    fraction_one = !FKS_NO_SKIP_PROOFS && bfly_sum(0.0 + term) * (1.0 + 1e-6) + 1e-12 < A.allowed_micro;
                }
                double step_fraction = 1.0;
                bool applied = false; /* cfg_act and Tcur already hold the corrected state */
                if (!fraction_one) {
                    apply_input<RT>(s, cfg_act, x, cfg_tmp, false, 0);
                    fk<RT>(s, cfg_tmp, Ttmp);
                    const double est = max_point_motion(s, Tcur, Ttmp);
                    step_fraction = dmax(est / A.allowed_micro, 1.0);
                    applied = step_fraction == 1.0 && dabs(kScalingLds ? *scaling_p : scaling_reg) == 1.0;
                    if (applied) {
                        /* real_correction_step = (x / 1) * 1 == x bit for bit (SPCS:1681-1682): the
                         * corrected configuration is cfg_tmp and its transforms are Ttmp */
                        if (ln < W) cfg_act[ln] = cfg_tmp[ln];
                        for (int e = ln; e < 12 * RDIM(R, L); e += kWave) Tcur[e] = Ttmp[e];
                        wsync();
                    }
                }
                if (!applied) {
                    if (ln < D) real[ln] = (x[ln] / step_fraction) * dabs(kScalingLds ? *scaling_p : scaling_reg);
                    wsync();
                    apply_input<RT>(s, cfg_act, real, cfg_tmp, false, 0);
                    if (ln < W) cfg_act[ln] = cfg_tmp[ln];
                    wsync();
                    fk<RT>(s, cfg_act, Tcur);
                }
                tock(s, FKS_PHASE_RESOLVE_APPLY, t0);
                in_collision = check_collision<RT, COOP>(s, Tprev, Tcur, cfg_act);
                if (s.err) return 1;
                trace_config<TR>(s, cfg_act, micro, FKS_TRACE_RESOLVER_STEP);
                iters++;
                if (iters > A.S.max_resolver_iterations) {
                    trace_config<TR>(s, cfg_prev, micro, FKS_TRACE_RESOLVE_FAILED);
                    if (ln == 0) {
                        s.stats()[kCntUnsuccessful]++;
                        s.stats()[s.self_nonempty ? kCntUnsuccessfulSelf : kCntUnsuccessfulEnv]++;
                    }
                    if (ln < W) res_cfg[ln] = cfg_prev[ln];
                    wsync();
                    *out_collided = true;
                    *out_failed = true;
                    return 0;
                }
                if ((iters % A.S.resolve_correction_step_scaling_decay_iterations) == 0u) {
                    double scaling = kScalingLds ? *scaling_p : scaling_reg;
                    if (scaling >= 0.0) {
                        scaling = scaling * A.S.resolve_correction_step_scaling_decay_rate;
                        if (scaling < A.S.resolve_correction_min_step_scaling) scaling = -A.S.resolve_correction_min_step_scaling;
                    } else {
                        scaling = -A.S.resolve_correction_min_step_scaling;
                    }
                    if (kScalingLds) {
                        if (ln == 0) *scaling_p = scaling;
                        wsync();
                    } else {
                        scaling_reg = scaling;
                    }
                }
            }
            if (ln < W) cfg[ln] = cfg_act[ln];
            wsync();
            /* the resolved configuration's check came back free (Tcur = FK(cfg)) */
        } else if (in_collision && !allow_contacts) {
            trace_config<TR>(s, cfg_prev, micro, FKS_TRACE_CONTACT_STOP);
            if (s.lane() == 0) s.stats()[kCntSuccessful]++;
            if (ln < W) res_cfg[ln] = cfg_prev[ln];
            wsync();
            *out_collided = true;
            return 0;
        }
    }
    if (ln == 0) {
        s.stats()[kCntSuccessful]++;
        s.stats()[collided ? kCntCollision : kCntFree]++;
    }
    if (ln < W) res_cfg[ln] = cfg[ln];
    wsync();
    *out_collided = collided;
    s.tcur_valid = true; /* the step's last check came back free at Tcur = FK(cfg) */
    return 0;
}

}  // namespace fksd

using namespace fksd;

/* workgroup prologue shared by the kernels: one LDS copy of the robot tables the
 * inner loops read, then this wave's view of its LDS block and scratch */
template <int RT>
__device__ __forceinline__ void setup_wave(const SimArgs* __restrict__ args, double* lds_mem, Sim& s) {
    const SimArgs& A = *args;
    const RobotDev& R = A.R;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); /* wave-uniform: LDS bases stay in SGPRs */
    double* shared = lds_mem;
    {
        const int t = (int)threadIdx.x, nt = (int)blockDim.x;
        uint64_t* dj = reinterpret_cast<uint64_t*>(shared + LAY(A).joints);
        const uint64_t* sj = reinterpret_cast<const uint64_t*>(R.joints);
        for (int k = t; k < RDIM(R, J) * kJointWords; k += nt) dj[k] = sj[k];
        uint64_t* dc = reinterpret_cast<uint64_t*>(shared + LAY(A).ctrl);
        const uint64_t* sc = reinterpret_cast<const uint64_t*>(R.ctrl);
        for (int k = t; k < RDIM(R, D) * kCtrlWords; k += nt) dc[k] = sc[k];
        int32_t* dd = reinterpret_cast<int32_t*>(shared + LAY(A).dofj);
        if (RT == FKS_ROBOT_LINKED && t < RDIM(R, D)) dd[t] = gp(R.dof_joint)[t];
        if (t < 12) shared[LAY(A).base + t] = R.base[t];
        if (RT == FKS_ROBOT_LINKED) {
            for (int k = t; k < 8 * RDIM(R, G); k += nt)
                shared[LAY(A).gbox + k] = (k % 8 == 7) ? (double)gp(R.geom_link)[k / 8] : gp(R.geom_box)[7 * (k / 8) + k % 8];
            uint32_t* lp = reinterpret_cast<uint32_t*>(shared + LAY(A).gpairs);
            for (int k = t; k < RDIM(R, npairs) && k < kLdsPairs; k += nt)
                lp[k] = (uint32_t)gp(R.pairs)[2 * k] | ((uint32_t)gp(R.pairs)[2 * k + 1] << 16);
        }
        if (t < RDIM(R, nrounds) && t < kWave) {
            const RoundDev rd = load_round(R.rounds, t);
            shared[LAY(A).rounds + 2 * t] = (double)rd.link;
            shared[LAY(A).rounds + 2 * t + 1] = rd.radius;
        }
        __syncthreads();
    }
    s.A = args;
    s.lds_block = lds_mem + LAY(A).shared_total + (uint64_t)wave * LAY(A).total;
    s.scratch = A.scratch + ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (uint64_t)wave) * A.scratch_per_wave;
    s.lane_v = lane_id();
    s.rstate = s.lds() + LAY(A).rstate; /* (the check / kinematics kernels keep no skip-proof cache) */
    s.err = 0;
    s.lane_bytes = 0;
    s.self_nonempty = false;
    s.tcur_valid = false;
}

/* SetPosition(src) into cfg (LDS): joint limits / angle wrap as SetConfig does */
template <int RT>
__device__ __forceinline__ void set_position(Sim& s, const double* src, double* cfg) {
    const int ln = s.lane();
    if constexpr (RT == FKS_ROBOT_LINKED) {
        if (ln < RDIM(s.A->R, D)) {
            const JointDev& jd = s.joints()[s.dofj()[ln]];
            cfg[ln] = (jd.type == FKS_JOINT_CONTINUOUS) ? fks_math::wrap_revolute(src[ln])
                                                        : clamp(src[ln], jd.lo, jd.hi);
        }
    } else if constexpr (RT == FKS_ROBOT_SE2) {
        if (ln < 3) cfg[ln] = (ln == 2) ? fks_math::wrap_revolute(src[2]) : src[ln];
    } else {
        if (ln < 12) cfg[ln] = src[ln];
    }
    wsync();
}

/* CheckSelfCollisions (SPCS:1324-1396) at extended cells of size `res`: true iff one
 * cell holds points of two geometries whose pair is disallowed (CheckPointsForSelfCollision,
 * SPCS:1277-1322).  Conservative per-geometry key boxes (one lane per geometry) reject
 * pairs; overlapping pairs compare exact keys: a point of b can share a cell with a point of
 * a only if its key lies in a's box (and the a point's in b's), so b's points in a's box are
 * taken by ballot, their keys held in registers and broadcast one by one (readlane) to the
 * lanes holding a's points in b's box — no memory round trip per comparison.  env_hit: the
 * configuration already collides with the environment, so only the error bits of the key
 * computation (which the reference's keying would raise) are still needed. */
__device__ __forceinline__ int64_t readlane_i64(int64_t v, int lane) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __noinline__ uint32_t config_self_collision(const SimArgs* __restrict__ Ap, const double* shared, double* lds,
                                                       double* scratch, int ln, const double* Tc, double res, bool env_hit) {
    const SimArgs& A = *Ap;
    const RobotDev& R = A.R;
    double* box = lds + LAY(A).box;
    bool bad = false;
    if (ln < RDIM(R, G)) {
        const double* gb = shared + LAY(A).gbox + 8 * ln;
        const double* T = Tc + 12 * (int)gb[7];
        double lo[3], hi[3];
        if (gb[6] != 0.0) {
            const D3 wc = xform3(T, D3{gb[0], gb[1], gb[2]});
            double wh[3];
            for (int i = 0; i < 3; ++i)
                wh[i] = (dabs(T[4 * i]) * gb[3] + dabs(T[4 * i + 1]) * gb[4]) + dabs(T[4 * i + 2]) * gb[5];
            const D3 gc = xform3(A.env_g.inv, wc);
            const double gcv[3] = {gc.x, gc.y, gc.z};
            for (int i = 0; i < 3; ++i) {
                const double* Ir = A.env_g.inv + 4 * i;
                const double gh = (dabs(Ir[0]) * wh[0] + dabs(Ir[1]) * wh[1]) + dabs(Ir[2]) * wh[2];
                const double margin = 1e-6 + 1e-9 * (dabs(gcv[i]) + gh);
                const double l = (gcv[i] - gh - margin) / res;
                const double h = (gcv[i] + gh + margin) / res;
                if (!(l > -1e18 && l < 1e18 && h > -1e18 && h < 1e18)) bad = true;
                lo[i] = __builtin_trunc(l);
                hi[i] = __builtin_trunc(h);
            }
        } else {
            bad = true;
        }
        for (int i = 0; i < 3; ++i) {
            box[6 * ln + i] = bad ? -__builtin_huge_val() : lo[i];
            box[6 * ln + 3 + i] = bad ? __builtin_huge_val() : hi[i];
        }
    }
    wsync();
    /* the geometries whose keys matter: those of overlapping pairs, and every geometry whose box
     * is not finite.  A non-finite point (the only source of FKS_PARTICLE_ERR_KEY_RANGE, which
     * the reference's keying of every point would raise) lies on a link with a non-finite box,
     * so keying these gives the error bits of keying all points.  After an environment hit only
     * the error bits are still needed. */
    const uint64_t bad_geoms = __ballot(ln < RDIM(R, G) && bad);
    uint64_t need = bad_geoms;
    if (!env_hit) {
        for (int k0 = 0; k0 < RDIM(R, npairs); k0 += kWave) {
            const int k = k0 + ln;
            int a = 0, b = 0;
            bool ov = false;
            if (k < RDIM(R, npairs)) {
                a = gp(R.pairs)[2 * k];
                b = gp(R.pairs)[2 * k + 1];
                ov = true;
                for (int i = 0; i < 3; ++i) ov = ov && (box[6 * a + i] <= box[6 * b + 3 + i]) && (box[6 * b + i] <= box[6 * a + 3 + i]);
            }
            uint64_t m = __ballot(ov);
            while (m) {
                const int bit = __ffsll((unsigned long long)m) - 1;
                m &= m - 1ull;
                need |= (1ull << readlane_i32(a, bit)) | (1ull << readlane_i32(b, bit));
            }
        }
    }
    if (!need) return 0u;
    /* exact keys (LocationToExtendedGridIndex SPCS:1173-1181: trunc of the quotient by `res`) of
     * the needed geometries' points.  The quotient is taken as a product with 1/res unless an
     * integer lies within 8 ulp of it (then the division): the product is within 2.5 ulp of the
     * correctly rounded quotient, so away from integers both truncate alike */
    int64_t* keys = reinterpret_cast<int64_t*>(scratch + SLAY(A).keys);
    uint32_t err = 0;
    const double inv = 1.0 / res;
    auto quotient = [&](double v) {
        const double r = v * inv;
        return (dabs(r) < 4.0e15 && dabs(r - __builtin_rint(r)) > dabs(r) * 0x1p-49) ? r : v / res;
    };
    for (uint64_t gm = need; gm; gm &= gm - 1ull) {
        const int g0 = __ffsll((unsigned long long)gm) - 1;
        for (int i = (int)gp(R.geom_off)[g0] + ln; i < (int)gp(R.geom_off)[g0 + 1]; i += kWave) {
            const D4 x = xform4(Tc + 12 * (int)gp(R.point_link)[i], load_point(R, i));
            const D4 g = xform4(A.env_g.inv, x);
            const double q[3] = {quotient(g.x), quotient(g.y), quotient(g.z)};
            for (int a = 0; a < 3; ++a) {
                int64_t k;
                if (q[a] != q[a] || q[a] == __builtin_huge_val() || q[a] == -__builtin_huge_val()) {
                    err |= FKS_PARTICLE_ERR_KEY_RANGE;
                    k = 0;
                } else if (q[a] >= 9.0e18) {
                    k = (int64_t)9000000000000000000ll;
                } else if (q[a] <= -9.0e18) {
                    k = -(int64_t)9000000000000000000ll;
                } else {
                    k = (int64_t)q[a];
                }
                keys[3 * i + a] = k;
            }
        }
    }
    err = wave_or(err);
    if (env_hit) return err << 1; /* collided either way: the pairs need not be compared */
    wsync();
    auto in_box = [&](int i, int g) {
        bool in = true;
        for (int a = 0; a < 3; ++a) {
            const double k = (double)keys[3 * i + a];
            in = in && box[6 * g + a] <= k && k <= box[6 * g + 3 + a];
        }
        return in;
    };
    bool hit = false;
    for (int k = 0; k < RDIM(R, npairs) && !wave_any(hit); ++k) {
        const int a = gp(R.pairs)[2 * k], b = gp(R.pairs)[2 * k + 1];
        bool ov = true;
        for (int i = 0; i < 3; ++i) ov = ov && (box[6 * a + i] <= box[6 * b + 3 + i]) && (box[6 * b + i] <= box[6 * a + 3 + i]);
        if (!ov) continue;
        const int a0 = (int)gp(R.geom_off)[a], a1 = (int)gp(R.geom_off)[a + 1];
        const int b0 = (int)gp(R.geom_off)[b], b1 = (int)gp(R.geom_off)[b + 1];
        if (a1 - a0 <= kWave && b1 - b0 <= kWave) {
            /* one chunk each (every robot here: <= 64 points per geometry): both sides' keys in
             * one memory round trip */
            const int j = b0 + ln, i = a0 + ln;
            int64_t bx = 0, by = 0, bz = 0, ax = 0, ay = 0, az = 0;
            if (j < b1) {
                bx = keys[3 * j];
                by = keys[3 * j + 1];
                bz = keys[3 * j + 2];
            }
            if (i < a1) {
                ax = keys[3 * i];
                ay = keys[3 * i + 1];
                az = keys[3 * i + 2];
            }
            auto in_box_k = [&](int64_t kx, int64_t ky, int64_t kz, int g) {
                return box[6 * g] <= (double)kx && (double)kx <= box[6 * g + 3] && box[6 * g + 1] <= (double)ky &&
                       (double)ky <= box[6 * g + 4] && box[6 * g + 2] <= (double)kz && (double)kz <= box[6 * g + 5];
            };
            const bool jin = j < b1 && in_box_k(bx, by, bz, a);
            const bool iin = i < a1 && in_box_k(ax, ay, az, b);
            uint64_t m = __ballot(jin);
            if (!m || !wave_any(iin)) continue;
            bool h = false;
            while (m) {
                const int t = __ffsll((unsigned long long)m) - 1;
                m &= m - 1ull;
                h = h || (ax == readlane_i64(bx, t) && ay == readlane_i64(by, t) && az == readlane_i64(bz, t));
            }
            hit = hit || (iin && h);
            continue;
        }
        for (int j0 = b0; j0 < b1 && !wave_any(hit); j0 += kWave) {
            const int j = j0 + ln;
            const bool jin = j < b1 && in_box(j, a);
            const int64_t bx = jin ? keys[3 * j] : 0, by = jin ? keys[3 * j + 1] : 0, bz = jin ? keys[3 * j + 2] : 0;
            const uint64_t mb = __ballot(jin);
            if (!mb) continue;
            for (int i0 = a0; i0 < a1 && !wave_any(hit); i0 += kWave) {
                const int i = i0 + ln;
                const bool iin = i < a1 && in_box(i, b);
                if (!wave_any(iin)) continue;
                const int64_t ax = iin ? keys[3 * i] : 0, ay = iin ? keys[3 * i + 1] : 0, az = iin ? keys[3 * i + 2] : 0;
                uint64_t m = mb;
                bool h = false;
                while (m) {
                    const int t = __ffsll((unsigned long long)m) - 1;
                    m &= m - 1ull;
                    h = h || (ax == readlane_i64(bx, t) && ay == readlane_i64(by, t) && az == readlane_i64(bz, t));
                }
                hit = hit || (iin && h);
            }
        }
    }
    return (err << 1) | (wave_any(hit) ? 1u : 0u);
}

/* CheckEnvironmentCollision (SPCS:921-981) for the batched configuration check: the
 * nearest-cell values of NB rounds of points are gathered at once (one memory round trip for
 * the whole robot at cfg3's 8 rounds, instead of one per pair of rounds), then examined in
 * point order; EstimateDistance4d only where the nearest value cannot decide, as env_point.
 * Bytes are counted up to the first colliding point, as the reference reads them. */
template <int NB>
__device__ __forceinline__ bool check_env_rounds(const SimArgs& A, const double* T, int ln, uint64_t* lane_bytes) {
    const RobotDev& R = A.R;
    const GridDev& g = A.sdf_g;
    const double thr = A.thr_env;
    const int P = RDIM(R, P);
    for (int base = 0; base < P; base += NB * kWave) {
        float d[NB];
        uint32_t okm = 0; /* bit k: round k's point of this lane is in the grid */
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int i = base + k * kWave + ln;
            d[k] = A.oob;
            if (i < P) {
                const D4 x = xform4(T + 12 * gp(R.point_link)[i], load_point(R, i));
                int32_t idx[3];
                if (grid_index(g, x, idx)) {
                    d[k] = gp(A.sdf)[grid_brick(g, idx[0], idx[1], idx[2])];
                    okm |= 1u << k;
                }
            }
        }
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            if (base + k * kWave >= P) break;
            const int i = base + k * kWave + ln;
            uint64_t b = ((okm >> k) & 1u) ? 4 : 0;
            bool c = false;
            if (i < P && (double)d[k] < thr) {
                if ((double)d[k] < thr - g.res) {
                    c = true;
                } else {
                    const D4 x = xform4(T + 12 * gp(R.point_link)[i], load_point(R, i));
                    bool inb;
                    c = estimate_distance(A, x, &inb, &b) < thr;
                }
            }
            const uint64_t m = __ballot(c);
            if (m) {
                if (ln <= __ffsll((unsigned long long)m) - 1) *lane_bytes += b;
                return true;
            }
            *lane_bytes += b;
        }
    }
    return false;
}

/* batched CheckConfigCollision (SPCS:1398-1416): one wave per configuration,
 * grid-stride over the batch.  A.thr_env holds inflation_ratio * res - tolerance *
 * sdf_res (SPCS:1403 + 923), A.self_res = (inflation_ratio + 1) * res (SPCS:1404). */
template <int RT>
__device__ __forceinline__ void check_configs(const SimArgs* __restrict__ args, double* lds_mem) {
    Sim s;
    setup_wave<RT>(args, lds_mem, s);
    const SimArgs& A = *args;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    double* cfg = s.lds() + LAY(A).cfg;
    double* T = s.lds() + LAY(A).Tcur;
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t bytes_total = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c < A.n; c += stride) {
        set_position<RT>(s, A.starts + c * (uint64_t)RDIM(R, W), cfg);
        fk<RT>(s, cfg, T);
        /* CheckEnvironmentCollision: bytes up to the first colliding point (its loop returns
         * there), eight rounds' nearest-cell reads in flight at once */
        uint64_t lane_bytes = 0;
#if defined(FKS_PROBE_CHECK_NO_ENV)
        const bool env = false; /* A/B probe only: what the environment leg costs (results change) */
#else
        const bool env = check_env_rounds<8>(A, T, ln, &lane_bytes);
#endif
        uint32_t r = 0;
        if constexpr (RT == FKS_ROBOT_LINKED) {
#if !defined(FKS_PROBE_CHECK_NO_SELF) /* A/B probe only: what the self-collision leg costs */
            if (RDIM(R, self_possible)) r = config_self_collision(args, s.shared(), s.lds(), s.scratch, ln, T, A.self_res, env);
#endif
        }
        const uint64_t bytes = wave_sum_u64(lane_bytes);
        if (ln == 0) {
            A.out_collided[c] = (env || (r & 1u)) ? 1 : 0;
            if (A.out_err) A.out_err[c] = r >> 1;
            bytes_total += bytes;
        }
        wsync();
    }
    if (ln == 0 && bytes_total) atomicAdd(A.counters + kCntSdfBytes, (unsigned long long)bytes_total);
}

/* fks_kinematics (host-side helpers of the reference interface: GetLinkTransform for
 * Get3dPointForConfig SPCS:776-786, the point positions of MakeConfigurationDisplayRep
 * SPCS:634-688, the clean ApplyControlInput of MakeControlInputDisplayRep SPCS:719-774):
 * one wave per configuration, SetPosition then FK / point transforms / clean input */
template <int RT>
__device__ __forceinline__ void kinematics(const SimArgs* __restrict__ args, double* lds_mem) {
    Sim s;
    setup_wave<RT>(args, lds_mem, s);
    const SimArgs& A = *args;
    const RobotDev& R = A.R;
    const int ln = s.lane();
    double* cfg = s.lds() + LAY(A).cfg;
    double* out_cfg = s.lds() + LAY(A).cfg_tmp;
    double* T = s.lds() + LAY(A).Tcur;
    const uint64_t stride = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t c = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); c < A.n; c += stride) {
        set_position<RT>(s, A.starts + c * (uint64_t)RDIM(R, W), cfg);
        if (A.kin_mode == FKS_KIN_APPLY_CONTROL_INPUT) {
            double* in = s.lds() + LAY(A).u;
            if (ln < RDIM(R, D)) in[ln] = A.targets[c * (uint64_t)RDIM(R, D) + ln];
            wsync();
            apply_input<RT>(s, cfg, in, out_cfg, false, 0);
            if (ln < RDIM(R, W)) A.kin_out[c * (uint64_t)RDIM(R, W) + ln] = out_cfg[ln];
        } else {
            fk<RT>(s, cfg, T);
            if (A.kin_mode == FKS_KIN_LINK_TRANSFORMS) {
                for (int e = ln; e < 12 * RDIM(R, L); e += kWave) A.kin_out[c * 12ull * (uint64_t)RDIM(R, L) + e] = T[e];
            } else {
                for (int i = ln; i < RDIM(R, P); i += kWave) {
                    const D4 x = xform4(T + 12 * gp(R.point_link)[i], load_point(R, i));
                    double* o = A.kin_out + (c * (uint64_t)RDIM(R, P) + (uint64_t)i) * 3ull;
                    o[0] = x.x;
                    o[1] = x.y;
                    o[2] = x.z;
                }
            }
        }
        wsync();
    }
}

template <int RT, bool TR, bool IND = false, bool LEAN = false, int COOP = 0>
__device__ __forceinline__ void simulate_particles(const SimArgs* __restrict__ args, double* lds_mem) {
    const SimArgs& A = *args;
    const RobotDev& R = A.R;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); /* wave-uniform: LDS bases stay in SGPRs */
    double* shared = lds_mem;
    {
        /* one copy per workgroup of the robot tables read in the inner loops */
        const int t = (int)threadIdx.x, nt = (int)blockDim.x;
        uint64_t* dj = reinterpret_cast<uint64_t*>(shared + LAY(A).joints);
        const uint64_t* sj = reinterpret_cast<const uint64_t*>(R.joints);
        for (int k = t; k < RDIM(R, J) * kJointWords; k += nt) dj[k] = sj[k];
        uint64_t* dc = reinterpret_cast<uint64_t*>(shared + LAY(A).ctrl);
        const uint64_t* sc = reinterpret_cast<const uint64_t*>(R.ctrl);
        for (int k = t; k < RDIM(R, D) * kCtrlWords; k += nt) dc[k] = sc[k];
        int32_t* dd = reinterpret_cast<int32_t*>(shared + LAY(A).dofj);
        if (RT == FKS_ROBOT_LINKED && t < RDIM(R, D)) dd[t] = gp(R.dof_joint)[t];
        if (t < 12) shared[LAY(A).base + t] = R.base[t];
        if (RT == FKS_ROBOT_LINKED) {
            for (int k = t; k < 8 * RDIM(R, G); k += nt)
                shared[LAY(A).gbox + k] = (k % 8 == 7) ? (double)gp(R.geom_link)[k / 8] : gp(R.geom_box)[7 * (k / 8) + k % 8];
            uint32_t* lp = reinterpret_cast<uint32_t*>(shared + LAY(A).gpairs);
            for (int k = t; k < RDIM(R, npairs) && k < kLdsPairs; k += nt)
                lp[k] = (uint32_t)gp(R.pairs)[2 * k] | ((uint32_t)gp(R.pairs)[2 * k + 1] << 16);
        }
        if (t < RDIM(R, nrounds) && t < kWave) {
            const RoundDev rd = load_round(R.rounds, t);
            shared[LAY(A).rounds + 2 * t] = (double)rd.link;
            shared[LAY(A).rounds + 2 * t + 1] = rd.radius;
        }
        __syncthreads(); /* the only workgroup barrier: waves run independently afterwards (except COOP's) */
    }
    if constexpr (COOP > 0) {
        /* one particle per workgroup: wave 0 runs it, the others help with its point loops */
        if (wave != 0) {
            coop_helper<RT, COOP>(args, lds_mem, wave);
            return;
        }
    }
    Sim s;
    s.A = args;
    s.lds_block = lds_mem + LAY(A).shared_total + (uint64_t)wave * LAY(A).total;
    s.scratch = A.scratch + ((uint64_t)blockIdx.x * (COOP > 0 ? 1u : (blockDim.x >> 6)) + (uint64_t)wave) * A.scratch_per_wave;
    s.lane_v = lane_id();
    /* skip-proof cache of the first 64 rounds (the skip masks are 64-bit; later rounds are always
     * read): in the wave's LDS block, or in its scratch for a lean block (fixed per kernel, so
     * each instantiation addresses it with one kind of load) */
    s.rstate = LEAN ? s.scratch + SLAY(A).rstate : s.lds() + LAY(A).rstate;
    s.selfref = LEAN ? s.scratch + SLAY(A).selfref : s.lds() + LAY(A).selfref;
    if (s.lane() < RDIM(R, nrounds)) s.rstate[kRoundState * s.lane() + 12] = kInvalidRound;
    wsync();
    const int ln = s.lane();
    const int W = RDIM(R, W), D = RDIM(R, D);
    double* cfg = s.lds() + LAY(*s.A).cfg;
    double* res_cfg = s.lds() + LAY(*s.A).cfg_res;
    double* u = s.lds() + LAY(*s.A).u;
    unsigned long long* next_particle = reinterpret_cast<unsigned long long*>(s.lds() + LAY(*s.A).misc + 31);
    uint32_t* seg_seen = reinterpret_cast<uint32_t*>(s.lds() + LAY(*s.A).misc + 30);
    const uint32_t nseg = A.nseg;
    uint64_t carry = kNoTicket; /* the next segment of the particle just run, claimed by this wave */
    bool carry_heavy = false;   /* ... and whether the segment just run was contact-heavy */
    /* call counters are summed per wave and flushed once when the queue is drained
     * (per-segment device atomics on a handful of shared addresses would serialise) */
    if (ln < 8) s.stats()[ln] = 0;
    if (ln < FKS_NUM_PHASES) s.phase()[ln] = 0;
    if (ln < kWaveTotals) s.totals()[ln] = 0;
    s.lane_bytes = 0;
    if (ln < 2) self_counters(s)[ln] = 0;
    if (ln == 0) *reinterpret_cast<uint64_t*>(s.lds() + LAY(*s.A).misc + 6) = 0; /* relative heavy test: pending sums */
    /* timestamps are folded into their LDS sums at once (end - start = (0 - start) + end),
     * so none stays live across the particle loop */
    if (ln == 0) s.phase()[FKS_PHASE_WAVE_RESIDENCY] = 0ull - __builtin_amdgcn_s_memrealtime();
    wsync();
    while (true) {
        /* ticket t: segment t / n of particle t % n, so every particle's first segment is
         * handed out before any second one (processor sharing over the persistent grid:
         * a contact-heavy particle no longer starts late and sets the batch's tail).
         * Segment k >= 1 runs on whichever wave claims it first (seg_done CAS): the
         * ticket's holder if segment k-1 has finished, else the wave finishing k-1 —
         * no wave ever waits for another. */
        uint64_t ticket;
        uint32_t prio = 0;
        if (carry != kNoTicket) {
            ticket = carry;
            carry = kNoTicket;
            /* a wave carrying a contact-heavy particle issues first on its SIMD: the
             * longest particles finish sooner, the batch's tail shrinks */
            prio = carry_heavy ? 2u : (A.seg_heavy_prio > 1u ? 1u : 0u);
        } else {
            if (ln == 0) {
                const uint64_t t = __hip_atomic_fetch_add(A.queue, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t sg = (A.n > 0) ? t / A.n : (uint64_t)nseg;
                uint32_t run = 1;
                if (sg > 0 && sg < (uint64_t)nseg) {
                    uint32_t* done = A.seg_done + (t - sg * A.n);
                    uint32_t v = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    run = (v == (uint32_t)sg &&
                           __hip_atomic_compare_exchange_strong(done, &v, (uint32_t)sg | kSegClaimed, __ATOMIC_RELAXED,
                                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                              ? 1u
                              : 0u;
                }
                *next_particle = t;
                *seg_seen = run;
            }
            wsync();
            ticket = *next_particle;
            const uint32_t run = *seg_seen;
            wsync();
            if ((A.n > 0 ? ticket / A.n : (uint64_t)nseg) >= (uint64_t)nseg) {
                /* the queue is drained: this wave slot idles from here to the kernel's end */
                const uint64_t bytes = wave_sum_u64(s.lane_bytes);
                if (ln == 0) {
                    s.phase()[FKS_PHASE_WAVE_RESIDENCY] += __builtin_amdgcn_s_memrealtime();
                    for (int k = 0; k < 8; ++k)
                        if (s.stats()[k]) atomicAdd(A.counters + k, (unsigned long long)s.stats()[k]);
                    const uint64_t* wt = s.totals();
                    if (wt[kTotSteps]) atomicAdd(A.counters + kCntSteps, (unsigned long long)wt[kTotSteps]);
                    if (wt[kTotMicro]) atomicAdd(A.counters + kCntMicrosteps, (unsigned long long)wt[kTotMicro]);
                    if (wt[kTotResolver]) atomicAdd(A.counters + kCntResolver, (unsigned long long)wt[kTotResolver]);
                    if (wt[kTotLsq]) atomicAdd(A.counters + kCntLsqRows, (unsigned long long)wt[kTotLsq]);
                    if (bytes) atomicAdd(A.counters + kCntSdfBytes, (unsigned long long)bytes);
                    if (wt[kTotErrors]) atomicAdd(A.counters + kCntErrorParticles, (unsigned long long)wt[kTotErrors]);
                    const uint64_t* sc = self_counters(s);
                    if (sc[0]) atomicAdd(A.counters + kCntSelfChecks, (unsigned long long)sc[0]);
                    if (sc[1]) atomicAdd(A.counters + kCntSelfPoints, (unsigned long long)sc[1]);
                    for (int k = 0; k < FKS_NUM_PHASES; ++k)
                        if (s.phase()[k]) atomicAdd(A.counters + kPhaseBase + k, (unsigned long long)s.phase()[k]);
                }
                if constexpr (COOP > 0) {
                    /* release the helpers (every wave of the workgroup meets this barrier last) */
                    if (ln == 0) coop_box(s)->cmd = kCoopExit;
                    coop_sync();
                }
                break;
            }
            if (!run) continue; /* segment already run, being run, or left to the wave finishing its predecessor */
            claim_fence(); /* the resting state is read after the claim */
        }
        /* the issue priority is set afresh for every segment (0 unless carried heavy) */
        if (A.seg_heavy_prio) {
            if (prio == 2u)
                __builtin_amdgcn_s_setprio(2);
            else if (prio == 1u)
                __builtin_amdgcn_s_setprio(1); /* a particle that fell behind the round-robin */
            else
                __builtin_amdgcn_s_setprio(0);
        }
        const uint64_t seg = ticket / A.n;
        const uint64_t local = ticket - seg * A.n;
        const uint32_t step_begin = (uint32_t)seg * A.seg_steps;
        const uint32_t step_end = (seg + 1 == (uint64_t)nseg) ? A.T : step_begin + A.seg_steps;
        double* st = A.seg_state + local * (uint64_t)A.seg_stride; /* nseg > 1 only */
        s.local = local;
        s.tr_steps = 0;
        s.tr_cfgs = 0;
        s.err = 0;
        s.micro_count = 0;
        s.resolver_count = 0;
        s.lsq_rows = 0;
        s.step_count = 0;
        if (ln == 0) s.phase()[FKS_PHASE_PARTICLE] -= __builtin_amdgcn_s_memtime();
        s.self_nonempty = false;
        s.tcur_valid = false;
        if (ln == 0) s.selfref[RDIM(R, D)] = -1.0; /* no self-collision proof reference for this particle yet */
        const double* start = A.starts + local * (uint64_t)W;
        const double* target = (A.num_targets == A.n) ? A.targets + local * (uint64_t)W : A.targets;
        bool collided = false;
        bool any_failed = false;
        if (seg == 0) {
            /* ResetPosition zeroes the controllers (TNUVA:524-536); ForwardSimulateMutableRobot
             * continues the robot's own (SPCS:843-919, fks_forward_simulate_mutable) */
            if (ln < D)
                pid_set<RT>(s, ln, A.pid_io ? A.pid_io[local * 2ull * (uint64_t)D + ln] : 0.0,
                            A.pid_io ? A.pid_io[local * 2ull * (uint64_t)D + D + ln] : 0.0);
            /* ResetPosition(start): SetPosition enforces joint limits / angle wrap */
            if constexpr (RT == FKS_ROBOT_LINKED) {
                if (ln < D) {
                    const JointDev& jd = s.joints()[s.dofj()[ln]];
                    cfg[ln] = (jd.type == FKS_JOINT_CONTINUOUS) ? fks_math::wrap_revolute(start[ln])
                                                                : clamp(start[ln], jd.lo, jd.hi);
                }
            } else if constexpr (RT == FKS_ROBOT_SE2) {
                if (ln < 3) cfg[ln] = (ln == 2) ? fks_math::wrap_revolute(start[2]) : start[ln];
            } else {
                if (ln < 12) cfg[ln] = start[ln];
            }
        } else {
            /* resume: configuration from out_q, controller state and per-particle totals
             * from seg_state (bit-exact: the step loop below recomputes FK at its start) */
            if (ln < W) cfg[ln] = load_coherent(A.out_q + local * (uint64_t)W + ln);
            if (ln < D) pid_set<RT>(s, ln, load_coherent(st + ln), load_coherent(st + D + ln));
            const uint64_t* sw = reinterpret_cast<const uint64_t*>(st + 2 * D);
            const uint64_t flags = load_coherent_u64(sw);
            collided = (flags & 1ull) != 0;
            any_failed = (flags & 2ull) != 0;
            /* the particle's totals so far (sw + 1, + 2) are read again at the segment's end */
            /* the particle's own skip-proof cache (the rounds' last full evaluations) */
            const int nrc = kRoundState * (RDIM(R, nrounds) < kWave ? RDIM(R, nrounds) : kWave);
            for (int e = ln; e < nrc; e += kWave) s.rstate[e] = load_coherent(st + 2 * D + 4 + e);
        }
        wsync();
        double* Tcur = s.lds() + LAY(*s.A).Tcur;
        double* Tprev = s.lds() + LAY(*s.A).Tprev;
        bool ended = false;
        /* ForwardSimulateMutableRobot (SPCS:843-919) */
        for (uint32_t step = step_begin; step < step_end; ++step) {
            s.lane_v = opaque_lane(s.lane_v);
            const int ln = s.lane();
            s.step = step;
            s.step_count++;
            double* tgt_lds = s.lds() + LAY(*s.A).tgt;
            const uint64_t t0 = tick();
            const double uc = control_action<RT>(s, cfg, target);
            if (ln < D) u[ln] = uc * A.dt;
            wsync();
            tock(s, FKS_PHASE_CONTROL, t0);
            bool rc = false, rf = false;
            const int status = resolve_step<RT, TR, IND, COOP>(s, cfg, res_cfg, A.allow_contacts != 0, &rc, &rf, Tcur, Tprev);
            s.err = wave_or(s.err);
            if (status != 0 || s.err) {
                ended = true;
                break;
            }
            if (A.allow_contacts || !rc) {
                if (ln < W) cfg[ln] = res_cfg[ln];
                wsync();
                if (rc) collided = true;
                if (rf) {
                    if (A.S.failed_resolves_end_motion) {
                        ended = true;
                        break;
                    }
                    any_failed = true;
                } else if (any_failed) {
                    if (s.lane() == 0) s.stats()[kCntRecovered]++;
                }
                if (A.S.simulation_shortcut_distance > 0.0 || A.S.simulation_shortcut_distance != A.S.simulation_shortcut_distance) {
                    if (ln < W) tgt_lds[ln] = target[ln];
                    wsync();
                    const double dist = config_distance<RT>(s, cfg, tgt_lds);
                    wsync();
                    if (dist < A.S.simulation_shortcut_distance) {
                        ended = true;
                        break;
                    }
                }
            } else {
                ended = true;
                break;
            }
        }
        if (step_end == A.T) ended = true;
        /* outputs (the configuration doubles as the resting state between segments) */
        const uint64_t t_out = __builtin_amdgcn_s_memtime();
        if (ln < W) store_coherent(A.out_q + local * (uint64_t)W + ln, cfg[ln]);
        uint64_t micro_total = s.micro_count, resolver_total = s.resolver_count;
        if (seg > 0) {
            const uint64_t* sw = reinterpret_cast<const uint64_t*>(st + 2 * D);
            micro_total += load_coherent_u64(sw + 1);
            resolver_total += load_coherent_u64(sw + 2);
        }
        if (!ended) {
            if (ln < D) {
                double integral, last;
                pid_get<RT>(s, ln, &integral, &last);
                store_coherent(st + ln, integral);
                store_coherent(st + D + ln, last);
            }
            if (ln == 0) {
                uint64_t* sw = reinterpret_cast<uint64_t*>(st + 2 * D);
                store_coherent_u64(sw, (collided ? 1ull : 0ull) | (any_failed ? 2ull : 0ull));
                store_coherent_u64(sw + 1, micro_total);
                store_coherent_u64(sw + 2, resolver_total);
            }
            const int nrc = kRoundState * (RDIM(R, nrounds) < kWave ? RDIM(R, nrounds) : kWave);
            for (int e = ln; e < nrc; e += kWave) store_coherent(st + 2 * D + 4 + e, s.rstate[e]);
        }
        if (ln == 0) {
            uint64_t* wt = s.totals();
            wt[kTotSteps] += s.step_count;
            wt[kTotMicro] += s.micro_count;
            wt[kTotResolver] += s.resolver_count;
            wt[kTotLsq] += s.lsq_rows;
            if (s.err) wt[kTotErrors]++;
        }
        if (ended && A.pid_io && ln < D) {
            double integral, last;
            pid_get<RT>(s, ln, &integral, &last);
            A.pid_io[local * 2ull * (uint64_t)D + ln] = integral;
            A.pid_io[local * 2ull * (uint64_t)D + D + ln] = last;
        }
        if (ln == 0) {
            if (ended) {
                if (A.out_collided) A.out_collided[local] = collided ? 1 : 0;
                if (A.out_micro) A.out_micro[local] = (uint32_t)micro_total;
                if (A.out_resolver) A.out_resolver[local] = (uint32_t)resolver_total;
                if (A.out_err) A.out_err[local] = s.err;
                if constexpr (TR) {
                    A.tr_nsteps[local] = s.tr_steps;
                    A.tr_ncfg[local] = s.tr_cfgs;
                }
            }
            const uint64_t t_end = __builtin_amdgcn_s_memtime();
            s.phase()[FKS_PHASE_OUTPUT] += t_end - t_out;
            s.phase()[FKS_PHASE_PARTICLE] += t_end;
        }
        if (nseg > 1) {
            /* publish the resting state; if the next segment's ticket is already out, claim
             * the segment and run it here (its holder, if it looked earlier, skipped it) */
            publish_fence(); /* every lane's state stores have completed */
            wsync();
            if (ln == 0) {
                uint32_t nv = ended ? nseg : (uint32_t)seg + 1u;
                __hip_atomic_store(A.seg_done + local, nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                publish_fence(); /* the store is visible before the ticket counter is read (Dekker with the holder) */
                uint32_t cont = 0;
                /* a contact-heavy segment (many resolver iterations) keeps its wave: the
                 * particle's next segment is claimed at once instead of waiting for its
                 * ticket, so the longest particles are not paced by the round-robin */
                bool heavy = !ended && A.seg_heavy_resolver != 0 && s.resolver_count >= A.seg_heavy_resolver;
                if (A.seg_heavy_rel) {
                    /* relative to the batch: in a contact-heavy batch (its mean so far at or above
                     * the absolute threshold: most segments resolve contacts) only the outliers
                     * are carried.  The wave sums its segments in LDS (misc + 6) and adds them to
                     * the batch's running sums when it has 16 or a candidate needs the mean */
                    uint64_t* pend = reinterpret_cast<uint64_t*>(s.lds() + LAY(*s.A).misc + 6);
                    const uint64_t mine = *pend + (((uint64_t)s.resolver_count << 24) | 1ull);
                    unsigned long long* sums = A.counters + kSchedWord;
                    if (heavy) {
                        const uint64_t prior = __hip_atomic_fetch_add(sums, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint64_t segs = prior & 0xffffffull, iters = prior >> 24;
                        heavy = segs < 256u || iters < (uint64_t)A.seg_heavy_resolver * segs ||
                                (uint64_t)s.resolver_count * segs >= (uint64_t)A.seg_heavy_rel * iters;
                        *pend = 0;
                    } else if ((mine & 0xffffffull) >= 16u) {
                        (void)__hip_atomic_fetch_add(sums, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        *pend = 0;
                    } else {
                        *pend = mine;
                    }
                }
                if (!ended) {
                    const uint64_t next_ticket = (seg + 1) * A.n + local;
                    const uint64_t issued =
                        heavy ? ~0ull : __hip_atomic_load(A.queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (issued > next_ticket &&
                        __hip_atomic_compare_exchange_strong(A.seg_done + local, &nv, nv | kSegClaimed, __ATOMIC_RELAXED,
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        cont = heavy ? 2u : 1u;
                }
                *seg_seen = cont;
            }
            wsync();
            const uint32_t cont = *seg_seen;
            if (cont) {
                carry = (seg + 1) * A.n + local;
                carry_heavy = cont == 2u;
            }
        }
        wsync();
    }
}

/* one kernel per robot family so each carries only its own FK / Jacobian code.
 * The occupancy target bounds the VGPR budget of the kernel and of its out-of-line
 * callees (the rare self-contact path would otherwise set the budget for all). */
#ifndef FKS_WAVES_PER_EU
#define FKS_WAVES_PER_EU 5 /* fksd::kThroughputWavesPerEU */
#endif
#define FKS_KERNEL_ATTRS __launch_bounds__(64 * kMaxWavesPerGroup) __attribute__((amdgpu_waves_per_eu(FKS_WAVES_PER_EU)))
#if defined(FKS_SHAPE_L)
/* the shape-specialised build (fks_specialize.cpp, hiprtc): one throughput kernel for one
 * robot shape, the same template and launch attributes as the generic kernel it replaces
 * (fks_simulate_<family>[_lean]); a robot whose LDS block keeps fewer waves resident than
 * the register budget allows gets the registers of the absent waves (FKS_WAVES_PER_EU) */
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_shaped(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_SHAPE_TYPE, false, false, FKS_SHAPE_LEAN != 0>(args, lds_mem);
}
/* the batched CheckConfigCollision of the same shape (same module, same LDS block) */
extern "C" __global__ void FKS_KERNEL_ATTRS fks_check_configs_shaped(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    check_configs<FKS_SHAPE_TYPE>(args, lds_mem);
}
#if !FKS_SHAPE_LEAN
/* the small-batch instantiation of the same shape (two waves per SIMD; see
 * fks_simulate_<family>_small below), for calls that fit its resident waves once the module
 * is built */
extern "C" __global__ void __launch_bounds__(64 * kMaxWavesPerGroup) __attribute__((amdgpu_waves_per_eu(2)))
fks_simulate_shaped_small(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_SHAPE_TYPE, false>(args, lds_mem);
}
#endif
#else
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se2(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE2, false>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se3(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE3, false>(args, lds_mem);
}

/* small batches (fks_set_small_batch_kernel): at most two waves per SIMD, so the register
 * budget holds the whole working set without spills.  One particle per wave and no
 * segments, chosen only when the batch fits its resident waves: such a batch is the
 * latency of its slowest particle, not a throughput problem (cfg1: 3.8-3.9 ms against
 * 4.2-4.35, profiles/r04j_occupancy_ab_cfg1.log). */
#define FKS_SMALL_KERNEL_ATTRS __launch_bounds__(64 * kMaxWavesPerGroup) __attribute__((amdgpu_waves_per_eu(2)))
extern "C" __global__ void FKS_SMALL_KERNEL_ATTRS fks_simulate_linked_small(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false>(args, lds_mem);
}
extern "C" __global__ void FKS_SMALL_KERNEL_ATTRS fks_simulate_se2_small(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE2, false>(args, lds_mem);
}
extern "C" __global__ void FKS_SMALL_KERNEL_ATTRS fks_simulate_se3_small(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE3, false>(args, lds_mem);
}

/* cooperative small batches (fks_set_cooperative_waves): one particle per workgroup of
 * FKS_COOP_WAVES waves, whose environment checks and correction passes are shared out over
 * them (COOP above); for batches up to one particle per workgroup slot */
#define FKS_COOP_KERNEL_ATTRS __launch_bounds__(64 * FKS_COOP_WAVES) __attribute__((amdgpu_waves_per_eu(2)))
extern "C" __global__ void FKS_COOP_KERNEL_ATTRS fks_simulate_linked_coop(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false, false, false, FKS_COOP_WAVES>(args, lds_mem);
}
extern "C" __global__ void FKS_COOP_KERNEL_ATTRS fks_simulate_se2_coop(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE2, false, false, false, FKS_COOP_WAVES>(args, lds_mem);
}
extern "C" __global__ void FKS_COOP_KERNEL_ATTRS fks_simulate_se3_coop(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE3, false, false, false, FKS_COOP_WAVES>(args, lds_mem);
}

/* simulate_with_individual_jacobians = true (SPCS:420, 1629; fks_set_individual_jacobians) */
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked_indiv(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se2_indiv(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE2, false, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se3_indiv(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE3, false, true>(args, lds_mem);
}

/* traced instantiations: ForwardSimulateRobot with enable_tracing (fks_forward_simulate_traced) */
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked_traced(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se2_traced(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE2, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_se3_traced(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_SE3, true>(args, lds_mem);
}

/* lean LDS blocks (LdsLayout.lean: the round skip-proof cache in the wave's scratch), chosen by
 * fks_set_robot for linked robots whose LDS block limits the resident waves (14-dof cfg5) */
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked_lean(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false, false, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked_lean_indiv(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, false, true, true>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_simulate_linked_lean_traced(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    simulate_particles<FKS_ROBOT_LINKED, true, false, true>(args, lds_mem);
}

extern "C" __global__ void FKS_KERNEL_ATTRS fks_check_configs_linked(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    check_configs<FKS_ROBOT_LINKED>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_check_configs_se2(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    check_configs<FKS_ROBOT_SE2>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_check_configs_se3(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    check_configs<FKS_ROBOT_SE3>(args, lds_mem);
}

extern "C" __global__ void FKS_KERNEL_ATTRS fks_kinematics_linked(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    kinematics<FKS_ROBOT_LINKED>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_kinematics_se2(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    kinematics<FKS_ROBOT_SE2>(args, lds_mem);
}
extern "C" __global__ void FKS_KERNEL_ATTRS fks_kinematics_se3(const SimArgs* __restrict__ args) {
    extern __shared__ __attribute__((aligned(16))) double lds_mem[];
    kinematics<FKS_ROBOT_SE3>(args, lds_mem);
}

#endif /* FKS_SHAPE_L */

#if !defined(FKS_SHAPE_L)
/* device self-test of the portable libm (fks_selftest_math) */
extern "C" __global__ void fks_math_probe(const double* a, const double* b, double* out, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = a[i], y = b[i];
    out[8 * i + 0] = fks_math::sin(x);
    out[8 * i + 1] = fks_math::cos(x);
    out[8 * i + 2] = fks_math::log(fks_math::dabs(y) + 1e-300);
    out[8 * i + 3] = fks_math::atan2(x, y);
    out[8 * i + 4] = fks_math::dsqrt(fks_math::dabs(y));
    out[8 * i + 5] = x / y;
    out[8 * i + 6] = fks_math::wrap_revolute(x / y); /* |x / y| from 1e-7 to beyond 1e9: the long division's every length */
    out[8 * i + 7] = (x * y + x) * y - x * x;
}
#endif
