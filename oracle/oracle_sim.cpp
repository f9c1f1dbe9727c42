/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle of the particle forward-simulation path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (as the checker / reported CPU baseline); the product never does.
 *
 * A restatement of SimpleParticleContactSimulator (reference
 * include/fast_kinematic_simulator/simple_particle_contact_simulator.hpp = SPCS)
 * keeping the reference's call structure: per-check robot Clone() + full FK,
 * name-based link lookups, std::unordered_map self-collision grid, row-by-row
 * grown dynamic Jacobian, column-pivoting Householder QR.  Function-by-function
 * citations are on each function.  External-library primitives (sdf_tools,
 * arc_utilities, Eigen) are restated in oracle_geometry.h / oracle_models.h and
 * below with the evaluation orders documented in DESIGN.md.
 *
 * Parity status: UNPINNED against the reference binary (it cannot be built
 * here, SURVEY.md §8c: Eigen/arc_utilities/sdf_tools/ROS absent).  Pinned
 * pieces: PID against golden vectors produced by the reference header itself
 * (tests/golden/pid_golden.json), Philox against the Random123 KATs, the
 * portable libm against glibc (<= 1 ulp).
 */
#include <omp.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

#include "fks_capi.h"
#include "fks_portable_math.h"
#include "oracle_geometry.h"
#include "oracle_models.h"
#include "oracle_rng.h"

namespace oracle {

/* ---------------- counters ---------------- */
struct ParticleCounters {
    uint64_t microsteps = 0;
    uint64_t resolver_iterations = 0;
    uint64_t controller_steps = 0;
    uint64_t sdf_bytes = 0;
    uint64_t lsq_rows = 0;
    uint64_t self_checks = 0; /* CheckCollision calls with a non-empty self-collision map */
    uint64_t self_points = 0; /* corrected points holding a self-collision term */
    uint32_t error_flags = 0;
    fks_statistics stats;
    struct TraceSink* trace = nullptr; /* ForwardSimulationStepTrace of this particle (traced calls only) */
    ParticleCounters() { std::memset(&stats, 0, sizeof(stats)); }
};

/* ForwardSimulationStepTrace (simple_simulator_interface) flattened as in
 * include/fks_capi.h fks_trace: one record per resolver_steps entry
 * (SPCS:1583-1588) and one per contact_resolution_steps push (SPCS:1617,
 * 1703, 1714, 1778), tagged with (controller step, microstep, kind) */
struct TraceSink {
    std::vector<double> step_inputs; /* per step: real_control_input, control_input_step */
    std::vector<uint32_t> step_microsteps;
    std::vector<double> configs;
    std::vector<uint32_t> config_tags;
    uint32_t step = 0;
    void add_step(const std::vector<double>& u, const std::vector<double>& ustep, uint32_t m) {
        step_inputs.insert(step_inputs.end(), u.begin(), u.end());
        step_inputs.insert(step_inputs.end(), ustep.begin(), ustep.end());
        step_microsteps.push_back(m);
    }
    void add_config(const std::vector<double>& q, uint32_t micro, uint32_t kind) {
        configs.insert(configs.end(), q.begin(), q.end());
        config_tags.push_back(step);
        config_tags.push_back(micro);
        config_tags.push_back(kind);
    }
};

/* truncate toward zero like (int64_t)x; non-finite/huge values are rejected
 * explicitly (the C++ cast would be undefined there) */
static inline bool trunc_index(double v, int64_t* out) {
    if (!(v > -9.0e18 && v < 9.0e18)) return false;
    *out = (int64_t)v;
    return true;
}

/* ---------------- canonical wave reduction ----------------
 * sum_{r in [begin,end)} terms[r], evaluated as 64 lane-strided partial sums
 * (lane l accumulates rows r = l mod 64 in ascending r, starting from +0.0),
 * then an xor-butterfly over offsets 1,2,4,8,16,32.  This is the order the HIP
 * kernel's 64-lane wavefront reduction (DPP within rows, readlane across rows) produces; it is the oracle's definition
 * of every long sum in the least-squares solve (DESIGN.md §Canonical sums). */
static double canon_sum(const std::vector<double>& terms, size_t begin, size_t end) {
#ifdef ORACLE_AUDIT_SEQUENTIAL_SUMS /* restatement audit alternative: ascending scalar sum */
    double acc = 0.0;
    for (size_t r = begin; r < end; ++r) acc = acc + terms[r];
    return acc;
#endif
    double partial[64];
    for (int l = 0; l < 64; ++l) partial[l] = 0.0;
    for (size_t r = begin; r < end; ++r) partial[r % 64] = partial[r % 64] + terms[r];
    for (int off = 1; off <= 32; off <<= 1) {
        double next[64];
        for (int l = 0; l < 64; ++l) next[l] = partial[l] + partial[l ^ off];
        for (int l = 0; l < 64; ++l) partial[l] = next[l];
    }
    return partial[0];
}

/* ---------------- voxel grids (arc_utilities VoxelGrid restated) ---------------- */
struct GridGeom {
    Iso origin, inverse_origin;
    double res, inv_res;
    int64_t n[3];
    explicit GridGeom(const fks_grid_geometry& g) {
        origin = iso_from12(g.origin);
        inverse_origin = inverse(origin);
        res = g.resolution;
        inv_res = 1.0 / g.resolution;
        n[0] = g.num_cells[0];
        n[1] = g.num_cells[1];
        n[2] = g.num_cells[2];
    }
    /* LocationToGridIndex4d + IndexInBounds */
    bool LocationToGridIndex4d(const V4& p, int64_t idx[3]) const {
        const V4 g = xform4(inverse_origin, p);
        if (!trunc_index(g.x * inv_res, &idx[0]) || !trunc_index(g.y * inv_res, &idx[1]) ||
            !trunc_index(g.z * inv_res, &idx[2]))
            return false;
        return idx[0] >= 0 && idx[1] >= 0 && idx[2] >= 0 && idx[0] < n[0] && idx[1] < n[1] && idx[2] < n[2];
    }
    size_t Linear(int64_t i, int64_t j, int64_t k) const { return ((size_t)i * (size_t)n[1] + (size_t)j) * (size_t)n[2] + (size_t)k; }
    /* GridIndexToLocation: cell centre */
    V3 GridIndexToLocation(int64_t i, int64_t j, int64_t k) const {
        return xform3(origin, V3{res * ((double)i + 0.5), res * ((double)j + 0.5), res * ((double)k + 0.5)});
    }
};

/* sdf_tools::SignedDistanceField restated (GetImmutable4d, GetGradient, EstimateDistance4d) */
struct SDF {
    GridGeom g;
    const float* data;
    float oob;
    SDF(const fks_grid_geometry& geom, const float* d, float o) : g(geom), data(d), oob(o) {}
    float Get(int64_t i, int64_t j, int64_t k) const { return data[g.Linear(i, j, k)]; }
    std::pair<float, bool> GetImmutable4d(const V4& p, uint64_t* bytes) const {
        int64_t idx[3];
        if (!g.LocationToGridIndex4d(p, idx)) return std::make_pair(oob, false);
        *bytes += 4;
        return std::make_pair(Get(idx[0], idx[1], idx[2]), true);
    }
    /* GetGradient(x, y, z, enable_edge_gradients = true): central differences of
     * float values (float subtraction, then scaled in double); one-sided at edges.
     * Interior cells use 1/(res*2) which is bitwise 1/(2*res). */
    V3 GetGradient(int64_t i, int64_t j, int64_t k) const {
        const int64_t idx[3] = {i, j, k};
        double grad[3];
        for (int a = 0; a < 3; ++a) {
            int64_t lo[3] = {i, j, k}, hi[3] = {i, j, k};
            lo[a] = (idx[a] - 1 > 0) ? idx[a] - 1 : 0;
            hi[a] = (idx[a] + 1 < g.n[a] - 1) ? idx[a] + 1 : g.n[a] - 1;
            const double inv = 1.0 / (g.res * (double)(hi[a] - lo[a]));
            const float diff = Get(hi[0], hi[1], hi[2]) - Get(lo[0], lo[1], lo[2]);
            grad[a] = (double)diff * inv;
        }
        return V3{grad[0], grad[1], grad[2]};
    }
    /* EstimateDistance4d: nominal cell value moved half a cell toward zero plus the
     * gradient projection of the offset from the cell centre; a sign flip against the
     * nominal value is replaced by +-res/16 */
    std::pair<double, bool> EstimateDistance4d(const V4& p, uint64_t* bytes) const {
        int64_t idx[3];
        if (!g.LocationToGridIndex4d(p, idx)) return std::make_pair((double)oob, false);
        *bytes += 28;
        const V3 grad = GetGradient(idx[0], idx[1], idx[2]);
        const V3 c = g.GridIndexToLocation(idx[0], idx[1], idx[2]);
        const double dx = p.x - c.x, dy = p.y - c.y, dz = p.z - c.z;
        const double nominal = (double)Get(idx[0], idx[1], idx[2]);
        const double corrected = (nominal >= 0.0) ? nominal - (g.res * 0.5) : nominal + (g.res * 0.5);
        const double adjustment = (dx * grad.x + dy * grad.y) + dz * grad.z;
        const double estimate = corrected + adjustment;
        if ((corrected >= 0.0) == (estimate >= 0.0)) return std::make_pair(estimate, true);
        if (corrected >= 0.0) return std::make_pair(g.res * 0.0625, true);
        return std::make_pair(g.res * -0.0625, true);
    }
};

/* SurfaceNormalGrid (SPCS:44-343) over CSR storage */
struct NormalGrid {
    GridGeom g;
    const uint32_t* offsets;
    const double* entries;
    NormalGrid(const fks_grid_geometry& geom, const uint32_t* o, const double* e) : g(geom), offsets(o), entries(e) {}
    /* LookupSurfaceNormal(Vector4d location, Vector4d direction) SPCS:186-198,235-256 with
     * GetBestSurfaceNormal(.., Vector4d) SPCS:111-132: first strict maximum of
     * entry_direction . (direction / |direction|).  Returns in_bounds. */
    bool Lookup(const V4& location, const V4& direction, V3* out, uint32_t* err, uint64_t* bytes) const {
        int64_t idx[3];
        *out = V3{0.0, 0.0, 0.0};
        if (offsets == nullptr || !g.LocationToGridIndex4d(location, idx)) return false;
        const size_t lin = g.Linear(idx[0], idx[1], idx[2]);
        const uint32_t begin = offsets[lin], end = offsets[lin + 1];
        /* 4 B for the cell, 56 B per entry examined (a StoredSurfaceNormal is a
         * Vector4d entry direction + Vector3d normal, SPCS:52-53) */
        *bytes += 4;
        if (begin == end) return true;
        *bytes += 56ull * (uint64_t)(end - begin);
        const double direction_norm = fks_math::dsqrt(sqnorm4(direction));
        if (!(direction_norm > 0.0)) {
            *err |= FKS_PARTICLE_ERR_ZERO_DIRECTION; /* assert(direction_norm > 0.0), SPCS:115 */
            return true;
        }
        const double ux = direction.x / direction_norm, uy = direction.y / direction_norm,
                     uz = direction.z / direction_norm;
        int64_t best = -1;
        double best_dot = -HUGE_VAL;
        for (uint32_t e = begin; e < end; ++e) {
            const double* ent = entries + 6 * (size_t)e;
            /* EntryDirection4d().dot(unit_direction) SPCS:122 in Eigen's packet order; both
             * w terms are +0 (SPCS:62 stores (entry, 0); the motion's w is 1 - 1) */
#ifdef ORACLE_AUDIT_V4_SEQUENTIAL
            const double dot = (ent[0] * ux + ent[1] * uy) + ent[2] * uz;
#else
            const double dot = (ent[0] * ux + ent[2] * uz) + ent[1] * uy;
#endif
            if (dot > best_dot) {
                best_dot = dot;
                best = (int64_t)e;
            }
        }
        if (best < 0) {
            *err |= FKS_PARTICLE_ERR_ZERO_DIRECTION; /* assert(best_stored_index >= 0), SPCS:129 */
            return true;
        }
        const double* ent = entries + 6 * (size_t)best;
        *out = V3{ent[3], ent[4], ent[5]};
        return true;
    }
};

/* ---------------- dense helpers for the self-collision impulse solve ---------------- */
struct Dense {
    size_t rows, cols;
    std::vector<double> a;
    Dense(size_t r, size_t c) : rows(r), cols(c), a(r * c, 0.0) {}
    double& operator()(size_t i, size_t j) { return a[i * cols + j]; }
    double operator()(size_t i, size_t j) const { return a[i * cols + j]; }
};
static Dense matmul(const Dense& A, const Dense& B) {
    Dense C(A.rows, B.cols);
    for (size_t i = 0; i < A.rows; ++i)
        for (size_t j = 0; j < B.cols; ++j) {
            double acc = 0.0;
            for (size_t k = 0; k < A.cols; ++k) acc = acc + A(i, k) * B(k, j);
            C(i, j) = acc;
        }
    return C;
}
static Dense transpose(const Dense& A) {
    Dense T(A.cols, A.rows);
    for (size_t i = 0; i < A.rows; ++i)
        for (size_t j = 0; j < A.cols; ++j) T(j, i) = A(i, j);
    return T;
}
/* MatrixXd::inverse() restated as Gauss-Jordan with partial pivoting (first max) */
static Dense inverse(const Dense& A) {
    const size_t n = A.rows;
    Dense aug(n, 2 * n);
    for (size_t i = 0; i < n; ++i) {
        for (size_t j = 0; j < n; ++j) aug(i, j) = A(i, j);
        aug(i, n + i) = 1.0;
    }
    for (size_t c = 0; c < n; ++c) {
        size_t p = c;
        double best = fks_math::dabs(aug(c, c));
        for (size_t r = c + 1; r < n; ++r)
            if (fks_math::dabs(aug(r, c)) > best) {
                best = fks_math::dabs(aug(r, c));
                p = r;
            }
        if (p != c)
            for (size_t j = 0; j < 2 * n; ++j) std::swap(aug(c, j), aug(p, j));
        const double piv = aug(c, c);
        for (size_t j = 0; j < 2 * n; ++j) aug(c, j) = aug(c, j) / piv;
        for (size_t r = 0; r < n; ++r) {
            if (r == c) continue;
            const double f = aug(r, c);
            for (size_t j = 0; j < 2 * n; ++j) aug(r, j) = aug(r, j) - f * aug(c, j);
        }
    }
    Dense inv(n, n);
    for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < n; ++j) inv(i, j) = aug(i, n + j);
    return inv;
}

/* ---------------- ColPivHouseholderQR::solve restated (Eigen 3.2 / 3.3-beta1) ----------------
 * J is R x D (row-major), returns x (D).  Squared column norms with downdate and
 * recompute of the selected column, Householder vectors per makeHouseholder
 * (tol = DBL_MIN), nonzero pivots by threshold maxColSqNorm*eps^2/R*(R-k), Q^T b
 * applied for k < nonzero pivots, column-oriented back substitution, basic
 * solution (zeros in non-pivot unknowns).  Long sums are canon_sum(). */
std::vector<double> colpiv_qr_solve(const std::vector<double>& Jrm, size_t R, size_t D, const std::vector<double>& b,
                                    std::vector<size_t>* perm_out = nullptr, size_t* nonzero_out = nullptr) {
    std::vector<double> x(D, 0.0);
    if (perm_out) perm_out->assign(D, 0);
    if (nonzero_out) *nonzero_out = 0;
    if (D == 0) return x;
    /* column-major working copy */
    std::vector<double> qr(R * D);
    for (size_t r = 0; r < R; ++r)
        for (size_t c = 0; c < D; ++c) qr[c * R + r] = Jrm[r * D + c];
    auto col = [&](size_t c) { return &qr[c * R]; };
    const size_t size = (R < D) ? R : D;
    std::vector<double> hcoeffs(size, 0.0), colsq(D, 0.0);
    std::vector<size_t> transpositions(D, 0);
    std::vector<double> terms(R, 0.0);
    auto tail_sqnorm = [&](size_t c, size_t begin) {
        for (size_t r = begin; r < R; ++r) terms[r] = col(c)[r] * col(c)[r];
        return canon_sum(terms, begin, R);
    };
    for (size_t c = 0; c < D; ++c) colsq[c] = tail_sqnorm(c, 0);
    double maxsq = colsq[0];
    for (size_t c = 1; c < D; ++c)
        if (colsq[c] > maxsq) maxsq = colsq[c];
    const double eps = 2.220446049250313e-16;
    const double threshold_helper = maxsq * (eps * eps) / (double)R;
    size_t nonzero_pivots = size;
    for (size_t k = 0; k < size; ++k) {
        size_t biggest = k;
        double biggest_sq = colsq[k];
        for (size_t c = k + 1; c < D; ++c)
            if (colsq[c] > biggest_sq) {
                biggest_sq = colsq[c];
                biggest = c;
            }
        biggest_sq = tail_sqnorm(biggest, k);
        colsq[biggest] = biggest_sq;
        if (nonzero_pivots == size && biggest_sq < threshold_helper * (double)(R - k)) nonzero_pivots = k;
        transpositions[k] = biggest;
        if (k != biggest) {
            for (size_t r = 0; r < R; ++r) std::swap(col(k)[r], col(biggest)[r]);
            std::swap(colsq[k], colsq[biggest]);
        }
        /* makeHouseholderInPlace on col(k)[k..R) */
        const double c0 = col(k)[k];
        const double tail = (R - k == 1) ? 0.0 : tail_sqnorm(k, k + 1);
        double tau, beta;
        if (tail <= 2.2250738585072014e-308) {
            tau = 0.0;
            beta = c0;
            for (size_t r = k + 1; r < R; ++r) col(k)[r] = 0.0;
        } else {
            beta = fks_math::dsqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double denom = c0 - beta;
            for (size_t r = k + 1; r < R; ++r) col(k)[r] = col(k)[r] / denom;
            tau = (beta - c0) / beta;
        }
        hcoeffs[k] = tau;
        col(k)[k] = beta;
        /* applyHouseholderOnTheLeft to the bottom-right corner */
        if (R - k == 1) {
            for (size_t j = k + 1; j < D; ++j) col(j)[k] = col(j)[k] * (1.0 - tau);
        } else if (tau != 0.0) {
            for (size_t j = k + 1; j < D; ++j) {
                for (size_t r = k + 1; r < R; ++r) terms[r] = col(k)[r] * col(j)[r];
                double tmp = canon_sum(terms, k + 1, R);
                tmp = tmp + col(j)[k];
                col(j)[k] = col(j)[k] - tau * tmp;
                for (size_t r = k + 1; r < R; ++r) col(j)[r] = col(j)[r] - (tau * col(k)[r]) * tmp;
            }
        }
        /* squared-norm downdate */
        for (size_t j = k + 1; j < D; ++j) colsq[j] = colsq[j] - col(j)[k] * col(j)[k];
    }
    std::vector<size_t> perm(D);
    for (size_t i = 0; i < D; ++i) perm[i] = i;
    for (size_t k = 0; k < size; ++k) std::swap(perm[k], perm[transpositions[k]]);
    if (perm_out) *perm_out = perm;
    if (nonzero_out) *nonzero_out = nonzero_pivots;
    if (nonzero_pivots == 0) return x;
    std::vector<double> c(b);
    for (size_t k = 0; k < nonzero_pivots; ++k) {
        const double tau = hcoeffs[k];
        if (R - k == 1) {
            c[k] = c[k] * (1.0 - tau);
        } else if (tau != 0.0) {
            for (size_t r = k + 1; r < R; ++r) terms[r] = col(k)[r] * c[r];
            double tmp = canon_sum(terms, k + 1, R);
            tmp = tmp + c[k];
            c[k] = c[k] - tau * tmp;
            for (size_t r = k + 1; r < R; ++r) c[r] = c[r] - (tau * col(k)[r]) * tmp;
        }
    }
    /* upper-triangular solve, column oriented */
    for (size_t ii = nonzero_pivots; ii-- > 0;) {
        if (c[ii] != 0.0) {
            c[ii] = c[ii] / col(ii)[ii];
            for (size_t r = 0; r < ii; ++r) c[r] = c[r] - c[ii] * col(ii)[r];
        }
    }
    for (size_t i = 0; i < nonzero_pivots; ++i) x[perm[i]] = c[i];
    for (size_t i = nonzero_pivots; i < D; ++i) x[perm[i]] = 0.0;
    return x;
}

/* Capture of the stacked least-squares systems the simulator solves (SPCS:1990-1998),
 * for the pivot-rule pin against LAPACK dgeqp3 (tests/golden/make_qr_golden.py): every
 * `stride`-th system with at most `max_rows` rows, up to `max_systems` of them. */
struct SystemCapture {
    std::mutex mu;
    uint64_t max_systems = 0, stride = 1, max_rows = 0, seen = 0;
    std::vector<double> J, b;
    std::vector<uint64_t> shape; /* rows, cols per system */
};
static SystemCapture g_capture;

static void capture_system(const std::vector<double>& Jrm, size_t R, size_t D, const std::vector<double>& b) {
    if (g_capture.max_systems == 0) return;
    std::lock_guard<std::mutex> lock(g_capture.mu);
    if (g_capture.shape.size() / 2 >= g_capture.max_systems || R == 0 || R > g_capture.max_rows) return;
    if ((g_capture.seen++ % g_capture.stride) != 0) return;
    g_capture.J.insert(g_capture.J.end(), Jrm.begin(), Jrm.begin() + (long)(R * D));
    g_capture.b.insert(g_capture.b.end(), b.begin(), b.begin() + (long)R);
    g_capture.shape.push_back(R);
    g_capture.shape.push_back(D);
}

/* ComputeResolverCorrectionStepIndividualJacobians (SPCS:1966-1988): each corrected
 * point's 3 x D block solved on its own, the steps summed in point order (the first
 * assigned, later ones raw + step).  No corrected point: the zero step, as the stacked
 * solve of an empty system returns. */
std::vector<double> individual_jacobians_solve(const std::vector<double>& Jrm, size_t R, size_t D, const std::vector<double>& b) {
    std::vector<double> raw(D, 0.0);
    for (size_t r0 = 0; r0 < R; r0 += 3) {
        const std::vector<double> Jb(Jrm.begin() + (long)(r0 * D), Jrm.begin() + (long)((r0 + 3) * D));
        const std::vector<double> bb(b.begin() + (long)r0, b.begin() + (long)r0 + 3);
        const std::vector<double> step = colpiv_qr_solve(Jb, 3, D, bb);
        for (size_t i = 0; i < D; ++i) raw[i] = (r0 == 0) ? step[i] : raw[i] + step[i];
    }
    return raw;
}

/* ---------------- the simulator ---------------- */
struct PairHash {
    size_t operator()(const std::pair<size_t, size_t>& p) const {
        return std::hash<size_t>()(p.first) ^ (std::hash<size_t>()(p.second) << 1); /* SPCS:28-40 */
    }
};
struct GridIndex {
    int64_t x, y, z;
    bool operator==(const GridIndex& o) const { return x == o.x && y == o.y && z == o.z; }
};
struct GridIndexHash {
    size_t operator()(const GridIndex& g) const {
        size_t h = std::hash<int64_t>()(g.x);
        h ^= std::hash<int64_t>()(g.y) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        h ^= std::hash<int64_t>()(g.z) + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
        return h;
    }
};
typedef std::unordered_map<std::pair<size_t, size_t>, V3, PairHash> SelfMap;
typedef std::shared_ptr<RobotModel> RobotPtr;

struct ResolveResult {
    Config config;
    bool collided;
    bool failed;
    bool error;
};

class Simulator {
  public:
    Simulator(const fks_environment& env, const fks_solver_params& p, double freq, int32_t debug,
              bool simulate_with_individual_jacobians = false)
        : env_geom_(env.collision_map),
          sdf_(env.sdf, env.sdf_values, env.sdf_oob_value),
          normals_(env.normals, env.normal_offsets, env.normal_entries),
          solver_(p),
          debug_level_(debug),
          simulate_with_individual_jacobians_(simulate_with_individual_jacobians) {
        contact_distance_threshold_ = 0.0;
        resolution_distance_threshold_ = 0.0;
        simulation_controller_frequency_ = fks_math::dabs(freq);
        simulation_controller_interval_ = 1.0 / freq;
    }

    double GetResolution() const { return env_geom_.res; }

    /* SPCS:921-981 */
    bool CheckEnvironmentCollision(const RobotPtr& robot, const LinkGeometries& geoms, double collision_threshold,
                                   ParticleCounters& pc) const {
        const double real_collision_threshold =
            collision_threshold - (solver_.environment_collision_check_tolerance * sdf_.g.res);
        for (size_t link_idx = 0; link_idx < geoms.size(); ++link_idx) {
            const std::string& link_name = geoms[link_idx].first;
            const std::vector<V4>& link_points = *geoms[link_idx].second.points;
            const Iso link_transform = robot->GetLinkTransform(link_name);
            for (size_t point_idx = 0; point_idx < link_points.size(); ++point_idx) {
                const V4 p = xform4(link_transform, link_points[point_idx]);
                const std::pair<float, bool> sdf_check = sdf_.GetImmutable4d(p, &pc.sdf_bytes);
                if ((double)sdf_check.first < real_collision_threshold) {
                    if ((double)sdf_check.first < (real_collision_threshold - sdf_.g.res)) return true;
                    const double estimated = sdf_.EstimateDistance4d(p, &pc.sdf_bytes).first;
                    if (estimated < real_collision_threshold) return true;
                }
            }
        }
        return false;
    }

    /* ExtractSelfCollidingPoints SPCS:983-1171 */
    std::map<std::pair<size_t, size_t>, V3> ExtractSelfCollidingPoints(
        const RobotPtr& previous_robot, const RobotPtr& current_robot, const LinkGeometries& geoms,
        const std::vector<std::pair<size_t, size_t>>& candidate_points, const std::map<size_t, double>& link_masses,
        double time_interval, size_t* colliding_cells, ParticleCounters& pc) const {
        std::map<std::pair<size_t, size_t>, V3> result;
        if (candidate_points.size() <= 1) return result;
        std::map<size_t, std::vector<size_t>> by_link;
        for (size_t idx = 0; idx < candidate_points.size(); ++idx)
            by_link[candidate_points[idx].first].push_back(candidate_points[idx].second);
        if (by_link.size() < 2) return result;
        std::map<size_t, std::vector<size_t>> link_collisions;
        for (auto f = by_link.begin(); f != by_link.end(); ++f)
            for (auto s = by_link.begin(); s != by_link.end(); ++s)
                if (f != s && !current_robot->CheckIfSelfCollisionAllowed(f->first, s->first))
                    link_collisions[f->first].push_back(s->first);
        if (link_collisions.size() < 2) return result;
        (*colliding_cells)++;
        const double time_multiplier = 1.0 / time_interval;
        std::map<size_t, V4> momentum;
        for (auto it = by_link.begin(); it != by_link.end(); ++it) {
            const size_t link_idx = it->first;
            if (link_collisions.find(link_idx) == link_collisions.end()) continue;
            const Iso Tp = previous_robot->GetLinkTransform(geoms[link_idx].first);
            const Iso Tc = current_robot->GetLinkTransform(geoms[link_idx].first);
            V4 m{0.0, 0.0, 0.0, 0.0};
            for (size_t idx = 0; idx < it->second.size(); ++idx) {
                const V4& lp = (*geoms[link_idx].second.points)[it->second[idx]];
                const V4 prev = xform4(Tp, lp), cur = xform4(Tc, lp);
                const V4 vel{(cur.x - prev.x) * time_multiplier, (cur.y - prev.y) * time_multiplier,
                             (cur.z - prev.z) * time_multiplier, (cur.w - prev.w) * time_multiplier};
                m = V4{m.x + vel.x, m.y + vel.y, m.z + vel.z, m.w + vel.w};
            }
            momentum[link_idx] = m;
        }
        for (auto it = link_collisions.begin(); it != link_collisions.end(); ++it) {
            const size_t link_idx = it->first;
            const std::vector<size_t>& colliding = it->second;
            const size_t n = colliding.size();
            const Iso Tp = previous_robot->GetLinkTransform(geoms[link_idx].first);
            const V4 link_loc = xform4(Tp, (*geoms[link_idx].second.points)[by_link[link_idx].front()]);
            const V4 mom = momentum[link_idx];
            const double cnt = (double)by_link[link_idx].size();
            const V4 link_vel{mom.x / cnt, mom.y / cnt, mom.z / cnt, mom.w / cnt};
            Dense C((n + 1) * 3, n * 3);
            for (size_t l = 1; l <= n; ++l)
                for (size_t d = 0; d < 3; ++d) {
                    C(d, (l - 1) * 3 + d) = -1.0;
                    C(l * 3 + d, (l - 1) * 3 + d) = 1.0;
                }
            Dense N(n * 3, n);
            for (size_t c = 0; c < n; ++c) {
                const size_t other = colliding[c];
                const Iso Tpo = previous_robot->GetLinkTransform(geoms[other].first);
                const V4 other_loc = xform4(Tpo, (*geoms[other].second.points)[by_link[other].front()]);
                const V4 cn = safe_normal4(V4{other_loc.x - link_loc.x, other_loc.y - link_loc.y,
                                              other_loc.z - link_loc.z, other_loc.w - link_loc.w});
                N(c * 3 + 0, c) = cn.x;
                N(c * 3 + 1, c) = cn.y;
                N(c * 3 + 2, c) = cn.z;
            }
            Dense M((n + 1) * 3, (n + 1) * 3);
            const double link_mass = link_masses.find(link_idx)->second;
            for (size_t d = 0; d < 3; ++d) M(d, d) = link_mass;
            for (size_t l = 1; l <= n; ++l) {
                const double om = link_masses.find(colliding[l - 1])->second;
                for (size_t d = 0; d < 3; ++d) M(l * 3 + d, l * 3 + d) = om;
            }
            Dense V((n + 1) * 3, 1);
            V(0, 0) = link_vel.x;
            V(1, 0) = link_vel.y;
            V(2, 0) = link_vel.z;
            for (size_t l = 1; l <= n; ++l) {
                const size_t other = colliding[l - 1];
                const double oc = (double)by_link[other].size();
                const V4 om = momentum[other];
                V(l * 3 + 0, 0) = om.x / oc;
                V(l * 3 + 1, 0) = om.y / oc;
                V(l * 3 + 2, 0) = om.z / oc;
            }
            const Dense Nt = transpose(N), Ct = transpose(C), Minv = inverse(M);
            const Dense A = matmul(matmul(matmul(matmul(Nt, Ct), Minv), C), N);
            const Dense impulses = matmul(matmul(matmul(inverse(A), Nt), Ct), V);
            const Dense dv = matmul(matmul(matmul(Minv, C), N), impulses);
            const V3 corr{dv(0, 0) * -1.0, dv(1, 0) * -1.0, dv(2, 0) * -1.0};
            const std::vector<size_t>& link_points = by_link[link_idx];
            const double np = (double)link_points.size();
            for (size_t idx = 0; idx < link_points.size(); ++idx) {
                const V3 pcorr{corr.x / np, corr.y / np, corr.z / np};
                if (std::isnan(pcorr.x) || std::isnan(pcorr.y) || std::isnan(pcorr.z))
                    pc.error_flags |= FKS_PARTICLE_ERR_SELF_SINGULAR; /* assert(!isnan) SPCS:1151-1153 */
                result[std::make_pair(link_idx, link_points[idx])] = pcorr;
            }
        }
        return result;
    }

    /* LocationToExtendedGridIndex SPCS:1173-1181 (division by the extended resolution,
     * truncation toward zero) */
    GridIndex LocationToExtendedGridIndex(const V4& location, double extended_grid_resolution, ParticleCounters& pc) const {
        const V4 g = xform4(env_geom_.inverse_origin, location);
        const double q[3] = {g.x / extended_grid_resolution, g.y / extended_grid_resolution, g.z / extended_grid_resolution};
        int64_t k[3];
        for (int a = 0; a < 3; ++a) {
            if (q[a] != q[a] || q[a] == HUGE_VAL || q[a] == -HUGE_VAL) {
                pc.error_flags |= FKS_PARTICLE_ERR_KEY_RANGE;
                k[a] = 0;
            } else if (q[a] >= 9.0e18) {
                k[a] = (int64_t)9000000000000000000ll;
            } else if (q[a] <= -9.0e18) {
                k[a] = -(int64_t)9000000000000000000ll;
            } else {
                k[a] = (int64_t)q[a];
            }
        }
        return GridIndex{k[0], k[1], k[2]};
    }

    /* CollectSelfCollisions SPCS:1183-1275 */
    SelfMap CollectSelfCollisions(const RobotPtr& previous_robot, const RobotPtr& current_robot, const LinkGeometries& geoms,
                                  double time_interval, ParticleCounters& pc) const {
        if (geoms.size() == 1) return SelfMap();
        if (geoms.size() == 2 && current_robot->CheckIfSelfCollisionAllowed(0, 1)) return SelfMap();
        std::unordered_map<GridIndex, std::vector<std::pair<size_t, size_t>>, GridIndexHash> check_map;
        bool any_candidate = false;
        for (size_t link_idx = 0; link_idx < geoms.size(); ++link_idx) {
            const std::vector<V4>& link_points = *geoms[link_idx].second.points;
            const Iso T = current_robot->GetLinkTransform(geoms[link_idx].first);
            for (size_t point_idx = 0; point_idx < link_points.size(); ++point_idx) {
                const V4 p = xform4(T, link_points[point_idx]);
                const GridIndex key = LocationToExtendedGridIndex(p, env_geom_.res, pc);
                std::vector<std::pair<size_t, size_t>>& cell = check_map[key];
                if (cell.size() > 1) {
                    any_candidate = true;
                } else if (cell.size() == 1) {
                    if (cell[0].first != link_idx) any_candidate = true;
                }
                cell.push_back(std::make_pair(link_idx, point_idx));
            }
        }
        if (!any_candidate) return SelfMap();
        std::map<size_t, double> link_masses;
        double previous_link_masses = 0.0;
        for (int64_t link_idx = (int64_t)geoms.size() - 1; link_idx >= 0; --link_idx) {
            const double link_mass = (double)geoms[(size_t)link_idx].second.points->size();
            link_masses[(size_t)link_idx] = link_mass + previous_link_masses;
            previous_link_masses += link_mass;
        }
        SelfMap self_collisions;
        size_t colliding_cells = 0;
        for (auto it = check_map.begin(); it != check_map.end(); ++it) {
            const std::map<std::pair<size_t, size_t>, V3> points = ExtractSelfCollidingPoints(
                previous_robot, current_robot, geoms, it->second, link_masses, time_interval, &colliding_cells, pc);
            for (auto s = points.begin(); s != points.end(); ++s) self_collisions[s->first] = s->second;
        }
        return self_collisions;
    }

    /* CheckCollision SPCS:1418-1436 */
    std::pair<bool, SelfMap> CheckCollision(const RobotPtr& robot, const Config& previous_config, const Config& current_config,
                                            const LinkGeometries& geoms, double time_interval, ParticleCounters& pc) const {
        RobotPtr current_robot(robot->Clone());
        RobotPtr previous_robot(robot->Clone());
        current_robot->SetPosition(current_config);
        previous_robot->SetPosition(previous_config);
        const bool env_collision = CheckEnvironmentCollision(current_robot, geoms, contact_distance_threshold_, pc);
        SelfMap self = CollectSelfCollisions(previous_robot, current_robot, geoms, time_interval, pc);
        const bool collided = env_collision || (self.size() > 0);
        if (self.size() > 0) pc.self_checks++;
        return std::make_pair(collided, self);
    }

    /* CheckPointsForSelfCollision SPCS:1277-1322: the points of one extended cell
     * (geometry index, point index) collide if two of their geometries may not touch */
    bool CheckPointsForSelfCollision(const RobotPtr& current_robot, const std::vector<std::pair<size_t, size_t>>& candidate_points) const {
        if (candidate_points.size() <= 1) return false;
        std::map<size_t, std::vector<size_t>> by_link;
        for (size_t idx = 0; idx < candidate_points.size(); ++idx)
            by_link[candidate_points[idx].first].push_back(candidate_points[idx].second);
        if (by_link.size() < 2) return false;
        for (auto f = by_link.begin(); f != by_link.end(); ++f)
            for (auto s = by_link.begin(); s != by_link.end(); ++s)
                if (f != s && !current_robot->CheckIfSelfCollisionAllowed(f->first, s->first)) return true;
        return false;
    }

    /* CheckSelfCollisions SPCS:1324-1396 (extended cells of size check_resolution) */
    bool CheckSelfCollisions(const RobotPtr& current_robot, const LinkGeometries& geoms, double check_resolution,
                             ParticleCounters& pc) const {
        if (geoms.size() == 1) return false;
        if (geoms.size() == 2 && current_robot->CheckIfSelfCollisionAllowed(0, 1)) return false;
        std::unordered_map<GridIndex, std::vector<std::pair<size_t, size_t>>, GridIndexHash> check_map;
        bool any_candidate = false;
        for (size_t link_idx = 0; link_idx < geoms.size(); ++link_idx) {
            const std::vector<V4>& link_points = *geoms[link_idx].second.points;
            const Iso T = current_robot->GetLinkTransform(geoms[link_idx].first);
            for (size_t point_idx = 0; point_idx < link_points.size(); ++point_idx) {
                const V4 p = xform4(T, link_points[point_idx]);
                const GridIndex key = LocationToExtendedGridIndex(p, check_resolution, pc);
                std::vector<std::pair<size_t, size_t>>& cell = check_map[key];
                if (cell.size() > 1) {
                    any_candidate = true;
                } else if (cell.size() == 1) {
                    if (cell[0].first != link_idx) any_candidate = true;
                }
                cell.push_back(std::make_pair(link_idx, point_idx));
            }
        }
        if (!any_candidate) return false;
        for (auto it = check_map.begin(); it != check_map.end(); ++it)
            if (CheckPointsForSelfCollision(current_robot, it->second)) return true;
        return false;
    }

    /* CheckConfigCollision SPCS:1398-1416 */
    bool CheckConfigCollision(const RobotPtr& immutable_robot, const Config& config, double inflation_ratio,
                              ParticleCounters& pc) const {
        RobotPtr current_robot(immutable_robot->Clone());
        current_robot->SetPosition(config);
        const LinkGeometries& geoms = current_robot->GetLinkGeometries();
        const double environment_collision_distance_threshold = inflation_ratio * env_geom_.res;
        const double self_collision_check_resolution = (inflation_ratio + 1.0) * env_geom_.res;
        const bool env_collision = CheckEnvironmentCollision(current_robot, geoms, environment_collision_distance_threshold, pc);
        const bool self_collision = CheckSelfCollisions(current_robot, geoms, self_collision_check_resolution, pc);
        return env_collision || self_collision;
    }

    /* EstimateMaxControlInputWorkspaceMotion SPCS:1492-1544 */
    double EstimateMaxControlInputWorkspaceMotion(const RobotPtr& start_robot, const RobotPtr& end_robot) const {
        const LinkGeometries& geoms = start_robot->GetLinkGeometries();
        double max_sq = 0.0;
        for (size_t link_idx = 0; link_idx < geoms.size(); ++link_idx) {
            const std::vector<V4>& pts = *geoms[link_idx].second.points;
            const Iso Ts = start_robot->GetLinkTransform(geoms[link_idx].first);
            const Iso Te = end_robot->GetLinkTransform(geoms[link_idx].first);
            for (size_t i = 0; i < pts.size(); ++i) {
                const V4 a = xform4(Ts, pts[i]), b = xform4(Te, pts[i]);
                const double sq = sqnorm4(V4{b.x - a.x, b.y - a.y, b.z - a.z, b.w - a.w});
                if (sq > max_sq) max_sq = sq;
            }
        }
        return fks_math::dsqrt(max_sq);
    }
    double EstimateMaxControlInputWorkspaceMotion(const RobotPtr& current_robot, const std::vector<double>& control_input) const {
        RobotPtr next_robot(current_robot->Clone());
        next_robot->ApplyControlInput(control_input);
        return EstimateMaxControlInputWorkspaceMotion(current_robot, next_robot);
    }

    /* CollectPointCorrectionsAndJacobians SPCS:1818-1939 */
    void CollectPointCorrectionsAndJacobians(const RobotPtr& robot, const Config& previous_config, const Config& current_config,
                                             const LinkGeometries& geoms, const SelfMap& self_map, std::vector<double>& J,
                                             std::vector<double>& b, size_t& rows, ParticleCounters& pc) const {
        RobotPtr current_robot(robot->Clone());
        RobotPtr previous_robot(robot->Clone());
        current_robot->SetPosition(current_config);
        previous_robot->SetPosition(previous_config);
        const size_t D = robot->NumDofs();
        J.clear();
        b.clear();
        rows = 0;
        for (size_t link_idx = 0; link_idx < geoms.size(); ++link_idx) {
            const std::string& link_name = geoms[link_idx].first;
            const std::vector<V4>& link_points = *geoms[link_idx].second.points;
            const Iso Tp = previous_robot->GetLinkTransform(link_name);
            const Iso Tc = current_robot->GetLinkTransform(link_name);
            for (size_t point_idx = 0; point_idx < link_points.size(); ++point_idx) {
                bool has_self = false;
                V3 self_corr{0.0, 0.0, 0.0};
                const auto found = self_map.find(std::make_pair(link_idx, point_idx));
                if (found != self_map.end()) {
                    has_self = true;
                    self_corr = found->second;
                }
                bool has_env = false;
                V3 env_corr{0.0, 0.0, 0.0};
                const V4& lp = link_points[point_idx];
                const std::vector<double> point_jacobian = current_robot->ComputeLinkPointTranslationJacobian(link_name, lp);
                const V4 prev_loc = xform4(Tp, lp);
                const V4 cur_loc = xform4(Tc, lp);
                const std::pair<double, bool> sdf_check = sdf_.EstimateDistance4d(cur_loc, &pc.sdf_bytes);
                if (sdf_check.first < resolution_distance_threshold_ && sdf_check.second) {
                    const V4 motion{cur_loc.x - prev_loc.x, cur_loc.y - prev_loc.y, cur_loc.z - prev_loc.z, cur_loc.w - prev_loc.w};
                    const V4 normed_motion = safe_normal4(motion);
                    V3 raw_gradient;
                    const bool in_bounds = normals_.Lookup(cur_loc, normed_motion, &raw_gradient, &pc.error_flags, &pc.sdf_bytes);
                    if (!in_bounds) pc.error_flags |= FKS_PARTICLE_ERR_NORMAL_OOB; /* assert SPCS:1882 */
                    const V3 g = safe_normal3(raw_gradient);
                    const double penetration = fks_math::dabs(resolution_distance_threshold_ - sdf_check.first);
                    env_corr = V3{g.x * penetration, g.y * penetration, g.z * penetration};
                    has_env = true;
                }
                if (has_self) pc.self_points++;
                if (has_self || has_env) {
                    /* grow the dynamic Jacobian by copy, as the reference does (SPCS:1896-1906) */
                    std::vector<double> extended(J.size() + 3 * D);
                    std::copy(J.begin(), J.end(), extended.begin());
                    std::copy(point_jacobian.begin(), point_jacobian.end(), extended.begin() + (long)J.size());
                    J.swap(extended);
                    V3 point_correction{0.0, 0.0, 0.0};
                    if (has_self)
                        point_correction = V3{point_correction.x + self_corr.x, point_correction.y + self_corr.y,
                                              point_correction.z + self_corr.z};
                    if (has_env)
                        point_correction = V3{point_correction.x + env_corr.x, point_correction.y + env_corr.y,
                                              point_correction.z + env_corr.z};
                    std::vector<double> extended_b(b.size() + 3);
                    std::copy(b.begin(), b.end(), extended_b.begin());
                    extended_b[b.size() + 0] = point_correction.x;
                    extended_b[b.size() + 1] = point_correction.y;
                    extended_b[b.size() + 2] = point_correction.z;
                    b.swap(extended_b);
                    rows += 3;
                }
            }
        }
    }

    /* ResolveForwardSimulation SPCS:1546-1816 (stacked Jacobian, FKS.cpp:22,45,68) */
    ResolveResult ResolveForwardSimulation(const RobotPtr& immutable_robot, const std::vector<double>& control_input,
                                           double controller_interval, NoiseContext& rng, bool allow_contacts,
                                           ParticleCounters& pc) const {
        RobotPtr robot(immutable_robot->Clone());
        const size_t D = robot->NumDofs();
        std::vector<double> real_control_input(D);
        for (size_t i = 0; i < D; ++i) real_control_input[i] = control_input[i] * controller_interval;
        const LinkGeometries& geoms = robot->GetLinkGeometries();
        const double computed_step_motion = EstimateMaxControlInputWorkspaceMotion(robot, real_control_input);
        const double target_microstep_distance = GetResolution() * 0.125;
        const double allowed_microstep_distance = GetResolution() * 1.0;
        const double raw_steps = std::ceil(computed_step_motion / target_microstep_distance);
        if (!(raw_steps <= 1048576.0)) {
            pc.error_flags |= FKS_PARTICLE_ERR_MICROSTEP_CAP;
            return ResolveResult{robot->GetPosition(), false, false, true};
        }
        const uint32_t number_microsteps = std::max(1u, (uint32_t)raw_steps);
        std::vector<double> control_input_step(D);
        for (size_t i = 0; i < D; ++i) control_input_step[i] = real_control_input[i] / (double)number_microsteps;
        const double computed_microstep_motion = EstimateMaxControlInputWorkspaceMotion(robot, control_input_step);
        if (computed_microstep_motion > allowed_microstep_distance) {
            pc.error_flags |= FKS_PARTICLE_ERR_MICROSTEP_MOTION; /* assert(false), SPCS:1570-1575 */
            return ResolveResult{robot->GetPosition(), false, false, true};
        }
        if (pc.trace) pc.trace->add_step(real_control_input, control_input_step, number_microsteps); /* SPCS:1583-1588 */
        bool collided = false;
        std::vector<double> J, b;
        for (uint32_t micro_step = 0; micro_step < number_microsteps; ++micro_step) {
            pc.microsteps++;
            const Config previous_configuration = robot->GetPosition();
            rng.micro = micro_step;
            robot->ApplyControlInput(control_input_step, rng);
            if (pc.error_flags) return ResolveResult{previous_configuration, collided, false, true};
            const Config post_action_configuration = robot->GetPosition();
            robot->SetPosition(post_action_configuration);
            std::pair<bool, SelfMap> collision_check =
                CheckCollision(robot, previous_configuration, post_action_configuration, geoms, controller_interval, pc);
            if (pc.error_flags) return ResolveResult{previous_configuration, collided, false, true};
            SelfMap& self_collision_map = collision_check.second;
            bool in_collision = collision_check.first;
            if (in_collision) collided = true;
            if (pc.trace) pc.trace->add_config(post_action_configuration, micro_step, FKS_TRACE_POST_ACTION); /* SPCS:1615-1618 */
            if (in_collision && allow_contacts) {
                Config active_configuration = post_action_configuration;
                uint32_t resolver_iterations = 0;
                double correction_step_scaling = solver_.resolve_correction_initial_step_size;
                while (in_collision) {
                    pc.resolver_iterations++;
                    size_t rows = 0;
                    CollectPointCorrectionsAndJacobians(robot, previous_configuration, active_configuration, geoms,
                                                        self_collision_map, J, b, rows, pc);
                    pc.lsq_rows += rows;
                    if (pc.error_flags) return ResolveResult{previous_configuration, collided, false, true};
                    if (!simulate_with_individual_jacobians_) capture_system(J, rows, D, b);
                    /* SPCS:1629: individual (SPCS:1966-1988) or stacked (SPCS:1990-1998) solve */
                    const std::vector<double> raw_correction_step = simulate_with_individual_jacobians_
                                                                        ? individual_jacobians_solve(J, rows, D, b)
                                                                        : colpiv_qr_solve(J, rows, D, b);
                    const double correction_step_motion_estimate = EstimateMaxControlInputWorkspaceMotion(robot, raw_correction_step);
                    const double allowed_resolve_distance = allowed_microstep_distance;
                    const double step_fraction = fks_math::dmax(correction_step_motion_estimate / allowed_resolve_distance, 1.0);
                    std::vector<double> real_correction_step(D);
                    for (size_t i = 0; i < D; ++i)
                        real_correction_step[i] = (raw_correction_step[i] / step_fraction) * fks_math::dabs(correction_step_scaling);
                    robot->ApplyControlInput(real_correction_step);
                    const Config post_resolve_configuration = robot->GetPosition();
                    active_configuration = post_resolve_configuration;
                    std::pair<bool, SelfMap> new_check =
                        CheckCollision(robot, previous_configuration, active_configuration, geoms, controller_interval, pc);
                    if (pc.error_flags) return ResolveResult{previous_configuration, collided, false, true};
                    self_collision_map = new_check.second;
                    in_collision = new_check.first;
                    resolver_iterations++;
                    if (pc.trace) pc.trace->add_config(active_configuration, micro_step, FKS_TRACE_RESOLVER_STEP); /* SPCS:1701-1704 */
                    if (resolver_iterations > solver_.max_resolver_iterations) {
                        if (pc.trace) pc.trace->add_config(previous_configuration, micro_step, FKS_TRACE_RESOLVE_FAILED); /* SPCS:1712-1715 */
                        pc.stats.unsuccessful_resolves++;
                        if (self_collision_map.size() > 0)
                            pc.stats.unsuccessful_self_collision_resolves++;
                        else
                            pc.stats.unsuccessful_env_collision_resolves++;
                        return ResolveResult{previous_configuration, true, true, false};
                    }
                    if ((resolver_iterations % solver_.resolve_correction_step_scaling_decay_iterations) == 0) {
                        if (correction_step_scaling >= 0.0) {
                            correction_step_scaling = correction_step_scaling * solver_.resolve_correction_step_scaling_decay_rate;
                            if (correction_step_scaling < solver_.resolve_correction_min_step_scaling)
                                correction_step_scaling = -solver_.resolve_correction_min_step_scaling;
                        } else {
                            correction_step_scaling = -solver_.resolve_correction_min_step_scaling;
                        }
                    }
                }
            } else if (in_collision && !allow_contacts) {
                if (pc.trace) pc.trace->add_config(previous_configuration, micro_step, FKS_TRACE_CONTACT_STOP); /* SPCS:1776-1779 */
                pc.stats.successful_resolves++;
                return ResolveResult{previous_configuration, true, false, false};
            }
        }
        pc.stats.successful_resolves++;
        if (collided)
            pc.stats.collision_resolves++;
        else
            pc.stats.free_resolves++;
        return ResolveResult{robot->GetPosition(), collided, false, false};
    }

    /* ForwardSimulateMutableRobot SPCS:843-919 */
    std::pair<Config, bool> ForwardSimulateMutableRobot(const RobotPtr& robot, const Config& target_position, bool allow_contacts,
                                                        NoiseContext& rng, ParticleCounters& pc) const {
        bool collided = false;
        const uint32_t forward_simulation_steps = forward_steps(solver_.forward_simulation_time, simulation_controller_frequency_);
        bool any_resolve_failed = false;
        for (uint32_t step = 0; step < forward_simulation_steps; ++step) {
            pc.controller_steps++;
            rng.step = step;
            if (pc.trace) pc.trace->step = step;
            const std::vector<double> control_action = robot->GenerateControlAction(target_position, simulation_controller_interval_);
            const ResolveResult result =
                ResolveForwardSimulation(robot, control_action, simulation_controller_interval_, rng, allow_contacts, pc);
            if (result.error) break; /* particle terminated (assert in the reference) */
            if (allow_contacts || !result.collided) {
                robot->SetPosition(result.config);
                if (result.collided) collided = true;
                if (result.failed) {
                    if (solver_.failed_resolves_end_motion) break;
                    any_resolve_failed = true;
                } else if (any_resolve_failed) {
                    pc.stats.recovered_unsuccessful_resolves++;
                }
                const double target_distance = robot->ComputeConfigurationDistanceTo(target_position);
                if (target_distance < solver_.simulation_shortcut_distance) break;
            } else {
                break;
            }
        }
        return std::make_pair(robot->GetPosition(), collided);
    }

    static uint32_t forward_steps(double time, double frequency) {
        const double raw = time * frequency;
        if (!(raw < 4294967295.0)) return 0xffffffffu;
        const uint32_t steps = (raw > 0.0) ? (uint32_t)raw : 0u;
        return std::max(steps, 1u);
    }

  private:
    GridGeom env_geom_;
    SDF sdf_;
    NormalGrid normals_;
    fks_solver_params solver_;
    int32_t debug_level_;
    bool simulate_with_individual_jacobians_; /* SPCS:384, 423, 1629 */
    double contact_distance_threshold_, resolution_distance_threshold_;
    double simulation_controller_frequency_, simulation_controller_interval_;
};

static RobotModel* make_robot(const fks_robot_desc& d) {
    switch (d.robot_type) {
        case FKS_ROBOT_LINKED: return new LinkedRobot(d);
        case FKS_ROBOT_SE2: return new SE2Robot(d);
        case FKS_ROBOT_SE3: return new SE3Robot(d);
        default: return nullptr;
    }
}

static size_t config_width(const fks_robot_desc& d) {
    if (d.robot_type == FKS_ROBOT_SE2) return 3;
    if (d.robot_type == FKS_ROBOT_SE3) return 12;
    return (size_t)d.num_dofs;
}

}  // namespace oracle

using namespace oracle;

extern "C" {

/* ForwardSimulateRobots (SPCS:788-804) on the CPU.  rng_mode 0 = counter
 * (Philox, parity with the HIP path), 1 = reference (per-OpenMP-thread
 * std::mt19937_64 seeded as SPCS:431-441).  num_threads <= 0: OpenMP default. */
static int forward_simulate_impl(const fks_environment* env, const fks_solver_params* params, double frequency, uint64_t seed,
                                 uint64_t call_index, const fks_robot_desc* robot_desc, const double* starts, uint64_t n,
                                 const double* targets, uint64_t num_targets, uint64_t first_particle_id, int32_t allow_contacts,
                                 int32_t rng_mode, int32_t num_threads, double* out_positions, uint8_t* out_collided,
                                 uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                                 fks_statistics* out_stats, fks_call_counters* out_counters, const fks_trace* trace,
                                 int32_t individual_jacobians, double* controller_state) {
    if (!env || !params || !robot_desc || (n > 0 && (!starts || !targets || !out_positions))) return 1;
    if (n > 0 && num_targets != 1 && num_targets != n) return 1;
    if (params->resolve_correction_step_scaling_decay_iterations == 0) return 1;
    const Simulator sim(*env, *params, frequency, 0, individual_jacobians != 0);
    std::shared_ptr<RobotModel> immutable_robot(make_robot(*robot_desc));
    if (!immutable_robot) return 1;
    const size_t W = config_width(*robot_desc);
    const uint64_t key = call_key(seed, call_index);
    int nthreads = (num_threads > 0) ? num_threads : omp_get_max_threads();
    /* reference-mode generators: one per thread, SPCS:431-441 */
    std::vector<std::mt19937_64> rngs;
    {
        std::mt19937_64 prng(seed);
        std::uniform_int_distribution<uint64_t> seed_dist(0, std::numeric_limits<uint64_t>::max());
        for (int t = 0; t < nthreads; ++t) rngs.push_back(std::mt19937_64(seed_dist(prng)));
    }
    std::vector<ParticleCounters> counters((size_t)n);
    std::vector<TraceSink> sinks(trace ? (size_t)n : 0);
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (int64_t idx = 0; idx < (int64_t)n; ++idx) {
        ParticleCounters& pc = counters[(size_t)idx];
        if (trace) pc.trace = &sinks[(size_t)idx];
        const Config start(starts + (size_t)idx * W, starts + (size_t)idx * W + W);
        const double* tp = (num_targets == n) ? targets + (size_t)idx * W : targets;
        const Config target(tp, tp + W);
        NoiseContext rng;
        rng.mode = rng_mode;
        rng.key0 = (uint32_t)key;
        rng.key1 = (uint32_t)(key >> 32);
        rng.particle = first_particle_id + (uint64_t)idx;
        rng.step = 0;
        rng.micro = 0;
        rng.mt = &rngs[(size_t)omp_get_thread_num()];
        rng.error_flags = &pc.error_flags;
        /* ForwardSimulateRobot SPCS:824-829 */
        RobotPtr robot(immutable_robot->Clone());
        robot->ResetPosition(start);
        /* ForwardSimulateMutableRobot on a robot that keeps its controllers (SPCS:843-919) */
        const size_t D = robot->NumDofs();
        if (controller_state) robot->SetControllerState(controller_state + (size_t)idx * 2 * D);
        const std::pair<Config, bool> result = sim.ForwardSimulateMutableRobot(robot, target, allow_contacts != 0, rng, pc);
        if (controller_state) robot->GetControllerState(controller_state + (size_t)idx * 2 * D);
        std::memcpy(out_positions + (size_t)idx * W, result.first.data(), W * sizeof(double));
        if (out_collided) out_collided[idx] = result.second ? 1 : 0;
        if (out_microsteps) out_microsteps[idx] = (uint32_t)pc.microsteps;
        if (out_resolver_iterations) out_resolver_iterations[idx] = (uint32_t)pc.resolver_iterations;
        if (out_error_flags) out_error_flags[idx] = pc.error_flags;
        if (trace) {
            const TraceSink& ts = *pc.trace;
            const size_t D = ts.step_microsteps.empty() ? 0 : ts.step_inputs.size() / (2 * ts.step_microsteps.size());
            const uint32_t ns = (uint32_t)ts.step_microsteps.size(), nc = (uint32_t)ts.config_tags.size() / 3;
            trace->num_steps[idx] = ns;
            trace->num_configs[idx] = nc;
            for (uint32_t k = 0; k < ns && k < trace->step_capacity; ++k) {
                const size_t rec = (size_t)idx * trace->step_capacity + k;
                std::memcpy(trace->step_inputs + rec * 2 * D, ts.step_inputs.data() + (size_t)k * 2 * D, 2 * D * sizeof(double));
                trace->step_microsteps[rec] = ts.step_microsteps[k];
            }
            for (uint32_t k = 0; k < nc && k < trace->config_capacity; ++k) {
                const size_t rec = (size_t)idx * trace->config_capacity + k;
                std::memcpy(trace->configs + rec * W, ts.configs.data() + (size_t)k * W, W * sizeof(double));
                std::memcpy(trace->config_tags + rec * 3, ts.config_tags.data() + (size_t)k * 3, 3 * sizeof(uint32_t));
            }
        }
    }
    fks_statistics stats;
    std::memset(&stats, 0, sizeof(stats));
    fks_call_counters cc;
    std::memset(&cc, 0, sizeof(cc));
    cc.particles = n;
    cc.calls = 1;
    for (size_t i = 0; i < (size_t)n; ++i) {
        const ParticleCounters& pc = counters[i];
        stats.successful_resolves += pc.stats.successful_resolves;
        stats.unsuccessful_resolves += pc.stats.unsuccessful_resolves;
        stats.free_resolves += pc.stats.free_resolves;
        stats.collision_resolves += pc.stats.collision_resolves;
        stats.fallback_resolves += pc.stats.fallback_resolves;
        stats.unsuccessful_env_collision_resolves += pc.stats.unsuccessful_env_collision_resolves;
        stats.unsuccessful_self_collision_resolves += pc.stats.unsuccessful_self_collision_resolves;
        stats.recovered_unsuccessful_resolves += pc.stats.recovered_unsuccessful_resolves;
        cc.controller_steps += pc.controller_steps;
        cc.microsteps += pc.microsteps;
        cc.resolver_iterations += pc.resolver_iterations;
        cc.sdf_bytes += pc.sdf_bytes;
        cc.least_squares_rows += pc.lsq_rows;
        cc.self_collision_checks += pc.self_checks;
        cc.self_corrected_points += pc.self_points;
        cc.error_particles += pc.error_flags ? 1 : 0;
    }
    if (out_stats) *out_stats = stats;
    if (out_counters) *out_counters = cc;
    return 0;
}

int oracle_forward_simulate(const fks_environment* env, const fks_solver_params* params, double frequency, uint64_t seed,
                            uint64_t call_index, const fks_robot_desc* robot_desc, const double* starts, uint64_t n,
                            const double* targets, uint64_t num_targets, uint64_t first_particle_id, int32_t allow_contacts,
                            int32_t rng_mode, int32_t num_threads, double* out_positions, uint8_t* out_collided,
                            uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags,
                            fks_statistics* out_stats, fks_call_counters* out_counters, int32_t individual_jacobians,
                            double* controller_state) {
    return forward_simulate_impl(env, params, frequency, seed, call_index, robot_desc, starts, n, targets, num_targets,
                                 first_particle_id, allow_contacts, rng_mode, num_threads, out_positions, out_collided,
                                 out_microsteps, out_resolver_iterations, out_error_flags, out_stats, out_counters, nullptr,
                                 individual_jacobians, controller_state);
}

/* ForwardSimulateRobot(..., trace, enable_tracing = true, ...) (SPCS:824-829)
 * for a batch, the trace flattened into the caller's fks_trace buffers */
int oracle_forward_simulate_traced(const fks_environment* env, const fks_solver_params* params, double frequency,
                                   uint64_t seed, uint64_t call_index, const fks_robot_desc* robot_desc, const double* starts,
                                   uint64_t n, const double* targets, uint64_t num_targets, int32_t allow_contacts,
                                   int32_t num_threads, double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps,
                                   uint32_t* out_resolver_iterations, uint32_t* out_error_flags, const fks_trace* trace,
                                   uint64_t first_particle_id) {
    if (!trace || !trace->num_steps || !trace->num_configs) return 1;
    return forward_simulate_impl(env, params, frequency, seed, call_index, robot_desc, starts, n, targets, num_targets, first_particle_id,
                                 allow_contacts, 0, num_threads, out_positions, out_collided, out_microsteps,
                                 out_resolver_iterations, out_error_flags, nullptr, nullptr, trace, 0, nullptr);
}

/* CheckConfigCollision (SPCS:1398-1416) over a batch of configurations; the
 * reference checks one configuration per call, the planner calls it per sample.
 * out_sdf_bytes (optional): algorithmic SDF bytes per configuration. */
int oracle_check_config_collision(const fks_environment* env, const fks_solver_params* params, const fks_robot_desc* robot_desc,
                                  const double* configs, uint64_t n, double inflation_ratio, int32_t num_threads,
                                  uint8_t* out_collided, uint32_t* out_error_flags, uint64_t* out_sdf_bytes) {
    if (!env || !params || !robot_desc || (n > 0 && (!configs || !out_collided))) return 1;
    const Simulator sim(*env, *params, 1.0, 0);
    std::shared_ptr<RobotModel> immutable_robot(make_robot(*robot_desc));
    if (!immutable_robot) return 1;
    const size_t W = config_width(*robot_desc);
    const int nthreads = (num_threads > 0) ? num_threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
    for (int64_t idx = 0; idx < (int64_t)n; ++idx) {
        ParticleCounters pc;
        const Config config(configs + (size_t)idx * W, configs + (size_t)idx * W + W);
        const bool collided = sim.CheckConfigCollision(immutable_robot, config, inflation_ratio, pc);
        out_collided[idx] = collided ? 1 : 0;
        if (out_error_flags) out_error_flags[idx] = pc.error_flags;
        if (out_sdf_bytes) out_sdf_bytes[idx] = pc.sdf_bytes;
    }
    return 0;
}

/* ---- primitive entry points for the known-answer tests ---- */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    Philox4 c;
    for (int i = 0; i < 4; ++i) c.v[i] = ctr[i];
    const Philox4 r = philox4x32_10(c, key[0], key[1]);
    for (int i = 0; i < 4; ++i) out[i] = r.v[i];
}

/* runs SimplePIDController::ComputeFeedbackTerm over a sequence (PID:122-135) */
void oracle_pid_sequence(double kp, double ki, double kd, double iclamp, const double* errors, const double* dts, int32_t n,
                         double* out) {
    SimplePIDController pid(kp, ki, kd, iclamp);
    for (int32_t i = 0; i < n; ++i) out[i] = pid.ComputeFeedbackTerm(errors[i], dts[i]);
}

double oracle_counter_truncated_normal(uint64_t seed, uint64_t call_index, uint64_t particle, uint32_t step, uint32_t micro,
                                       uint32_t dof, uint32_t* error_flags) {
    const uint64_t key = call_key(seed, call_index);
    NoiseContext ctx;
    ctx.mode = RNG_COUNTER;
    ctx.key0 = (uint32_t)key;
    ctx.key1 = (uint32_t)(key >> 32);
    ctx.particle = particle;
    ctx.step = step;
    ctx.micro = micro;
    ctx.mt = nullptr;
    ctx.error_flags = error_flags;
    return counter_truncated_normal(ctx, dof, 0.0, 0.5, -2.0, 2.0);
}

/* J row-major R x D */
/* the column permutation (perm[i] = original column of pivot i) and nonzero-pivot count
 * of the oracle's ColPivHouseholderQR, with its basic solution */
void oracle_qr_info(const double* J, uint64_t R, uint64_t D, const double* b, double* x, uint64_t* perm, uint64_t* nonzero) {
    const std::vector<double> Jv(J, J + R * D), bv(b, b + R);
    std::vector<size_t> p;
    size_t nz = 0;
    const std::vector<double> xv = colpiv_qr_solve(Jv, (size_t)R, (size_t)D, bv, &p, &nz);
    for (size_t i = 0; i < (size_t)D; ++i) {
        x[i] = xv[i];
        perm[i] = p[i];
    }
    *nonzero = nz;
}

void oracle_capture_systems(uint64_t max_systems, uint64_t stride, uint64_t max_rows) {
    std::lock_guard<std::mutex> lock(g_capture.mu);
    g_capture.max_systems = max_systems;
    g_capture.stride = stride ? stride : 1;
    g_capture.max_rows = max_rows;
    g_capture.seen = 0;
    g_capture.J.clear();
    g_capture.b.clear();
    g_capture.shape.clear();
}

uint64_t oracle_captured_systems(uint64_t* nvalues_J, uint64_t* nvalues_b) {
    std::lock_guard<std::mutex> lock(g_capture.mu);
    *nvalues_J = g_capture.J.size();
    *nvalues_b = g_capture.b.size();
    return g_capture.shape.size() / 2;
}

void oracle_copy_captured(double* J, double* b, uint64_t* shape) {
    std::lock_guard<std::mutex> lock(g_capture.mu);
    std::copy(g_capture.J.begin(), g_capture.J.end(), J);
    std::copy(g_capture.b.begin(), g_capture.b.end(), b);
    std::copy(g_capture.shape.begin(), g_capture.shape.end(), shape);
}

void oracle_qr_solve(const double* J, uint64_t R, uint64_t D, const double* b, double* x) {
    const std::vector<double> Jv(J, J + R * D), bv(b, b + R);
    const std::vector<double> xv = colpiv_qr_solve(Jv, (size_t)R, (size_t)D, bv);
    for (size_t i = 0; i < (size_t)D; ++i) x[i] = xv[i];
}

void oracle_estimate_distance(const fks_environment* env, const double* points, uint64_t n, double* out_distance,
                              uint8_t* out_in_bounds, float* out_nearest) {
    const SDF sdf(env->sdf, env->sdf_values, env->sdf_oob_value);
    for (size_t i = 0; i < (size_t)n; ++i) {
        const V4 p{points[4 * i], points[4 * i + 1], points[4 * i + 2], points[4 * i + 3]};
        uint64_t bytes = 0;
        const std::pair<double, bool> e = sdf.EstimateDistance4d(p, &bytes);
        out_distance[i] = e.first;
        out_in_bounds[i] = e.second ? 1 : 0;
        out_nearest[i] = sdf.GetImmutable4d(p, &bytes).first;
    }
}

/* forward kinematics: link transforms (3x4 row-major) of geometry links after SetPosition */
int oracle_link_transforms(const fks_robot_desc* robot_desc, const double* config, double* out) {
    std::unique_ptr<RobotModel> robot(make_robot(*robot_desc));
    if (!robot) return 1;
    const size_t W = config_width(*robot_desc);
    robot->SetPosition(Config(config, config + W));
    const LinkGeometries& geoms = robot->GetLinkGeometries();
    for (size_t g = 0; g < geoms.size(); ++g) iso_to12(robot->GetLinkTransform(geoms[g].first), out + 12 * g);
    return 0;
}

/* SetPosition(config) then the clean ApplyControlInput(input) (TNUVA:538-566, SE2
 * 152-177, SE3 348-382): the configuration MakeControlInputDisplayRep draws to */
int oracle_apply_control_input(const fks_robot_desc* robot_desc, const double* config, const double* input, double* out) {
    std::unique_ptr<RobotModel> robot(make_robot(*robot_desc));
    if (!robot) return 1;
    const size_t W = config_width(*robot_desc);
    robot->SetPosition(Config(config, config + W));
    robot->ApplyControlInput(std::vector<double>(input, input + robot->NumDofs()));
    const Config& q = robot->GetPosition();
    std::memcpy(out, q.data(), W * sizeof(double));
    return 0;
}

/* One robot stepped by hand (the TnuvaRobot interface, TNUVA:15-23): ResetPosition(start),
 * then per step u = GenerateControlAction(target, controller_interval) and ApplyControlInput(u)
 * (clean) or, on the steps whose bit is set in noisy_mask, ApplyControlInput(u, rng) with one
 * std::mt19937_64(seed) as the generator (reference mode: each actuator's own
 * std::normal_distribution).  out_controls: steps x D, out_configs: steps x W, out_pid: 2D. */
int oracle_robot_steps(const fks_robot_desc* robot_desc, const double* start, const double* target, double controller_interval,
                       uint32_t steps, uint64_t seed, uint64_t noisy_mask, double* out_controls, double* out_configs,
                       double* out_pid) {
    std::unique_ptr<RobotModel> robot(make_robot(*robot_desc));
    if (!robot) return 1;
    const size_t W = config_width(*robot_desc), D = robot->NumDofs();
    robot->ResetPosition(Config(start, start + W));
    const Config tgt(target, target + W);
    std::mt19937_64 mt(seed);
    uint32_t err = 0;
    NoiseContext ctx{RNG_REFERENCE, 0, 0, 0, 0, 0, &mt, &err};
    for (uint32_t k = 0; k < steps; ++k) {
        const std::vector<double> u = robot->GenerateControlAction(tgt, controller_interval);
        for (size_t d = 0; d < D; ++d) out_controls[k * D + d] = u[d];
        if (k < 64 && ((noisy_mask >> k) & 1ull))
            robot->ApplyControlInput(u, ctx);
        else
            robot->ApplyControlInput(u);
        const Config& q = robot->GetPosition();
        std::memcpy(out_configs + k * W, q.data(), W * sizeof(double));
    }
    robot->GetControllerState(out_pid);
    return err ? 2 : 0;
}

/* point Jacobian (3 x D row-major) of point p (4 doubles) on geometry g */
int oracle_point_jacobian(const fks_robot_desc* robot_desc, const double* config, int32_t geometry, const double* p, double* out) {
    std::unique_ptr<RobotModel> robot(make_robot(*robot_desc));
    if (!robot) return 1;
    const size_t W = config_width(*robot_desc);
    robot->SetPosition(Config(config, config + W));
    const std::vector<double> J =
        robot->ComputeLinkPointTranslationJacobian(robot->GetLinkGeometries()[(size_t)geometry].first, V4{p[0], p[1], p[2], p[3]});
    for (size_t i = 0; i < J.size(); ++i) out[i] = J[i];
    return 0;
}

/* SE(3) helpers for tests */
void oracle_se3_exp(const double twist[6], double out[12]) { iso_to12(exp_twist(twist), out); }
void oracle_se3_log(const double pose[12], double twist[6]) { log_twist(iso_from12(pose), twist); }

int oracle_max_threads(void) { return omp_get_max_threads(); }

}  // extern "C"

extern "C" {
/* evaluate the shared portable libm (include/fks_portable_math.h) for tests:
 * fn 0 sin, 1 cos, 2 log, 3 atan, 4 atan2(x, y), 5 wrap, 6 fmod_two_pi and 7 wrap_revolute
 * (the kernel's libm-free wrap, checked against 5 and glibc) */
void oracle_portable_math(int32_t fn, const double* x, const double* y, uint64_t n, double* out) {
    for (uint64_t i = 0; i < n; ++i) {
        switch (fn) {
            case 0: out[i] = fks_math::sin(x[i]); break;
            case 1: out[i] = fks_math::cos(x[i]); break;
            case 2: out[i] = fks_math::log(x[i]); break;
            case 3: out[i] = fks_math::atan(x[i]); break;
            case 4: out[i] = fks_math::atan2(x[i], y[i]); break;
            case 6: out[i] = fks_math::fmod_two_pi(x[i]); break;
            case 7: out[i] = fks_math::wrap_revolute(x[i]); break;
            default: out[i] = fks_math::enforce_continuous_revolute_bounds(x[i]); break;
        }
    }
}
}
