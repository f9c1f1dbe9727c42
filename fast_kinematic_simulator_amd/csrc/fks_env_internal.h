/*
 * Shared pieces of the two environment builders (fks_env_builder.cpp on the host,
 * fks_env_gpu.hip on the device): the fks_env_handle layout, the grid indexing of
 * SEB.cpp / sdf_tools (truncating world -> cell index through the inverse origin)
 * and the obstacle sample lattice of DiscretizeObstacle (SEB.cpp:21-46).  Both
 * builders evaluate these with the same operation order (compiled with
 * -ffp-contract=off), so their outputs are bit-identical.
 */
#ifndef FKS_ENV_INTERNAL_H
#define FKS_ENV_INTERNAL_H

#include <stdint.h>

#include <vector>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#endif

#include "fks_capi.h"
#include "fks_portable_math.h"

struct fks_env_handle {
    fks_grid_geometry geometry;
    std::vector<float> sdf;
    std::vector<uint32_t> offsets;
    std::vector<double> entries;
    std::vector<uint8_t> occupancy;
    std::vector<fks_obstacle> obstacles; /* what fks_env_build was given (fks_env_cell_objects) */
};

/* an environment built on the GPU and kept there (fks_env_build_device) */
struct fks_device_env {
    int32_t device;
    fks_grid_geometry geometry;
    uint64_t cells;
    uint64_t num_entries;
    uint8_t* occupancy; /* device arrays */
    float* sdf;
    uint32_t* offsets;
    double* entries;
};

namespace fks_env {

/* the SDF analysis behind the kernels' skip proofs (fks_capi.cpp analyze_sdf) on a
 * device-resident SDF; false when a value is not finite or the analysis failed */
bool analyze_sdf_device(const float* d_sdf, int64_t nx, int64_t ny, int64_t nz, double res, double* lplus, double* cmax);

#if defined(__HIPCC__)
/* the simulation kernels' HBM layout (fks_device.h brick_cell): the VoxelGrid-order SDF
 * `lin` (n cells per axis) copied into 4x4x4-cell bricks (nb bricks per axis), and the
 * CSR offsets `off` (cells + 1) turned into a bricked [begin, end) range per cell; the
 * outputs are new device allocations the caller frees */
hipError_t brick_sdf_device(const float* lin, const int64_t n[3], const uint32_t nb[3], float** out);
hipError_t brick_normal_ranges_device(const uint32_t* off, const int64_t n[3], const uint32_t nb[3], uint2** out);
#endif

FKS_HD inline double dot3(double a0, double a1, double a2, double b0, double b1, double b2) {
    return (a0 * b0 + a1 * b1) + a2 * b2;
}

/* Isometry3d * Vector3d */
FKS_HD inline void xform3(const double* T, const double p[3], double out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = dot3(T[4 * i + 0], T[4 * i + 1], T[4 * i + 2], p[0], p[1], p[2]) + T[4 * i + 3];
}
FKS_HD inline void rotate3(const double* T, const double v[3], double out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = dot3(T[4 * i + 0], T[4 * i + 1], T[4 * i + 2], v[0], v[1], v[2]);
}
FKS_HD inline void inverse34(const double* T, double* I) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) I[4 * i + j] = T[4 * j + i];
    for (int i = 0; i < 3; ++i) I[4 * i + 3] = -dot3(I[4 * i + 0], I[4 * i + 1], I[4 * i + 2], T[3], T[7], T[11]);
}

struct Grid {
    double origin[12], inv_origin[12];
    double res, inv_res;
    int64_t n[3];
    /* VoxelGrid::LocationToGridIndex3d: truncation toward zero, bounds-checked */
    FKS_HD bool index(const double p[3], int64_t idx[3]) const {
        double g[3];
        xform3(inv_origin, p, g);
        for (int a = 0; a < 3; ++a) {
            const double q = g[a] * inv_res;
            if (!(q > -9.0e18 && q < 9.0e18)) return false;
            idx[a] = (int64_t)q;
            if (idx[a] < 0 || idx[a] >= n[a]) return false;
        }
        return true;
    }
    FKS_HD uint64_t linear(int64_t i, int64_t j, int64_t k) const {
        return ((uint64_t)i * (uint64_t)n[1] + (uint64_t)j) * (uint64_t)n[2] + (uint64_t)k;
    }
    FKS_HD uint64_t cells() const { return (uint64_t)n[0] * (uint64_t)n[1] * (uint64_t)n[2]; }
};

/* DiscretizeObstacle (SEB.cpp:21-46): samples per axis at half resolution */
FKS_HD inline void obstacle_samples(const fks_obstacle& ob, double resolution, int32_t nc[3]) {
    const double effective_resolution = resolution * 0.5;
    for (int a = 0; a < 3; ++a) nc[a] = (int32_t)(ob.extents[a] * 2.0 * (1.0 / effective_resolution));
}
/* world position of sample (xi, yi, zi); `inset` = resolution * 0.5 for the occupancy
 * lattice (SEB.cpp:33-35), effective_resolution for the surface lattice (SEB.cpp:295-297) */
FKS_HD inline void obstacle_sample_local(const fks_obstacle& ob, double resolution, double inset, int32_t xi, int32_t yi,
                                         int32_t zi, double local[3]) {
    const double effective_resolution = resolution * 0.5;
    local[0] = -(ob.extents[0] - inset) + (effective_resolution * xi);
    local[1] = -(ob.extents[1] - inset) + (effective_resolution * yi);
    local[2] = -(ob.extents[2] - inset) + (effective_resolution * zi);
}
FKS_HD inline void obstacle_sample_world(const fks_obstacle& ob, double resolution, double inset, int32_t xi, int32_t yi,
                                         int32_t zi, double w[3]) {
    double local[3];
    obstacle_sample_local(ob, resolution, inset, xi, yi, zi, local);
    xform3(ob.pose, local, w); /* obstacle.pose * relative_location (SEB.cpp:84-85) */
}

/* StoredSurfaceNormal entry of a boundary sample along axis a (SEB.cpp:300-460):
 * SafeNormal((entry, 0)) then SafeNormal(normal), rotated into the world.  The
 * Vector4d norm is Eigen's two-lane packet reduction (x^2 + z^2) + (y^2 + w^2)
 * (DESIGN.md §2.3); the Vector3d norm is sequential. */
FKS_HD inline void face_entry(const double* pose, int a, bool low_face, double E[6]) {
    double normal[3] = {0, 0, 0}, entry[3] = {0, 0, 0};
    normal[a] = low_face ? -1.0 : 1.0;
    entry[a] = low_face ? 1.0 : -1.0;
    double rn[3], re[3];
    rotate3(pose, normal, rn);
    rotate3(pose, entry, re);
    const double en = fks_math::dsqrt((re[0] * re[0] + re[2] * re[2]) + (re[1] * re[1] + 0.0 * 0.0));
    for (int b = 0; b < 3; ++b) E[b] = (en > 2.220446049250313e-16) ? re[b] / en : re[b];
    const double nn = fks_math::dsqrt((rn[0] * rn[0] + rn[1] * rn[1]) + rn[2] * rn[2]);
    for (int b = 0; b < 3; ++b) E[3 + b] = (nn > 2.220446049250313e-16) ? rn[b] / nn : rn[b];
}

/* surface-normal entry of an interior (d < 0) cell without a boundary sample:
 * normalised central-difference SDF gradient, one-sided at the grid edges
 * (SEB.cpp:263-277, GetGradient with edge gradients enabled) */
template <typename SdfAt>
FKS_HD inline void gradient_entry(const Grid& grid, int64_t i, int64_t j, int64_t k, const SdfAt& sdf_at, double E[6]) {
    const int64_t id3[3] = {i, j, k};
    double g[3];
    for (int a = 0; a < 3; ++a) {
        int64_t lo[3] = {i, j, k}, hi[3] = {i, j, k};
        lo[a] = (id3[a] - 1 > 0) ? id3[a] - 1 : 0;
        hi[a] = (id3[a] + 1 < grid.n[a] - 1) ? id3[a] + 1 : grid.n[a] - 1;
        const double inv = 1.0 / (grid.res * (double)(hi[a] - lo[a]));
        const float diff = sdf_at(hi[0], hi[1], hi[2]) - sdf_at(lo[0], lo[1], lo[2]);
        g[a] = (double)diff * inv;
    }
    const double gn = fks_math::dsqrt((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]);
    for (int b = 0; b < 3; ++b) E[b] = 0.0;
    for (int b = 0; b < 3; ++b) E[3 + b] = (gn > 2.220446049250313e-16) ? g[b] / gn : g[b];
}

/* SEB.cpp:128-149: grid sized to the samples' bounds, minimum keyed half a cell
 * out, plus a 3-cell border; (0, 10) when there is nothing to bound */
inline void auto_bounds(bool any, double mn[3], double mx[3], double resolution, Grid& grid) {
    if (!any) {
        for (int a = 0; a < 3; ++a) {
            mn[a] = 0.0;
            mx[a] = 10.0;
        }
    } else {
        for (int a = 0; a < 3; ++a) {
            mn[a] -= resolution * 0.5;
            mn[a] -= resolution * 3.0;
            mx[a] += resolution * 3.0;
        }
    }
    const double I[12] = {1, 0, 0, mn[0], 0, 1, 0, mn[1], 0, 0, 1, mn[2]};
    for (int t = 0; t < 12; ++t) grid.origin[t] = I[t];
    for (int a = 0; a < 3; ++a) grid.n[a] = (int64_t)__builtin_ceil((mx[a] - mn[a]) / resolution);
}

}  // namespace fks_env

#endif
