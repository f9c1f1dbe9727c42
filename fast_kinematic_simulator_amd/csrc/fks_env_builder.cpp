/*
 * Environment preprocessing on the host: obstacles -> collision grid -> signed
 * distance field -> surface-normal grid.  Restates
 * src/fast_kinematic_simulator/simulator_environment_builder.cpp (SEB.cpp):
 *   DiscretizeObstacle        SEB.cpp:21-46   (half-resolution sample lattice)
 *   BuildEnvironment          SEB.cpp:49-160  (auto bounds + 3-cell border, or a fixed box)
 *   ExtractSignedDistanceField SEB.cpp:473    (sdf_tools, absent: restated as an exact
 *                                             Euclidean distance transform, Felzenszwalb &
 *                                             Huttenlocher 2012, distance to the nearest
 *                                             opposite cell centre; +inf out of bounds)
 *   BuildSurfaceNormalsGrid   SEB.cpp:258-468 (SDF-gradient pass for d<0 cells, then the exact
 *                                             cuboid face/edge/corner normals, last write wins)
 * This is the input side of the hot path ("next" row f2 in SURVEY.md §8f);
 * fks_env_gpu.hip builds the same bytes on the GPU (fks_env_build_gpu).  Output
 * layout is the fks_environment CSR.
 */
#include <stdint.h>

#include <cmath>
#include <cstring>
#include <limits>
#include <new>
#include <unordered_map>
#include <vector>

#include "fks_capi.h"
#include "fks_env_internal.h"
#include "fks_portable_math.h"

namespace {

using fks_env::Grid;
using fks_env::inverse34;
using fks_env::rotate3;
using fks_env::xform3;

/* 1-D squared distance transform (lower envelope of parabolas rooted at the
 * finite samples), exact on integer grids */
void edt_1d(const double* f, double* d, int64_t n, int64_t* v, double* z) {
    const double INF = std::numeric_limits<double>::infinity();
    int64_t k = -1;
    for (int64_t q = 0; q < n; ++q) {
        if (!(f[q] < INF)) continue;
        if (k < 0) {
            k = 0;
            v[0] = q;
            z[0] = -INF;
            z[1] = INF;
            continue;
        }
        double s = ((f[q] + (double)(q * q)) - (f[v[k]] + (double)(v[k] * v[k]))) / (2.0 * (double)(q - v[k]));
        while (s <= z[k]) {
            k--;
            s = ((f[q] + (double)(q * q)) - (f[v[k]] + (double)(v[k] * v[k]))) / (2.0 * (double)(q - v[k]));
        }
        k++;
        v[k] = q;
        z[k] = s;
        z[k + 1] = INF;
    }
    if (k < 0) {
        for (int64_t q = 0; q < n; ++q) d[q] = INF;
        return;
    }
    k = 0;
    for (int64_t q = 0; q < n; ++q) {
        while (z[k + 1] < (double)q) k++;
        const double dq = (double)(q - v[k]);
        d[q] = dq * dq + f[v[k]];
    }
}

/* squared distance (in cells) from every cell to the nearest cell with seed[c] != 0 */
std::vector<double> edt_3d(const std::vector<uint8_t>& seed, const int64_t n[3]) {
    const double INF = std::numeric_limits<double>::infinity();
    const size_t total = (size_t)n[0] * (size_t)n[1] * (size_t)n[2];
    std::vector<double> D(total);
    for (size_t c = 0; c < total; ++c) D[c] = seed[c] ? 0.0 : INF;
    const int64_t maxn = std::max(n[0], std::max(n[1], n[2]));
    std::vector<double> f((size_t)maxn), d((size_t)maxn), z((size_t)maxn + 1);
    std::vector<int64_t> v((size_t)maxn);
    const int64_t sx = n[1] * n[2], sy = n[2];
    /* z */
    for (int64_t i = 0; i < n[0]; ++i)
        for (int64_t j = 0; j < n[1]; ++j) {
            const size_t base = (size_t)(i * sx + j * sy);
            for (int64_t k = 0; k < n[2]; ++k) f[(size_t)k] = D[base + (size_t)k];
            edt_1d(f.data(), d.data(), n[2], v.data(), z.data());
            for (int64_t k = 0; k < n[2]; ++k) D[base + (size_t)k] = d[(size_t)k];
        }
    /* y */
    for (int64_t i = 0; i < n[0]; ++i)
        for (int64_t k = 0; k < n[2]; ++k) {
            const size_t base = (size_t)(i * sx + k);
            for (int64_t j = 0; j < n[1]; ++j) f[(size_t)j] = D[base + (size_t)(j * sy)];
            edt_1d(f.data(), d.data(), n[1], v.data(), z.data());
            for (int64_t j = 0; j < n[1]; ++j) D[base + (size_t)(j * sy)] = d[(size_t)j];
        }
    /* x */
    for (int64_t j = 0; j < n[1]; ++j)
        for (int64_t k = 0; k < n[2]; ++k) {
            const size_t base = (size_t)(j * sy + k);
            for (int64_t i = 0; i < n[0]; ++i) f[(size_t)i] = D[base + (size_t)(i * sx)];
            edt_1d(f.data(), d.data(), n[0], v.data(), z.data());
            for (int64_t i = 0; i < n[0]; ++i) D[base + (size_t)(i * sx)] = d[(size_t)i];
        }
    return D;
}

struct Entry {
    double e[6];
};

/* BuildSurfaceNormalsGrid (SEB.cpp:258-468) on `sdf` (VoxelGrid order over `grid`): the
 * obstacles' boundary samples get their exact face / edge / corner entries (last write wins),
 * every other cell with a negative distance its SDF-gradient entry (pass 1) */
void build_normals(const fks_obstacle* obstacles, int32_t num_obstacles, const Grid& grid, const float* sdf,
                   std::vector<uint32_t>* offsets_out, std::vector<double>* entries_out) {
    const double resolution = grid.res;
    const double effective_resolution = resolution * 0.5;
    const size_t total = grid.cells();
    auto sdf_at = [&](int64_t i, int64_t j, int64_t k) { return sdf[grid.linear(i, j, k)]; };
    /* pass 2 first into a map (last write wins); pass 1 fills the rest */
    std::unordered_map<size_t, std::vector<Entry>> surface;
    for (int32_t o = 0; o < num_obstacles; ++o) {
        const fks_obstacle& ob = obstacles[o];
        int32_t nc[3];
        for (int a = 0; a < 3; ++a) nc[a] = (int32_t)(ob.extents[a] * 2.0 * (1.0 / effective_resolution));
        for (int32_t xi = 0; xi < nc[0]; ++xi)
            for (int32_t yi = 0; yi < nc[1]; ++yi)
                for (int32_t zi = 0; zi < nc[2]; ++zi) {
                    const int32_t id3[3] = {xi, yi, zi};
                    bool boundary = false;
                    for (int a = 0; a < 3; ++a) boundary = boundary || id3[a] == 0 || id3[a] == nc[a] - 1;
                    if (!boundary) continue;
                    const double local[3] = {-(ob.extents[0] - effective_resolution) + (effective_resolution * xi),
                                             -(ob.extents[1] - effective_resolution) + (effective_resolution * yi),
                                             -(ob.extents[2] - effective_resolution) + (effective_resolution * zi)};
                    double w[3];
                    xform3(ob.pose, local, w);
                    int64_t idx[3];
                    /* UpdateSurfaceNormalGridCell SEB.cpp:162-187 */
                    if (!grid.index(w, idx)) continue; /* GetImmutable3d OOB = +inf, then insert fails */
                    const float distance = sdf_at(idx[0], idx[1], idx[2]);
                    if (!((double)distance > -(resolution * 1.5))) continue;
                    std::vector<Entry> list;
                    for (int a = 0; a < 3; ++a) {
                        if (id3[a] != 0 && id3[a] != nc[a] - 1) continue;
                        /* StoredSurfaceNormal: SafeNormal(normal), SafeNormal((entry, 0)) */
                        Entry E;
                        fks_env::face_entry(ob.pose, a, id3[a] == 0, E.e);
                        list.push_back(E);
                    }
                    surface[grid.linear(idx[0], idx[1], idx[2])] = list;
                }
    }
    offsets_out->assign(total + 1, 0);
    uint64_t count = 0;
    for (int64_t i = 0; i < grid.n[0]; ++i)
        for (int64_t j = 0; j < grid.n[1]; ++j)
            for (int64_t k = 0; k < grid.n[2]; ++k) {
                const size_t c = grid.linear(i, j, k);
                (*offsets_out)[c] = (uint32_t)count;
                const auto it = surface.find(c);
                if (it != surface.end()) {
                    for (const Entry& E : it->second) entries_out->insert(entries_out->end(), E.e, E.e + 6);
                    count += it->second.size();
                } else if (sdf[c] < 0.0f) {
                    /* pass 1 (SEB.cpp:263-277): SDF gradient (edge gradients enabled), entry 0 */
                    Entry E;
                    fks_env::gradient_entry(grid, i, j, k, sdf_at, E.e);
                    entries_out->insert(entries_out->end(), E.e, E.e + 6);
                    count += 1;
                }
                if (count > 0xffffffffull) throw std::bad_alloc();
            }
    (*offsets_out)[total] = (uint32_t)count;
}

}  // namespace

extern "C" fks_status fks_env_build(const fks_obstacle* obstacles, int32_t num_obstacles, double resolution,
                                    const double* grid_origin, const int64_t* num_cells, fks_env_handle** out) {
    if (!out || !(resolution > 0.0) || num_obstacles < 0 || (num_obstacles > 0 && !obstacles)) return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    const double effective_resolution = resolution * 0.5;
    /* DiscretizeObstacle + world placement (SEB.cpp:21-46, 78-127) */
    std::vector<double> cells;  // xyz triples
    std::vector<uint32_t> cell_ids;
    double mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    bool init = false;
    for (int32_t o = 0; o < num_obstacles; ++o) {
        const fks_obstacle& ob = obstacles[o];
        int32_t nc[3];
        for (int a = 0; a < 3; ++a) nc[a] = (int32_t)(ob.extents[a] * 2.0 * (1.0 / effective_resolution));
        for (int32_t xi = 0; xi < nc[0]; ++xi)
            for (int32_t yi = 0; yi < nc[1]; ++yi)
                for (int32_t zi = 0; zi < nc[2]; ++zi) {
                    const double local[3] = {-(ob.extents[0] - (resolution * 0.5)) + (effective_resolution * xi),
                                             -(ob.extents[1] - (resolution * 0.5)) + (effective_resolution * yi),
                                             -(ob.extents[2] - (resolution * 0.5)) + (effective_resolution * zi)};
                    double w[3];
                    xform3(ob.pose, local, w);
                    cells.insert(cells.end(), w, w + 3);
                    cell_ids.push_back(ob.object_id);
                    if (!init) {
                        for (int a = 0; a < 3; ++a) mn[a] = mx[a] = w[a];
                        init = true;
                    } else {
                        for (int a = 0; a < 3; ++a) {
                            if (w[a] < mn[a]) mn[a] = w[a];
                            else if (w[a] > mx[a]) mx[a] = w[a];
                        }
                    }
                }
    }
    Grid grid;
    grid.res = resolution;
    grid.inv_res = 1.0 / resolution;
    if (grid_origin && num_cells) {
        std::memcpy(grid.origin, grid_origin, sizeof(grid.origin));
        for (int a = 0; a < 3; ++a) grid.n[a] = num_cells[a];
    } else {
        fks_env::auto_bounds(init, mn, mx, resolution, grid);
    }
    for (int a = 0; a < 3; ++a)
        if (grid.n[a] < 2 || grid.n[a] > 4096) return FKS_ERR_INVALID_ARGUMENT;
    inverse34(grid.origin, grid.inv_origin);

    fks_env_handle* env = new (std::nothrow) fks_env_handle();
    if (!env) return FKS_ERR_OUT_OF_MEMORY;
    try {
        const size_t total = grid.cells();
        env->occupancy.assign(total, 0);
        for (size_t c = 0; c < cell_ids.size(); ++c) {
            int64_t idx[3];
            if (grid.index(&cells[3 * c], idx)) env->occupancy[grid.linear(idx[0], idx[1], idx[2])] = 1;
        }
        /* signed distance field: + distance to the nearest filled cell for free cells,
         * - distance to the nearest free cell for filled cells (sdf_tools convention) */
        std::vector<uint8_t> free_seed(total);
        for (size_t c = 0; c < total; ++c) free_seed[c] = env->occupancy[c] ? 0 : 1;
        const std::vector<double> to_filled = edt_3d(env->occupancy, grid.n);
        const std::vector<double> to_free = edt_3d(free_seed, grid.n);
        env->sdf.resize(total);
        for (size_t c = 0; c < total; ++c) {
            const double filled_distance = fks_math::dsqrt(to_filled[c]) * resolution;
            const double free_distance = fks_math::dsqrt(to_free[c]) * resolution;
            env->sdf[c] = (float)(filled_distance - free_distance);
        }
        build_normals(obstacles, num_obstacles, grid, env->sdf.data(), &env->offsets, &env->entries);
        env->obstacles.assign(obstacles, obstacles + num_obstacles);
    } catch (const std::bad_alloc&) {
        delete env;
        return FKS_ERR_OUT_OF_MEMORY;
    }
    std::memcpy(env->geometry.origin, grid.origin, sizeof(grid.origin));
    env->geometry.resolution = resolution;
    for (int a = 0; a < 3; ++a) env->geometry.num_cells[a] = grid.n[a];
    *out = env;
    return FKS_OK;
}

extern "C" fks_status fks_env_view(const fks_env_handle* env, fks_environment* out) {
    if (!env || !out) return FKS_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    out->collision_map = env->geometry;
    out->sdf = env->geometry;
    out->normals = env->geometry;
    out->sdf_values = env->sdf.data();
    out->sdf_oob_value = std::numeric_limits<float>::infinity();
    out->normal_offsets = env->offsets.data();
    out->normal_entries = env->entries.data();
    return FKS_OK;
}

extern "C" fks_status fks_env_occupancy(const fks_env_handle* env, uint8_t* out, uint64_t num_cells) {
    if (!env || (num_cells > 0 && !out) || num_cells != (uint64_t)env->occupancy.size()) return FKS_ERR_INVALID_ARGUMENT;
    if (num_cells) std::memcpy(out, env->occupancy.data(), (size_t)num_cells);
    return FKS_OK;
}

extern "C" void fks_env_free(fks_env_handle* env) { delete env; }

/* DiscretizeObstacle (SEB.cpp:21-46): the positions, relative to the obstacle, of its half-resolution
 * sample lattice, x then y then z (the order BuildEnvironment's SetValue calls take) */
extern "C" fks_status fks_env_discretize_obstacle(const fks_obstacle* obstacle, double resolution, double* out_xyz,
                                                  uint64_t capacity, uint64_t* count) {
    if (!obstacle || !count || !(resolution > 0.0)) return FKS_ERR_INVALID_ARGUMENT;
    int32_t nc[3];
    fks_env::obstacle_samples(*obstacle, resolution, nc);
    const uint64_t n = (nc[0] > 0 && nc[1] > 0 && nc[2] > 0) ? (uint64_t)nc[0] * (uint64_t)nc[1] * (uint64_t)nc[2] : 0;
    *count = n;
    if (!out_xyz) return FKS_OK;
    if (capacity < n) return FKS_ERR_INVALID_ARGUMENT;
    uint64_t k = 0;
    for (int32_t xi = 0; xi < nc[0]; ++xi)
        for (int32_t yi = 0; yi < nc[1]; ++yi)
            for (int32_t zi = 0; zi < nc[2]; ++zi, ++k)
                fks_env::obstacle_sample_local(*obstacle, resolution, resolution * 0.5, xi, yi, zi, out_xyz + 3 * k);
    return FKS_OK;
}

/* BuildSurfaceNormalsGrid (SEB.cpp:258-468) on a caller's SDF (any SignedDistanceField, e.g.
 * the planner's own sdf_tools ExtractSignedDistanceField result, SEB.cpp:473-475): a handle
 * holding only the normal CSR over the SDF's geometry (fks_env_view: sdf_values NULL) */
extern "C" fks_status fks_env_build_normals(const fks_obstacle* obstacles, int32_t num_obstacles,
                                            const fks_grid_geometry* sdf_geometry, const float* sdf_values,
                                            fks_env_handle** out) {
    if (!out || !sdf_geometry || !sdf_values || num_obstacles < 0 || (num_obstacles > 0 && !obstacles) ||
        !(sdf_geometry->resolution > 0.0))
        return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Grid grid;
    grid.res = sdf_geometry->resolution;
    grid.inv_res = 1.0 / grid.res;
    std::memcpy(grid.origin, sdf_geometry->origin, sizeof(grid.origin));
    for (int a = 0; a < 3; ++a) {
        grid.n[a] = sdf_geometry->num_cells[a];
        if (grid.n[a] < 1 || grid.n[a] > 4096) return FKS_ERR_INVALID_ARGUMENT;
    }
    inverse34(grid.origin, grid.inv_origin);
    fks_env_handle* env = new (std::nothrow) fks_env_handle();
    if (!env) return FKS_ERR_OUT_OF_MEMORY;
    try {
        build_normals(obstacles, num_obstacles, grid, sdf_values, &env->offsets, &env->entries);
        env->obstacles.assign(obstacles, obstacles + num_obstacles);
    } catch (const std::bad_alloc&) {
        delete env;
        return FKS_ERR_OUT_OF_MEMORY;
    }
    env->geometry = *sdf_geometry;
    *out = env;
    return FKS_OK;
}

/* the object id BuildEnvironment leaves in each cell (SEB.cpp:151-155: every obstacle's
 * samples SetValue(1.0, object_id) in obstacle order, the last write wins; 0 = free) */
extern "C" fks_status fks_env_cell_objects(const fks_env_handle* env, uint32_t* out, uint64_t num_cells) {
    if (!env || (num_cells > 0 && !out)) return FKS_ERR_INVALID_ARGUMENT;
    Grid grid;
    grid.res = env->geometry.resolution;
    grid.inv_res = 1.0 / grid.res;
    std::memcpy(grid.origin, env->geometry.origin, sizeof(grid.origin));
    for (int a = 0; a < 3; ++a) grid.n[a] = env->geometry.num_cells[a];
    if (num_cells != grid.cells()) return FKS_ERR_INVALID_ARGUMENT;
    if (env->occupancy.size() != num_cells) return FKS_ERR_UNSUPPORTED; /* a normals-only handle */
    if (env->obstacles.empty())                                          /* a device build's copy */
        for (uint8_t o : env->occupancy)
            if (o) return FKS_ERR_UNSUPPORTED;
    inverse34(grid.origin, grid.inv_origin);
    std::memset(out, 0, (size_t)num_cells * sizeof(uint32_t));
    for (const fks_obstacle& ob : env->obstacles) {
        int32_t nc[3];
        fks_env::obstacle_samples(ob, grid.res, nc);
        for (int32_t xi = 0; xi < nc[0]; ++xi)
            for (int32_t yi = 0; yi < nc[1]; ++yi)
                for (int32_t zi = 0; zi < nc[2]; ++zi) {
                    double w[3];
                    fks_env::obstacle_sample_world(ob, grid.res, grid.res * 0.5, xi, yi, zi, w);
                    int64_t idx[3];
                    if (grid.index(w, idx)) out[grid.linear(idx[0], idx[1], idx[2])] = ob.object_id;
                }
    }
    return FKS_OK;
}
