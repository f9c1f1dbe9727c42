/*
 * environment.hpp — the environment the simulator is built from: the reference's
 * SurfaceNormalGrid (SPCS:44-343) and its environment builder
 * (simulator_environment_builder, SEB.hpp / SEB.cpp:470-476), over the builder of the
 * C-ABI (fks_env_build, the restatement of SEB.cpp).
 *
 * The factories take sdf_tools::TaggedObjectCollisionMapGrid, sdf_tools::SignedDistanceField
 * and simple_particle_contact_simulator::SurfaceNormalGrid (FKS.hpp:18-22).  The two
 * sdf_tools types are the real ones in a planner workspace and stand-ins otherwise
 * (fks_external_types.hpp); SurfaceNormalGrid belongs to the reference package itself and
 * is defined here with its public API (SPCS:138-343: the VoxelGrid-shaped constructor,
 * IsInitialized, LookupSurfaceNormal, InsertSurfaceNormal, ClearStoredSurfaceNormals): a
 * grid built by the environment builder keeps the builder's CSR of (entry direction,
 * normal) pairs per cell, and becomes an editable sparse copy on its first insert or clear.
 * The builder's public steps (SEB.hpp:39-70): OBSTACLE_CONFIG (both constructors),
 * RawCellSurfaceNormal, DiscretizeObstacle, BuildEnvironment, UpdateSurfaceNormalGridCell,
 * AdjustSurfaceNormalGridForAllFlatSurfaces, BuildSurfaceNormalsGrid and
 * BuildCompleteEnvironment, which returns the three objects as SEB.cpp:470-476 does:
 *   - stand-in mode: the collision map, SDF and normals of one fks_env_build call;
 *   - workspace mode: BuildEnvironment's collision map (SEB.cpp:148-153: constructor,
 *     SetValue(1.0, object_id) at each filled cell's centre), the SDF from its own
 *     ExtractSignedDistanceField(+inf, {}, true, false) (SEB.cpp:473), and the normals
 *     BuildSurfaceNormalsGrid derives from that same SDF (SEB.cpp:474-475).
 * ToFksEnvironment turns the three objects into the fks_environment the C-ABI takes,
 * reading the SDF through GetImmutable (SPCS:941) and the normals from any initialized
 * grid, built or edited.  The host arithmetic here (normalisation, rotation, grid index)
 * uses the evaluation orders of the builder and the kernels; like the reference's own
 * build (CMakeLists.txt:66, no -march) it assumes no floating-point contraction.
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_ENVIRONMENT_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_ENVIRONMENT_HPP

#include <array>
#include <cmath>
#include <cstdint>
#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/fks_external_types.hpp"
#include "fks_capi.h"
#include "fks_portable_math.h"

namespace fks_detail {

/* one built environment (fks_env_handle): the surface-normal CSR lives here */
struct EnvironmentHolder {
    fks_env_handle* handle = nullptr;
    fks_environment view{};
    EnvironmentHolder() {}
    EnvironmentHolder(const EnvironmentHolder&) = delete;
    EnvironmentHolder& operator=(const EnvironmentHolder&) = delete;
    ~EnvironmentHolder() {
        if (handle) fks_env_free(handle);
    }
};

inline std::shared_ptr<EnvironmentHolder> build_environment(const std::vector<fks_obstacle>& obs, double resolution,
                                                            const double* grid_origin, const int64_t* num_cells) {
    auto holder = std::make_shared<EnvironmentHolder>();
    fks_status st = fks_env_build(obs.empty() ? nullptr : obs.data(), (int32_t)obs.size(), resolution, grid_origin, num_cells,
                                  &holder->handle);
    if (st != FKS_OK) throw std::runtime_error(std::string("BuildCompleteEnvironment: ") + fks_status_string(st));
    if ((st = fks_env_view(holder->handle, &holder->view)) != FKS_OK)
        throw std::runtime_error(std::string("fks_env_view: ") + fks_status_string(st));
    return holder;
}

/* VoxelGrid sizes in metres that give exactly n cells under ceil(size / resolution) */
inline double grid_size(int64_t n, double resolution) { return ((double)n - 0.5) * resolution; }

template <typename Grid>
inline void expect_cells(const Grid& g, const fks_grid_geometry& want, const char* what) {
    if (g.GetNumXCells() != want.num_cells[0] || g.GetNumYCells() != want.num_cells[1] || g.GetNumZCells() != want.num_cells[2])
        throw std::runtime_error(std::string(what) + ": grid has an unexpected cell count");
}

/* the holder of a handle whose view is already filled (fks_env_build_normals) */
inline std::shared_ptr<EnvironmentHolder> hold(fks_env_handle* handle, const char* what) {
    auto holder = std::make_shared<EnvironmentHolder>();
    holder->handle = handle;
    const fks_status st = fks_env_view(handle, &holder->view);
    if (st != FKS_OK) throw std::runtime_error(std::string(what) + ": fks_env_view: " + fks_status_string(st));
    return holder;
}

constexpr double kEps = 2.220446049250313e-16; /* std::numeric_limits<double>::epsilon(), EigenHelpers::SafeNormal */

/* StoredSurfaceNormal (SPCS:59-63): SafeNormal((entry direction, 0)) as a Vector4d (Eigen's
 * two-lane packet norm (x^2 + z^2) + (y^2 + w^2)), then SafeNormal(normal) as
 * a Vector3d; the builder's entries (fks_env_internal.h face_entry) take the same steps */
inline std::array<double, 6> stored_entry(const double normal[3], const double direction[3]) {
    std::array<double, 6> E;
    const double en = fks_math::dsqrt((direction[0] * direction[0] + direction[2] * direction[2]) +
                                      (direction[1] * direction[1] + 0.0 * 0.0));
    for (int b = 0; b < 3; ++b) E[(size_t)b] = (en > kEps) ? direction[b] / en : direction[b];
    const double nn = fks_math::dsqrt((normal[0] * normal[0] + normal[1] * normal[1]) + normal[2] * normal[2]);
    for (int b = 0; b < 3; ++b) E[(size_t)(3 + b)] = (nn > kEps) ? normal[b] / nn : normal[b];
    return E;
}

/* the 3x3 rotation of a 3x4 row-major transform times v (Eigen's coefficient order) */
inline void rotate34(const double* T, const double v[3], double out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = (T[4 * i] * v[0] + T[4 * i + 1] * v[1]) + T[4 * i + 2] * v[2];
}
inline void xform34(const double* T, const double v[3], double out[3]) {
    for (int i = 0; i < 3; ++i) out[i] = ((T[4 * i] * v[0] + T[4 * i + 1] * v[1]) + T[4 * i + 2] * v[2]) + T[4 * i + 3];
}

/* VoxelGrid::LocationToGridIndex3d + IndexInBounds over a grid geometry: the inverse origin
 * applied, scaled by 1 / resolution, truncated toward zero (the builder's Grid::index) */
inline bool location_to_index(const fks_grid_geometry& g, const double p[3], int64_t idx[3]) {
    double inv[12];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) inv[4 * i + j] = g.origin[4 * j + i];
    for (int i = 0; i < 3; ++i)
        inv[4 * i + 3] = -((inv[4 * i] * g.origin[3] + inv[4 * i + 1] * g.origin[7]) + inv[4 * i + 2] * g.origin[11]);
    double q[3];
    xform34(inv, p, q);
    const double inv_res = 1.0 / g.resolution;
    for (int a = 0; a < 3; ++a) {
        const double v = q[a] * inv_res;
        if (!(v > -9.0e18 && v < 9.0e18)) return false;
        idx[a] = (int64_t)v;
        if (idx[a] < 0 || idx[a] >= g.num_cells[a]) return false;
    }
    return true;
}

/* the surface-normal CSR of an edited grid (ToFksEnvironment) */
struct NormalCsr {
    std::vector<uint32_t> offsets;
    std::vector<double> entries;
};

}  // namespace fks_detail

namespace simple_particle_contact_simulator {

/* SurfaceNormalGrid (SPCS:44-343): per cell, (entry direction, normal) pairs in insertion order */
class SurfaceNormalGrid {
  public:
    typedef std::array<double, 6> Entry; /* unit entry direction xyz, unit normal xyz */
    typedef std::pair<fks_planner_types::Vector3d, bool> LookupResult;

    SurfaceNormalGrid() {}
    /* SPCS:138-142: an empty grid of ceil(size / resolution) cells per axis at origin_transform */
    SurfaceNormalGrid(const fks_planner_types::Isometry3d& origin_transform, const double resolution, const double x_size,
                      const double y_size, const double z_size, const std::string& frame = "world")
        : frame_(frame), initialized_(true) {
        if (!(resolution > 0.0)) throw std::invalid_argument("SurfaceNormalGrid: resolution must be > 0");
        const std::array<double, 12> o = fks_ext::iso_to_row_major34(origin_transform);
        for (int k = 0; k < 12; ++k) geom_.origin[k] = o[(size_t)k];
        geom_.resolution = resolution;
        const double sizes[3] = {x_size, y_size, z_size};
        for (int a = 0; a < 3; ++a) geom_.num_cells[a] = (int64_t)std::ceil(std::fabs(sizes[a]) / resolution);
        cells_ = std::make_shared<std::map<uint64_t, std::vector<Entry>>>();
    }
    /* a grid the environment builder made (its CSR, shared and immutable until edited) */
    SurfaceNormalGrid(std::shared_ptr<const fks_detail::EnvironmentHolder> env, const std::string& frame)
        : env_(std::move(env)), frame_(frame), initialized_(true) {
        if (!env_) throw std::invalid_argument("SurfaceNormalGrid: null environment");
        geom_ = env_->view.normals;
    }

    bool IsInitialized() const { return initialized_; }
    double GetResolution() const { return Geometry().resolution; }
    fks_planner_types::Isometry3d GetOriginTransform() const { return fks_ext::iso_from_row_major34(Geometry().origin); }
    int64_t GetNumXCells() const { return Geometry().num_cells[0]; }
    int64_t GetNumYCells() const { return Geometry().num_cells[1]; }
    int64_t GetNumZCells() const { return Geometry().num_cells[2]; }
    const std::string& GetFrame() const { return frame_; }
    bool IndexInBounds(int64_t x, int64_t y, int64_t z) const {
        const fks_grid_geometry& g = Geometry();
        return x >= 0 && y >= 0 && z >= 0 && x < g.num_cells[0] && y < g.num_cells[1] && z < g.num_cells[2];
    }
    const fks_grid_geometry& Geometry() const {
        if (!initialized_) throw std::logic_error("SurfaceNormalGrid is not initialized");
        return geom_;
    }

    /* LookupSurfaceNormal (SPCS:152-262): the normal of the stored entry whose entry direction
     * best matches `direction` (GetBestSurfaceNormal SPCS:91-130, strict > so the first best
     * wins); (0, true) for an empty cell, (0, false) out of bounds */
    LookupResult LookupSurfaceNormal(const double x, const double y, const double z,
                                     const fks_planner_types::Vector3d& direction) const {
        return LookupSurfaceNormal(fks_planner_types::Vector3d(x, y, z), direction);
    }
    LookupResult LookupSurfaceNormal(const fks_planner_types::Vector3d& location, const fks_planner_types::Vector3d& direction) const {
        int64_t i[3];
        if (!Index(location(0), location(1), location(2), i)) return Miss();
        return LookupSurfaceNormal(i[0], i[1], i[2], direction);
    }
    LookupResult LookupSurfaceNormal(const fks_planner_types::Vector4d& location, const fks_planner_types::Vector3d& direction) const {
        int64_t i[3];
        if (!Index(location(0), location(1), location(2), i)) return Miss();
        return LookupSurfaceNormal(i[0], i[1], i[2], direction);
    }
    LookupResult LookupSurfaceNormal(const fks_planner_types::Vector4d& location, const fks_planner_types::Vector4d& direction) const {
        int64_t i[3];
        if (!Index(location(0), location(1), location(2), i)) return Miss();
        return LookupSurfaceNormal(i[0], i[1], i[2], direction);
    }
    LookupResult LookupSurfaceNormal(const int64_t x, const int64_t y, const int64_t z, const fks_planner_types::Vector3d& direction) const {
        if (!IndexInBounds(x, y, z)) return Miss();
        const double d[4] = {direction(0), direction(1), direction(2), 0.0};
        return Best(x, y, z, d, false);
    }
    LookupResult LookupSurfaceNormal(const int64_t x, const int64_t y, const int64_t z, const fks_planner_types::Vector4d& direction) const {
        if (!IndexInBounds(x, y, z)) return Miss();
        const double d[4] = {direction(0), direction(1), direction(2), direction(3)};
        return Best(x, y, z, d, true);
    }

    /* InsertSurfaceNormal (SPCS:264-300): append (SafeNormal(entry_direction), SafeNormal(normal))
     * to the cell; false out of bounds */
    bool InsertSurfaceNormal(const double x, const double y, const double z, const fks_planner_types::Vector3d& surface_normal,
                             const fks_planner_types::Vector3d& entry_direction) {
        return InsertSurfaceNormal(fks_planner_types::Vector3d(x, y, z), surface_normal, entry_direction);
    }
    bool InsertSurfaceNormal(const fks_planner_types::Vector3d& location, const fks_planner_types::Vector3d& surface_normal,
                             const fks_planner_types::Vector3d& entry_direction) {
        int64_t i[3];
        if (!Index(location(0), location(1), location(2), i)) return false;
        return InsertSurfaceNormal(i[0], i[1], i[2], surface_normal, entry_direction);
    }
    bool InsertSurfaceNormal(const int64_t x, const int64_t y, const int64_t z, const fks_planner_types::Vector3d& surface_normal,
                             const fks_planner_types::Vector3d& entry_direction) {
        if (!IndexInBounds(x, y, z)) return false;
        const double n[3] = {surface_normal(0), surface_normal(1), surface_normal(2)};
        const double e[3] = {entry_direction(0), entry_direction(1), entry_direction(2)};
        Editable()[Linear(x, y, z)].push_back(fks_detail::stored_entry(n, e));
        return true;
    }

    /* ClearStoredSurfaceNormals (SPCS:302-338): empty the cell; false out of bounds */
    bool ClearStoredSurfaceNormals(const double x, const double y, const double z) {
        return ClearStoredSurfaceNormals(fks_planner_types::Vector3d(x, y, z));
    }
    bool ClearStoredSurfaceNormals(const fks_planner_types::Vector3d& location) {
        int64_t i[3];
        if (!Index(location(0), location(1), location(2), i)) return false;
        return ClearStoredSurfaceNormals(i[0], i[1], i[2]);
    }
    bool ClearStoredSurfaceNormals(const int64_t x, const int64_t y, const int64_t z) {
        if (!IndexInBounds(x, y, z)) return false;
        Editable().erase(Linear(x, y, z));
        return true;
    }

    /* the stored (entry direction, normal) pairs of a cell, in insertion order */
    std::vector<std::pair<fks_planner_types::Vector4d, fks_planner_types::Vector3d>> GetCellEntries(int64_t x, int64_t y,
                                                                                                        int64_t z) const {
        std::vector<std::pair<fks_planner_types::Vector4d, fks_planner_types::Vector3d>> out;
        if (!initialized_ || !IndexInBounds(x, y, z)) return out;
        size_t n = 0;
        const double* p = CellEntries(Linear(x, y, z), &n);
        for (size_t e = 0; e < n; ++e, p += 6)
            out.emplace_back(fks_planner_types::Vector4d(p[0], p[1], p[2], 0.0), fks_planner_types::Vector3d(p[3], p[4], p[5]));
        return out;
    }

    /* the CSR the C-ABI reads (fks_environment.normal_offsets [cells + 1], 6 doubles per
     * entry): the builder's own arrays while unedited, else built once per edit state */
    const uint32_t* CsrOffsets() const { return Csr().first; }
    const double* CsrEntries() const { return Csr().second; }

  private:
    static LookupResult Miss() { return LookupResult(fks_planner_types::Vector3d(0.0, 0.0, 0.0), false); }
    bool Index(double x, double y, double z, int64_t idx[3]) const {
        const double p[3] = {x, y, z};
        return fks_detail::location_to_index(Geometry(), p, idx);
    }
    uint64_t Linear(int64_t x, int64_t y, int64_t z) const {
        return ((uint64_t)x * (uint64_t)geom_.num_cells[1] + (uint64_t)y) * (uint64_t)geom_.num_cells[2] + (uint64_t)z;
    }
    const double* CellEntries(uint64_t c, size_t* n) const {
        if (cells_) {
            const auto it = cells_->find(c);
            *n = (it == cells_->end()) ? 0 : it->second.size();
            return *n ? it->second.front().data() : nullptr;
        }
        if (!env_ || !env_->view.normal_offsets) {
            *n = 0;
            return nullptr;
        }
        const uint32_t b = env_->view.normal_offsets[c], e = env_->view.normal_offsets[c + 1];
        *n = e - b;
        return env_->view.normal_entries + 6 * (size_t)b;
    }
    LookupResult Best(int64_t x, int64_t y, int64_t z, const double d[4], bool four) const {
        size_t n = 0;
        const double* p = CellEntries(Linear(x, y, z), &n);
        if (n == 0) return LookupResult(fks_planner_types::Vector3d(0.0, 0.0, 0.0), true);
        /* GetBestSurfaceNormal: Vector3d norm / dot sequential, Vector4d in packet order */
        const double norm = four ? fks_math::dsqrt((d[0] * d[0] + d[2] * d[2]) + (d[1] * d[1] + d[3] * d[3]))
                                 : fks_math::dsqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]);
        if (!(norm > 0.0)) throw std::invalid_argument("LookupSurfaceNormal: zero direction (SPCS:113-114 assert)");
        const double u[4] = {d[0] / norm, d[1] / norm, d[2] / norm, d[3] / norm};
        int64_t best = -1;
        double best_dot = -std::numeric_limits<double>::infinity();
        for (size_t e = 0; e < n; ++e) {
            const double* q = p + 6 * e;
            const double dot = four ? (q[0] * u[0] + q[2] * u[2]) + (q[1] * u[1] + 0.0 * u[3]) : (q[0] * u[0] + q[1] * u[1]) + q[2] * u[2];
            if (dot > best_dot) {
                best_dot = dot;
                best = (int64_t)e;
            }
        }
        if (best < 0) throw std::invalid_argument("LookupSurfaceNormal: no comparable entry (SPCS:127 assert)");
        const double* q = p + 6 * (size_t)best;
        return LookupResult(fks_planner_types::Vector3d(q[3], q[4], q[5]), true);
    }
    /* the editable cells: the builder's CSR copied on the first edit; copies of this grid
     * share nothing they can change */
    std::map<uint64_t, std::vector<Entry>>& Editable() {
        if (!initialized_) throw std::logic_error("SurfaceNormalGrid is not initialized");
        if (!cells_) {
            auto cells = std::make_shared<std::map<uint64_t, std::vector<Entry>>>();
            if (env_ && env_->view.normal_offsets) {
                const uint64_t total = (uint64_t)geom_.num_cells[0] * (uint64_t)geom_.num_cells[1] * (uint64_t)geom_.num_cells[2];
                for (uint64_t c = 0; c < total; ++c)
                    for (uint32_t e = env_->view.normal_offsets[c]; e < env_->view.normal_offsets[c + 1]; ++e) {
                        Entry E;
                        for (int k = 0; k < 6; ++k) E[(size_t)k] = env_->view.normal_entries[6 * (size_t)e + (size_t)k];
                        (*cells)[c].push_back(E);
                    }
            }
            cells_ = cells;
            env_.reset();
        } else if (cells_.use_count() > 1) {
            cells_ = std::make_shared<std::map<uint64_t, std::vector<Entry>>>(*cells_);
        }
        csr_.reset();
        return *cells_;
    }
    std::pair<const uint32_t*, const double*> Csr() const {
        const fks_grid_geometry& g = Geometry();
        if (!cells_ && env_) return {env_->view.normal_offsets, env_->view.normal_entries};
        if (!csr_) {
            auto csr = std::make_shared<fks_detail::NormalCsr>();
            const uint64_t total = (uint64_t)g.num_cells[0] * (uint64_t)g.num_cells[1] * (uint64_t)g.num_cells[2];
            csr->offsets.assign(total + 1, 0);
            uint64_t count = 0, c = 0;
            for (const auto& kv : *cells_) {
                for (; c <= kv.first; ++c) csr->offsets[c] = (uint32_t)count;
                for (const Entry& E : kv.second) csr->entries.insert(csr->entries.end(), E.begin(), E.end());
                count += kv.second.size();
                if (count > 0xffffffffull) throw std::length_error("SurfaceNormalGrid: more than 2^32 entries");
            }
            for (; c <= total; ++c) csr->offsets[c] = (uint32_t)count;
            csr_ = csr;
        }
        return {csr_->offsets.data(), csr_->entries.empty() ? nullptr : csr_->entries.data()};
    }

    std::shared_ptr<const fks_detail::EnvironmentHolder> env_;
    std::shared_ptr<std::map<uint64_t, std::vector<Entry>>> cells_;
    mutable std::shared_ptr<const fks_detail::NormalCsr> csr_;
    fks_grid_geometry geom_{};
    std::string frame_ = "world";
    bool initialized_ = false;
};

}  // namespace simple_particle_contact_simulator

namespace simulator_environment_builder {

/* OBSTACLE_CONFIG (SEB.hpp:25-48): object id > 0, pose, half extents */
struct OBSTACLE_CONFIG {
    fks_planner_types::Isometry3d pose;
    fks_planner_types::Vector3d extents;
    uint32_t object_id = 0;
    OBSTACLE_CONFIG() : pose(fks_planner_types::Isometry3d::Identity()), extents(0.0, 0.0, 0.0) {}
    OBSTACLE_CONFIG(const uint32_t in_object_id, const fks_planner_types::Isometry3d& in_pose,
                    const fks_planner_types::Vector3d& in_extents)
        : pose(in_pose), extents(in_extents), object_id(in_object_id) {
        if (in_object_id == 0) throw std::invalid_argument("object id must be > 0 (SEB.hpp assert)");
    }
    /* SEB.hpp:39-45: pose = Translation3d(translation) * orientation, the rotation by Eigen's
     * Quaternion::toRotationMatrix formula */
    OBSTACLE_CONFIG(const uint32_t in_object_id, const fks_planner_types::Vector3d& in_translation,
                    const fks_planner_types::Quaterniond& in_orientation, const fks_planner_types::Vector3d& in_extents)
        : pose(fks_planner_types::Isometry3d::Identity()), extents(in_extents), object_id(in_object_id) {
        if (in_object_id == 0) throw std::invalid_argument("object id must be > 0 (SEB.hpp assert)");
        const double w = in_orientation.w(), x = in_orientation.x(), y = in_orientation.y(), z = in_orientation.z();
        const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
        const double twx = tx * w, twy = ty * w, twz = tz * w;
        const double txx = tx * x, txy = ty * x, txz = tz * x;
        const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
        const double R[9] = {1.0 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.0 - (txx + tzz),
                             tyz - twx, txz - twy, tyz + twx, 1.0 - (txx + tyy)};
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) pose.matrix()(r, c) = R[3 * r + c];
            pose.matrix()(r, 3) = in_translation(r);
        }
    }
};

/* RawCellSurfaceNormal (SEB.hpp:50-57) */
struct RawCellSurfaceNormal {
    fks_planner_types::Vector3d normal;
    fks_planner_types::Vector3d entry_direction;
    RawCellSurfaceNormal(const fks_planner_types::Vector3d& in_normal, const fks_planner_types::Vector3d& in_direction)
        : normal(in_normal), entry_direction(in_direction) {}
    RawCellSurfaceNormal() : normal(0.0, 0.0, 0.0), entry_direction(0.0, 0.0, 0.0) {}
};

/* EnvironmentComponents (SEB.hpp:72-98) */
class EnvironmentComponents {
  public:
    EnvironmentComponents(const sdf_tools::TaggedObjectCollisionMapGrid& environment, const sdf_tools::SignedDistanceField& environment_sdf,
                          const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid)
        : environment_(environment), environment_sdf_(environment_sdf), surface_normals_grid_(surface_normals_grid) {}
    const sdf_tools::TaggedObjectCollisionMapGrid& GetEnvironment() const { return environment_; }
    const sdf_tools::SignedDistanceField& GetEnvironmentSDF() const { return environment_sdf_; }
    const simple_particle_contact_simulator::SurfaceNormalGrid& GetSurfaceNormalsGrid() const { return surface_normals_grid_; }

  private:
    sdf_tools::TaggedObjectCollisionMapGrid environment_;
    sdf_tools::SignedDistanceField environment_sdf_;
    simple_particle_contact_simulator::SurfaceNormalGrid surface_normals_grid_;
};

namespace detail {
inline std::vector<fks_obstacle> to_fks(const std::vector<OBSTACLE_CONFIG>& obstacles) {
    std::vector<fks_obstacle> obs(obstacles.size());
    for (size_t i = 0; i < obstacles.size(); ++i) {
        const std::array<double, 12> pose = fks_ext::iso_to_row_major34(obstacles[i].pose);
        for (int k = 0; k < 12; ++k) obs[i].pose[k] = pose[(size_t)k];
        for (int k = 0; k < 3; ++k) obs[i].extents[k] = obstacles[i].extents(k);
        obs[i].object_id = obstacles[i].object_id;
        obs[i].reserved = 0;
    }
    return obs;
}

/* the collision map of a built environment (SEB.cpp:148-155): every filled cell gets
 * TAGGED_OBJECT_COLLISION_CELL(1.0, object id of the last obstacle that filled it) */
inline sdf_tools::TaggedObjectCollisionMapGrid collision_map(const fks_detail::EnvironmentHolder& holder, const std::string& frame) {
    const fks_grid_geometry& g = holder.view.collision_map;
    const size_t cells = (size_t)(g.num_cells[0] * g.num_cells[1] * g.num_cells[2]);
    std::vector<uint32_t> ids(cells);
    const fks_status st = fks_env_cell_objects(holder.handle, ids.data(), ids.size());
    if (st != FKS_OK) throw std::runtime_error(std::string("fks_env_cell_objects: ") + fks_status_string(st));
    const fks_planner_types::Isometry3d origin = fks_ext::iso_from_row_major34(g.origin);
    const sdf_tools::TAGGED_OBJECT_COLLISION_CELL default_cell;
    sdf_tools::TaggedObjectCollisionMapGrid grid(origin, frame, g.resolution, fks_detail::grid_size(g.num_cells[0], g.resolution),
                                                 fks_detail::grid_size(g.num_cells[1], g.resolution),
                                                 fks_detail::grid_size(g.num_cells[2], g.resolution), default_cell);
    fks_detail::expect_cells(grid, g, "BuildEnvironment");
#if FKS_EXTERNAL_PLANNER_TYPES
    size_t k = 0;
    for (int64_t x = 0; x < g.num_cells[0]; ++x)
        for (int64_t y = 0; y < g.num_cells[1]; ++y)
            for (int64_t z = 0; z < g.num_cells[2]; ++z, ++k) {
                if (!ids[k]) continue;
                const fks_planner_types::Vector3d c(g.resolution * ((double)x + 0.5), g.resolution * ((double)y + 0.5),
                                                    g.resolution * ((double)z + 0.5));
                const fks_planner_types::Vector3d w = origin * c;
                grid.SetValue(w.x(), w.y(), w.z(), sdf_tools::TAGGED_OBJECT_COLLISION_CELL(1.0f, ids[k]));
            }
#else
    auto& cells_out = grid.GetMutableRawData();
    for (size_t k = 0; k < cells; ++k)
        if (ids[k]) cells_out[k] = sdf_tools::TAGGED_OBJECT_COLLISION_CELL(1.0f, ids[k]);
#endif
    return grid;
}

/* the SDF's values in VoxelGrid order */
inline std::vector<float> sdf_values(const sdf_tools::SignedDistanceField& sdf) {
#if FKS_EXTERNAL_PLANNER_TYPES
    return fks_ext::sdf_values(sdf);
#else
    return sdf.GetImmutableRawData();
#endif
}

/* the SDF value at a world location (sdf_tools GetImmutable3d: the OOB value outside) */
inline float sdf_at(const sdf_tools::SignedDistanceField& sdf, const double p[3]) {
    const fks_grid_geometry g = fks_ext::grid_geometry(sdf);
    int64_t i[3];
    if (!fks_detail::location_to_index(g, p, i)) return sdf.GetOOBValue();
    return sdf.GetImmutable(i[0], i[1], i[2]).first;
}
}  // namespace detail

/* DiscretizeObstacle (SEB.cpp:21-46): the obstacle's half-resolution sample positions relative
 * to the obstacle (BuildEnvironment places them with obstacle.pose, SEB.cpp:84-85), each with
 * TAGGED_OBJECT_COLLISION_CELL(1.0, object_id) */
inline std::vector<std::pair<fks_planner_types::Vector3d, sdf_tools::TAGGED_OBJECT_COLLISION_CELL>> DiscretizeObstacle(
    const OBSTACLE_CONFIG& obstacle, const double resolution) {
    const fks_obstacle ob = detail::to_fks({obstacle})[0];
    uint64_t n = 0;
    fks_status st = fks_env_discretize_obstacle(&ob, resolution, nullptr, 0, &n);
    std::vector<double> xyz(3 * (size_t)n);
    if (st == FKS_OK && n) st = fks_env_discretize_obstacle(&ob, resolution, xyz.data(), n, &n);
    if (st != FKS_OK) throw std::runtime_error(std::string("DiscretizeObstacle: ") + fks_status_string(st));
    std::vector<std::pair<fks_planner_types::Vector3d, sdf_tools::TAGGED_OBJECT_COLLISION_CELL>> out;
    out.reserve((size_t)n);
    for (uint64_t k = 0; k < n; ++k)
        out.emplace_back(fks_planner_types::Vector3d(xyz[3 * k], xyz[3 * k + 1], xyz[3 * k + 2]),
                         sdf_tools::TAGGED_OBJECT_COLLISION_CELL(1.0f, obstacle.object_id));
    return out;
}

/* BuildEnvironment (SEB.cpp:49-160): the grid sized to the obstacles plus a 3-cell border
 * (or, with grid_origin (3x4 row-major) and num_cells, that fixed box), each obstacle's
 * samples set to (1.0, object_id) in obstacle order */
inline sdf_tools::TaggedObjectCollisionMapGrid BuildEnvironment(const std::vector<OBSTACLE_CONFIG>& obstacles, const double resolution,
                                                                const double* grid_origin = nullptr, const int64_t* num_cells = nullptr,
                                                                const std::string& frame = "uncertainty_planning_simulator") {
    const std::shared_ptr<fks_detail::EnvironmentHolder> holder =
        fks_detail::build_environment(detail::to_fks(obstacles), resolution, grid_origin, num_cells);
    return detail::collision_map(*holder, frame);
}

/* UpdateSurfaceNormalGridCell (SEB.cpp:162-187): at transform * cell_location, if the SDF
 * there is above -1.5 resolution, replace the cell's entries with the raw normals rotated by
 * the transform */
inline void UpdateSurfaceNormalGridCell(const std::vector<RawCellSurfaceNormal>& raw_surface_normals,
                                        const fks_planner_types::Isometry3d& transform, const fks_planner_types::Vector3d& cell_location,
                                        const sdf_tools::SignedDistanceField& environment_sdf,
                                        simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid) {
    const std::array<double, 12> T = fks_ext::iso_to_row_major34(transform);
    const double c[3] = {cell_location(0), cell_location(1), cell_location(2)};
    double w[3];
    fks_detail::xform34(T.data(), c, w);
    const float distance = detail::sdf_at(environment_sdf, w);
    if (!(distance > -(environment_sdf.GetResolution() * 1.5))) return;
    const fks_planner_types::Vector3d world(w[0], w[1], w[2]);
    surface_normals_grid.ClearStoredSurfaceNormals(world);
    for (const RawCellSurfaceNormal& raw : raw_surface_normals) {
        const double n[3] = {raw.normal(0), raw.normal(1), raw.normal(2)};
        const double e[3] = {raw.entry_direction(0), raw.entry_direction(1), raw.entry_direction(2)};
        double rn[3], re[3];
        fks_detail::rotate34(T.data(), n, rn);
        fks_detail::rotate34(T.data(), e, re);
        surface_normals_grid.InsertSurfaceNormal(world, fks_planner_types::Vector3d(rn[0], rn[1], rn[2]),
                                                 fks_planner_types::Vector3d(re[0], re[1], re[2]));
    }
}

/* AdjustSurfaceNormalGridForAllFlatSurfaces (SEB.cpp:189-256): every filled cell next to a
 * free one gets the axis-aligned face normals of its free neighbours */
inline void AdjustSurfaceNormalGridForAllFlatSurfaces(const sdf_tools::SignedDistanceField& environment_sdf,
                                                      simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid) {
    typedef fks_planner_types::Vector3d V;
    for (int64_t x = 0; x < environment_sdf.GetNumXCells(); ++x)
        for (int64_t y = 0; y < environment_sdf.GetNumYCells(); ++y)
            for (int64_t z = 0; z < environment_sdf.GetNumZCells(); ++z) {
                if (!(environment_sdf.GetImmutable(x, y, z).first < 0.0)) continue;
                const bool edge[6] = {environment_sdf.GetImmutable(x - 1, y, z).first > 0.0, environment_sdf.GetImmutable(x + 1, y, z).first > 0.0,
                                      environment_sdf.GetImmutable(x, y - 1, z).first > 0.0, environment_sdf.GetImmutable(x, y + 1, z).first > 0.0,
                                      environment_sdf.GetImmutable(x, y, z - 1).first > 0.0, environment_sdf.GetImmutable(x, y, z + 1).first > 0.0};
                if (!(edge[0] || edge[1] || edge[2] || edge[3] || edge[4] || edge[5])) continue;
                surface_normals_grid.ClearStoredSurfaceNormals(x, y, z);
                for (int f = 0; f < 6; ++f) {
                    if (!edge[f]) continue;
                    double n[3] = {0.0, 0.0, 0.0}, e[3] = {0.0, 0.0, 0.0};
                    n[f / 2] = (f % 2) ? 1.0 : -1.0;
                    e[f / 2] = (f % 2) ? -1.0 : 1.0;
                    surface_normals_grid.InsertSurfaceNormal(x, y, z, V(n[0], n[1], n[2]), V(e[0], e[1], e[2]));
                }
            }
}

/* BuildSurfaceNormalsGrid (SEB.cpp:258-468) on the given SDF: the SDF-gradient entry of every
 * cell with a negative distance, then the obstacles' exact face / edge / corner normals */
inline simple_particle_contact_simulator::SurfaceNormalGrid BuildSurfaceNormalsGrid(const std::vector<OBSTACLE_CONFIG>& obstacles,
                                                                                   const sdf_tools::SignedDistanceField& environment_sdf) {
    const std::vector<fks_obstacle> obs = detail::to_fks(obstacles);
    const fks_grid_geometry g = fks_ext::grid_geometry(environment_sdf);
    const std::vector<float> values = detail::sdf_values(environment_sdf);
    fks_env_handle* h = nullptr;
    const fks_status st = fks_env_build_normals(obs.empty() ? nullptr : obs.data(), (int32_t)obs.size(), &g, values.data(), &h);
    if (st != FKS_OK) throw std::runtime_error(std::string("BuildSurfaceNormalsGrid: ") + fks_status_string(st));
    return simple_particle_contact_simulator::SurfaceNormalGrid(fks_detail::hold(h, "BuildSurfaceNormalsGrid"),
                                                                environment_sdf.GetFrame());
}

/* BuildCompleteEnvironment (SEB.cpp:470-476): the grid sized to the obstacles plus a
 * 3-cell border; with grid_origin (3x4 row-major) and num_cells, that fixed box.  frame:
 * GetFrame() of the three objects (the reference names it "uncertainty_planning_simulator",
 * SEB.cpp:148). */
inline EnvironmentComponents BuildCompleteEnvironment(const std::vector<OBSTACLE_CONFIG>& obstacles, const double resolution,
                                                      const double* grid_origin = nullptr, const int64_t* num_cells = nullptr,
                                                      const std::string& frame = "uncertainty_planning_simulator") {
    const std::shared_ptr<fks_detail::EnvironmentHolder> holder =
        fks_detail::build_environment(detail::to_fks(obstacles), resolution, grid_origin, num_cells);
    const sdf_tools::TaggedObjectCollisionMapGrid grid = detail::collision_map(*holder, frame);
#if FKS_EXTERNAL_PLANNER_TYPES
    /* SEB.cpp:473-475: the SDF from sdf_tools, the normals from that same SDF */
    const sdf_tools::SignedDistanceField sdf =
        grid.ExtractSignedDistanceField(std::numeric_limits<float>::infinity(), std::vector<uint32_t>(), true, false).first;
    fks_detail::expect_cells(sdf, holder->view.sdf, "ExtractSignedDistanceField");
    return EnvironmentComponents(grid, sdf, BuildSurfaceNormalsGrid(obstacles, sdf));
#else
    const fks_grid_geometry& sg = holder->view.sdf;
    const size_t cells = (size_t)(sg.num_cells[0] * sg.num_cells[1] * sg.num_cells[2]);
    sdf_tools::SignedDistanceField sdf(fks_ext::iso_from_row_major34(sg.origin), frame, sg.resolution,
                                       fks_detail::grid_size(sg.num_cells[0], sg.resolution),
                                       fks_detail::grid_size(sg.num_cells[1], sg.resolution),
                                       fks_detail::grid_size(sg.num_cells[2], sg.resolution), holder->view.sdf_oob_value);
    fks_detail::expect_cells(sdf, sg, "BuildCompleteEnvironment");
    sdf.GetMutableRawData().assign(holder->view.sdf_values, holder->view.sdf_values + cells);
    return EnvironmentComponents(grid, sdf, simple_particle_contact_simulator::SurfaceNormalGrid(holder, frame));
#endif
}

/* the fks_environment the C-ABI takes, from the three objects.  With the real sdf_tools the
 * SDF values are read into `sdf_storage`; with the stand-in the result points into
 * `environment_sdf`.  Either must outlive the call that uses the result; the normal CSR is
 * a view into the SurfaceNormalGrid (any initialized grid: built, or made and filled through
 * InsertSurfaceNormal). */
inline fks_environment ToFksEnvironment(const sdf_tools::TaggedObjectCollisionMapGrid& environment,
                                        const sdf_tools::SignedDistanceField& environment_sdf,
                                        const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid,
                                        std::vector<float>& sdf_storage) {
    if (!surface_normals_grid.IsInitialized()) throw std::invalid_argument("the surface normal grid is not initialized");
    fks_environment e{};
    e.collision_map = fks_ext::grid_geometry(environment);
    e.sdf = fks_ext::grid_geometry(environment_sdf);
#if FKS_EXTERNAL_PLANNER_TYPES
    sdf_storage = fks_ext::sdf_values(environment_sdf);
    e.sdf_values = sdf_storage.data();
#else
    (void)sdf_storage; /* the stand-in's cells are already in VoxelGrid order */
    e.sdf_values = environment_sdf.GetImmutableRawData().data();
#endif
    e.sdf_oob_value = environment_sdf.GetOOBValue();
    e.normals = surface_normals_grid.Geometry();
    e.normal_offsets = surface_normals_grid.CsrOffsets();
    e.normal_entries = surface_normals_grid.CsrEntries();
    return e;
}

}  // namespace simulator_environment_builder

#endif
