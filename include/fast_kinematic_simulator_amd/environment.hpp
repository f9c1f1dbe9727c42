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
 * is defined here (a CSR of (entry direction, normal) pairs per cell, insertion order).
 * BuildCompleteEnvironment returns the three objects as SEB.cpp:470-476 does:
 *   - stand-in mode: the collision map and SDF of fks_env_build copied into the stand-in
 *     VoxelGrid containers;
 *   - workspace mode: the collision map built as SEB.cpp:148-153 builds it (constructor,
 *     SetValue at each filled cell's centre) and the SDF from its own
 *     ExtractSignedDistanceField(+inf, {}, true, false) (SEB.cpp:473), as the reference
 *     does; the surface normals from fks_env_build's exact EDT (equal to sdf_tools' exact
 *     EDT on the same grid).
 * ToFksEnvironment turns the three objects into the fks_environment the C-ABI takes,
 * reading the SDF through GetImmutable (SPCS:941).
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_ENVIRONMENT_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_ENVIRONMENT_HPP

#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/fks_external_types.hpp"
#include "fks_capi.h"

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

}  // namespace fks_detail

namespace simple_particle_contact_simulator {

/* SurfaceNormalGrid (SPCS:44-343): per cell, (entry direction, normal) pairs in insertion order */
class SurfaceNormalGrid {
  public:
    SurfaceNormalGrid() {}
    SurfaceNormalGrid(std::shared_ptr<const fks_detail::EnvironmentHolder> env, const std::string& frame)
        : env_(std::move(env)), frame_(frame) {}
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
    std::vector<std::pair<fks_planner_types::Vector4d, fks_planner_types::Vector3d>> GetCellEntries(int64_t x, int64_t y,
                                                                                                        int64_t z) const {
        std::vector<std::pair<fks_planner_types::Vector4d, fks_planner_types::Vector3d>> out;
        if (!env_ || !IndexInBounds(x, y, z) || !env_->view.normal_offsets) return out;
        const fks_grid_geometry& g = Geometry();
        const size_t c = ((size_t)x * (size_t)g.num_cells[1] + (size_t)y) * (size_t)g.num_cells[2] + (size_t)z;
        for (uint32_t e = env_->view.normal_offsets[c]; e < env_->view.normal_offsets[c + 1]; ++e) {
            const double* p = env_->view.normal_entries + 6 * (size_t)e;
            out.emplace_back(fks_planner_types::Vector4d(p[0], p[1], p[2], 0.0), fks_planner_types::Vector3d(p[3], p[4], p[5]));
        }
        return out;
    }
    /* the CSR the C-ABI reads (offsets[cells + 1], 6 doubles per entry) */
    const std::shared_ptr<const fks_detail::EnvironmentHolder>& Holder() const { return env_; }
    const fks_grid_geometry& Geometry() const {
        if (!env_) throw std::logic_error("empty SurfaceNormalGrid");
        return env_->view.normals;
    }

  private:
    std::shared_ptr<const fks_detail::EnvironmentHolder> env_;
    std::string frame_ = "world";
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

/* BuildCompleteEnvironment (SEB.cpp:470-476): the grid sized to the obstacles plus a
 * 3-cell border; with grid_origin (3x4 row-major) and num_cells, that fixed box.  frame:
 * GetFrame() of the three objects (the reference names it "uncertainty_planning_simulator",
 * SEB.cpp:148). */
inline EnvironmentComponents BuildCompleteEnvironment(const std::vector<OBSTACLE_CONFIG>& obstacles, const double resolution,
                                                      const double* grid_origin = nullptr, const int64_t* num_cells = nullptr,
                                                      const std::string& frame = "uncertainty_planning_simulator") {
    std::vector<fks_obstacle> obs(obstacles.size());
    for (size_t i = 0; i < obstacles.size(); ++i) {
        const std::array<double, 12> pose = fks_ext::iso_to_row_major34(obstacles[i].pose);
        for (int k = 0; k < 12; ++k) obs[i].pose[k] = pose[(size_t)k];
        for (int k = 0; k < 3; ++k) obs[i].extents[k] = obstacles[i].extents(k);
        obs[i].object_id = obstacles[i].object_id;
        obs[i].reserved = 0;
    }
    std::shared_ptr<fks_detail::EnvironmentHolder> holder = fks_detail::build_environment(obs, resolution, grid_origin, num_cells);
    const fks_grid_geometry& g = holder->view.collision_map;
    const size_t cells = (size_t)(g.num_cells[0] * g.num_cells[1] * g.num_cells[2]);
    std::vector<uint8_t> occupancy(cells);
    fks_status st = fks_env_occupancy(holder->handle, occupancy.data(), occupancy.size());
    if (st != FKS_OK) throw std::runtime_error(std::string("fks_env_occupancy: ") + fks_status_string(st));
    const fks_planner_types::Isometry3d origin = fks_ext::iso_from_row_major34(g.origin);
    const sdf_tools::TAGGED_OBJECT_COLLISION_CELL default_cell;
    sdf_tools::TaggedObjectCollisionMapGrid grid(origin, frame, g.resolution, fks_detail::grid_size(g.num_cells[0], g.resolution),
                                                 fks_detail::grid_size(g.num_cells[1], g.resolution),
                                                 fks_detail::grid_size(g.num_cells[2], g.resolution), default_cell);
    fks_detail::expect_cells(grid, g, "BuildCompleteEnvironment");
#if FKS_EXTERNAL_PLANNER_TYPES
    /* SEB.cpp:148-153, then SEB.cpp:473 */
    size_t k = 0;
    for (int64_t x = 0; x < g.num_cells[0]; ++x)
        for (int64_t y = 0; y < g.num_cells[1]; ++y)
            for (int64_t z = 0; z < g.num_cells[2]; ++z, ++k) {
                if (!occupancy[k]) continue;
                const fks_planner_types::Vector3d c(g.resolution * ((double)x + 0.5), g.resolution * ((double)y + 0.5),
                                                    g.resolution * ((double)z + 0.5));
                const fks_planner_types::Vector3d w = origin * c;
                grid.SetValue(w.x(), w.y(), w.z(), sdf_tools::TAGGED_OBJECT_COLLISION_CELL(1.0f, 1u));
            }
    const sdf_tools::SignedDistanceField sdf =
        grid.ExtractSignedDistanceField(std::numeric_limits<float>::infinity(), std::vector<uint32_t>(), true, false).first;
    fks_detail::expect_cells(sdf, g, "ExtractSignedDistanceField");
#else
    {
        auto& cells_out = grid.GetMutableRawData();
        for (size_t k = 0; k < cells; ++k)
            if (occupancy[k]) cells_out[k] = sdf_tools::TAGGED_OBJECT_COLLISION_CELL(1.0f, 0u);
    }
    const fks_grid_geometry& sg = holder->view.sdf;
    sdf_tools::SignedDistanceField sdf(fks_ext::iso_from_row_major34(sg.origin), frame, sg.resolution,
                                       fks_detail::grid_size(sg.num_cells[0], sg.resolution),
                                       fks_detail::grid_size(sg.num_cells[1], sg.resolution),
                                       fks_detail::grid_size(sg.num_cells[2], sg.resolution), holder->view.sdf_oob_value);
    fks_detail::expect_cells(sdf, sg, "BuildCompleteEnvironment");
    sdf.GetMutableRawData().assign(holder->view.sdf_values, holder->view.sdf_values + cells);
#endif
    return EnvironmentComponents(grid, sdf, simple_particle_contact_simulator::SurfaceNormalGrid(holder, frame));
}

/* the fks_environment the C-ABI takes, from the three objects.  With the real sdf_tools the
 * SDF values are read into `sdf_storage`; with the stand-in the result points into
 * `environment_sdf`.  Either must outlive the call that uses the result; the normal CSR is
 * a view into the SurfaceNormalGrid. */
inline fks_environment ToFksEnvironment(const sdf_tools::TaggedObjectCollisionMapGrid& environment,
                                        const sdf_tools::SignedDistanceField& environment_sdf,
                                        const simple_particle_contact_simulator::SurfaceNormalGrid& surface_normals_grid,
                                        std::vector<float>& sdf_storage) {
    if (!surface_normals_grid.Holder()) throw std::invalid_argument("the surface normal grid must come from BuildCompleteEnvironment");
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
    e.normal_offsets = surface_normals_grid.Holder()->view.normal_offsets;
    e.normal_entries = surface_normals_grid.Holder()->view.normal_entries;
    return e;
}

}  // namespace simulator_environment_builder

#endif
