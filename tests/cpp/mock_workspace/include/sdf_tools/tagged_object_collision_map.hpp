/* Mock of sdf_tools::TaggedObjectCollisionMapGrid as the reference builds and reads it
 * (test only; tests/cpp/mock_workspace/README.md): the constructor and SetValue of
 * SEB.cpp:147-153, ExtractSignedDistanceField of SEB.cpp:473 (exact Euclidean distance
 * transform by brute-force 1-D minimisation per axis: + distance to the nearest filled cell
 * for free cells, - distance to the nearest free cell for filled cells). */
#ifndef MOCK_SDF_TOOLS_TAGGED_OBJECT_COLLISION_MAP
#define MOCK_SDF_TOOLS_TAGGED_OBJECT_COLLISION_MAP
#include <cmath>
#include <cstdint>
#include <limits>
#include <utility>
#include <vector>
#include <sdf_tools/sdf.hpp>

namespace sdf_tools {
struct TAGGED_OBJECT_COLLISION_CELL {
    float occupancy = 0.0f;
    uint32_t component = 0u;
    uint32_t object_id = 0u;
    uint32_t convex_segment = 0u;
    TAGGED_OBJECT_COLLISION_CELL() {}
    TAGGED_OBJECT_COLLISION_CELL(const float in_occupancy, const uint32_t in_object_id) : occupancy(in_occupancy), object_id(in_object_id) {}
};

class TaggedObjectCollisionMapGrid : public mock::VoxelGrid<TAGGED_OBJECT_COLLISION_CELL> {
  public:
    using mock::VoxelGrid<TAGGED_OBJECT_COLLISION_CELL>::VoxelGrid;

    std::pair<SignedDistanceField, std::pair<double, double>> ExtractSignedDistanceField(const float oob_value,
                                                                                        const std::vector<uint32_t>&, const bool,
                                                                                        const bool) const {
        const size_t total = data_.size();
        std::vector<double> to_filled(total), to_free(total);
        const double INF = std::numeric_limits<double>::infinity();
        for (size_t c = 0; c < total; ++c) {
            const bool filled = data_[c].occupancy > 0.5f;
            to_filled[c] = filled ? 0.0 : INF;
            to_free[c] = filled ? INF : 0.0;
        }
        Edt(to_filled);
        Edt(to_free);
        SignedDistanceField sdf(origin_, frame_, resolution_, ((double)n_[0] - 0.5) * resolution_, ((double)n_[1] - 0.5) * resolution_,
                                ((double)n_[2] - 0.5) * resolution_, oob_value);
        size_t c = 0;
        for (int64_t x = 0; x < n_[0]; ++x)
            for (int64_t y = 0; y < n_[1]; ++y)
                for (int64_t z = 0; z < n_[2]; ++z, ++c)
                    sdf.SetCell(x, y, z, (float)(std::sqrt(to_filled[c]) * resolution_ - std::sqrt(to_free[c]) * resolution_));
        return {sdf, {0.0, 0.0}};
    }

  private:
    void Edt(std::vector<double>& D) const {
        const int64_t stride[3] = {n_[1] * n_[2], n_[2], 1};
        for (int axis = 2; axis >= 0; --axis) {
            const int64_t n = n_[axis];
            std::vector<double> f((size_t)n);
            for (size_t base = 0; base < D.size(); ++base) {
                if ((int64_t)(base / (size_t)stride[axis]) % n != 0) continue; /* first cell of a line along `axis` */
                for (int64_t q = 0; q < n; ++q) f[(size_t)q] = D[base + (size_t)(q * stride[axis])];
                for (int64_t q = 0; q < n; ++q) {
                    double best = std::numeric_limits<double>::infinity();
                    for (int64_t p = 0; p < n; ++p) {
                        const double v = f[(size_t)p] + (double)((q - p) * (q - p));
                        if (v < best) best = v;
                    }
                    D[base + (size_t)(q * stride[axis])] = best;
                }
            }
        }
    }
};
}  // namespace sdf_tools
#endif
