/* Mock of sdf_tools::SignedDistanceField as the reference reads it (test only;
 * tests/cpp/mock_workspace/README.md): GetImmutable (SEB.cpp:197), GetImmutable4d
 * (SPCS:941), grid geometry accessors, OOB value. */
#ifndef MOCK_SDF_TOOLS_SDF
#define MOCK_SDF_TOOLS_SDF
#include <cmath>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>
#include <Eigen/Geometry>

namespace sdf_tools {
namespace mock {
template <typename T>
class VoxelGrid {
  public:
    VoxelGrid() {}
    VoxelGrid(const Eigen::Isometry3d& origin, const std::string& frame, const double resolution, const double x_size,
              const double y_size, const double z_size, const T& oob_value)
        : origin_(origin), frame_(frame), resolution_(resolution), oob_(oob_value) {
        n_[0] = (int64_t)std::ceil(std::fabs(x_size) / resolution);
        n_[1] = (int64_t)std::ceil(std::fabs(y_size) / resolution);
        n_[2] = (int64_t)std::ceil(std::fabs(z_size) / resolution);
        data_.assign((size_t)(n_[0] * n_[1] * n_[2]), oob_value);
    }
    double GetResolution() const { return resolution_; }
    int64_t GetNumXCells() const { return n_[0]; }
    int64_t GetNumYCells() const { return n_[1]; }
    int64_t GetNumZCells() const { return n_[2]; }
    const std::string& GetFrame() const { return frame_; }
    T GetOOBValue() const { return oob_; }
    const Eigen::Isometry3d& GetOriginTransform() const { return origin_; }
    std::pair<const T&, bool> GetImmutable(const int64_t x, const int64_t y, const int64_t z) const {
        if (x < 0 || y < 0 || z < 0 || x >= n_[0] || y >= n_[1] || z >= n_[2]) return std::pair<const T&, bool>(oob_, false);
        return std::pair<const T&, bool>(data_[Linear(x, y, z)], true);
    }
    /* world location -> cell (the origin is a translation in these tests) */
    bool SetValue(const double x, const double y, const double z, const T& value) {
        const int64_t i = (int64_t)std::floor((x - origin_.matrix()(0, 3)) / resolution_);
        const int64_t j = (int64_t)std::floor((y - origin_.matrix()(1, 3)) / resolution_);
        const int64_t k = (int64_t)std::floor((z - origin_.matrix()(2, 3)) / resolution_);
        if (i < 0 || j < 0 || k < 0 || i >= n_[0] || j >= n_[1] || k >= n_[2]) return false;
        data_[Linear(i, j, k)] = value;
        return true;
    }

  protected:
    size_t Linear(int64_t x, int64_t y, int64_t z) const { return ((size_t)x * (size_t)n_[1] + (size_t)y) * (size_t)n_[2] + (size_t)z; }
    Eigen::Isometry3d origin_ = Eigen::Isometry3d::Identity();
    std::string frame_;
    double resolution_ = 1.0;
    T oob_{};
    int64_t n_[3] = {0, 0, 0};
    std::vector<T> data_;
};
}  // namespace mock

class SignedDistanceField : public mock::VoxelGrid<float> {
  public:
    using mock::VoxelGrid<float>::VoxelGrid;
    void SetCell(int64_t x, int64_t y, int64_t z, float v) { data_[Linear(x, y, z)] = v; }
};
}  // namespace sdf_tools
#endif
