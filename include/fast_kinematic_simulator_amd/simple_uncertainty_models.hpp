/*
 * simple_uncertainty_models.hpp — the reference's sensor and actuator uncertainty models
 * (UNC:18-281) with their interface unchanged, for planner and execution code that includes
 * <fast_kinematic_simulator/simple_uncertainty_models.hpp>:
 *
 *   TruncatedNormalUncertainSensor            UNC:20-46
 *   TruncatedNormalUncertainVelocityActuator  UNC:48-121
 *   JointUncertaintySampleModel, DownsampleBin, GetMatchingBin, LoadModel   UNC:123-222
 *   SampledUncertainVelocityActuator          UNC:224-281
 *
 * The actuator arithmetic is fks_control.h's (the simulation kernels' own expression trees);
 * the truncated-normal draws come from fks::TruncatedNormalDistribution (truncated_normal.hpp,
 * a restatement of arc_helpers' sampler: parity unpinned).  ToSampledActuator turns a
 * LoadModel result into the per-dof bins the GPU simulation samples from (fks_sampled_actuator,
 * fks::RobotDescription::SetSampledActuator).  Differences from the reference, by design:
 *   - a command outside every bin throws std::out_of_range (the reference prints and asserts,
 *     UNC:150-153);
 *   - LoadModel has an overload with a seed for reproducible bins (the reference seeds
 *     DownsampleBin from std::random_device, UNC:130, which the seedless overloads keep).
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_SIMPLE_UNCERTAINTY_MODELS_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_SIMPLE_UNCERTAINTY_MODELS_HPP

#include <cassert>
#include <cmath>
#include <cstdint>
#include <fstream>
#include <iostream>
#include <limits>
#include <memory>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp"
#include "fast_kinematic_simulator_amd/truncated_normal.hpp"
#include "fks_capi.h"
#include "fks_control.h"

namespace simple_uncertainty_models {

/* UNC:20-46 */
class TruncatedNormalUncertainSensor {
  protected:
    bool initialized_;
    mutable fks::TruncatedNormalDistribution noise_distribution_;

  public:
    TruncatedNormalUncertainSensor(const double noise_lower_bound, const double noise_upper_bound)
        : initialized_(true),
          noise_distribution_(0.0, std::max((std::abs(noise_lower_bound) * 0.5), (std::abs(noise_upper_bound) * 0.5)), noise_lower_bound,
                              noise_upper_bound) {}
    TruncatedNormalUncertainSensor() : initialized_(false), noise_distribution_(0.0, 1.0, 0.0, 0.0) {}

    inline bool IsInitialized() const { return initialized_; }

    template <typename RNG>
    inline double GetSensorValue(const double process_value, RNG& rng) const {
        assert(!std::isnan(process_value) && !std::isinf(process_value));
        const double noise = noise_distribution_(rng);
        return process_value + noise;
    }
};

/* UNC:48-121 */
class TruncatedNormalUncertainVelocityActuator {
  protected:
    bool initialized_;
    mutable fks::TruncatedNormalDistribution noise_distribution_;
    double velocity_limit_;
    double acceleration_limit_;
    double proportional_noise_bound_;
    double minimum_noise_bound_;

  public:
    TruncatedNormalUncertainVelocityActuator(const double velocity_limit, const double acceleration_limit,
                                             const double proportional_noise_bound, const double minimum_noise_bound,
                                             const double percent_variance)
        : initialized_(true),
          noise_distribution_(0.0, std::min(std::max(std::abs(percent_variance), 0.0), 1.0), -1.0, 1.0),
          velocity_limit_(std::abs(velocity_limit)),
          acceleration_limit_(std::abs(acceleration_limit)),
          proportional_noise_bound_(std::abs(proportional_noise_bound)),
          minimum_noise_bound_(std::abs(minimum_noise_bound)) {}
    TruncatedNormalUncertainVelocityActuator()
        : initialized_(false), noise_distribution_(0.0, 1.0, 0.0, 0.0), velocity_limit_(0.0), acceleration_limit_(0.0),
          proportional_noise_bound_(0.0), minimum_noise_bound_(0.0) {}

    inline bool IsInitialized() const { return initialized_; }

    /* UNC:70-75 */
    inline double GetControlValue(const double control_input) const {
        assert(!std::isnan(control_input) && !std::isinf(control_input));
        return fks_control::actuator_clamp(control_input, velocity_limit_);
    }
    /* UNC:77-90: noise proportional to the command with a floor, as the simulation kernels */
    template <typename RNG>
    inline double GetControlValue(const double control_input, RNG& rng) const {
        const double real_control_input = GetControlValue(control_input);
        const double real_noise_bound =
            fks_control::actuator_noise_bound(real_control_input, proportional_noise_bound_, minimum_noise_bound_, velocity_limit_);
        const double real_noise = noise_distribution_(rng) * real_noise_bound;
        return real_control_input + real_noise;
    }
    inline double GetMaxVelocity() const { return velocity_limit_; }
    inline double GetMaxAcceleration() const { return acceleration_limit_; }
    /* UNC:102-115 */
    inline double GetMaxVelocityNoise(const double velocity) const {
        const double real_control_input = GetControlValue(velocity);
        if (real_control_input >= 0.0)
            return std::max((proportional_noise_bound_ * real_control_input), (minimum_noise_bound_ * velocity_limit_));
        return std::min((proportional_noise_bound_ * real_control_input), (minimum_noise_bound_ * -velocity_limit_));
    }
    inline double GetMaxVelocityNoise() const { return GetMaxVelocityNoise(GetMaxVelocity()); }
};

/* UNC:123: per bin, the (lower, upper) commanded-velocity bounds and its velocity errors */
typedef std::vector<std::pair<std::pair<double, double>, std::vector<double>>> JointUncertaintySampleModel;

/* UNC:125-138: `downsampled_size` items drawn with replacement */
template <typename RNG>
inline std::vector<double> DownsampleBin(const std::vector<double>& raw_bin, const uint32_t downsampled_size, RNG& rng) {
    if (raw_bin.empty()) throw std::invalid_argument("DownsampleBin: an empty bin");
    std::vector<double> downsampled_bin(downsampled_size, 0.0);
    std::uniform_int_distribution<size_t> pick_dist(0, raw_bin.size() - 1);
    for (uint32_t idx = 0; idx < downsampled_size; idx++) downsampled_bin[idx] = raw_bin[pick_dist(rng)];
    return downsampled_bin;
}
inline std::vector<double> DownsampleBin(const std::vector<double>& raw_bin, const uint32_t downsampled_size) {
    std::random_device rd; /* as the reference (UNC:130) */
    std::mt19937 rng(rd());
    return DownsampleBin(raw_bin, downsampled_size, rng);
}

/* UNC:140-154: the first bin whose closed interval holds the command */
inline size_t GetMatchingBin(const JointUncertaintySampleModel& bins, const double commanded_velocity) {
    for (size_t idx = 0; idx < bins.size(); idx++) {
        const std::pair<double, double>& bin_bounds = bins[idx].first;
        if (commanded_velocity >= bin_bounds.first && commanded_velocity <= bin_bounds.second) return idx;
    }
    throw std::out_of_range("GetMatchingBin: value " + std::to_string(commanded_velocity) + " is not in any bin");
}

namespace unc_detail {
/* the model file's rows, each `commanded velocity, velocity error` (blank lines skipped) */
inline std::vector<std::pair<double, double>> read_error_rows(const std::string& path) {
    std::ifstream file(path);
    if (!file) throw std::runtime_error("LoadModel: cannot read " + path);
    std::vector<std::pair<double, double>> rows;
    for (std::string text; std::getline(file, text);) {
        if (text.empty()) continue;
        std::vector<double> cells;
        std::stringstream fields(text);
        for (std::string field; std::getline(fields, field, ',');) cells.push_back(std::stod(field));
        if (cells.size() != 2) throw std::runtime_error("LoadModel: rows are `commanded velocity, velocity error`");
        rows.emplace_back(cells[0], cells[1]);
    }
    return rows;
}
/* the upper edge of each of `count` bins over [-limit, limit]: the width accumulated from -limit
 * one bin at a time (the reference's edges, bit for bit), the last edge open (+inf) */
inline std::vector<double> bin_upper_edges(const double limit, const uint32_t count) {
    const double width = (limit * 2.0) / (double)count;
    std::vector<double> upper(count);
    double edge = -limit;
    for (uint32_t k = 0; k < count; k++) {
        edge = edge + width;
        upper[k] = (k + 1 >= count) ? std::numeric_limits<double>::infinity() : edge;
    }
    return upper;
}
}  // namespace unc_detail

/* UNC:156-222: the (commanded velocity, velocity error) rows of `model_file` sorted into
 * num_bins bins over [-actuator_limit, actuator_limit] (the outer two open to -inf / +inf),
 * each bin then downsampled to bin_elements entries with `rng` */
template <typename RNG>
inline std::shared_ptr<JointUncertaintySampleModel> LoadModel(const std::string& model_file, const double actuator_limit,
                                                              const uint32_t num_bins, const uint32_t bin_elements, RNG& rng) {
    const std::vector<std::pair<double, double>> rows = unc_detail::read_error_rows(model_file);
    const std::vector<double> upper = unc_detail::bin_upper_edges(actuator_limit, num_bins);
    auto model = std::make_shared<JointUncertaintySampleModel>();
    model->reserve(num_bins);
    for (uint32_t k = 0; k < num_bins; k++) {
        const double lower = (k == 0) ? -std::numeric_limits<double>::infinity() : upper[k - 1];
        model->emplace_back(std::make_pair(lower, upper[k]), std::vector<double>());
    }
    for (const std::pair<double, double>& row : rows) (*model)[GetMatchingBin(*model, row.first)].second.push_back(row.second);
    for (auto& bin : *model) bin.second = DownsampleBin(bin.second, bin_elements, rng);
    return model;
}
/* reproducible bins: the downsampling generator seeded with `seed` */
inline std::shared_ptr<JointUncertaintySampleModel> LoadModel(const std::string& model_file, const double actuator_limit,
                                                              const uint32_t num_bins, const uint32_t bin_elements, const uint64_t seed) {
    std::mt19937_64 rng(seed);
    return LoadModel(model_file, actuator_limit, num_bins, bin_elements, rng);
}
/* the reference's signature: DownsampleBin seeded from std::random_device */
inline std::shared_ptr<JointUncertaintySampleModel> LoadModel(const std::string& model_file, const double actuator_limit,
                                                              const uint32_t num_bins, const uint32_t bin_elements) {
    std::random_device rd;
    std::mt19937 rng(rd());
    return LoadModel(model_file, actuator_limit, num_bins, bin_elements, rng);
}

/* UNC:224-281 */
class SampledUncertainVelocityActuator {
    bool initialized_;
    double actuator_limit_;
    std::shared_ptr<JointUncertaintySampleModel> model_ptr_;

    /* UNC:230-246: the generator is taken by value, as the reference does, so the caller's is
     * not advanced */
    template <typename RNG>
    inline double GetNoiseValue(const double commanded_velocity, RNG rng) const {
        if (!model_ptr_) return 0.0;
        const std::vector<double>& best_match_bin = (*model_ptr_)[GetMatchingBin(*model_ptr_, commanded_velocity)].second;
        std::uniform_int_distribution<size_t> pick_dist(0, best_match_bin.size() - 1);
        return best_match_bin[pick_dist(rng)];
    }

  public:
    SampledUncertainVelocityActuator(const std::shared_ptr<JointUncertaintySampleModel> model_ptr, const double max_velocity)
        : initialized_(true), actuator_limit_(std::abs(max_velocity)), model_ptr_(model_ptr) {}
    SampledUncertainVelocityActuator(const double max_velocity) : initialized_(true), actuator_limit_(std::abs(max_velocity)) {}
    SampledUncertainVelocityActuator() : initialized_(true), actuator_limit_(0.0) {}

    inline bool IsInitialized() const { return initialized_; }
    /* UNC:262-269 */
    inline double GetControlValue(const double control_input) const {
        assert(!std::isnan(control_input) && !std::isinf(control_input));
        return fks_control::actuator_clamp(control_input, actuator_limit_);
    }
    /* UNC:271-279 */
    template <typename RNG>
    inline double GetControlValue(const double control_input, RNG& rng) const {
        const double real_control_input = GetControlValue(control_input);
        const double noise = GetNoiseValue(real_control_input, rng);
        return real_control_input + noise;
    }
    inline double GetMaxVelocity() const { return actuator_limit_; }
    const std::shared_ptr<JointUncertaintySampleModel>& Model() const { return model_ptr_; }
};

/* A LoadModel result as the flat bins the GPU simulation samples from (fks_sampled_actuator:
 * bounds then samples per bin; every bin must hold the same number of samples, as
 * DownsampleBin makes them).  `storage` owns the arrays the descriptor points to. */
struct SampledActuatorBins {
    std::vector<double> bounds;  /* num_bins x (lower, upper) */
    std::vector<double> samples; /* num_bins x bin_elements */
    fks_sampled_actuator View() const {
        fks_sampled_actuator a{};
        a.num_bins = (uint32_t)(bounds.size() / 2);
        a.bin_elements = a.num_bins ? (uint32_t)(samples.size() / a.num_bins) : 0u;
        a.bin_bounds = bounds.empty() ? nullptr : bounds.data();
        a.bin_samples = samples.empty() ? nullptr : samples.data();
        return a;
    }
};
inline std::shared_ptr<const SampledActuatorBins> ToSampledActuator(const JointUncertaintySampleModel& model) {
    auto out = std::make_shared<SampledActuatorBins>();
    const size_t elements = model.empty() ? 0 : model.front().second.size();
    for (const auto& bin : model) {
        if (bin.second.size() != elements || elements == 0)
            throw std::invalid_argument("ToSampledActuator: every bin needs the same, non-zero number of samples");
        out->bounds.push_back(bin.first.first);
        out->bounds.push_back(bin.first.second);
        out->samples.insert(out->samples.end(), bin.second.begin(), bin.second.end());
    }
    return out;
}

/* dof `dof` of `robot` samples its actuation noise from `model` on the GPU (the
 * SampledUncertainVelocityActuator of UNC:224-281 inside the simulation kernels) */
inline void SetSampledActuator(fks::RobotDescription& robot, const int32_t dof, const JointUncertaintySampleModel& model) {
    const std::shared_ptr<const SampledActuatorBins> bins = ToSampledActuator(model);
    robot.SetSampledActuator(dof, bins->View(), bins);
}

}  // namespace simple_uncertainty_models

#endif
