/*
 * device_set.hpp — the MI355X devices one simulator object runs on.
 *
 * The reference runs every batch over the host's cores (`#pragma omp parallel for` over
 * particles, SPCS:795-802).  A DeviceSet runs it over a list of devices: one fks_context
 * for a single device, an fks_multi_context (fks_multi.cpp) for several.  A batch is split
 * into contiguous shards by global particle id over the first devices_for(n) devices — as
 * many as keep at least shard_threshold() particles each — each simulated with
 * first_particle_id = the shard's start and the call index the first device would have used,
 * so the counter RNG streams and therefore the results are bit-identical to one device
 * (DESIGN.md §6).  A launch lasts at least as long as its slowest particle's chain, so a shard
 * smaller than a few times one device's resident waves gains little from another device
 * (the strong-scaling projection in DESIGN.md §6 sets the default).  Batches that keep one
 * device and every single-particle call (mutable robots, traced runs, kinematics) run on
 * devices[0], whose call index is the simulator's.  Statistics are summed over the devices.
 *
 * Used by the planner-facing HipParticleContactSimulator (fast_kinematic_simulator.hpp) and
 * the plain C++ wrapper (hip_particle_contact_simulator.hpp).
 */
#ifndef FAST_KINEMATIC_SIMULATOR_AMD_DEVICE_SET_HPP
#define FAST_KINEMATIC_SIMULATOR_AMD_DEVICE_SET_HPP

#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "fks_capi.h"

namespace fks {

/* a failed C-ABI call: the status and the library's message */
class SimulatorError : public std::runtime_error {
  public:
    SimulatorError(fks_status status, const std::string& what) : std::runtime_error(what), status_(status) {}
    fks_status status() const { return status_; }

  private:
    fks_status status_;
};

/* The robot-shape-specialised kernel of the current robot on every device
 * (fks_get_specialization): whether all of them run it, and why not when a build failed (the
 * calls then run the generic kernel: same results, 10-20 % slower). */
struct SpecializationStatus {
    bool active = false;  /* every device runs the shaped kernel for the current robot */
    bool pending = false; /* some device builds it at its first throughput call */
    bool failed = false;  /* some device's build failed */
    std::string shape;    /* the shape key */
    std::string message;  /* the first failure's log, else empty */
    std::vector<fks_specialization_info> per_device;
};

/* every device visible to the process (HIP_VISIBLE_DEVICES applies), {0} when there is none
 * (fks_create then reports FKS_ERR_NO_DEVICE) */
inline std::vector<int32_t> AllVisibleDevices() {
    const int32_t n = fks_device_count();
    std::vector<int32_t> d;
    for (int32_t g = 0; g < (n > 0 ? n : 1); ++g) d.push_back(g);
    return d;
}

class DeviceSet {
  public:
    DeviceSet(const fks_environment& env, const fks_solver_params& params, double simulation_controller_frequency, uint64_t prng_seed,
              int32_t debug_level, const std::vector<int32_t>& devices)
        : devices_(devices) {
        if (devices_.empty()) throw std::invalid_argument("a simulator needs at least one device");
        if (devices_.size() == 1) {
            fks_context* ctx = nullptr;
            Check(fks_create(&env, &params, simulation_controller_frequency, prng_seed, debug_level, devices_[0], &ctx), nullptr,
                  "fks_create");
            own_.reset(ctx);
            ctx_ = ctx;
        } else {
            fks_multi_context* m = nullptr;
            const fks_status st = fks_create_multi(&env, &params, simulation_controller_frequency, prng_seed, debug_level,
                                                   devices_.data(), (int32_t)devices_.size(), &m);
            if (st != FKS_OK) throw SimulatorError(st, std::string("fks_create_multi: ") + fks_status_string(st));
            multi_.reset(m);
            ctx_ = fks_multi_device_context(m, 0);
        }
    }

    /* devices[0]'s context: single-particle calls and batches below shard_threshold() */
    fks_context* primary() const { return ctx_; }
    fks_multi_context* multi() const { return multi_.get(); }
    const std::vector<int32_t>& devices() const { return devices_; }

    template <typename F>
    void for_each(F f) const {
        if (!multi_) {
            f(ctx_);
            return;
        }
        for (int32_t g = 0; g < fks_multi_num_devices(multi_.get()); ++g) f(fks_multi_device_context(multi_.get(), g));
    }

    void set_robot(const fks_robot_desc& d) {
        if (multi_)
            MultiCheck(fks_multi_set_robot(multi_.get(), &d), "fks_set_robot");
        else
            Check(fks_set_robot(ctx_, &d), ctx_, "fks_set_robot");
    }

    /* the particles each device must get before a batch takes it on (0: automatic =
     * kShardWavesPerDevice x the resident waves of devices[0] for the current robot; 1 shards
     * every batch of at least as many particles as devices over all of them) */
    static constexpr uint64_t kShardWavesPerDevice = 3;
    void set_shard_threshold(uint64_t particles_per_device) { shard_threshold_ = particles_per_device; }
    uint64_t shard_threshold() const {
        if (shard_threshold_ > 0) return shard_threshold_;
        uint32_t waves = 0;
        uint64_t lds = 0;
        Check(fks_get_launch_geometry(ctx_, &waves, &lds), ctx_, "fks_get_launch_geometry");
        return waves > 0 ? kShardWavesPerDevice * waves : 1;
    }
    /* the devices a batch of n particles is sharded over: min(devices, n / shard_threshold()), >= 1 */
    int32_t devices_for(uint64_t n) const {
        if (!multi_ || n == 0) return 1;
        const uint64_t g = n / shard_threshold();
        const uint64_t nd = (uint64_t)fks_multi_num_devices(multi_.get());
        return (int32_t)(g < 1 ? 1 : (g > nd ? nd : g));
    }
    bool shards(uint64_t n) const { return devices_for(n) >= 2; }
    /* how many devices the last batch ran on (1: devices[0] alone) */
    int32_t last_devices() const { return last_devices_; }
    bool last_sharded() const { return last_devices_ >= 2; }

    /* ForwardSimulateRobots / ReverseSimulateRobots (SPCS:788-822) over host buffers; the
     * arguments are those of fks_forward_simulate */
    void simulate(bool reverse, const double* starts, uint64_t n, const double* targets, uint64_t num_targets, bool allow_contacts,
                  double* out_positions, uint8_t* out_collided, uint32_t* out_microsteps, uint32_t* out_resolver_iterations,
                  uint32_t* out_error_flags, const char* what) {
        last_devices_ = devices_for(n);
        if (last_devices_ >= 2) {
            /* every device uses the call index devices[0] would have used */
            const uint64_t call = fks_get_call_index(ctx_);
            MultiCheck(fks_multi_set_active_devices(multi_.get(), last_devices_), what);
            MultiCheck(fks_multi_set_call_index(multi_.get(), call), what);
            MultiCheck(fks_multi_forward_simulate(multi_.get(), starts, n, targets, num_targets, allow_contacts ? 1 : 0, out_positions,
                                                  out_collided, out_microsteps, out_resolver_iterations, out_error_flags),
                       what);
            Check(fks_set_call_index(ctx_, call + 1), ctx_, what);
            return;
        }
        auto fn = reverse ? fks_reverse_simulate : fks_forward_simulate;
        Check(fn(ctx_, starts, n, targets, num_targets, allow_contacts ? 1 : 0, out_positions, out_collided, out_microsteps,
                 out_resolver_iterations, out_error_flags),
              ctx_, what);
    }

    /* batched CheckConfigCollision (SPCS:1398-1416) */
    void check_configs(const double* configs, uint64_t n, double inflation_ratio, uint8_t* out_collided, uint32_t* out_error_flags,
                       const char* what) const {
        const int32_t g = devices_for(n);
        if (g >= 2) {
            MultiCheck(fks_multi_set_active_devices(multi_.get(), g), what);
            MultiCheck(fks_multi_check_config_collision(multi_.get(), configs, n, inflation_ratio, out_collided, out_error_flags), what);
        } else
            Check(fks_check_config_collision(ctx_, configs, n, inflation_ratio, out_collided, out_error_flags), ctx_, what);
    }

    /* GetStatistics (SPCS:488-500), summed over the devices */
    fks_statistics statistics() const {
        fks_statistics s{};
        if (multi_)
            MultiCheck(fks_multi_get_statistics(multi_.get(), &s), "GetStatistics");
        else
            Check(fks_get_statistics(ctx_, &s), ctx_, "GetStatistics");
        return s;
    }
    void reset_statistics() const {
        for_each([&](fks_context* c) { Check(fks_reset_statistics(c), c, "ResetStatistics"); });
    }
    /* ResetGenerators (SPCS:457-471): every device re-keyed by the seed, call index 0 */
    void reset_generators(uint64_t prng_seed) const {
        for_each([&](fks_context* c) { Check(fks_reset_generators(c, prng_seed), c, "ResetGenerators"); });
    }
    int32_t set_debug_level(int32_t level) const {
        int32_t previous = fks_get_debug_level(ctx_);
        for_each([&](fks_context* c) { (void)fks_set_debug_level(c, level); });
        return previous;
    }
    void set_individual_jacobians(bool on) const {
        for_each([&](fks_context* c) { Check(fks_set_individual_jacobians(c, on ? 1 : 0), c, "fks_set_individual_jacobians"); });
    }

    /* build the current robot's shape-specialised kernel on every device now (construction
     * time, where a planner expects setup cost) instead of inside the first large batch.  A
     * failed build is not an error: the calls keep the generic kernel and the returned status
     * says why.  mode: FKS_SPECIALIZE_OFF / _ON / _NO_PROOFS */
    SpecializationStatus prepare_kernels(int32_t mode = FKS_SPECIALIZE_ON) const {
        for_each([&](fks_context* c) {
            const fks_status st = fks_set_specialization(c, mode);
            if (st != FKS_OK && st != FKS_ERR_UNSUPPORTED) Check(st, c, "fks_set_specialization");
        });
        return specialization_status();
    }
    SpecializationStatus specialization_status() const {
        SpecializationStatus s;
        s.active = true;
        for_each([&](fks_context* c) {
            fks_specialization_info i{};
            Check(fks_get_specialization(c, &i), c, "fks_get_specialization");
            s.active = s.active && i.active != 0;
            s.pending = s.pending || i.pending != 0;
            if (i.failed && !s.failed) s.message = i.message;
            s.failed = s.failed || i.failed != 0;
            if (s.shape.empty()) s.shape = i.shape;
            s.per_device.push_back(i);
        });
        return s;
    }

    static void Check(fks_status st, const fks_context* ctx, const char* what) {
        if (st == FKS_OK) return;
        std::string msg = std::string(what) + ": " + fks_status_string(st);
        if (ctx) {
            const char* detail = fks_get_last_error(ctx);
            if (detail && detail[0]) msg += std::string(" (") + detail + ")";
        }
        throw SimulatorError(st, msg);
    }

  private:
    struct Destroy {
        void operator()(fks_context* c) const { fks_destroy(c); }
    };
    struct DestroyMulti {
        void operator()(fks_multi_context* m) const { fks_destroy_multi(m); }
    };
    void MultiCheck(fks_status st, const char* what) const {
        if (st == FKS_OK) return;
        throw SimulatorError(st, std::string(what) + ": " + fks_status_string(st) + " (" + fks_multi_get_last_error(multi_.get()) + ")");
    }

    std::vector<int32_t> devices_;
    std::unique_ptr<fks_context, Destroy> own_;
    std::unique_ptr<fks_multi_context, DestroyMulti> multi_;
    fks_context* ctx_ = nullptr;
    uint64_t shard_threshold_ = 0;
    int32_t last_devices_ = 1;
};

}  // namespace fks

#endif
