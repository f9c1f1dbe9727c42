/*
 * fks_multi.cpp — one process driving several MI355X devices through the C-ABI
 * (fks_create_multi and friends, include/fks_capi.h).
 *
 * Replaces the reference's `#pragma omp parallel for` over particles (SPCS:795)
 * at device granularity: particle i of a call belongs to the device whose contiguous,
 * balanced range holds it (fks_shard_bounds), and that device
 * simulates it with first_particle_id = the range start, so the counter RNG stream of
 * every particle is the one a single device would use and the results are
 * bit-identical for any device count.  All devices share one call
 * index per logical call.  Each device gets its inputs by its own H2D copy, runs on
 * its own stream, and copies its outcomes straight into the caller's buffers at its
 * offset — the gather of per-particle outcomes is per-device D2H into host memory,
 * which is where the planner consumes them; the statistics and call counters are
 * summed over the devices (kernel_ms is the slowest device's).  Device-resident
 * multi-process use (one rank per GPU, RCCL gather) is bench.py / sharding.py.
 *
 * Host side of a call: one std::thread per active device runs that device's whole pipeline
 * (copy of its shard into its own pinned staging buffer, H2D, kernel, D2H into pinned memory,
 * copy out to the caller), so no device's copies or host memcpys wait for another device's
 * (a pageable hipMemcpyAsync blocks its caller until the copy is done, which serialised the
 * devices' copies in device order before ABI 9).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "fks_capi.h"

struct fks_multi_context {
    struct Device {
        int32_t device = 0;
        fks_context* ctx = nullptr;
        hipStream_t stream = nullptr;
        double* d_starts = nullptr;
        double* d_targets = nullptr;
        double* d_out = nullptr;
        uint8_t* d_coll = nullptr;
        uint32_t* d_micro = nullptr;
        uint32_t* d_res = nullptr;
        uint32_t* d_err = nullptr;
        size_t cap = 0, cap_targets = 0;
        /* pinned host staging of the shard: inputs (starts, targets), outputs (positions,
         * then collided bytes, microsteps, resolver iterations, error bits) */
        unsigned char* h_in = nullptr;
        unsigned char* h_out = nullptr;
        size_t cap_h_in = 0, cap_h_out = 0;
        fks_status status = FKS_OK; /* the device thread's outcome */
        std::string error;
        fks_call_counters counters{};
    };
    std::vector<Device> devices;
    std::string last_error;
    uint64_t call_index = 0;
    int32_t width = 0;
    int32_t active = 0; /* devices the batches are sharded over (0 = all) */
    fks_call_counters last{};
};

namespace {

fks_status mfail(fks_multi_context* m, fks_status st, const std::string& msg) {
    if (m) m->last_error = msg;
    return st;
}
fks_status mctx(fks_multi_context* m, fks_status st, const fks_context* ctx, const char* where) {
    return mfail(m, st, std::string(where) + ": " + fks_status_string(st) + " (" + fks_get_last_error(ctx) + ")");
}

template <typename T>
hipError_t grow(T** p, size_t count) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    return hipMalloc((void**)p, (count > 0 ? count : 1) * sizeof(T));
}
hipError_t grow_pinned(unsigned char** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *p) return hipSuccess;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const hipError_t e = hipHostMalloc((void**)p, bytes > 0 ? bytes : 1, hipHostMallocDefault);
    if (e == hipSuccess) *cap = bytes;
    return e;
}

void free_device(fks_multi_context::Device& d) {
    (void)hipSetDevice(d.device);
    void* ptrs[] = {d.d_starts, d.d_targets, d.d_out, d.d_coll, d.d_micro, d.d_res, d.d_err};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (d.h_in) (void)hipHostFree(d.h_in);
    if (d.h_out) (void)hipHostFree(d.h_out);
    if (d.stream) (void)hipStreamDestroy(d.stream);
    if (d.ctx) fks_destroy(d.ctx);
    d = fks_multi_context::Device();
}

int32_t active_count(const fks_multi_context* m) {
    const int32_t n = (int32_t)m->devices.size();
    return (m->active > 0 && m->active < n) ? m->active : n;
}

/* run f(device index) on one host thread per device (inline when there is one) */
template <typename F>
void on_device_threads(int32_t ndev, F f) {
    if (ndev == 1) {
        f(0);
        return;
    }
    std::vector<std::thread> threads;
    threads.reserve((size_t)ndev);
    for (int32_t g = 0; g < ndev; ++g) threads.emplace_back(f, g);
    for (auto& t : threads) t.join();
}

#define DHIP(d, expr)                                                                              \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            (d).status = FKS_ERR_HIP;                                                              \
            (d).error = std::string(#expr) + ": " + hipGetErrorString(_e);                         \
            return;                                                                                \
        }                                                                                          \
    } while (0)
#define DCTX(d, st, what)                                                                          \
    do {                                                                                           \
        const fks_status _s = (st);                                                                \
        if (_s != FKS_OK) {                                                                        \
            (d).status = _s;                                                                       \
            (d).error = std::string(what) + ": " + fks_status_string(_s) + " (" + fks_get_last_error((d).ctx) + ")"; \
            return;                                                                                \
        }                                                                                          \
    } while (0)

/* the first failing device's error, in device order */
fks_status collect_status(fks_multi_context* m, int32_t ndev) {
    for (int32_t g = 0; g < ndev; ++g) {
        const auto& d = m->devices[(size_t)g];
        if (d.status != FKS_OK) return mfail(m, d.status, "device " + std::to_string(d.device) + ": " + d.error);
    }
    return FKS_OK;
}

}  // namespace

extern "C" {

fks_status fks_shard_bounds(uint64_t n, int32_t ndev, int32_t shard, uint64_t* begin, uint64_t* end) {
    if (ndev < 1 || shard < 0 || shard >= ndev || !begin || !end) return FKS_ERR_INVALID_ARGUMENT;
    /* balanced contiguous ranges, the first n % ndev shards one particle longer
     * (fast_kinematic_simulator_amd/sharding.py shard_bounds is the same rule) */
    const uint64_t base = n / (uint64_t)ndev, extra = n % (uint64_t)ndev, g = (uint64_t)shard;
    *begin = g * base + (g < extra ? g : extra);
    *end = *begin + base + (g < extra ? 1u : 0u);
    return FKS_OK;
}

fks_status fks_create_multi(const fks_environment* env, const fks_solver_params* params, double simulation_controller_frequency,
                            uint64_t prng_seed, int32_t debug_level, const int32_t* devices, int32_t ndev,
                            fks_multi_context** out) {
    if (!out) return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (!env || !params || !devices || ndev < 1 || ndev > 64) return FKS_ERR_INVALID_ARGUMENT;
    fks_multi_context* m = new (std::nothrow) fks_multi_context();
    if (!m) return FKS_ERR_OUT_OF_MEMORY;
    for (int32_t g = 0; g < ndev; ++g) {
        fks_multi_context::Device d;
        d.device = devices[g];
        fks_status st = fks_create(env, params, simulation_controller_frequency, prng_seed, debug_level, d.device, &d.ctx);
        if (st == FKS_OK && hipSetDevice(d.device) != hipSuccess) st = FKS_ERR_HIP;
        if (st == FKS_OK && hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking) != hipSuccess) st = FKS_ERR_HIP;
        m->devices.push_back(d);
        if (st != FKS_OK) {
            fks_destroy_multi(m);
            return st;
        }
    }
    *out = m;
    return FKS_OK;
}

void fks_destroy_multi(fks_multi_context* m) {
    if (!m) return;
    for (auto& d : m->devices) free_device(d);
    delete m;
}

const char* fks_multi_get_last_error(const fks_multi_context* m) { return m ? m->last_error.c_str() : "null context"; }

int32_t fks_multi_num_devices(const fks_multi_context* m) { return m ? (int32_t)m->devices.size() : 0; }

fks_context* fks_multi_device_context(fks_multi_context* m, int32_t shard) {
    if (!m || shard < 0 || shard >= (int32_t)m->devices.size()) return nullptr;
    return m->devices[(size_t)shard].ctx;
}

fks_status fks_multi_set_robot(fks_multi_context* m, const fks_robot_desc* robot) {
    if (!m) return FKS_ERR_INVALID_ARGUMENT;
    for (auto& d : m->devices) {
        const fks_status st = fks_set_robot(d.ctx, robot);
        if (st != FKS_OK) return mctx(m, st, d.ctx, "fks_set_robot");
    }
    m->width = fks_config_width(m->devices[0].ctx);
    return FKS_OK;
}

fks_status fks_multi_forward_simulate(fks_multi_context* m, const double* starts, uint64_t n, const double* targets,
                                      uint64_t num_targets, int32_t allow_contacts, double* out_positions, uint8_t* out_collided,
                                      uint32_t* out_microsteps, uint32_t* out_resolver_iterations, uint32_t* out_error_flags) {
    if (!m) return FKS_ERR_INVALID_ARGUMENT;
    if (m->width <= 0) return mfail(m, FKS_ERR_NO_ROBOT, "fks_multi_set_robot has not been called");
    if (n > 0 && (!starts || !targets || !out_positions)) return mfail(m, FKS_ERR_INVALID_ARGUMENT, "null host buffer");
    if (n > 0 && num_targets != 1 && num_targets != n) return mfail(m, FKS_ERR_INVALID_ARGUMENT, "targets must be 1 or n (SPCS:792)");
    const auto t0 = std::chrono::steady_clock::now();
    const size_t W = (size_t)m->width;
    const int32_t ndev = active_count(m);
    const uint64_t call = m->call_index++;
    /* one host thread per device: stage in, launch, stage out (the devices run concurrently) */
    on_device_threads(ndev, [&](int32_t g) {
        auto& d = m->devices[(size_t)g];
        d.status = FKS_OK;
        d.error.clear();
        std::memset(&d.counters, 0, sizeof(d.counters));
        uint64_t lo = 0, hi = 0;
        fks_shard_bounds(n, ndev, g, &lo, &hi);
        const uint64_t k = hi - lo;
        DCTX(d, fks_set_call_index(d.ctx, call), "fks_set_call_index");
        DHIP(d, hipSetDevice(d.device));
        if (k > d.cap) {
            DHIP(d, grow(&d.d_starts, k * W));
            DHIP(d, grow(&d.d_out, k * W));
            DHIP(d, grow(&d.d_coll, k));
            DHIP(d, grow(&d.d_micro, k));
            DHIP(d, grow(&d.d_res, k));
            DHIP(d, grow(&d.d_err, k));
            d.cap = k;
        }
        const uint64_t nt = (num_targets == n) ? k : 1;
        if (nt > d.cap_targets) {
            DHIP(d, grow(&d.d_targets, nt * W));
            d.cap_targets = nt;
        }
        if (k == 0) {
            DCTX(d, fks_get_last_call_counters(d.ctx, &d.counters), "fks_get_last_call_counters"); /* settles */
            std::memset(&d.counters, 0, sizeof(d.counters));
            return;
        }
        const size_t in_bytes = (k + nt) * W * sizeof(double);
        const size_t out_bytes = k * W * sizeof(double) + k * (1 + 3 * sizeof(uint32_t));
        DHIP(d, grow_pinned(&d.h_in, &d.cap_h_in, in_bytes));
        DHIP(d, grow_pinned(&d.h_out, &d.cap_h_out, out_bytes));
        double* h_starts = reinterpret_cast<double*>(d.h_in);
        double* h_targets = h_starts + k * W;
        std::memcpy(h_starts, starts + lo * W, k * W * sizeof(double));
        std::memcpy(h_targets, targets + (num_targets == n ? lo * W : 0), nt * W * sizeof(double));
        DHIP(d, hipMemcpyAsync(d.d_starts, h_starts, k * W * sizeof(double), hipMemcpyHostToDevice, d.stream));
        DHIP(d, hipMemcpyAsync(d.d_targets, h_targets, nt * W * sizeof(double), hipMemcpyHostToDevice, d.stream));
        DCTX(d, fks_forward_simulate_device(d.ctx, d.d_starts, k, d.d_targets, nt, lo, allow_contacts, d.d_out, d.d_coll, d.d_micro,
                                            d.d_res, d.d_err, d.stream, 0),
             "fks_forward_simulate_device");
        double* h_q = reinterpret_cast<double*>(d.h_out);
        uint32_t* h_micro = reinterpret_cast<uint32_t*>(h_q + k * W);
        uint32_t* h_res = h_micro + k;
        uint32_t* h_err = h_res + k;
        uint8_t* h_coll = reinterpret_cast<uint8_t*>(h_err + k);
        DHIP(d, hipMemcpyAsync(h_q, d.d_out, k * W * sizeof(double), hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipMemcpyAsync(h_micro, d.d_micro, k * sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipMemcpyAsync(h_res, d.d_res, k * sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipMemcpyAsync(h_err, d.d_err, k * sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipMemcpyAsync(h_coll, d.d_coll, k, hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipStreamSynchronize(d.stream));
        std::memcpy(out_positions + lo * W, h_q, k * W * sizeof(double));
        if (out_collided) std::memcpy(out_collided + lo, h_coll, k);
        if (out_microsteps) std::memcpy(out_microsteps + lo, h_micro, k * sizeof(uint32_t));
        if (out_resolver_iterations) std::memcpy(out_resolver_iterations + lo, h_res, k * sizeof(uint32_t));
        if (out_error_flags) std::memcpy(out_error_flags + lo, h_err, k * sizeof(uint32_t));
        DCTX(d, fks_get_last_call_counters(d.ctx, &d.counters), "fks_get_last_call_counters"); /* settles the launch */
    });
    const fks_status st = collect_status(m, ndev);
    if (st != FKS_OK) return st;
    std::memset(&m->last, 0, sizeof(m->last));
    for (int32_t g = 0; g < ndev; ++g) {
        const fks_call_counters& c = m->devices[(size_t)g].counters;
        m->last.particles += c.particles;
        m->last.controller_steps += c.controller_steps;
        m->last.microsteps += c.microsteps;
        m->last.resolver_iterations += c.resolver_iterations;
        m->last.sdf_bytes += c.sdf_bytes;
        m->last.error_particles += c.error_particles;
        m->last.least_squares_rows += c.least_squares_rows;
        m->last.self_collision_checks += c.self_collision_checks;
        m->last.self_corrected_points += c.self_corrected_points;
        m->last.kernel_ms = std::max(m->last.kernel_ms, c.kernel_ms);
    }
    m->last.calls = 1;
    m->last.call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return FKS_OK;
}

fks_status fks_multi_set_active_devices(fks_multi_context* m, int32_t count) {
    if (!m || count < 0 || count > (int32_t)m->devices.size()) return FKS_ERR_INVALID_ARGUMENT;
    m->active = count;
    return FKS_OK;
}

int32_t fks_multi_active_devices(const fks_multi_context* m) { return m ? active_count(m) : 0; }

fks_status fks_multi_get_statistics(const fks_multi_context* m, fks_statistics* out) {
    if (!m || !out) return FKS_ERR_INVALID_ARGUMENT;
    std::memset(out, 0, sizeof(*out));
    for (const auto& d : m->devices) {
        fks_statistics s;
        const fks_status st = fks_get_statistics(d.ctx, &s);
        if (st != FKS_OK) return st;
        out->successful_resolves += s.successful_resolves;
        out->unsuccessful_resolves += s.unsuccessful_resolves;
        out->free_resolves += s.free_resolves;
        out->collision_resolves += s.collision_resolves;
        out->fallback_resolves += s.fallback_resolves;
        out->unsuccessful_env_collision_resolves += s.unsuccessful_env_collision_resolves;
        out->unsuccessful_self_collision_resolves += s.unsuccessful_self_collision_resolves;
        out->recovered_unsuccessful_resolves += s.recovered_unsuccessful_resolves;
    }
    return FKS_OK;
}

fks_status fks_multi_reset_statistics(fks_multi_context* m) {
    if (!m) return FKS_ERR_INVALID_ARGUMENT;
    for (auto& d : m->devices) {
        const fks_status st = fks_reset_statistics(d.ctx);
        if (st != FKS_OK) return mctx(m, st, d.ctx, "fks_reset_statistics");
    }
    return FKS_OK;
}

fks_status fks_multi_get_last_call_counters(const fks_multi_context* m, fks_call_counters* out) {
    if (!m || !out) return FKS_ERR_INVALID_ARGUMENT;
    *out = m->last;
    return FKS_OK;
}

fks_status fks_multi_set_call_index(fks_multi_context* m, uint64_t call_index) {
    if (!m) return FKS_ERR_INVALID_ARGUMENT;
    m->call_index = call_index;
    return FKS_OK;
}

fks_status fks_multi_check_config_collision(fks_multi_context* m, const double* configs, uint64_t n, double inflation_ratio,
                                            uint8_t* out_collided, uint32_t* out_error_flags) {
    if (!m) return FKS_ERR_INVALID_ARGUMENT;
    if (m->width <= 0) return mfail(m, FKS_ERR_NO_ROBOT, "fks_multi_set_robot has not been called");
    if (n > 0 && (!configs || !out_collided)) return mfail(m, FKS_ERR_INVALID_ARGUMENT, "null host buffer");
    const size_t W = (size_t)m->width;
    const int32_t ndev = active_count(m);
    /* the configurations and flags reuse the simulation buffers (starts, collided, errors) */
    on_device_threads(ndev, [&](int32_t g) {
        auto& d = m->devices[(size_t)g];
        d.status = FKS_OK;
        d.error.clear();
        uint64_t lo = 0, hi = 0;
        fks_shard_bounds(n, ndev, g, &lo, &hi);
        const uint64_t k = hi - lo;
        DHIP(d, hipSetDevice(d.device));
        if (k > d.cap) {
            DHIP(d, grow(&d.d_starts, k * W));
            DHIP(d, grow(&d.d_out, k * W));
            DHIP(d, grow(&d.d_coll, k));
            DHIP(d, grow(&d.d_micro, k));
            DHIP(d, grow(&d.d_res, k));
            DHIP(d, grow(&d.d_err, k));
            d.cap = k;
        }
        if (k == 0) return;
        DHIP(d, grow_pinned(&d.h_in, &d.cap_h_in, k * W * sizeof(double)));
        DHIP(d, grow_pinned(&d.h_out, &d.cap_h_out, k * (1 + sizeof(uint32_t))));
        std::memcpy(d.h_in, configs + lo * W, k * W * sizeof(double));
        DHIP(d, hipMemcpyAsync(d.d_starts, d.h_in, k * W * sizeof(double), hipMemcpyHostToDevice, d.stream));
        DCTX(d, fks_check_config_collision_device(d.ctx, d.d_starts, k, inflation_ratio, d.d_coll, d.d_err, d.stream, 0),
             "fks_check_config_collision_device");
        uint32_t* h_err = reinterpret_cast<uint32_t*>(d.h_out);
        uint8_t* h_coll = reinterpret_cast<uint8_t*>(h_err + k);
        DHIP(d, hipMemcpyAsync(h_coll, d.d_coll, k, hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipMemcpyAsync(h_err, d.d_err, k * sizeof(uint32_t), hipMemcpyDeviceToHost, d.stream));
        DHIP(d, hipStreamSynchronize(d.stream));
        std::memcpy(out_collided + lo, h_coll, k);
        if (out_error_flags) std::memcpy(out_error_flags + lo, h_err, k * sizeof(uint32_t));
        fks_call_counters c;
        DCTX(d, fks_get_last_check_counters(d.ctx, &c), "fks_get_last_check_counters"); /* settles the device's check */
    });
    return collect_status(m, ndev);
}

int32_t fks_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
