/*
 * Environment preprocessing on the GPU:
 *   obstacles -> collision grid -> signed distance field -> surface-normal CSR,
 * the same bytes as the host builder fks_env_build (fks_env_builder.cpp), which
 * restates src/fast_kinematic_simulator/simulator_environment_builder.cpp (SEB.cpp):
 *   DiscretizeObstacle / BuildEnvironment  SEB.cpp:21-160  -> env_bounds, env_occupancy
 *   ExtractSignedDistanceField             SEB.cpp:473     -> env_seed_lines + 2 x env_envelope + env_sdf
 *   BuildSurfaceNormalsGrid                SEB.cpp:258-468 -> env_surface_winner, env_count_blocks,
 *                                                             env_scan_blocks, env_fill
 *
 * Layout in HBM: cells are z-fastest (index (i * ny + j) * nz + k), the layout the
 * simulation kernels read.  The distance transform is the exact separable squared
 * EDT: a seed pass along z (distance to the nearest seed in the line), then the
 * lower envelope of parabolas (Felzenszwalb & Huttenlocher) along y and x.  Every
 * line is one thread; the y and x lines of neighbouring threads are neighbouring
 * columns, so every load and store of those passes is coalesced across the wave.
 * Squared distances are exact integers (uint32, 0xffffffff = no seed) and the
 * envelope's intersection tests are exact int64 cross-multiplications, so the
 * result is the true minimum, identical to the host's double-precision envelope.
 *
 * Roofline: every pass is a handful of streaming reads/writes per cell (HBM-bound,
 * ~45 B/cell in total at one read of the occupancy + 2 x (write + 2 x read-write of a
 * uint32 field) + scratch traffic of the envelope + the SDF write); there is no
 * matrix work.  "Last write wins" of the reference's surface map becomes an
 * atomicMax over the boundary samples' sequence numbers (obstacle-major, then xi,
 * yi, zi: the host loop order).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <cstring>
#include <limits>
#include <new>
#include <vector>

#include "fks_capi.h"
#include "fks_device.h"
#include "fks_env_internal.h"
#include "fks_portable_math.h"

namespace {

using fks_env::Grid;

constexpr uint32_t kNoSeed = 0xffffffffu;
constexpr int kScanThreads = 256;
constexpr int kScanItems = 16; /* cells per thread in the CSR scan */
constexpr uint64_t kCellsPerScanBlock = (uint64_t)kScanThreads * kScanItems;

struct ObstacleDev {
    fks_obstacle ob;
    int32_t nc[3];
    int32_t pad;
    uint64_t first; /* first global sample index */
    uint64_t count;
};

struct EnvArgs {
    Grid grid;
    const ObstacleDev* obs;
    int32_t num_obstacles;
    uint64_t samples;
    double resolution;
};

/* global sample index -> (obstacle, xi, yi, zi) in the host's loop order */
__device__ __forceinline__ int decode_sample(const EnvArgs& A, uint64_t s, int32_t id3[3]) {
    int lo = 0, hi = A.num_obstacles - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (A.obs[mid].first <= s) lo = mid;
        else hi = mid - 1;
    }
    const ObstacleDev& O = A.obs[lo];
    const uint64_t local = s - O.first;
    const uint64_t yz = (uint64_t)O.nc[1] * (uint64_t)O.nc[2];
    id3[0] = (int32_t)(local / yz);
    const uint64_t r = local - (uint64_t)id3[0] * yz;
    id3[1] = (int32_t)(r / (uint64_t)O.nc[2]);
    id3[2] = (int32_t)(r - (uint64_t)id3[1] * (uint64_t)O.nc[2]);
    return lo;
}

/* order-preserving map of doubles onto uint64 (for exact atomic min / max) */
__device__ __forceinline__ unsigned long long order_key(double x) {
    const unsigned long long b = (unsigned long long)fks_math::bits(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__global__ void env_bounds(const EnvArgs A, unsigned long long* keys /* order keys: min x, y, z then max x, y, z */) {
    unsigned long long mn[3] = {~0ull, ~0ull, ~0ull}, mx[3] = {0, 0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < A.samples; s += stride) {
        int32_t id3[3];
        const int o = decode_sample(A, s, id3);
        double w[3];
        fks_env::obstacle_sample_world(A.obs[o].ob, A.resolution, A.resolution * 0.5, id3[0], id3[1], id3[2], w);
        for (int a = 0; a < 3; ++a) {
            const unsigned long long k = order_key(w[a]);
            mn[a] = k < mn[a] ? k : mn[a];
            mx[a] = k > mx[a] ? k : mx[a];
        }
    }
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long om = __shfl_xor(mn[a], off, 64), oM = __shfl_xor(mx[a], off, 64);
            mn[a] = om < mn[a] ? om : mn[a];
            mx[a] = oM > mx[a] ? oM : mx[a];
        }
    }
    if ((threadIdx.x & 63) == 0) {
        for (int a = 0; a < 3; ++a) {
            atomicMin(keys + a, mn[a]);
            atomicMax(keys + 3 + a, mx[a]);
        }
    }
}

__global__ void env_occupancy(const EnvArgs A, uint8_t* __restrict__ occ) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < A.samples; s += stride) {
        int32_t id3[3];
        const int o = decode_sample(A, s, id3);
        double w[3];
        fks_env::obstacle_sample_world(A.obs[o].ob, A.resolution, A.resolution * 0.5, id3[0], id3[1], id3[2], w);
        int64_t idx[3];
        if (A.grid.index(w, idx)) occ[A.grid.linear(idx[0], idx[1], idx[2])] = 1;
    }
}

/* pass 1 (z lines): squared distance to the nearest filled cell (to_filled) and to
 * the nearest free cell (to_free) within the line */
__global__ void env_seed_lines(const EnvArgs A, const uint8_t* __restrict__ occ, uint32_t* __restrict__ to_filled,
                               uint32_t* __restrict__ to_free) {
    const int64_t nz = A.grid.n[2];
    const uint64_t lines = (uint64_t)A.grid.n[0] * (uint64_t)A.grid.n[1];
    const uint64_t line = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (line >= lines) return;
    const uint64_t base = line * (uint64_t)nz;
    int64_t last_filled = -1, last_free = -1;
    for (int64_t k = 0; k < nz; ++k) {
        const bool filled = occ[base + k] != 0;
        if (filled) last_filled = k;
        else last_free = k;
        to_filled[base + k] = last_filled < 0 ? kNoSeed : (uint32_t)((k - last_filled) * (k - last_filled));
        to_free[base + k] = last_free < 0 ? kNoSeed : (uint32_t)((k - last_free) * (k - last_free));
    }
    int64_t next_filled = -1, next_free = -1;
    for (int64_t k = nz - 1; k >= 0; --k) {
        const bool filled = occ[base + k] != 0;
        if (filled) next_filled = k;
        else next_free = k;
        if (next_filled >= 0) {
            const uint32_t d = (uint32_t)((next_filled - k) * (next_filled - k));
            if (d < to_filled[base + k]) to_filled[base + k] = d;
        }
        if (next_free >= 0) {
            const uint32_t d = (uint32_t)((next_free - k) * (next_free - k));
            if (d < to_free[base + k]) to_free[base + k] = d;
        }
    }
}

/* s(a, b) > s(c, d) style comparisons of the parabola intersections
 * s(a, b) = ((f_a + a^2) - (f_b + b^2)) / (2 (a - b)), a > b, exactly in int64 */
__device__ __forceinline__ int64_t isect_num(int64_t a, int64_t fa, int64_t b, int64_t fb) { return (fa + a * a) - (fb + b * b); }

/* one squared-EDT pass along lines of `len` cells spaced `stride` apart; line l
 * starts at (l / inner) * outer + (l % inner).  scratch: per line the envelope's
 * (position, value) pairs, stored position-major so a wave's accesses coalesce. */
__global__ void env_envelope(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t* __restrict__ scratch,
                             uint64_t lines, int64_t len, uint64_t stride, uint64_t inner, uint64_t outer) {
    const uint64_t l = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= lines) return;
    const uint64_t base = (l / inner) * outer + (l % inner);
    auto V = [&](int64_t k) -> uint64_t& { return scratch[(uint64_t)k * lines + l]; };
    int64_t k = -1;
    for (int64_t q = 0; q < len; ++q) {
        const uint32_t fq = in[base + (uint64_t)q * stride];
        if (fq == kNoSeed) continue;
        if (k >= 0) {
            /* pop while s(q, v_k) <= s(v_k, v_{k-1}) (z_0 = -inf never pops) */
            while (k > 0) {
                const uint64_t pk = V(k), pk1 = V(k - 1);
                const int64_t vk = (int64_t)(pk & 0xffff), fk = (int64_t)(pk >> 16);
                const int64_t vk1 = (int64_t)(pk1 & 0xffff), fk1 = (int64_t)(pk1 >> 16);
                const int64_t n1 = isect_num(q, (int64_t)fq, vk, fk), d1 = 2 * (q - vk);
                const int64_t n2 = isect_num(vk, fk, vk1, fk1), d2 = 2 * (vk - vk1);
                if (n1 * d2 <= n2 * d1) k--;
                else break;
            }
        }
        k++;
        V(k) = ((uint64_t)fq << 16) | (uint64_t)q;
    }
    if (k < 0) {
        for (int64_t q = 0; q < len; ++q) out[base + (uint64_t)q * stride] = kNoSeed;
        return;
    }
    int64_t j = 0;
    uint64_t pj = V(0);
    for (int64_t q = 0; q < len; ++q) {
        /* advance while z_{j+1} = s(v_{j+1}, v_j) < q */
        while (j < k) {
            const uint64_t pn = V(j + 1);
            const int64_t vn = (int64_t)(pn & 0xffff), fn = (int64_t)(pn >> 16);
            const int64_t vj = (int64_t)(pj & 0xffff), fj = (int64_t)(pj >> 16);
            if (isect_num(vn, fn, vj, fj) < q * (2 * (vn - vj))) {
                j++;
                pj = pn;
            } else {
                break;
            }
        }
        const int64_t vj = (int64_t)(pj & 0xffff), fj = (int64_t)(pj >> 16);
        out[base + (uint64_t)q * stride] = (uint32_t)((q - vj) * (q - vj) + fj);
    }
}

/* + distance to the nearest filled cell for free cells, - distance to the nearest
 * free cell for filled cells (sdf_tools convention; fks_env_builder.cpp) */
__global__ void env_sdf(const EnvArgs A, const uint32_t* __restrict__ to_filled, const uint32_t* __restrict__ to_free,
                        float* __restrict__ sdf) {
    const uint64_t total = A.grid.cells();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const double INF = __builtin_inf();
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total; c += stride) {
        const uint32_t a = to_filled[c], b = to_free[c];
        const double filled_distance = (a == kNoSeed ? INF : fks_math::dsqrt((double)a)) * A.resolution;
        const double free_distance = (b == kNoSeed ? INF : fks_math::dsqrt((double)b)) * A.resolution;
        sdf[c] = (float)(filled_distance - free_distance);
    }
}

__device__ __forceinline__ bool sample_is_boundary(const ObstacleDev& O, const int32_t id3[3]) {
    bool boundary = false;
    for (int a = 0; a < 3; ++a) boundary = boundary || id3[a] == 0 || id3[a] == O.nc[a] - 1;
    return boundary;
}

/* second pass of BuildSurfaceNormalsGrid (SEB.cpp:279-466) through
 * UpdateSurfaceNormalGridCell (SEB.cpp:162-187): the last boundary sample that lands
 * in a cell with d > -1.5 res owns the cell's list */
__global__ void env_surface_winner(const EnvArgs A, const float* __restrict__ sdf, uint32_t* __restrict__ winner) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < A.samples; s += stride) {
        int32_t id3[3];
        const int o = decode_sample(A, s, id3);
        const ObstacleDev& O = A.obs[o];
        if (!sample_is_boundary(O, id3)) continue;
        double w[3];
        fks_env::obstacle_sample_world(O.ob, A.resolution, A.resolution * 0.5, id3[0], id3[1], id3[2], w);
        int64_t idx[3];
        if (!A.grid.index(w, idx)) continue;
        const uint64_t c = A.grid.linear(idx[0], idx[1], idx[2]);
        if (!((double)sdf[c] > -(A.resolution * 1.5))) continue;
        atomicMax(winner + c, (uint32_t)(s + 1));
    }
}

__device__ __forceinline__ uint32_t cell_count(const EnvArgs& A, uint64_t c, const uint32_t* winner, const float* sdf) {
    const uint32_t w = winner[c];
    if (w) {
        int32_t id3[3];
        const int o = decode_sample(A, (uint64_t)(w - 1), id3);
        const ObstacleDev& O = A.obs[o];
        uint32_t n = 0;
        for (int a = 0; a < 3; ++a) n += (id3[a] == 0 || id3[a] == O.nc[a] - 1) ? 1u : 0u;
        return n;
    }
    return sdf[c] < 0.0f ? 1u : 0u;
}

/* exclusive scan of 256 per-thread sums in LDS; returns this thread's prefix and the block total */
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* lds, uint64_t* total) {
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    for (int off = 1; off < kScanThreads; off <<= 1) {
        const uint64_t add = (t >= off) ? lds[t - off] : 0;
        __syncthreads();
        lds[t] += add;
        __syncthreads();
    }
    const uint64_t inclusive = lds[t];
    *total = lds[kScanThreads - 1];
    __syncthreads();
    return inclusive - v;
}

__global__ void __launch_bounds__(kScanThreads) env_count_blocks(const EnvArgs A, const uint32_t* __restrict__ winner,
                                                                 const float* __restrict__ sdf, uint64_t* __restrict__ block_sums) {
    __shared__ uint64_t lds[kScanThreads];
    const uint64_t total = A.grid.cells();
    const uint64_t c0 = (uint64_t)blockIdx.x * kCellsPerScanBlock + (uint64_t)threadIdx.x * kScanItems;
    uint64_t sum = 0;
    for (int i = 0; i < kScanItems; ++i)
        if (c0 + i < total) sum += cell_count(A, c0 + i, winner, sdf);
    uint64_t block_total;
    (void)block_exclusive_scan(sum, lds, &block_total);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = block_total;
}

/* exclusive scan of the block sums in place (one workgroup, chunked with a carry) */
__global__ void __launch_bounds__(kScanThreads) env_scan_blocks(uint64_t* __restrict__ block_sums, uint64_t nblocks,
                                                                uint64_t* __restrict__ grand_total) {
    __shared__ uint64_t lds[kScanThreads];
    uint64_t carry = 0;
    for (uint64_t start = 0; start < nblocks; start += kScanThreads) {
        const uint64_t i = start + threadIdx.x;
        const uint64_t v = i < nblocks ? block_sums[i] : 0;
        uint64_t chunk_total;
        const uint64_t ex = block_exclusive_scan(v, lds, &chunk_total);
        if (i < nblocks) block_sums[i] = carry + ex;
        carry += chunk_total;
    }
    if (threadIdx.x == 0) *grand_total = carry;
}

/* CSR offsets and entries: boundary-owned cells get one face entry per boundary
 * axis in axis order (SEB.cpp:300-460), other d < 0 cells the gradient entry
 * (SEB.cpp:263-277) */
__global__ void __launch_bounds__(kScanThreads) env_fill(const EnvArgs A, const uint32_t* __restrict__ winner,
                                                         const float* __restrict__ sdf, const uint64_t* __restrict__ block_offsets,
                                                         uint32_t* __restrict__ offsets, double* __restrict__ entries) {
    __shared__ uint64_t lds[kScanThreads];
    const uint64_t total = A.grid.cells();
    const uint64_t c0 = (uint64_t)blockIdx.x * kCellsPerScanBlock + (uint64_t)threadIdx.x * kScanItems;
    uint32_t counts[kScanItems];
    uint64_t sum = 0;
    for (int i = 0; i < kScanItems; ++i) {
        counts[i] = (c0 + i < total) ? cell_count(A, c0 + i, winner, sdf) : 0u;
        sum += counts[i];
    }
    uint64_t block_total;
    uint64_t off = block_offsets[blockIdx.x] + block_exclusive_scan(sum, lds, &block_total);
    const int64_t nyz = A.grid.n[1] * A.grid.n[2];
    auto sdf_at = [&](int64_t i, int64_t j, int64_t k) { return sdf[A.grid.linear(i, j, k)]; };
    for (int it = 0; it < kScanItems; ++it) {
        const uint64_t c = c0 + it;
        if (c >= total) break;
        offsets[c] = (uint32_t)off;
        if (counts[it] == 0) continue;
        double* E = entries + 6 * off;
        const uint32_t w = winner[c];
        if (w) {
            int32_t id3[3];
            const int o = decode_sample(A, (uint64_t)(w - 1), id3);
            const ObstacleDev& O = A.obs[o];
            for (int a = 0; a < 3; ++a) {
                const bool low = id3[a] == 0;
                if (!low && id3[a] != O.nc[a] - 1) continue;
                fks_env::face_entry(O.ob.pose, a, low, E);
                E += 6;
            }
        } else {
            const int64_t i = (int64_t)(c / (uint64_t)nyz);
            const int64_t r = (int64_t)(c - (uint64_t)i * (uint64_t)nyz);
            const int64_t j = r / A.grid.n[2], k = r - j * A.grid.n[2];
            fks_env::gradient_entry(A.grid, i, j, k, sdf_at, E);
        }
        off += counts[it];
    }
}

struct DeviceBuffers {
    std::vector<void*> ptrs;
    ~DeviceBuffers() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    /* hand a buffer over to the caller: it is no longer freed here */
    void keep(void* p) {
        for (void*& q : ptrs)
            if (q == p) q = nullptr;
    }
    template <typename T>
    hipError_t alloc(T** p, uint64_t count) {
        *p = nullptr;
        hipError_t e = hipMalloc((void**)p, (size_t)(count > 0 ? count : 1) * sizeof(T));
        if (e == hipSuccess) ptrs.push_back(*p);
        return e;
    }
};

inline unsigned grid_for(uint64_t work, unsigned threads, unsigned cap) {
    const uint64_t g = (work + threads - 1) / threads;
    return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

fks_status to_status(hipError_t e) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return FKS_ERR_OUT_OF_MEMORY;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return FKS_ERR_NO_DEVICE;
    return FKS_ERR_HIP;
}

/* the host's analyze_sdf (fks_capi.cpp) per cell: lplus = max |a - b| / res over axis
 * neighbours both positive, cmax = max positive value / res next to a non-positive
 * one; keys are the doubles' bits (all values >= 0, so bit order is value order) */
__global__ void env_analyze(const float* __restrict__ sdf, int64_t nx, int64_t ny, int64_t nz, double inv,
                            unsigned long long* out /* lplus bits, cmax bits, bad */) {
    const uint64_t total = (uint64_t)nx * (uint64_t)ny * (uint64_t)nz;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    double lp = 0.0, cm = 0.0;
    unsigned long long bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const double a = sdf[i];
        if (!__builtin_isfinite(a)) {
            bad = 1;
            continue;
        }
        const int64_t z = (int64_t)(i % (uint64_t)nz), y = (int64_t)((i / (uint64_t)nz) % (uint64_t)ny),
                      x = (int64_t)(i / ((uint64_t)ny * (uint64_t)nz));
        const uint64_t nb[3] = {x + 1 < nx ? i + (uint64_t)ny * (uint64_t)nz : i, y + 1 < ny ? i + (uint64_t)nz : i,
                                z + 1 < nz ? i + 1 : i};
        for (int k = 0; k < 3; ++k) {
            if (nb[k] == i) continue;
            const double b = sdf[nb[k]];
            if (!__builtin_isfinite(b)) continue;
            if (a > 0.0 && b > 0.0) {
                const double v = __builtin_fabs(a - b) * inv;
                lp = v > lp ? v : lp;
            } else if (a > 0.0) {
                const double v = a * inv;
                cm = v > cm ? v : cm;
            } else if (b > 0.0) {
                const double v = b * inv;
                cm = v > cm ? v : cm;
            }
        }
    }
    unsigned long long klp = (unsigned long long)fks_math::bits(lp), kcm = (unsigned long long)fks_math::bits(cm);
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o1 = __shfl_xor(klp, off, 64), o2 = __shfl_xor(kcm, off, 64), o3 = __shfl_xor(bad, off, 64);
        klp = o1 > klp ? o1 : klp;
        kcm = o2 > kcm ? o2 : kcm;
        bad |= o3;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(out, klp);
        atomicMax(out + 1, kcm);
        if (bad) atomicOr(out + 2, bad);
    }
}

__global__ void env_brick_sdf(const float* __restrict__ lin, float* __restrict__ out, int64_t nx, int64_t ny, int64_t nz, uint32_t nb0,
                              uint32_t nb1, uint32_t nb2) {
    const uint64_t total = (uint64_t)nx * (uint64_t)ny * (uint64_t)nz;
    const uint32_t nb[3] = {nb0, nb1, nb2};
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total; c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = c % (uint64_t)nz, j = (c / (uint64_t)nz) % (uint64_t)ny, i = c / ((uint64_t)ny * (uint64_t)nz);
        out[fksd::brick_cell(nb, (uint32_t)i, (uint32_t)j, (uint32_t)k)] = lin[c];
    }
}

__global__ void env_brick_ranges(const uint32_t* __restrict__ off, uint2* __restrict__ out, int64_t nx, int64_t ny, int64_t nz,
                                 uint32_t nb0, uint32_t nb1, uint32_t nb2) {
    const uint64_t total = (uint64_t)nx * (uint64_t)ny * (uint64_t)nz;
    const uint32_t nb[3] = {nb0, nb1, nb2};
    for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < total; c += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t k = c % (uint64_t)nz, j = (c / (uint64_t)nz) % (uint64_t)ny, i = c / ((uint64_t)ny * (uint64_t)nz);
        out[fksd::brick_cell(nb, (uint32_t)i, (uint32_t)j, (uint32_t)k)] = make_uint2(off[c], off[c + 1]);
    }
}

}  // namespace

hipError_t fks_env::brick_sdf_device(const float* lin, const int64_t n[3], const uint32_t nb[3], float** out) {
    *out = nullptr;
    const uint64_t padded = fksd::brick_total(nb), total = (uint64_t)n[0] * (uint64_t)n[1] * (uint64_t)n[2];
    hipError_t e = hipMalloc((void**)out, padded * sizeof(float));
    if (e == hipSuccess) e = hipMemset(*out, 0, padded * sizeof(float));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(env_brick_sdf, dim3(grid_for(total, 256, 65536)), dim3(256), 0, nullptr, lin, *out, n[0], n[1], n[2], nb[0],
                           nb[1], nb[2]);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess && *out) {
        (void)hipFree(*out);
        *out = nullptr;
    }
    return e;
}

hipError_t fks_env::brick_normal_ranges_device(const uint32_t* off, const int64_t n[3], const uint32_t nb[3], uint2** out) {
    *out = nullptr;
    const uint64_t padded = fksd::brick_total(nb), total = (uint64_t)n[0] * (uint64_t)n[1] * (uint64_t)n[2];
    hipError_t e = hipMalloc((void**)out, padded * sizeof(uint2));
    if (e == hipSuccess) e = hipMemset(*out, 0, padded * sizeof(uint2));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(env_brick_ranges, dim3(grid_for(total, 256, 65536)), dim3(256), 0, nullptr, off, *out, n[0], n[1], n[2], nb[0],
                           nb[1], nb[2]);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess && *out) {
        (void)hipFree(*out);
        *out = nullptr;
    }
    return e;
}

bool fks_env::analyze_sdf_device(const float* d_sdf, int64_t nx, int64_t ny, int64_t nz, double res, double* lplus,
                                 double* cmax) {
    unsigned long long* d_out = nullptr;
    if (hipMalloc((void**)&d_out, 3 * sizeof(unsigned long long)) != hipSuccess) return false;
    bool ok = hipMemset(d_out, 0, 3 * sizeof(unsigned long long)) == hipSuccess;
    if (ok) {
        const uint64_t total = (uint64_t)nx * (uint64_t)ny * (uint64_t)nz;
        const uint64_t blocks = (total + 255) / 256;
        hipLaunchKernelGGL(env_analyze, dim3((unsigned)(blocks < 65536 ? (blocks ? blocks : 1) : 65536)), dim3(256), 0, nullptr,
                           d_sdf, nx, ny, nz, 1.0 / res, d_out);
        ok = hipGetLastError() == hipSuccess;
    }
    unsigned long long h[3] = {0, 0, 1};
    if (ok) ok = hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d_out);
    if (!ok || h[2]) return false;
    *lplus = fks_math::from_bits((uint64_t)h[0]);
    *cmax = fks_math::from_bits((uint64_t)h[1]);
    return *lplus > 0.0;
}

#define ENV_TRY(expr)                            \
    do {                                         \
        hipError_t _e = (expr);                  \
        if (_e != hipSuccess) return to_status(_e); \
    } while (0)

extern "C" fks_status fks_env_build_device(const fks_obstacle* obstacles, int32_t num_obstacles, double resolution,
                                           const double* grid_origin, const int64_t* num_cells, int32_t device,
                                           fks_device_env** out, fks_env_build_stats* stats) {
    if (!out || !(resolution > 0.0) || num_obstacles < 0 || (num_obstacles > 0 && !obstacles)) return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FKS_ERR_NO_DEVICE;
    if (device < 0 || device >= ndev) return FKS_ERR_INVALID_ARGUMENT;
    ENV_TRY(hipSetDevice(device));

    /* obstacle table: DiscretizeObstacle sample counts, prefix offsets */
    std::vector<ObstacleDev> obs;
    uint64_t samples = 0;
    for (int32_t o = 0; o < num_obstacles; ++o) {
        ObstacleDev d;
        std::memset(&d, 0, sizeof(d));
        d.ob = obstacles[o];
        fks_env::obstacle_samples(d.ob, resolution, d.nc);
        d.first = samples;
        d.count = (d.nc[0] > 0 && d.nc[1] > 0 && d.nc[2] > 0) ? (uint64_t)d.nc[0] * (uint64_t)d.nc[1] * (uint64_t)d.nc[2] : 0;
        samples += d.count;
        obs.push_back(d);
    }
    if (samples >= 0xffffffffull) return FKS_ERR_UNSUPPORTED; /* surface winners are 32-bit sequence numbers */

    DeviceBuffers B;
    EnvArgs A;
    std::memset(&A, 0, sizeof(A));
    A.num_obstacles = num_obstacles;
    A.samples = samples;
    A.resolution = resolution;
    A.grid.res = resolution;
    A.grid.inv_res = 1.0 / resolution;
    ObstacleDev* d_obs = nullptr;
    ENV_TRY(B.alloc(&d_obs, obs.size()));
    if (!obs.empty()) ENV_TRY(hipMemcpy(d_obs, obs.data(), obs.size() * sizeof(ObstacleDev), hipMemcpyHostToDevice));
    A.obs = d_obs;

    hipEvent_t ev0, ev1;
    ENV_TRY(hipEventCreate(&ev0));
    ENV_TRY(hipEventCreate(&ev1));
    struct EventGuard {
        hipEvent_t a, b;
        ~EventGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } eg{ev0, ev1};
    ENV_TRY(hipEventRecord(ev0, nullptr));

    if (grid_origin && num_cells) {
        std::memcpy(A.grid.origin, grid_origin, sizeof(A.grid.origin));
        for (int a = 0; a < 3; ++a) A.grid.n[a] = num_cells[a];
    } else {
        double mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
        if (samples > 0) {
            unsigned long long* d_keys = nullptr;
            ENV_TRY(B.alloc(&d_keys, 6));
            const unsigned long long init[6] = {~0ull, ~0ull, ~0ull, 0, 0, 0};
            ENV_TRY(hipMemcpy(d_keys, init, sizeof(init), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(env_bounds, dim3(grid_for(samples, 256, 8192)), dim3(256), 0, nullptr, A, d_keys);
            ENV_TRY(hipGetLastError());
            unsigned long long keys[6];
            ENV_TRY(hipMemcpy(keys, d_keys, sizeof(keys), hipMemcpyDeviceToHost));
            for (int a = 0; a < 6; ++a) {
                const uint64_t k = keys[a];
                const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
                double v;
                std::memcpy(&v, &b, sizeof(v));
                (a < 3 ? mn[a] : mx[a - 3]) = v;
            }
        }
        fks_env::auto_bounds(samples > 0, mn, mx, resolution, A.grid);
    }
    for (int a = 0; a < 3; ++a)
        if (A.grid.n[a] < 2 || A.grid.n[a] > 4096) return FKS_ERR_INVALID_ARGUMENT;
    fks_env::inverse34(A.grid.origin, A.grid.inv_origin);

    const uint64_t total = A.grid.cells();
    const int64_t nx = A.grid.n[0], ny = A.grid.n[1], nz = A.grid.n[2];
    uint8_t* d_occ = nullptr;
    uint32_t *d_filled = nullptr, *d_free = nullptr, *d_tmp = nullptr, *d_offsets = nullptr;
    uint64_t* d_scratch = nullptr;
    float* d_sdf = nullptr;
    ENV_TRY(B.alloc(&d_occ, total));
    ENV_TRY(B.alloc(&d_filled, total));
    ENV_TRY(B.alloc(&d_free, total));
    ENV_TRY(B.alloc(&d_tmp, total));
    ENV_TRY(B.alloc(&d_scratch, total));
    ENV_TRY(B.alloc(&d_sdf, total));
    ENV_TRY(hipMemsetAsync(d_occ, 0, total, nullptr));
    if (samples > 0) {
        hipLaunchKernelGGL(env_occupancy, dim3(grid_for(samples, 256, 65536)), dim3(256), 0, nullptr, A, d_occ);
        ENV_TRY(hipGetLastError());
    }
    /* squared EDT: z seeds, then y and x envelopes (ping-pong through d_tmp) */
    hipLaunchKernelGGL(env_seed_lines, dim3(grid_for((uint64_t)nx * ny, 64, 1u << 30)), dim3(64), 0, nullptr, A, d_occ, d_filled,
                       d_free);
    ENV_TRY(hipGetLastError());
    uint32_t* fields[2] = {d_filled, d_free};
    for (uint32_t* f : fields) {
        const uint64_t ylines = (uint64_t)nx * nz, xlines = (uint64_t)ny * nz;
        hipLaunchKernelGGL(env_envelope, dim3(grid_for(ylines, 64, 1u << 30)), dim3(64), 0, nullptr, f, d_tmp, d_scratch, ylines,
                           ny, (uint64_t)nz, (uint64_t)nz, (uint64_t)ny * nz);
        ENV_TRY(hipGetLastError());
        hipLaunchKernelGGL(env_envelope, dim3(grid_for(xlines, 64, 1u << 30)), dim3(64), 0, nullptr, d_tmp, f, d_scratch, xlines,
                           nx, (uint64_t)ny * nz, xlines, (uint64_t)0);
        ENV_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(env_sdf, dim3(grid_for(total, 256, 65536)), dim3(256), 0, nullptr, A, d_filled, d_free, d_sdf);
    ENV_TRY(hipGetLastError());

    /* surface-normal CSR; the EDT fields are dead now: reuse d_tmp as winners, d_filled as offsets */
    uint32_t* d_winner = d_tmp;
    ENV_TRY(hipMemsetAsync(d_winner, 0, total * sizeof(uint32_t), nullptr));
    if (samples > 0) {
        hipLaunchKernelGGL(env_surface_winner, dim3(grid_for(samples, 256, 65536)), dim3(256), 0, nullptr, A, d_sdf, d_winner);
        ENV_TRY(hipGetLastError());
    }
    const uint64_t nblocks = (total + kCellsPerScanBlock - 1) / kCellsPerScanBlock;
    uint64_t *d_block = nullptr, *d_grand = nullptr;
    ENV_TRY(B.alloc(&d_block, nblocks));
    ENV_TRY(B.alloc(&d_grand, 1));
    ENV_TRY(B.alloc(&d_offsets, total + 1));
    hipLaunchKernelGGL(env_count_blocks, dim3((unsigned)nblocks), dim3(kScanThreads), 0, nullptr, A, d_winner, d_sdf, d_block);
    ENV_TRY(hipGetLastError());
    hipLaunchKernelGGL(env_scan_blocks, dim3(1), dim3(kScanThreads), 0, nullptr, d_block, nblocks, d_grand);
    ENV_TRY(hipGetLastError());
    uint64_t nentries = 0;
    ENV_TRY(hipMemcpy(&nentries, d_grand, sizeof(nentries), hipMemcpyDeviceToHost));
    if (nentries > 0xffffffffull) return FKS_ERR_OUT_OF_MEMORY; /* offsets are uint32 (fks_environment) */
    double* d_entries = nullptr;
    ENV_TRY(B.alloc(&d_entries, 6 * nentries));
    hipLaunchKernelGGL(env_fill, dim3((unsigned)nblocks), dim3(kScanThreads), 0, nullptr, A, d_winner, d_sdf, d_block, d_offsets,
                       d_entries);
    ENV_TRY(hipGetLastError());
    const uint32_t last = (uint32_t)nentries;
    ENV_TRY(hipMemcpy(d_offsets + total, &last, sizeof(last), hipMemcpyHostToDevice));
    ENV_TRY(hipEventRecord(ev1, nullptr));
    ENV_TRY(hipEventSynchronize(ev1));
    float gpu_ms = 0.0f;
    ENV_TRY(hipEventElapsedTime(&gpu_ms, ev0, ev1));

    fks_device_env* env = new (std::nothrow) fks_device_env();
    if (!env) return FKS_ERR_OUT_OF_MEMORY;
    env->device = device;
    std::memcpy(env->geometry.origin, A.grid.origin, sizeof(A.grid.origin));
    env->geometry.resolution = resolution;
    for (int a = 0; a < 3; ++a) env->geometry.num_cells[a] = A.grid.n[a];
    env->cells = total;
    env->num_entries = nentries;
    env->occupancy = d_occ;
    env->sdf = d_sdf;
    env->offsets = d_offsets;
    env->entries = d_entries;
    B.keep(d_occ);
    B.keep(d_sdf);
    B.keep(d_offsets);
    B.keep(d_entries);
    if (stats) {
        stats->cells = total;
        stats->obstacle_samples = samples;
        stats->normal_entries = nentries;
        stats->gpu_ms = gpu_ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    *out = env;
    return FKS_OK;
}

extern "C" fks_status fks_device_env_geometry(const fks_device_env* env, fks_grid_geometry* out) {
    if (!env || !out) return FKS_ERR_INVALID_ARGUMENT;
    *out = env->geometry;
    return FKS_OK;
}

extern "C" void fks_device_env_free(fks_device_env* env) {
    if (!env) return;
    (void)hipSetDevice(env->device);
    void* ptrs[] = {env->occupancy, env->sdf, env->offsets, env->entries};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    delete env;
}

extern "C" fks_status fks_device_env_download(const fks_device_env* denv, fks_env_handle** out) {
    if (!denv || !out) return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    ENV_TRY(hipSetDevice(denv->device));
    fks_env_handle* env = new (std::nothrow) fks_env_handle();
    if (!env) return FKS_ERR_OUT_OF_MEMORY;
    const uint64_t total = denv->cells, nentries = denv->num_entries;
    try {
        env->occupancy.resize(total);
        env->sdf.resize(total);
        env->offsets.resize(total + 1);
        env->entries.resize(6 * nentries);
    } catch (const std::bad_alloc&) {
        delete env;
        return FKS_ERR_OUT_OF_MEMORY;
    }
    hipError_t e = hipMemcpy(env->occupancy.data(), denv->occupancy, total, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(env->sdf.data(), denv->sdf, total * sizeof(float), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(env->offsets.data(), denv->offsets, (total + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e == hipSuccess && nentries)
        e = hipMemcpy(env->entries.data(), denv->entries, 6 * nentries * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        delete env;
        return to_status(e);
    }
    env->geometry = denv->geometry;
    *out = env;
    return FKS_OK;
}

extern "C" fks_status fks_env_build_gpu(const fks_obstacle* obstacles, int32_t num_obstacles, double resolution,
                                        const double* grid_origin, const int64_t* num_cells, int32_t device,
                                        fks_env_handle** out, fks_env_build_stats* stats) {
    if (!out) return FKS_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    const auto t_start = std::chrono::steady_clock::now();
    fks_device_env* denv = nullptr;
    fks_status st = fks_env_build_device(obstacles, num_obstacles, resolution, grid_origin, num_cells, device, &denv, stats);
    if (st != FKS_OK) return st;
    st = fks_device_env_download(denv, out);
    fks_device_env_free(denv);
    if (st == FKS_OK && stats)
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return st;
}
