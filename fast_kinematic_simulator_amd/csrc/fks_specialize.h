/*
 * fks_specialize.h — robot-shape-specialised simulation kernels, compiled at run time.
 *
 * The generic kernels (fks_kernels.hip) read the robot's dimensions and the LDS / scratch
 * carve-outs from SimArgs.  For one robot shape the same source compiled with those values
 * as constants (FKS_SHAPE_*, see the "robot shape" block of fks_kernels.hip) keeps far fewer
 * wave-uniform values live: on cfg3's 7-dof arm the throughput kernel runs 11-12 % faster,
 * bit for bit the same results.  hiprtc compiles the kernel source the
 * library carries (fks_spec_sources.inc, generated at build time from the very sources the
 * library was built from) for gfx950 with the library's flags; code objects are kept per
 * process and, unless FKS_KERNEL_CACHE=off, on disk (FKS_KERNEL_CACHE, else
 * $XDG_CACHE_HOME or ~/.cache, /fast_kinematic_simulator_amd), keyed by a hash of the
 * sources and the compile options.
 */
#ifndef FKS_SPECIALIZE_H
#define FKS_SPECIALIZE_H

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace fks_spec {

/* everything the specialised build fixes at compile time */
struct Shape {
    int32_t type;   /* FKS_ROBOT_* */
    int32_t L, J, D, W, G, P;
    int32_t pair;   /* LdsLayout.fk_pair */
    int32_t lean;   /* LdsLayout.lean (the fks_simulate_linked_lean variant) */
    int32_t waves_per_eu = 0; /* 0: the library's register budget (fksd::kThroughputWavesPerEU waves
                               * per SIMD); fewer when the LDS block caps the resident waves lower,
                               * so the kernel may use the registers those absent waves leave */
    int32_t no_proofs = 0;    /* validation build: every skip proof compiled out (FKS_NO_SKIP_PROOFS) */
};

/* "t0-L8-J7-D7-W7-G8-P512-p1-l0" (+ "-w4" for a raised register budget, "-np" for the
 * validation build without skip proofs): names the shape in logs and cache files */
std::string shape_key(const Shape& s);

struct CodeObject {
    std::vector<char> bytes;
    double compile_seconds = 0.0; /* 0 when it came from a cache */
    bool from_disk = false;
};

/* The code object of `fks_simulate_shaped` for shape `s`: from the process cache, the disk
 * cache, or a hiprtc compile (seconds; one compile at a time per process; *compiled says
 * which).  refresh: drop the cached copies and compile.  On failure returns null and sets
 * *log.  The disk cache is used only when its directory belongs to this user and is not
 * writable by others; the key covers every source byte, every option, the device
 * architecture and the identity (size, mtime) of the fks_shapec binary that compiles. */
std::shared_ptr<const CodeObject> code_object(const Shape& s, std::string* log, bool* compiled, bool refresh = false);

/* an unsigned field of the (single) kernel's entry in a code object's AMDGPU metadata note
 * (MessagePack: the key string followed by a positive integer), e.g. ".vgpr_count"; -1 if
 * absent */
int metadata_uint(const std::vector<char>& code_object, const char* key);
/* the same field of the entry of kernel `name` (the module also carries the shaped
 * configuration check): the first `key` after the entry's ".name" (the keys of a kernel's
 * metadata map are emitted in sorted order, ".name" before ".sgpr_count" / ".vgpr_count") */
int kernel_metadata_uint(const std::vector<char>& code_object, const char* name, const char* key);

}  // namespace fks_spec

#endif
