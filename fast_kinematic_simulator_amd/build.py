"""In-tree build of libfks_hip.so (HIP kernels for gfx950 + the C-ABI host code).

hipcc cross-compiles here without a GPU; the .so travels to the GPU box with the
repository snapshot.  Every translation unit is compiled with -ffp-contract=off:
bit-exact parity with the CPU oracle depends on the absence of fused multiply-adds.
"""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SOURCES = ["csrc/fks_kernels.hip", "csrc/fks_capi.cpp", "csrc/fks_env_builder.cpp", "csrc/fks_env_gpu.hip"]
HEADERS = ["csrc/fks_device.h", "csrc/fks_env_internal.h", "../include/fks_capi.h", "../include/fks_portable_math.h"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def hipcc() -> str:
    return shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def build_command(output: str, defines=()) -> list:
    return [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
            *[f"-D{d}" for d in defines],
            f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(PKG, 'csrc')}", "-x", "hip",
            *[os.path.join(PKG, s) for s in SOURCES], "-o", output]


def _stale(target: str) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = [os.path.join(PKG, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_library(force: bool = False, verbose: bool = False) -> str:
    target = os.path.join(PKG, "libfks_hip.so")
    if not force and not _stale(target):
        return target
    tmp = target + ".tmp"
    proc = subprocess.run(build_command(tmp), cwd=PKG, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + proc.stdout[-6000:])
    if verbose:
        print(proc.stdout)
    os.replace(tmp, target)
    return target


def build_variant(output: str, defines) -> str:
    """Build a tuning variant (e.g. FKS_WAVES_PER_EU=3) to a separate path; load it
    with FKS_LIB_PATH=<output> (tools/variant_bench.py)."""
    output = os.path.abspath(output)
    proc = subprocess.run(build_command(output, defines), cwd=PKG, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + proc.stdout[-6000:])
    return output


def build_example(force: bool = False) -> str:
    """Compile examples/cpp_forward_simulate.cpp (C++ host code over the C-ABI and
    include/fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp)."""
    lib = build_library()
    src = os.path.join(ROOT, "examples", "cpp_forward_simulate.cpp")
    out_dir = os.path.join(ROOT, "build")
    os.makedirs(out_dir, exist_ok=True)
    target = os.path.join(out_dir, "cpp_forward_simulate")
    hdr = os.path.join(ROOT, "include", "fast_kinematic_simulator_amd", "hip_particle_contact_simulator.hpp")
    capi = os.path.join(ROOT, "include", "fks_capi.h")
    if not force and os.path.exists(target) and all(os.path.getmtime(target) >= os.path.getmtime(p)
                                                    for p in (src, hdr, capi, lib)):
        return target
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", f"-I{os.path.join(ROOT, 'include')}", src, "-o", target, f"-L{PKG}",
           "-lfks_hip", "-Wl,-rpath,$ORIGIN/../fast_kinematic_simulator_amd", "-Wl,-rpath-link,/opt/rocm/lib"]
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("g++ failed:\n" + proc.stdout[-6000:])
    return target


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
