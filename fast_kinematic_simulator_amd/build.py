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
SOURCES = ["csrc/fks_kernels.hip", "csrc/fks_capi.cpp", "csrc/fks_multi.cpp", "csrc/fks_env_builder.cpp", "csrc/fks_env_gpu.hip",
           "csrc/fks_robot_control.cpp", "csrc/fks_specialize.cpp"]
HEADERS = ["csrc/fks_device.h", "csrc/fks_env_internal.h", "csrc/fks_se3.h", "csrc/fks_specialize.h", "../include/fks_capi.h",
           "../include/fks_portable_math.h", "../include/fks_control.h"]
# the kernel source and the headers it includes, carried inside the library for the run-time
# compilation of shape-specialised kernels (fks_specialize.cpp): name as included -> path
EMBEDDED = [("fks_kernels.hip", "csrc/fks_kernels.hip"), ("fks_device.h", "csrc/fks_device.h"), ("fks_se3.h", "csrc/fks_se3.h"),
            ("fks_capi.h", "../include/fks_capi.h"), ("fks_portable_math.h", "../include/fks_portable_math.h"),
            ("fks_control.h", "../include/fks_control.h")]
GENERATED = os.path.join(ROOT, "build", "generated")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"


def hipcc() -> str:
    return shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def write_embedded_sources(directory: str = GENERATED, defines=()) -> str:
    """fks_spec_sources.inc: the EMBEDDED files as byte arrays (cmake/fks_embed_sources.cmake
    writes the same file for the CMake build).  A variant build's defines (build_variant) are
    prepended to the kernel source, so its shape-specialised kernels are built the same way."""
    os.makedirs(directory, exist_ok=True)
    lines = ["/* generated from the library's sources by fast_kinematic_simulator_amd/build.py: do not edit */"]
    entries = []
    for k, (name, rel) in enumerate(EMBEDDED):
        data = open(os.path.join(PKG, rel), "rb").read()
        if name == "fks_kernels.hip" and defines:
            prelude = "".join("#define " + d.replace("=", " ", 1) + "\n" for d in defines)
            data = prelude.encode() + data
        body = ",".join(f"0x{b:02x}" for b in data)
        lines.append(f"static const unsigned char kFksSrc{k}[] = {{{body}}};")
        entries.append(f'{{"{name}", kFksSrc{k}, sizeof(kFksSrc{k})}}')
    lines.append("struct FksEmbeddedSource {\n    const char* name;\n    const unsigned char* data;\n    unsigned long size;\n};")
    lines.append("static const FksEmbeddedSource kFksEmbeddedSources[] = {" + ", ".join(entries) + "};")
    lines.append(f"static const int kFksEmbeddedSourceCount = {len(EMBEDDED)};")
    out = os.path.join(directory, "fks_spec_sources.inc")
    text = "\n".join(lines) + "\n"
    if not os.path.exists(out) or open(out).read() != text:
        with open(out + ".tmp", "w") as f:
            f.write(text)
        os.replace(out + ".tmp", out)
    return out


def generated_dir(output: str) -> str:
    """Where the embedded-sources include of the library at `output` is written: the product's
    under build/generated, each variant's in a directory of its own (concurrent variant builds
    must not embed each other's defines)."""
    if os.path.basename(output) in ("libfks_hip.so", "libfks_hip.so.tmp"):
        return GENERATED
    return os.path.join(GENERATED, "variant-" + os.path.basename(output).replace(".tmp", ""))


def build_command(output: str, defines=(), flags=()) -> list:
    gen = generated_dir(output)
    write_embedded_sources(gen, defines=defines)
    return [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=off",
            *[f"-D{d}" for d in defines], *flags,
            f"-I{os.path.join(ROOT, 'include')}", f"-I{os.path.join(PKG, 'csrc')}", f"-I{gen}", "-x", "hip",
            *[os.path.join(PKG, s) for s in SOURCES], "-o", output]


SHAPEC = os.path.join(PKG, "fks_shapec")


def build_shapec(force: bool = False) -> str:
    """The compiler process of the shape specialisation (csrc/fks_shapec.cpp): a host program
    over ROCm's hiprtc, next to libfks_hip.so; it compiles the sources the calling library
    writes out for it, so one helper serves the product and every variant build."""
    src = os.path.join(PKG, "csrc", "fks_shapec.cpp")
    if not force and os.path.exists(SHAPEC) and os.path.getmtime(SHAPEC) >= os.path.getmtime(src):
        return SHAPEC
    cmd = ["g++", "-std=c++17", "-O2", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", src, "-o", SHAPEC + ".tmp",
           "-L/opt/rocm/lib", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"]
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("g++ (fks_shapec) failed:\n" + proc.stdout[-6000:])
    os.replace(SHAPEC + ".tmp", SHAPEC)
    return SHAPEC


def _stale(target: str) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = [os.path.join(PKG, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_library(force: bool = False, verbose: bool = False) -> str:
    target = os.path.join(PKG, "libfks_hip.so")
    build_shapec(force)
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


def build_variant(output: str, defines=(), flags=()) -> str:
    """Build a tuning or diagnostic variant (e.g. FKS_WAVES_PER_EU=3, FKS_PHASE_TIMERS=1, or
    extra compiler flags) to a separate path; load it with FKS_LIB_PATH=<output> and
    FKS_VARIANT_LIB=1 (tools/variant_bench.py).  A variant never takes the product's name.
    Its defines reach its shape-specialised kernels (they are prepended to the embedded kernel
    source, and a source-defined FKS_WAVES_PER_EU wins over the layout's budget); extra
    `flags` do not (hiprtc compiles with the library's fixed options)."""
    output = os.path.abspath(output)
    if os.path.basename(output) == "libfks_hip.so":
        raise ValueError("a build variant must not be named libfks_hip.so (the product library)")
    proc = subprocess.run(build_command(output, defines, flags), cwd=PKG, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                          text=True)
    if proc.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + proc.stdout[-6000:])
    return output


def _headers(directory: str) -> list:
    return [os.path.join(d, f) for d, _, fs in os.walk(directory) for f in fs]


def build_cpp_program(src: str, name: str, force: bool = False, extra_flags=(), extra_deps=()) -> str:
    """Compile a host C++ program over the public headers (include/) and link
    libfks_hip.so: g++ only, no HIP toolchain, as a planner would build against the
    drop-in.  Output: build/<name>."""
    lib = build_library()
    src = os.path.join(ROOT, src)
    out_dir = os.path.join(ROOT, "build")
    os.makedirs(out_dir, exist_ok=True)
    target = os.path.join(out_dir, name)
    inc = os.path.join(ROOT, "include")
    headers = _headers(inc) + list(extra_deps)
    if not force and os.path.exists(target) and all(os.path.getmtime(target) >= os.path.getmtime(p)
                                                    for p in [src, lib] + headers):
        return target
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-ffp-contract=off", *extra_flags, f"-I{inc}", src, "-o", target,
           f"-L{PKG}", "-lfks_hip", "-Wl,-rpath,$ORIGIN/../fast_kinematic_simulator_amd", "-Wl,-rpath-link,/opt/rocm/lib"]
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("g++ failed:\n" + proc.stdout[-6000:])
    return target


def build_example(force: bool = False) -> str:
    """Compile examples/cpp_forward_simulate.cpp (C++ host code over the C-ABI and
    include/fast_kinematic_simulator_amd/hip_particle_contact_simulator.hpp)."""
    return build_cpp_program(os.path.join("examples", "cpp_forward_simulate.cpp"), "cpp_forward_simulate", force)


MOCK_WORKSPACE = os.path.join(ROOT, "tests", "cpp", "mock_workspace", "include")


def build_planner_test(force: bool = False, workspace: bool = False) -> str:
    """Compile tests/cpp/planner_interface_test.cpp: the planner-side drop-in driven only
    through std::shared_ptr<SimulatorInterface<...>> (fast_kinematic_simulator.hpp).
    workspace=True puts the mock planner workspace (tests/cpp/mock_workspace) on the
    include path, so fks_external_types.hpp takes the real-libraries branch."""
    if workspace:
        return build_cpp_program(os.path.join("tests", "cpp", "planner_interface_test.cpp"), "planner_interface_test_workspace",
                                 force, extra_flags=(f"-I{MOCK_WORKSPACE}",), extra_deps=_headers(MOCK_WORKSPACE))
    return build_cpp_program(os.path.join("tests", "cpp", "planner_interface_test.cpp"), "planner_interface_test", force)


if __name__ == "__main__":
    print(build_library(force=True, verbose=True))
