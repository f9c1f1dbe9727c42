"""The catkin-compatible CMake package (CMakeLists.txt, package.xml): the drop-in for the
reference's fast_kinematic_simulator catkin package (reference CMakeLists.txt:75-92,
package.xml).  Configured and built here with cmake (HIP language, gfx950, no GPU needed):
the library exports every symbol of include/fks_capi.h, the planner-side test program built
through it hands the GPU the same robot as the build.py-built one, and an installed package
is found by find_package() from a separate consumer project."""
import os
import subprocess
import tempfile

import pytest

from test_capi import declared_symbols

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, **kw):
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, **kw)
    assert p.returncode == 0, " ".join(cmd) + "\n" + p.stdout[-4000:]
    return p.stdout


@pytest.fixture(scope="module")
def cmake_build():
    with tempfile.TemporaryDirectory(prefix="fks_cmake_") as d:
        build, prefix = os.path.join(d, "build"), os.path.join(d, "prefix")
        _run(["cmake", "-S", ROOT, "-B", build, "-DFKS_BUILD_TESTS=ON", f"-DCMAKE_INSTALL_PREFIX={prefix}"], timeout=300)
        _run(["cmake", "--build", build, "-j8"], timeout=900)
        _run(["cmake", "--install", build], timeout=300)
        yield d, build, prefix


def test_package_xml_names_the_reference_package():
    text = open(os.path.join(ROOT, "package.xml")).read()
    assert "<name>fast_kinematic_simulator</name>" in text and "<buildtool_depend>catkin</buildtool_depend>" in text
    cm = open(os.path.join(ROOT, "CMakeLists.txt")).read()
    assert "project(fast_kinematic_simulator " in cm and "catkin_package(INCLUDE_DIRS include LIBRARIES ${PROJECT_NAME}" in cm


def test_cmake_library_flags_and_exports(cmake_build):
    _, build, prefix = cmake_build
    flags = open(os.path.join(build, "CMakeFiles", "fast_kinematic_simulator.dir", "flags.make")).read()
    assert "--offload-arch=gfx950" in flags and "-ffp-contract=off" in flags
    lib = os.path.join(prefix, "lib", "libfast_kinematic_simulator.so")
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not sorted(declared_symbols() - exported)
    for h in ("fks_capi.h", "fast_kinematic_simulator/fast_kinematic_simulator.hpp",
              "fast_kinematic_simulator_amd/fks_external_types.hpp"):
        assert os.path.exists(os.path.join(prefix, "include", h)), h


def test_cmake_built_planner_program_matches_build_py(cmake_build):
    from test_planner_interface import _dump, _scene, _write_scene

    _, build, _ = cmake_build
    exe = os.path.join(build, "planner_interface_test")
    for name in ("linked", "se3"):
        family, wl, obstacles, grid = _scene(name)
        with tempfile.TemporaryDirectory() as d:
            path = os.path.join(d, "scene.txt")
            _write_scene(path, family, wl, obstacles, grid)
            got = _run([exe, path, "--dump"], timeout=300)
        assert got == _dump(name, False), name


def test_installed_package_is_found_by_a_consumer(cmake_build):
    """A planner-side project written as the reference's users write theirs: includes
    <fast_kinematic_simulator/fast_kinematic_simulator.hpp>, calls the factory, links the
    exported target.  Without a GPU the factory throws FKS_ERR_NO_DEVICE (exit 3)."""
    d, _, prefix = cmake_build
    src = os.path.join(d, "consumer")
    os.makedirs(src)
    with open(os.path.join(src, "CMakeLists.txt"), "w") as f:
        f.write("cmake_minimum_required(VERSION 3.21)\nproject(consumer LANGUAGES CXX)\n"
                "find_package(fast_kinematic_simulator 3 REQUIRED)\nadd_executable(consumer main.cpp)\n"
                "target_link_libraries(consumer PRIVATE fast_kinematic_simulator::fast_kinematic_simulator)\n")
    with open(os.path.join(src, "main.cpp"), "w") as f:
        f.write("#include <fast_kinematic_simulator/fast_kinematic_simulator.hpp>\n#include <cstdio>\n"
                "int main() {\n"
                "  using namespace simulator_environment_builder;\n"
                "  std::vector<OBSTACLE_CONFIG> obs{OBSTACLE_CONFIG(1u, fks_planner_types::Isometry3d::Identity(),"
                " fks_planner_types::Vector3d(0.1, 0.1, 0.1))};\n"
                "  const EnvironmentComponents env = BuildCompleteEnvironment(obs, 0.05);\n"
                "  try {\n"
                "    uncertainty_planning_core::LinkedSimulatorPtr sim = fast_kinematic_simulator::MakeLinkedSimulator(\n"
                "        env.GetEnvironment(), env.GetEnvironmentSDF(), env.GetSurfaceNormalsGrid(),\n"
                "        fast_kinematic_simulator::GetDefaultSolverParameters(), 100.0, 42u, 0);\n"
                "    std::printf(\"frame %s\\n\", sim->GetFrame().c_str());\n"
                "    return 0;\n"
                "  } catch (const fks::SimulatorError& e) {\n"
                "    std::printf(\"%s\\n\", e.what());\n"
                "    return e.status() == FKS_ERR_NO_DEVICE ? 3 : 1;\n"
                "  }\n}\n")
    cb = os.path.join(d, "consumer_build")
    _run(["cmake", "-S", src, "-B", cb, f"-DCMAKE_PREFIX_PATH={prefix}"], timeout=300)
    _run(["cmake", "--build", cb], timeout=300)
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(prefix, "lib") + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    p = subprocess.run([os.path.join(cb, "consumer")], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=120)
    assert p.returncode in (0, 3), p.stdout
    if p.returncode == 0:
        assert "frame uncertainty_planning_simulator" in p.stdout
