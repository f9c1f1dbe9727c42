"""CPU AddressSanitizer + UndefinedBehaviorSanitizer run of the host code (VERDICT r01:
no sanitizer build existed): the oracle, the product's host environment builder and the
planner-facing host headers, built by `make -C oracle sanitize` and driven by
tests/cpp/sanitize_driver.cpp.  Any sanitizer report fails the run (halt_on_error)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_clean_under_asan_ubsan():
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "sanitize"], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600)
    assert b.returncode == 0, b.stdout[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="2")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "sanitize_driver")], stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-6000:]
    assert "sanitize driver ok" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
