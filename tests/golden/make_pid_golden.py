"""Regenerate tests/golden/pid_golden.json from the reference's own PID header.

Builds oracle/_ref/pid_golden (oracle/Makefile target `ref`, compiling
oracle/ref/pid_golden_driver.cpp against /root/reference/include) and captures
its output.  Needs /root/reference (this container only)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

if __name__ == "__main__":
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "pid_golden")], check=True, capture_output=True, text=True).stdout
    with open(os.path.join(HERE, "pid_golden.json"), "w") as f:
        f.write(out)
    print("wrote", os.path.join(HERE, "pid_golden.json"))
