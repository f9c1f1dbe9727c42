"""Compare kernel build variants on the GPU: runs bench.py once per library.

    python tools/variant_bench.py build/variants/libfks_w2.so build/variants/libfks_w4.so ...

Each variant runs in its own process (FKS_LIB_PATH selects the library), one after
another; prints one summary line per variant.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    extra = []
    libs = []
    for a in sys.argv[1:]:
        # "lib.so+flag" runs that library with bench.py --flag (e.g. libfks_hip.so+segment-steps=10);
        # "lib.so+env:NAME=VALUE" with that environment variable set
        (extra if a.startswith("--") or (extra and ".so" not in a) else libs).append(a)
    for spec in libs:
        lib, _, flag = spec.partition("+")
        env = dict(os.environ, FKS_LIB_PATH=os.path.abspath(lib), FKS_VARIANT_LIB="1")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--pipeline-batches", "0", "--no-projection", *extra]
        if flag.startswith("env:"):
            name, _, value = flag[4:].partition("=")
            env[name] = value
        elif flag:
            cmd.append("--" + flag)
        p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=900)
        if p.returncode != 0:
            print(f"{lib}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
            sys.exit(p.returncode)
        line = json.loads(p.stdout.strip().splitlines()[-1])
        print(json.dumps({"lib": os.path.basename(lib) + ("+" + flag if flag else ""), "value": line["value"], "kernel_ms": line["roofline"]["avg_kernel_ms"],
                          "frac": line["roofline"]["frac"], "error_particles": line["config"].get("error_particles"),
                          "busy": line.get("wave_slots", {}).get("busy_fraction"), "phases": line.get("kernel_phases"),
                          "config_check": (line.get("config_check") or {}).get("value"),
                          "config_check_ms": (line.get("config_check") or {}).get("kernel_ms")}),
              flush=True)


if __name__ == "__main__":
    main()
