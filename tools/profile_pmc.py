"""Summarise rocprofv3 PMC passes of bench.py into profiles/<round>_pmc.json.

Usage (after the three passes FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum,
each its own `rocprofv3 --pmc ... --kernel-trace --output-format csv` run of
`python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline`):

    python tools/profile_pmc.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_tcc r01
    python tools/profile_pmc.py <fetch> <write> <tcc> r04_cfg5 fks_simulate_linked_lean   # another kernel

Only the headline kernel's summary (no kernel argument) is also written as latest_pmc.json,
which bench.py reads for `roofline.traffic` — and only when the profile names the kernel and
shape its own timed launches ran (`--shape t0-L8-...`, the bench line's specialization.shape)
and the kernel sources it was built from (kernel_source_sha16, checked against the tree).

HBM traffic per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 bytes, averaged over the
kernel's dispatches: MI355X_MICROARCH.md §HBM prescribes doubling FETCH_SIZE on gfx950
(128-B read requests tallied at 64 B) and reading WRITE_SIZE as is.  FETCH_SIZE counts
L2->fabric read requests, Infinity-Cache hits included.  The doubling is calibrated on
16-B-per-lane streaming reads; this kernel's reads are 4-32-B gathers and scratch
reloads, so the corrected figure is an upper bound and the raw counts are kept
beside it."""
import csv
import json
import os
import sys

KERNEL = "fks_simulate_shaped"


def counters(path, kernel=KERNEL):
    vals = {}
    with open(os.path.join(path, "bench_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"] != kernel:
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return vals


def kernel_source_sha16():
    """A hash of the kernel source and the headers it includes (build.EMBEDDED): a profile of
    another kernel version is not quoted by bench.py."""
    import hashlib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from fast_kinematic_simulator_amd import build

    h = hashlib.sha256()
    for name, rel in build.EMBEDDED:
        h.update(name.encode() + b"\0")
        h.update(open(os.path.join(build.PKG, rel), "rb").read())
    return h.hexdigest()[:16]


def main():
    argv = list(sys.argv[1:])
    shape = None
    if "--shape" in argv:
        i = argv.index("--shape")
        shape = argv[i + 1]
        del argv[i:i + 2]
    fetch_dir, write_dir, tcc_dir, tag = argv[:4]
    kernel = argv[4] if len(argv) > 4 else KERNEL
    f = counters(fetch_dir, kernel)["FETCH_SIZE"]
    w = counters(write_dir, kernel)["WRITE_SIZE"]
    t = counters(tcc_dir, kernel)
    hits, misses = t["TCC_HIT_sum"], t["TCC_MISS_sum"]
    fetch_raw = sum(f) / len(f) * 1024.0
    fetch_b = 2.0 * fetch_raw
    write_b = sum(w) / len(w) * 1024.0
    out = {
        "kernel": f"{kernel} ({shape})" if shape else kernel,
        "kernel_source_sha16": kernel_source_sha16(),
        "dispatches": len(f),
        "fetch_bytes_per_launch": fetch_b,
        "fetch_size_raw_bytes_per_launch": fetch_raw,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "l2_hit_rate": sum(hits) / (sum(hits) + sum(misses)),
        "note": "FETCH_SIZE/WRITE_SIZE from separate rocprofv3 --pmc passes of bench.py --steps 2 --warmup 1; fetch doubled "
                "per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at 64 B; an upper bound for this kernel's gathers)",
        "source": f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum+TCC_MISS_sum passes of "
                  "bench.py --steps 2 --warmup 1, tools/profile_pmc.py)",
    }
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for name in (f"{tag}_pmc.json", "latest_pmc.json") if kernel == KERNEL else (f"{tag}_pmc.json",):
        with open(os.path.join(root, "profiles", name), "w") as fo:
            json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
