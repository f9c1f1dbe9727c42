# Kernel build variants: bench line + rocprofv3 WRITE_SIZE / FETCH_SIZE pass per variant.
# usage: bash tools/variant_pmc.sh <tag> lib1.so lib2.so ...   (run on the GPU box)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check"
for lib in "$@"; do
  n=$(basename $lib .so)
  FKS_LIB_PATH=$PWD/$lib timeout -k 10 200 $B > gpurun_out/$TAG/$n.bench.json 2> gpurun_out/$TAG/$n.bench.err || exit 1
  FKS_LIB_PATH=$PWD/$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/$TAG/$n.write -o bench -- $B > /dev/null 2> gpurun_out/$TAG/$n.write.err || exit 1
  FKS_LIB_PATH=$PWD/$lib timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/$TAG/$n.fetch -o bench -- $B > /dev/null 2> gpurun_out/$TAG/$n.fetch.err || exit 1
  python3 - "$TAG" "$n" <<'PY'
import csv, glob, json, sys
tag, n = sys.argv[1], sys.argv[2]
line = json.loads(open(f"gpurun_out/{tag}/{n}.bench.json").read().strip().splitlines()[-1])
out = {"lib": n, "value": line["value"], "kernel_ms": line["roofline"]["avg_kernel_ms"]}
for c in ("write", "fetch"):
    for f in glob.glob(f"gpurun_out/{tag}/{n}.{c}/**/*counter_collection.csv", recursive=True):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("fks_simulate_linked")]
        if vals:
            out[c + "_GB_per_launch"] = sum(vals) / len(vals) * 1024 / 1e9
print(json.dumps(out), flush=True)
PY
done
