# SQ instruction-count A/B of kernel builds on a 16k-particle cfg3 bench (one --pmc pass per lib).
# usage: bash tools/sq_ab.sh <tag> <lib> [<lib> ...]
TAG=${1:-sqab}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  FKS_LIB_PATH=$(readlink -f $lib) timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM --kernel-trace --output-format csv -d gpurun_out/${TAG}_$i -o bench -- python3 bench.py --particles 16384 --steps 1 --warmup 0 --no-cpu-baseline --no-config-check > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "$lib rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$TAG" "$@" <<'PY'
import csv, glob, sys, json
tag = sys.argv[1]
for i, lib in enumerate(sys.argv[2:], 1):
    f = glob.glob(f"gpurun_out/{tag}_{i}/**/*counter_collection.csv", recursive=True)
    tot = {}
    for row in csv.DictReader(open(f[0])):
        if "fks_simulate_linked" not in row.get("Kernel_Name", ""):
            continue
        tot[row["Counter_Name"]] = tot.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    print(lib, json.dumps({k: f"{v:.4g}" for k, v in sorted(tot.items())}))
PY
