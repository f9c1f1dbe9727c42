# Round-end GPU evidence: tools/gpu_round.sh (suite, smoke, bench, rocprof trace + PMC), the
# other workloads' bench lines, and the joint-space proof A/B against a baseline build.
# usage: bash tools/final_round.sh <tag> [baseline.so]
TAG=${1:-rXX}
BASE=${2:-build/variants/libfks_head.so}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh $TAG || exit $?
for w in cfg1 cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --workload $w --no-config-check > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || exit $?
done
timeout -k 10 700 python tools/variant_bench.py $BASE fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+joint-proof $BASE fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+joint-proof > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
echo final_done
