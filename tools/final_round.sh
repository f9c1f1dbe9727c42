# Round-end GPU evidence: tools/gpu_round.sh (suite, smoke, bench, rocprof trace + PMC) and
# the other workloads' bench lines.
# usage: bash tools/final_round.sh <tag>
TAG=${1:-rXX}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round.sh $TAG || exit $?
for w in cfg1 cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --workload $w --no-config-check > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || exit $?
done
echo final_done
