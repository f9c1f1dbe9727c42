# One GPU call for a candidate build: the whole -m gpu suite, then interleaved A/B bench lines
# (cfg3, cfg4) of the candidate against the listed baselines.
# usage: bash tools/round_check.sh <tag> <baseline.so> [<baseline2.so>]
set -e
TAG=$1; B1=$2; B2=${3:-$2}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=fast_kinematic_simulator_amd/libfks_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B1 $NEW $B2 $B1 $NEW $B2 > gpurun_out/${TAG}_ab_cfg3.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B2 $NEW $B2 $NEW --workload cfg4 --no-config-check > gpurun_out/${TAG}_ab_cfg4.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B2 $NEW $B2 $NEW --workload cfg5 --no-config-check > gpurun_out/${TAG}_ab_cfg5.log 2>&1
echo done
