# candidate build: whole GPU suite, then interleaved cfg3 / cfg4 / cfg5 A/B against a baseline build
# usage: bash tools/ab_check.sh <tag> <baseline.so>
set -e
TAG=$1; B=$2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=fast_kinematic_simulator_amd/libfks_hip.so
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
timeout -k 10 700 python tools/variant_bench.py $B $NEW $B $NEW $B $NEW > gpurun_out/${TAG}_ab_cfg3.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B $NEW $B $NEW --workload cfg4 --no-config-check > gpurun_out/${TAG}_ab_cfg4.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B $NEW --workload cfg5 --no-config-check > gpurun_out/${TAG}_ab_cfg5.log 2>&1
echo done
