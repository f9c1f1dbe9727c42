# lean LDS blocks: whole GPU suite, then cfg5 / cfg3 A/B against the previous build (+ a variant)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
NEW=fast_kinematic_simulator_amd/libfks_hip.so
B=build/variants/libfks_tile.so
V=build/variants/libfks_selfid.so
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03l_pytest_gpu.log 2>&1
timeout -k 10 600 python tools/variant_bench.py $B $NEW $B $NEW --workload cfg5 --no-config-check > gpurun_out/r03l_ab_cfg5.log 2>&1
timeout -k 10 700 python tools/variant_bench.py $B $NEW $V $B $NEW $V > gpurun_out/r03l_ab_cfg3.log 2>&1
echo done
