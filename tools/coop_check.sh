# Cooperative point rounds: parity suite subset + A/B of cfg3/cfg2 against the round-start library.
# usage: bash tools/coop_check.sh <tag>
set -e
TAG=${1:-rXX}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_cooperative.py tests/test_gpu_parity.py tests/test_capi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
timeout -k 10 400 python tools/variant_bench.py build/variants/libfks_head.so fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+no-coop build/variants/libfks_head.so fast_kinematic_simulator_amd/libfks_hip.so > gpurun_out/${TAG}_ab_cfg3.log 2>&1
timeout -k 10 300 python tools/variant_bench.py build/variants/libfks_head.so fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+no-coop --workload cfg2 --no-config-check > gpurun_out/${TAG}_ab_cfg2.log 2>&1
echo done
