cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
FKS_LIB_PATH=$PWD/build/variants/libfks_phase.so FKS_VARIANT_LIB=1 timeout -k 10 200 python tools/tail_latency.py --top 2 --json gpurun_out/r03e_tail_coop.json > gpurun_out/r03e_tail_coop.log 2>&1 &&
FKS_LIB_PATH=$PWD/build/variants/libfks_phase.so FKS_VARIANT_LIB=1 timeout -k 10 200 python tools/tail_latency.py --top 2 --no-coop --json gpurun_out/r03e_tail_nocoop.json > gpurun_out/r03e_tail_nocoop.log 2>&1 &&
timeout -k 10 200 python tools/tail_latency.py --top 2 --json gpurun_out/r03e_tail_plain_coop.json > gpurun_out/r03e_tail_plain_coop.log 2>&1 &&
timeout -k 10 200 python tools/tail_latency.py --top 2 --no-coop --json gpurun_out/r03e_tail_plain_nocoop.json > gpurun_out/r03e_tail_plain_nocoop.log 2>&1 && echo done
timeout -k 10 500 python -u -m pytest tests/test_cooperative.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1 &&
timeout -k 10 400 python tools/variant_bench.py build/variants/libfks_head.so fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+no-coop build/variants/libfks_head.so fast_kinematic_simulator_amd/libfks_hip.so fast_kinematic_simulator_amd/libfks_hip.so+no-coop > gpurun_out/r03e_ab_cfg3.log 2>&1 && echo done2
