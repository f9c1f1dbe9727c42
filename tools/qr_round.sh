# A/B of two builds: parity subset, the heaviest cfg3 particles alone (tools/tail_latency.py),
# cfg3 and cfg4 batches.  usage: bash tools/qr_round.sh <baseline.so>
BASE=${1:-build/variants/libfks_head.so}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_branch_coverage.py tests/test_trace.py tests/test_sampled_actuator.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/qr_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/qr_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  FKS_LIB_PATH=$PWD/$BASE timeout -k 10 200 python tools/tail_latency.py --top 2 > gpurun_out/qr_tail_base$i.log 2>&1 || exit 1
  timeout -k 10 200 python tools/tail_latency.py --top 2 > gpurun_out/qr_tail_new$i.log 2>&1 || exit 1
  for f in base$i new$i; do echo $f $(grep -h '"kernel_ms"' gpurun_out/qr_tail_$f.log | tr -d ' \n'); done
done
timeout -k 10 900 python tools/variant_bench.py $BASE fast_kinematic_simulator_amd/libfks_hip.so $BASE fast_kinematic_simulator_amd/libfks_hip.so 2>&1 | cut -c1-110
timeout -k 10 900 python tools/variant_bench.py $BASE fast_kinematic_simulator_amd/libfks_hip.so $BASE fast_kinematic_simulator_amd/libfks_hip.so --workload cfg4 --no-config-check 2>&1 | cut -c1-110
