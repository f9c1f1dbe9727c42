# joint-proof round: full GPU suite (stop on failure), verification build with the proof on
# (every proven microstep re-checked in full: error_particles must stay 0), A/B benches.
# usage: bash tools/jp_check.sh <tag> <lib[+flag]> [...]
# the verification build first, on the CPU side:
#   python -c "from fast_kinematic_simulator_amd.build import build_variant; \
#              build_variant('build/variants/libfks_verify.so', ['FKS_VERIFY_JP=1'])"
# (a baseline library for the A/B: the same sources at another commit, built with build_variant)
TAG=${1:-jpc}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { case $1 in 124|134|137|139) return 1;; *) return 0;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for w in cfg3 cfg2 cfg5; do
  timeout -k 10 300 python tools/variant_bench.py build/variants/libfks_verify.so+joint-proof --workload $w --no-config-check > gpurun_out/${TAG}_verify_$w.log 2>&1
  rc=$?; echo "verify $w rc=$rc"; cut -c1-300 gpurun_out/${TAG}_verify_$w.log; ok $rc || exit $rc
done
timeout -k 10 700 python tools/variant_bench.py "$@" "$@" > gpurun_out/${TAG}_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cut -c1-300 gpurun_out/${TAG}_ab.log
exit 0
