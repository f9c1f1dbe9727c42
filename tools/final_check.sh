# the round-end commands the driver runs, on the final tree: GPU suite, smoke, default bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03r_pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03r_bench.json 2> gpurun_out/r03r_bench.err
echo done
