# Interleaved A/B of kernel builds on one box (bench.py per library, tools/variant_bench.py).
# usage: bash tools/variant_ab.sh <tag> "<bench args>" lib1 lib2 ... (each lib may carry +flag)
TAG=$1; ARGS=$2; shift 2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python tools/variant_bench.py "$@" $ARGS > gpurun_out/${TAG}_ab.log 2>&1
