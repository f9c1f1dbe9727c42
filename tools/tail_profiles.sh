# heaviest particles alone + batch phase shares (profiling build) for cfg2 / cfg3 / cfg5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=$PWD/build/variants/libfks_phase.so
for w in cfg2 cfg3 cfg5; do
  FKS_LIB_PATH=$P FKS_VARIANT_LIB=1 timeout -k 10 400 python tools/tail_latency.py --workload $w --top 2 --json gpurun_out/r03s_tail_$w.json > gpurun_out/r03s_tail_$w.log 2>&1 || exit 1
done
echo done
