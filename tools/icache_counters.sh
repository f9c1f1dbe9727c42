set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES --kernel-trace --output-format csv -d gpurun_out/ic_E -o bench -- python3 bench.py --particles 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ic_E.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_WAVE32 SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_ACCUM_PREV_HIRES --kernel-trace --output-format csv -d gpurun_out/ic_F -o bench -- python3 bench.py --particles 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ic_F.log 2>&1 || true
echo done
