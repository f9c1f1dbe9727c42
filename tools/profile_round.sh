set -o pipefail
mkdir -p gpurun_out/${ROUND_TAG:-r01g}
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-check"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${ROUND_TAG:-r01g}/trace -o bench -- $B > gpurun_out/${ROUND_TAG:-r01g}/bench_under_rocprof.json 2> gpurun_out/${ROUND_TAG:-r01g}/trace.err && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${ROUND_TAG:-r01g}/pmc_fetch -o bench -- $B > gpurun_out/${ROUND_TAG:-r01g}/fetch.out 2> gpurun_out/${ROUND_TAG:-r01g}/fetch.err && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${ROUND_TAG:-r01g}/pmc_write -o bench -- $B > gpurun_out/${ROUND_TAG:-r01g}/write.out 2> gpurun_out/${ROUND_TAG:-r01g}/write.err && \
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/${ROUND_TAG:-r01g}/pmc_tcc -o bench -- $B > gpurun_out/${ROUND_TAG:-r01g}/tcc.out 2> gpurun_out/${ROUND_TAG:-r01g}/tcc.err && \
echo PROFILES_DONE
