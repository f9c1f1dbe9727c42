# VALU / issue utilisation of the simulation kernel (separate rocprofv3 --pmc passes)
set -o pipefail
T=${ROUND_TAG:-r01j}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check"
timeout -s KILL 180 rocprofv3 --pmc VALUBusy --kernel-trace --output-format csv -d gpurun_out/$T/pmc_valubusy -o bench -- $B > /dev/null 2> gpurun_out/$T/valubusy.err && \
timeout -s KILL 180 rocprofv3 --pmc VALUUtilization --kernel-trace --output-format csv -d gpurun_out/$T/pmc_valuutil -o bench -- $B > /dev/null 2> gpurun_out/$T/valuutil.err && \
timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/$T/pmc_issue -o bench -- $B > /dev/null 2> gpurun_out/$T/issue.err && \
echo VALU_DONE
