# SQ / TA / TCP / TCC counter passes of a 16k-particle cfg3 bench (separate --pmc runs, kernel-trace only).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq}
run() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/${TAG}_$name -o bench -- python3 bench.py --particles 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/${TAG}_$name.log 2>&1
}
run A SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES
run B SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA
run C TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_BUSY_avr GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
run D SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_IFETCH
echo done
