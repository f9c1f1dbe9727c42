# Phase cost by repetition (run on the GPU box): for each build of tools/phase_cost.py
# (FKS_PROF_DUP bit b = phase b run twice with identical inputs/outputs), one cfg3 bench
# launch under one rocprofv3 SQ instruction-count pass; tools/phase_cost.py turns the
# differences against the plain build into per-phase instruction and time costs.
# usage: bash tools/phase_cost.sh <tag> build/prof/p_*.so
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check"
for lib in "$@"; do
  n=$(basename $lib .so)
  FKS_LIB_PATH=$PWD/$lib timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/$TAG/$n -o bench -- $B > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || exit 1
  echo "$n done"
done
