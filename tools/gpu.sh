# One parametrised GPU-box tool (run through gpurun from the repository root).  Each step
# runs under its own time limit and the chain stops at the first failure.
#
# usage: bash tools/gpu.sh <tag> <task> [<task> ...]
#   suite              pytest -m gpu (whole suite)                  -> <tag>_pytest_gpu.log
#   suitelib:<lib>     the same suite against a variant library  -> <tag>_pytest_gpu_<lib>.log
#   tests:<file>       pytest -m gpu of one test file (tests/<file>.py) -> <tag>_pytest_<file>.log
#   testslib:<file>:<lib>  the same against a variant library -> <tag>_pytest_<file>_<lib>.log
#   smoke              __graft_entry__.smoke()                      -> <tag>_smoke.log
#   bench[:cfgN]       bench.py (default workload, or --workload cfgN) -> <tag>_bench[_cfgN].json
#   others             bench lines of cfg1 / cfg2 / cfg4 / cfg5
#   trace              rocprofv3 --kernel-trace --stats of bench.py -> <tag>_trace/
#   pmc                FETCH_SIZE / WRITE_SIZE / TCC hit+miss, one --pmc pass each -> <tag>_pmc_*/
#   pmc:<wl>           the same three passes on another workload  -> <tag>_pmc_<wl>_*/
#   counters           rocprofv3 --list-avail                        -> <tag>_counters.txt
#   icache             instruction-cache, instruction-wait and LDS-conflict counters, one pass -> <tag>_icache/
#   valu               VALUBusy / VALUUtilization / SQ issue counters, one pass each -> <tag>_valu/
#   ab:<wl>:<libs>     interleaved bench.py of comma-separated libraries (each may carry +flag;
#                      "L" = the product library) on workload <wl>  -> <tag>_ab_<wl>.log
#   tail:<wl>:<lib>    heaviest particles alone + phase shares (tools/tail_latency.py) -> <tag>_tail_<wl>_<lib>.json
#   tailsmall:<wl>:<lib>  the same, the lone particles on the one-wave small-batch kernel
#                      -> <tag>_tailsmall_<wl>_<lib>.json
#   tailcoop:<wl>:<lib>   the same, the lone particles on the cooperative kernel -> <tag>_tailcoop_<wl>_<lib>.json
#   tailpmc:<wl>:<lib> instruction-mix and wait counters of the batch and the heaviest particle
#                      alone (three --pmc passes over tools/tail_latency.py --top 1) -> <tag>_tailpmc_<wl>_<lib>/
#   sched:<wl>:<segs>:<heavy>[:<rel>]  scheduling sweep (tools/sched_sweep.py; comma lists of segment lengths,
#                      heavy thresholds and relative factors (default 3), priority 1) -> <tag>_sched_<wl>.json
#   torchrun1          bench.py through torch.distributed.run, world size 1 (RCCL) -> <tag>_torchrun_w1.json
#   inproc:<devices>   bench.py --in-process over a device list (e.g. 0 or 0,0) with the strong-scaling
#                      projection -> <tag>_inproc_<devices>.json
#   round              suite smoke bench trace pmc others
set -o pipefail
TAG=$1
shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
L=fast_kinematic_simulator_amd/libfks_hip.so
# variant libraries (build/variants) compile their shape-specialised kernels with the product's helper
export FKS_SHAPEC=$PWD/fast_kinematic_simulator_amd/fks_shapec
# profiled runs find their shape-specialised kernels compiled by an unprofiled run beforehand
# (warm), so no compiler process starts under rocprofv3
export FKS_KERNEL_CACHE=/tmp/fks_kernel_cache_$TAG
warm() { timeout -k 10 300 "$@" > /dev/null 2>&1; }
BP="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline-batches 0 --no-projection"
lib() { [ "$1" = L ] && echo $L || echo "$1"; }

run_task() {
  case "$1" in
  suite) timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/${TAG}_pytest_gpu.log 2>&1 ;;
  suitelib:*) l=$(lib ${1#suitelib:}); FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/${TAG}_pytest_gpu_$(basename $l .so).log 2>&1 ;;
  tests:*) f=${1#tests:}; timeout -k 10 600 python -u -m pytest tests/$f.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/${TAG}_pytest_$f.log 2>&1 ;;
  testslib:*) spec=${1#testslib:}; f=${spec%%:*}; l=$(lib ${spec#*:}); FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1 timeout -k 10 600 python -u -m pytest tests/$f.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/${TAG}_pytest_${f}_$(basename $l .so).log 2>&1 ;;
  smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 ;;
  bench) timeout -k 10 400 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err ;;
  bench:*) w=${1#bench:}; timeout -k 10 300 python bench.py --workload $w --no-config-check > $O/${TAG}_bench_$w.json 2> $O/${TAG}_bench_$w.err ;;
  others) for w in cfg1 cfg2 cfg4 cfg5; do run_task bench:$w || return $?; done ;;
  trace) warm $BP && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_trace -o bench -- $BP > $O/${TAG}_bench_under_rocprof.json 2> $O/${TAG}_trace.err ;;
  pmc)
    warm $BP &&
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${TAG}_pmc_fetch -o bench -- $BP > /dev/null 2> $O/${TAG}_pmc_fetch.err &&
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${TAG}_pmc_write -o bench -- $BP > /dev/null 2> $O/${TAG}_pmc_write.err &&
    timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/${TAG}_pmc_tcc -o bench -- $BP > /dev/null 2> $O/${TAG}_pmc_tcc.err ;;
  pmc:*)
    w=${1#pmc:}; BW="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config-check --pipeline-batches 0 --no-projection --workload $w"
    warm $BW &&
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${TAG}_pmc_${w}_fetch -o bench -- $BW > /dev/null 2> $O/${TAG}_pmc_${w}_fetch.err &&
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${TAG}_pmc_${w}_write -o bench -- $BW > /dev/null 2> $O/${TAG}_pmc_${w}_write.err &&
    timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/${TAG}_pmc_${w}_tcc -o bench -- $BW > /dev/null 2> $O/${TAG}_pmc_${w}_tcc.err ;;
  valu)
    B1="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check --pipeline-batches 0 --no-projection"
    mkdir -p $O/${TAG}_valu
    warm $B1 &&
    timeout -s KILL 180 rocprofv3 --pmc VALUBusy --kernel-trace --output-format csv -d $O/${TAG}_valu/valubusy -o bench -- $B1 > /dev/null 2> $O/${TAG}_valu/valubusy.err &&
    timeout -s KILL 180 rocprofv3 --pmc VALUUtilization --kernel-trace --output-format csv -d $O/${TAG}_valu/valuutil -o bench -- $B1 > /dev/null 2> $O/${TAG}_valu/valuutil.err &&
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/${TAG}_valu/issue -o bench -- $B1 > /dev/null 2> $O/${TAG}_valu/issue.err ;;
  counters) timeout -k 10 120 rocprofv3 --list-avail > $O/${TAG}_counters.txt 2>&1 ;;
  icache)
    B1="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check --pipeline-batches 0 --no-projection"
    mkdir -p $O/${TAG}_icache
    warm $B1 &&
    timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/${TAG}_icache/ic -o bench -- $B1 > /dev/null 2> $O/${TAG}_icache/ic.err ;;
  ab:*)
    spec=${1#ab:}; w=${spec%%:*}; libs=${spec#*:}; args=()
    for x in ${libs//,/ }; do args+=("$(lib ${x%%+*})${x#${x%%+*}}"); done
    extra=""; [ "$w" != cfg3 ] && extra="--workload $w --no-config-check"
    timeout -k 10 1000 python tools/variant_bench.py "${args[@]}" $extra > $O/${TAG}_ab_$w.log 2>&1 ;;
  tail:*)
    spec=${1#tail:}; w=${spec%%:*}; l=$(lib ${spec#*:}); n=$(basename $l .so)
    FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1 timeout -k 10 400 python tools/tail_latency.py --workload $w --top 3 --json $O/${TAG}_tail_${w}_$n.json > $O/${TAG}_tail_${w}_$n.log 2>&1 ;;
  tailsmall:*|tailcoop:*)
    kind=${1%%:*}; spec=${1#*:}; w=${spec%%:*}; l=$(lib ${spec#*:}); n=$(basename $l .so)
    lone=small; [ $kind = tailcoop ] && lone=cooperative
    FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1 timeout -k 10 400 python tools/tail_latency.py --workload $w --top 3 --lone $lone --json $O/${TAG}_${kind}_${w}_$n.json > $O/${TAG}_${kind}_${w}_$n.log 2>&1 ;;
  tailpmc:*)
    spec=${1#tailpmc:}; w=${spec%%:*}; l=$(lib ${spec#*:}); n=$(basename $l .so); D=$O/${TAG}_tailpmc_${w}_$n
    T1="python3 tools/tail_latency.py --workload $w --top 1"
    export FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1
    warm $T1 &&
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $D/mix -o tail -- $T1 > $D.mix.log 2>&1 &&
    timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $D/wait -o tail -- $T1 > $D.wait.log 2>&1 &&
    timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d $D/valu -o tail -- $T1 > $D.valu.log 2>&1
    rc=$?; unset FKS_LIB_PATH FKS_VARIANT_LIB; return $rc ;;
  mix:*)
    spec=${1#mix:}; w=${spec%%:*}; l=$(lib ${spec#*:}); n=$(basename $l .so); D=$O/${TAG}_mix_${w}_$n
    BM="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-config-check --pipeline-batches 0 --no-projection --workload $w"
    export FKS_LIB_PATH=$PWD/$l FKS_VARIANT_LIB=1
    warm $BM &&
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $D/mix -o m -- $BM > $D.mix.log 2>&1 &&
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $D/wait -o m -- $BM > $D.wait.log 2>&1 &&
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $D/more -o m -- $BM > $D.more.log 2>&1
    rc=$?; unset FKS_LIB_PATH FKS_VARIANT_LIB; return $rc ;;
  sched:*)
    spec=${1#sched:}; w=${spec%%:*}; rest=${spec#*:}; seg=${rest%%:*}; rest=${rest#*:}; heavy=${rest%%:*}; rel=3
    [ "$rest" != "$heavy" ] && rel=${rest#*:}
    np=""; [ "$w" = cfg4 -o "$w" = cfg5 ] && np="--particles 131072"
    timeout -k 10 600 python tools/sched_sweep.py --workload $w $np --segments $seg --heavy $heavy --prio 1 --rel $rel --json $O/${TAG}_sched_$w.json > $O/${TAG}_sched_$w.log 2>&1 ;;
  inproc:*) d=${1#inproc:}; timeout -k 10 400 python bench.py --in-process --devices $d --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_inproc_${d//,/}.json 2> $O/${TAG}_inproc_${d//,/}.err ;;
  torchrun1) timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/${TAG}_torchrun_w1.json 2> $O/${TAG}_torchrun_w1.err ;;
  round) for t in suite smoke bench trace pmc others; do run_task $t || return $?; done ;;
  *) echo "unknown task $1" >&2; return 2 ;;
  esac
}

for t in "$@"; do
  echo "[$(date +%T)] $t"
  run_task "$t" || { rc=$?; echo "task $t failed: $rc"; exit $rc; }
done
echo done
