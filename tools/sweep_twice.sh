# two passes of tools/sched_sweep.py over the knobs near the defaults (noise check)
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in a b; do
  timeout -k 10 300 python tools/sched_sweep.py --segments ${SEGS:-8,10,14} --heavy ${HEAVY:-1,2,3} --prio ${PRIO:-1,2} --json gpurun_out/r02ar_sched_sweep_$p.json > gpurun_out/sweep_$p.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
a = json.load(open("gpurun_out/r02ar_sched_sweep_a.json"))["rows"]
b = json.load(open("gpurun_out/r02ar_sched_sweep_b.json"))["rows"]
for x, y in zip(a, b):
    print(x["segment_steps"], x["heavy_resolver_per_step"], x["heavy_priority"], round(x["kernel_ms"], 1), round(y["kernel_ms"], 1))
PY
