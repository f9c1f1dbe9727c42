# bench.py A/B: automatic segment length vs a fixed one, interleaved (cfg3)
# usage: bash tools/seg_ab.sh <k> [reps]
K=${1:-14}; REPS=${2:-3}
export TMPDIR=/tmp
for i in $(seq $REPS); do
  for k in -1 $K; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-config-check --steps 3 --segment-steps $k 2>/dev/null > /tmp/seg_ab.json || exit 1
    python3 -c "import json; d=json.loads(open('/tmp/seg_ab.json').read().strip().splitlines()[-1]); print($k, round(d['value']/1e6,2), round(d['roofline']['avg_kernel_ms'],2), round(d['wave_slots']['busy_fraction'],3))"
  done
done
