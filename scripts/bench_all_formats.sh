#!/bin/bash
# Every format through bench.py on one GPU, stream and HBM-resident modes.
# usage: scripts/bench_all_formats.sh <outdir> [formats...]
set -o pipefail
OUT=${1:-gpurun_out/formats}
shift
FORMATS=${@:-libsvm libfm csv recordio}
mkdir -p "$OUT"
for f in $FORMATS; do
  for mode in stream hbm; do
    timeout -k 10 400 python bench.py --format $f --mode $mode --steps 10 --warmup 3 \
      > "$OUT/bench_${f}_${mode}.json" 2> "$OUT/bench_${f}_${mode}.err" || { echo "$f $mode failed"; tail -5 "$OUT/bench_${f}_${mode}.err"; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_${f}_${mode}.json').read().strip().splitlines()[-1]); print('$f $mode', round(d['value']/1e6,2), d['unit'], d['input_GBps'], 'GB/s', 'x', d['vs_baseline'])"
  done
done
