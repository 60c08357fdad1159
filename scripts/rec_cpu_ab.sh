#!/usr/bin/env bash
# RecordIO split A/B on the GPU box's CPU: reference vs this repo with chunks
# as file-mapping views (DMLC_SPLIT_MMAP=1) and read into buffers (=0),
# alternating, REPS rounds.  Lines "mode threads impl records_per_sec".
set -euo pipefail
OUT=${OUT:-gpurun_out/rec_ab}
DATA=${DATA:-/tmp/dmlc_cpu_baseline}
REPS=${REPS:-3}
mkdir -p "$OUT" "$DATA"
[ -e "$DATA/rec1m.done" ] || { timeout -k 10 300 build/dmlc_gen recordio 1000000 "$DATA/rec1m" 1 0 16 uniform && touch "$DATA/rec1m.done"; }
: > "$OUT/ab.txt"
for rep in $(seq "$REPS"); do
  for mode in record chunk; do
    for t in ${THREADS:-1 16}; do
      r=$(OMP_NUM_THREADS=$t timeout -k 10 120 build/refbench/ref_bench_split_cpu "$DATA/rec1m-0.rec" $mode 0 1 3 | grep -o 'records_per_sec": [0-9.]*' | cut -d' ' -f2)
      m=$(DMLC_SPLIT_MMAP=1 OMP_NUM_THREADS=$t timeout -k 10 120 build/dmlc_bench_split_cpu "$DATA/rec1m-0.rec" $mode 0 1 3 | grep -o 'records_per_sec": [0-9.]*' | cut -d' ' -f2)
      d=$(DMLC_SPLIT_MMAP=0 OMP_NUM_THREADS=$t timeout -k 10 120 build/dmlc_bench_split_cpu "$DATA/rec1m-0.rec" $mode 0 1 3 | grep -o 'records_per_sec": [0-9.]*' | cut -d' ' -f2)
      echo "$mode $t ref $r mmap $m read $d" | tee -a "$OUT/ab.txt"
    done
  done
done
