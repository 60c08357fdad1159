#!/usr/bin/env bash
# Text parser A/B on the GPU box's CPU: reference vs this repo's library in
# build/ab_old (LD_LIBRARY_PATH) vs the current one, alternating, REPS rounds.
# Lines "dataset threads ref R old O new N" (rows/s).
set -euo pipefail
OUT=${OUT:-gpurun_out/parser_ab}
DATA=${DATA:-/tmp/dmlc_cpu_baseline}
REPS=${REPS:-3}
mkdir -p "$OUT" "$DATA"
gen() { [ -e "$DATA/$3.done" ] || { timeout -k 10 300 build/dmlc_gen "$1" "$2" "$DATA/$3" 1 0 16 uniform && touch "$DATA/$3.done"; }; }
gen csv 1000000 csv1m
gen libsvm 1000000 ls1m
: > "$OUT/ab.txt"
rate() { grep -o 'rows_per_sec": [0-9.]*' | cut -d' ' -f2; }
for rep in $(seq "$REPS"); do
  for ds in "csv1m-0.csv?format=csv&label_column=0 csv" "ls1m-0.libsvm libsvm"; do
    set -- $ds
    for t in ${THREADS:-8 16}; do
      r=$(OMP_NUM_THREADS=$t timeout -k 10 120 build/refbench/ref_bench_cpu "$DATA/$1" $2 0 1 3 | rate)
      o=$(LD_LIBRARY_PATH=build/ab_old OMP_NUM_THREADS=$t timeout -k 10 120 build/dmlc_bench_cpu "$DATA/$1" $2 0 1 3 | rate)
      n=$(OMP_NUM_THREADS=$t timeout -k 10 120 build/dmlc_bench_cpu "$DATA/$1" $2 0 1 3 | rate)
      echo "$2 $t ref $r old $o new $n" | tee -a "$OUT/ab.txt"
    done
  done
done
