#!/usr/bin/env bash
# Same-host CPU baseline ("must be re-measured on the MI355X
# host's CPU before claiming speedups").
#
# On the GPU box: the reference's own parsers (built from /root/reference by
# `make refbench`, harness = tools/dmlc_bench_cpu.cc / dmlc_bench_split_cpu.cc,
# public API only) and this repo's parity CPU parsers, on the survey's dataset
# shapes (1 M rows: LibSVM 20-60 nnz, LibFM 20-60 triples, CSV 29 columns,
# RecordIO 512 B) plus the headline's 10 M-row LibSVM shard, at 1 / 8 / 16
# OpenMP threads (16 = this box's CPU share).  JSON lines -> $OUT/cpu.jsonl.
set -euo pipefail
OUT=${OUT:-gpurun_out/r06_cpu}
REPS=${REPS:-2}
DATA=${DATA:-/tmp/dmlc_cpu_baseline}
THREADS=${THREADS:-"1 8 16"}
mkdir -p "$OUT" "$DATA"
B=build
R=build/refbench
{
  echo "host: $(hostname)"
  lscpu | grep -E "Model name|^CPU\(s\)|NUMA node|Thread|Socket|MHz" || true
  echo "affinity: $(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"
} > "$OUT/host.txt"
gen() {  # format rows name
  [ -e "$DATA/$3.done" ] || { timeout -k 10 300 $B/dmlc_gen "$1" "$2" "$DATA/$3" 1 0 16 uniform && touch "$DATA/$3.done"; }
}
gen libsvm 1000000 ls1m
gen libfm 1000000 fm1m
gen csv 1000000 csv1m
gen recordio 1000000 rec1m
gen libsvm 10000000 ls10m
J="$OUT/cpu.jsonl"
: > "$J"
run() {  # tag threads cmd...
  local tag=$1 t=$2
  shift 2
  local line
  line=$(OMP_NUM_THREADS=$t timeout -k 10 300 "$@" | tail -1)
  echo "{\"impl\": \"$tag\", \"omp_threads\": $t, \"result\": $line}" | tee -a "$J"
}
# ref and repo alternate, REPS rounds (best of all of them is reported by
# scripts/cpu_table.py): a page-cache or clock swing hits both alike
for rep in $(seq "$REPS"); do
for t in $THREADS; do
  for impl in ref repo; do
    if [ $impl = ref ]; then P=$R/ref_bench_cpu; S=$R/ref_bench_split_cpu; else P=$B/dmlc_bench_cpu; S=$B/dmlc_bench_split_cpu; fi
    run $impl "$t" $P "$DATA/ls1m-0.libsvm" libsvm 0 1 3
    run $impl "$t" $P "$DATA/fm1m-0.libfm" libfm 0 1 3
    run $impl "$t" $P "$DATA/csv1m-0.csv?format=csv&label_column=0" csv 0 1 3
    run $impl "$t" $S "$DATA/rec1m-0.rec" record 0 1 3
    run $impl "$t" $S "$DATA/rec1m-0.rec" chunk 0 1 3
    run $impl "$t" $P "$DATA/ls10m-0.libsvm" libsvm 0 1 2
  done
done
done
python3 scripts/cpu_table.py "$J" > "$OUT/table.md" && cat "$OUT/table.md"
echo "cpu baseline done: $J"
