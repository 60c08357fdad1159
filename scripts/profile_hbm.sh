#!/bin/bash
# rocprofv3 kernel statistics of the HBM-resident parse (bench.py --mode hbm)
# for LibSVM, CSV and RecordIO, plus the plain bench JSON of each.
# usage (through gpurun): bash scripts/profile_hbm.sh OUTDIR [formats...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=gpurun_out/$1; shift
fmts=${*:-libsvm csv recordio}
mkdir -p "$out"
export TMPDIR=/tmp
for f in $fmts; do
  timeout -k 10 300 python bench.py --mode hbm --format $f --steps 10 --warmup 2 \
    > "$out/bench_$f.json" 2> "$out/bench_$f.err" || { tail -20 "$out/bench_$f.err"; exit 1; }
  tail -c 600 "$out/bench_$f.json"; echo
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$f" \
    -o run -- python "$GRAFT_REPO_ROOT/bench.py" --mode hbm --format $f --steps 5 --warmup 2 \
    > "$GRAFT_REPO_ROOT/$out/prof_$f.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$out/prof_$f.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
done
find "$out" -name "*kernel_stats.csv" | head
