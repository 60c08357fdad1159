#!/bin/bash
# Ingest on realistic row shapes: stream and HBM-resident
# epochs of uniform / skewed / mixed synthetic data, one JSON line each.
# usage (through gpurun): bash scripts/bench_shapes.sh OUTDIR [format] [rows]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=gpurun_out/$1
fmt=${2:-libsvm}
rows=${3:-10000000}
mkdir -p "$out"
export TMPDIR=/tmp
for shape in uniform skewed mixed; do
  # skewed / mixed rows are ~4x shorter (Pareto nnz): 4x the rows, so every
  # shape parses about the same bytes (fixed per-epoch costs weigh the same)
  n=$rows
  [ "$shape" != uniform ] && n=$((rows * 4))
  for mode in ${MODES:-stream hbm}; do
    timeout -k 10 400 python bench.py --format $fmt --shape $shape --mode $mode --rows $n \
      --steps 5 --warmup 2 > "$out/${fmt}_${shape}_${mode}.json" 2> "$out/${fmt}_${shape}_${mode}.err" \
      || { tail -20 "$out/${fmt}_${shape}_${mode}.err"; exit 1; }
    python - "$out/${fmt}_${shape}_${mode}.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d.get("parser_stats_last_rank0", {})
print(d["shape"], d["mode"], "rows/s %.3g" % d["value"], "GB/s %.1f" % d["input_GBps"],
      "exact_chunks %s/%s" % (st.get("exact_chunks"), st.get("chunks")), flush=True)
PY
  done
done
