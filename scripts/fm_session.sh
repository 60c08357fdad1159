#!/usr/bin/env bash
# HashedFM step on the GPU box: the FM numerics tests, the step timing of
# scripts/bench_hashed.py, a kernel trace and a VALU / MFMA counter pass of
# the fused step.  OUT=gpurun_out/fm TAG=...
set -uo pipefail
OUT=${OUT:-gpurun_out/fm}
TAG=${TAG:-fm}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_hashed.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "fm" > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -2 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_hashed.py --sweep 1024 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT/${TAG}_bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d[k] for k in d if k.startswith("hashed_fm")})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$TAG" -o run --output-format csv -- \
  python scripts/bench_hashed.py --sweep 1024 --steps 5 > "$OUT/${TAG}_trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$OUT/trace_$TAG" -name "*kernel_stats.csv" | head -1)
grep -E "k_fm|Name" "$f" | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$OUT/pmc_$TAG" -o run --output-format csv -- python scripts/bench_hashed.py --sweep 1024 --steps 2 \
  > "$OUT/${TAG}_pmc.log" 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 - "$OUT/pmc_$TAG" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "k_fm" not in r["Kernel_Name"]:
        continue
    k = r["Kernel_Name"].split("(")[0][-40:]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    acc[k]["_n"] += 1.0 / 6
for k, v in acc.items():
    w = v["SQ_WAVES"]
    print(k, {c: round(v[c] / w, 1) for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES")}, "waves", w)
PY
