#!/bin/bash
# One GPU iteration: parser parity tests, HBM-resident + stream benches, and a
# rocprofv3 kernel-time profile of the HBM bench.  Usage: scripts/gpu_iter.sh <outdir> [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/iter}
K=${2:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
fi
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --mode hbm > "$OUT/bench_hbm.json" 2> "$OUT/bench_hbm.err" || { echo "hbm bench failed"; tail "$OUT/bench_hbm.err"; exit 1; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench_stream.json" 2> "$OUT/bench_stream.err" || { echo "stream bench failed"; tail "$OUT/bench_stream.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --mode hbm > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; tail "$OUT/prof.log"; exit 1; }
python - "$OUT" <<'PY'
import json, sys, glob
out = sys.argv[1]
for f in ("bench_hbm.json", "bench_stream.json"):
    d = json.loads(open(f"{out}/{f}").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 1), "M rows/s", d["input_GBps"], "GB/s")
for p in glob.glob(f"{out}/prof/**/*kernel_stats.csv", recursive=True):
    print(open(p).read()[:3000])
PY
