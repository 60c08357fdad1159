#!/bin/bash
# r05: fused HashedFM step, transpose workspace, RecordIO chain count on one box.
set -o pipefail
out=gpurun_out/r05_fm
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_hashed.py -k "fm_" > $out/pytest.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_recordio.py > $out/pytest_rec.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_ops.py -k "transpose" > $out/pytest_transpose.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu -k "csv or CSV" > $out/pytest_csv.log 2>&1 &&
timeout -k 10 300 python -u bench.py --mode hbm --format csv --steps 10 --warmup 2 > $out/bench_csv.json 2> $out/bench_csv.err &&
timeout -k 10 400 python -u scripts/bench_hashed.py --sweep "" --steps 20 > $out/bench.json 2> $out/bench.err &&
timeout -k 10 300 python -u bench.py --mode hbm --format recordio --steps 10 --warmup 2 > $out/bench_rec.json 2> $out/bench_rec.err &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_hashed.py" --sweep "" --steps 10 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1) &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_rec" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --mode hbm --format recordio --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/$out/prof_rec.log" 2>&1) &&
timeout -k 10 400 python -u scripts/bench_linear.py > $out/bench_linear.json 2> $out/bench_linear.err &&
bash scripts/csv_pricing.sh r05_fm/csv > $out/csv_pricing.log 2>&1
