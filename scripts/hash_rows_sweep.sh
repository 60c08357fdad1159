#!/bin/bash
# fused hashed-batch kernel: rows built per LDS round (DMLC_HASH_ROWS) sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "hash" -p no:cacheprovider > gpurun_out/pytest_hash.log 2>&1
rc=$?; echo "pytest hash rc=$rc"; tail -3 gpurun_out/pytest_hash.log; [ $rc -eq 0 ] || exit $rc
for r in ${ROWS_LIST:-default 4 8 16 32}; do
  if [ $r = default ]; then unset DMLC_HASH_ROWS; else export DMLC_HASH_ROWS=$r; fi
  timeout -k 10 300 python scripts/bench_hashed.py > gpurun_out/hashed_rows_$r.json 2> gpurun_out/hashed_rows_$r.err
  rc=$?; echo "rows=$r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/hashed_rows_$r.json'));print({k:v for k,v in d['dim_sweep_ms'].items()})"
done
