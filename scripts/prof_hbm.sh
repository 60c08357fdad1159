#!/bin/bash
# GPU suite + kernel trace of the HBM-resident parse (bench --mode hbm)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_hbm
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hbm -o run --output-format csv -- \
  python3 bench.py --mode hbm --steps 3 --warmup 1 > gpurun_out/prof_hbm.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_hbm.log; [ $rc -eq 0 ] || exit $rc
if [ -n "${WITH_BENCH:-}" ]; then
  for m in stream hbm; do
    timeout -k 10 600 python bench.py --mode $m > gpurun_out/bench_$m.json 2> gpurun_out/bench_$m.err
    rc=$?; echo "bench $m rc=$rc"; cut -c1-300 gpurun_out/bench_$m.json; [ $rc -eq 0 ] || exit $rc
  done
fi
