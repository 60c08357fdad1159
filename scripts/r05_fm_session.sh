set -o pipefail
mkdir -p gpurun_out/r05_fm
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_hashed.py -k "fm_" > gpurun_out/r05_fm/pytest.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_hashed.py --sweep "" --steps 20 > gpurun_out/r05_fm/bench.json 2> gpurun_out/r05_fm/bench.err &&
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r05_fm/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_hashed.py" --sweep "" --steps 10 > "$GRAFT_REPO_ROOT/gpurun_out/r05_fm/prof.log" 2>&1)
