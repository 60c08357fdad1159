mkdir -p gpurun_out/hash1 && cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_hashed.py tests/test_gpu_parser.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hash1/pytest.log 2>&1 || { tail -30 gpurun_out/hash1/pytest.log; exit 1; }
tail -2 gpurun_out/hash1/pytest.log
timeout -k 10 400 python scripts/bench_hashed.py --sweep 128,256,512,1024 > gpurun_out/hash1/bench.json 2> gpurun_out/hash1/bench.err || { tail gpurun_out/hash1/bench.err; exit 1; }
cat gpurun_out/hash1/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hash1/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --mode hbm > gpurun_out/hash1/prof.log 2>&1 || exit 1
grep -E "k_tile_count|k_tile_fill" gpurun_out/hash1/prof/run_kernel_stats.csv | cut -d, -f2-4 | tail -4
tail -1 gpurun_out/hash1/prof.log | cut -c1-200
