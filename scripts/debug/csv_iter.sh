#!/bin/bash
# CSV parity tests, CSV benches (stream + HBM) and a kernel profile of the HBM run.
OUT=gpurun_out/${1:-csv_iter}
mkdir -p $OUT && cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_parser.py tests/test_gpu_public_api.py -x -q --timeout 120 --timeout-method thread -k "csv or shuffled" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash scripts/bench_all_formats.sh $OUT/f csv || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --format csv --mode hbm --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit 1
grep -E "k_csv" $OUT/prof/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-50,150-220
