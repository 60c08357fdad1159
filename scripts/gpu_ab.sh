set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests ${PYTEST_SEL:--m gpu} -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/ab/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 200 python bench.py --mode hbm --steps 10 --warmup 2 > gpurun_out/ab/bench_hbm_$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/ab/bench_hbm_$i.json'));print(d['value'],d['input_GBps'],d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof -o run --output-format csv -- python3 bench.py --mode hbm --steps 5 --warmup 1 > gpurun_out/ab/prof.log 2>&1 || exit $?
f=$(find gpurun_out/ab/prof -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -d, -f1-8
