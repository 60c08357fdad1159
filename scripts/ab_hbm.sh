set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parser.py tests/test_gpu_long_records.py tests/test_gpu_public_api.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 600 python bench.py --mode hbm > gpurun_out/bench_hbm_ab$i.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/bench_hbm_ab$i.json'));print(d['value'],d['ms_per_step'])"
done
