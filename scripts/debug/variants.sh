set -o pipefail
cp dmlc_core_amd/lib/libdmlc.so /tmp/libdmlc_orig.so
for v in ${VARIANTS}; do
  cp build/variants/libdmlc_$v.so dmlc_core_amd/lib/libdmlc.so
  for m in ${MODES:-0}; do
    DMLC_FILL_EXP=$m timeout -k 10 100 python bench.py --steps 10 --warmup 1 --mode hbm > gpurun_out/var_$v_$m.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/var_$v_$m.json').read().strip().splitlines()[-1]); print('variant $v mode $m', round(d['value']/1e6,1), d['input_GBps'])"
  done
done
cp /tmp/libdmlc_orig.so dmlc_core_amd/lib/libdmlc.so
