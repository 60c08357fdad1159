set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in ${MODES:-0 1}; do
  DMLC_FILL_EXP=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/exp_prof_$m -o run --output-format csv -- python bench.py --steps 10 --warmup 1 --mode hbm > gpurun_out/exp_$m.json 2>gpurun_out/exp_$m.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/exp_$m.json').read().strip().splitlines()[-1]); print('mode $m', d['value']/1e6, d['input_GBps'])"
  python - $m <<'PY'
import csv, glob, sys, collections, re
m = sys.argv[1]
f = glob.glob(f"gpurun_out/exp_prof_{m}/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for row in csv.DictReader(open(f)):
    k = re.search(r"(k_\w+)", row["Kernel_Name"])
    k = k.group(1) if k else row["Kernel_Name"][:30]
    agg[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    v.sort()
    print(f"  {k:32s} n={len(v):4d} total={sum(v)/1e3:8.2f}ms max={v[-1]:9.1f}us")
PY
done
