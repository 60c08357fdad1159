set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 1250000 2500000 5000000; do
  timeout -k 10 300 python bench.py --rows $r --steps 10 --warmup 2 > gpurun_out/probe_$r.json 2> gpurun_out/probe_$r.err || exit $?
  cut -c1-400 gpurun_out/probe_$r.json
done
