set -u
cd $GRAFT_REPO_ROOT
for args in "--depth 8" "--depth 1" "--depth 2" "--depth 8 --scene csg256_balanced" "--depth 1 --scene csg256_balanced"; do
  for bml in 2 100000; do
    WOLOLO_BOUND_MIN_LEAVES=$bml timeout -k 10 150 python bench.py --steps 5 --warmup 1 --no-cpu-baseline $args > gpurun_out/e.json 2>gpurun_out/e.err || { echo FAIL; tail -3 gpurun_out/e.err; exit 1; }
    python3 -c "import json; j=json.loads(open('gpurun_out/e.json').read().strip().splitlines()[-1]); print('$args bml=$bml', j['ms_per_step'], j['segments_per_frame'], round(j['ms_per_step']*1e6/j['segments_per_frame'],4), 'ns/seg')"
  done
done
