#!/usr/bin/env bash
# Runs bench.py once per case and appends "<label> <scene> <ms/frame> <kernel ms> <path>"
# to gpurun_out/matrix.txt.  A case is "label|ENV=V ENV2=V2|bench args"; stops at the
# first failing run.
#   tools/bench_matrix.sh "lanes|WOLOLO_TRACER=lanes|--scene rtiow_cover --steps 3" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    label="${spec%%|*}"
    rest="${spec#*|}"
    envs="${rest%%|*}"
    args="${rest#*|}"
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/m.json 2> gpurun_out/m.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$label] rc=$rc"; tail -5 gpurun_out/m.err; exit $rc; fi
    python3 -c "import json; j=json.loads(open('gpurun_out/m.json').read().strip().splitlines()[-1]); print('$label', j['config']['scene'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline'].get('trace_path'))" | tee -a gpurun_out/matrix.txt
done
