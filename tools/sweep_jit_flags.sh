#!/usr/bin/env bash
# Times the scene-specialised kernel under several WOLOLO_JIT_FLAGS settings
# (one bench process per setting), appending "<flags> <scene> <ms/frame> <kernel ms>"
# lines to gpurun_out/sweep.txt.  Stops at the first failing run.
#   tools/sweep_jit_flags.sh "<scenes>" "<flags 1>" "<flags 2>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
scenes="$1"
shift
for f in "$@"; do
  for sc in $scenes; do
    WOLOLO_JIT_FLAGS="$f" timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --scene "$sc" \
        > gpurun_out/sw.json 2> gpurun_out/sw.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$f] $sc rc=$rc"; tail -5 gpurun_out/sw.err; exit $rc; fi
    python3 -c "import json; j=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]); print('[$f]', '$sc', j['ms_per_step'], j['roofline']['kernel_ms'])" | tee -a gpurun_out/sweep.txt
  done
done
