#!/usr/bin/env bash
# bench.py once per (scene, WOLOLO_JIT_FLAGS) pair; appends "<flags> <scene> <ms/frame> <kernel ms>"
# to gpurun_out/jitab.txt.   tools/jit_flags_ab.sh "csg32|-DWO_JIT_MIN_WAVES=8" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    scene="${spec%%|*}"; flags="${spec#*|}"
    WOLOLO_JIT_FLAGS="$flags" timeout -k 10 300 python bench.py --no-cpu-baseline --scene "$scene" --steps 10 --warmup 2 > gpurun_out/j.json 2> gpurun_out/j.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$spec] rc=$rc"; tail -5 gpurun_out/j.err; exit $rc; fi
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/j.json').read().strip().splitlines()[-1]); print(repr(sys.argv[1]), j['config']['scene'], j['ms_per_step'], j['roofline']['kernel_ms'])" "$flags" | tee -a gpurun_out/jitab.txt
done
