#!/usr/bin/env bash
# bench.py once per (scene, environment) pair; appends "<env> <scene> <ms/frame> <kernel ms>"
# to gpurun_out/envab.txt.   tools/env_ab.sh "csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_NEXT_EAGER=4" ...
# A "%" inside a value stands for a space ("WOLOLO_JIT_FLAGS=-mllvm%-opt").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    scene="${spec%%|*}"; envs="${spec#*|}"
    assigns=()
    for a in $envs; do assigns+=("${a//%/ }"); done
    env "${assigns[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-count-work --no-draw-frame --side-scenes "" --scene "$scene" --steps 10 --warmup 2 > gpurun_out/e.json 2> gpurun_out/e.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$spec] rc=$rc"; tail -5 gpurun_out/e.err; exit $rc; fi
    python3 -c "import json,sys; j=json.loads(open('gpurun_out/e.json').read().strip().splitlines()[-1]); ko=j['roofline'].get('kernel_object') or {}; print(repr(sys.argv[1]), j['config']['scene'], j['ms_per_step'], j['roofline']['kernel_ms'], 'vgprs=%s scratch=%s' % (ko.get('vgprs'), ko.get('scratch_bytes')))" "$envs" | tee -a gpurun_out/envab.txt
done
