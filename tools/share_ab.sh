#!/usr/bin/env bash
# tools/rank_share.py at N = 8 once per (scene, environment) pair; appends
# "<env> <scene> <slowest rank ms>" to gpurun_out/shareab.txt.
#   tools/share_ab.sh "csg32|WOLOLO_TILE_SMALL=2x2 WOLOLO_TILE_TAIL=2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
    scene="${spec%%|*}"; envs="${spec#*|}"
    env $envs timeout -k 10 200 python tools/rank_share.py --scene "$scene" --worlds 8 --reps 5 > gpurun_out/s.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$spec] rc=$rc"; tail -5 gpurun_out/s.log; exit $rc; fi
    echo "'$envs' $scene $(grep '\[share\] N=8' gpurun_out/s.log | sed 's/.*max \([0-9.]*\) ms.*/\1/')" | tee -a gpurun_out/shareab.txt
done
