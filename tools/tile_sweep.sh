#!/usr/bin/env bash
# Per-rank kernel shares (tools/rank_share.py) for tile plans given as env
# settings, e.g. tools/tile_sweep.sh csg32 "WOLOLO_TILE=8x8 WOLOLO_TILE_TAIL=1" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
scene=$1; shift
for v in "$@"; do
  echo "== $v" | tee -a gpurun_out/tiles.txt
  env $v timeout -k 10 120 python tools/rank_share.py --scene "$scene" --worlds 1 2 4 8 --reps 5 ${RS_ARGS:-} > gpurun_out/tiles_one.log 2>&1
  rc=$?; grep "^\[share\]" gpurun_out/tiles_one.log | tee -a gpurun_out/tiles.txt
  [ "$rc" -ne 0 ] && { echo "FAIL rc=$rc"; tail -5 gpurun_out/tiles_one.log; exit $rc; }
done
exit 0
