cd "${GRAFT_REPO_ROOT}"
rs() { echo "== $1"; env $1 timeout -k 10 120 python tools/rank_share.py --scene csg32 --worlds 8 --reps 5 2>&1 | grep "share\]"; }
bash tools/gpu_session.sh \
 "t:600:$(declare -f rs); rs X=0; rs WOLOLO_TILE=8x4 WOLOLO_TILE_TAIL=2; rs WOLOLO_TILE=8x4 WOLOLO_TILE_TAIL=3; rs WOLOLO_TILE=8x8 WOLOLO_TILE_TAIL=3; rs WOLOLO_TILE=4x4; rs WOLOLO_TILE=8x4 WOLOLO_TILE_TAIL=1; rs X=0"
