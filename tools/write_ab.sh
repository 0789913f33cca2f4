#!/usr/bin/env bash
# HBM bytes written per path-tracer launch (rocprofv3 --pmc WRITE_SIZE, its own
# pass) for (scene, environment) pairs: tools/write_ab.sh "csg32|WOLOLO_JIT_FLAGS=-DX=1" ...
# ("%" in a value stands for a space, as in tools/env_ab.sh).  Appends
# "<env> <scene> <MB written per launch>" to gpurun_out/write_ab.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for spec in "$@"; do
    scene="${spec%%|*}"; envs="${spec#*|}"
    assigns=()
    for a in $envs; do assigns+=("${a//%/ }"); done
    i=$((i + 1))
    d="gpurun_out/wab_$i"
    env "${assigns[@]}" timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$d" -o w --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-count-work --no-draw-frame --side-scenes "" --scene "$scene" \
        --steps 5 --warmup 1 > "$d.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL [$spec] rc=$rc"; tail -5 "$d.log"; exit $rc; fi
    python3 - "$d" "$envs" "$scene" <<'PY' | tee -a gpurun_out/write_ab.txt
import csv, glob, sys
per = {}
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("wo_jit_pathtrace", "pathtrace_lanes_kernel", "pathtrace_kernel")):
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
v = sorted(per.values())
print(repr(sys.argv[2]), sys.argv[3], round(v[len(v) // 2] * 1024 / 1e6, 2) if v else None, "MB written (median launch)")
PY
done
