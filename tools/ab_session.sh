#!/usr/bin/env bash
# Round-2 closing session: full GPU suite on HEAD and the default bench line.
S=tools/gpu_session.sh
bash $S \
 "gt:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "b32:200:python bench.py > gpurun_out/r02_bench_csg32_final.json"
