#!/usr/bin/env bash
# Round-2 A/B session: incremental union count (csg256 balanced, WOLOLO_JIT_UNION_COUNT) and the
# deep-tree register window size (chain).
S=tools/gpu_session.sh
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-count-work"
bash $S \
 "bal_uc:200:$B --scene csg256_balanced > gpurun_out/ab_bal_uc.json" \
 "bal_nouc:200:WOLOLO_JIT_UNION_COUNT=0 $B --scene csg256_balanced > gpurun_out/ab_bal_nouc.json" \
 "bal_uc2:200:$B --scene csg256_balanced > gpurun_out/ab_bal_uc2.json" \
 "bal_nouc2:200:WOLOLO_JIT_UNION_COUNT=0 $B --scene csg256_balanced > gpurun_out/ab_bal_nouc2.json" \
 "chain_w6:200:$B --scene csg256_chain > gpurun_out/ab_chain_w6.json" \
 "chain_w5:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=5 $B --scene csg256_chain > gpurun_out/ab_chain_w5.json" \
 "chain_w4:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=4 $B --scene csg256_chain > gpurun_out/ab_chain_w4.json" \
 "chain_w5b:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=5 $B --scene csg256_chain > gpurun_out/ab_chain_w5b.json" \
 "chain_w6b:200:$B --scene csg256_chain > gpurun_out/ab_chain_w6b.json" \
 "par:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'balanced'"
