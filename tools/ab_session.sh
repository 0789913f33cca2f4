#!/usr/bin/env bash
# Round-2 A/B session: decision-list root evaluation on the chain (WOLOLO_JIT_DL_EVAL).
S=tools/gpu_session.sh
bash $S \
 "chain_dl:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_chain_dl.json" \
 "chain_nodl:200:WOLOLO_JIT_DL_EVAL=0 python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_chain_nodl.json" \
 "chain_dl_lds:200:WOLOLO_JIT_LDS_EVENTS=1 python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_chain_dl_lds.json" \
 "chain_w5:200:WOLOLO_JIT_FLAGS=-DWO_WINDOW=5 python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_chain_w5.json" \
 "chain_dl2:200:python bench.py --scene csg256_chain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_chain_dl2.json" \
 "par:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'chain or jit_event or knobs or lanes'"
