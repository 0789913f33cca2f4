#!/usr/bin/env bash
# Round-2 A/B session: leaf children intersected at their parent in the lane walk
# (abtest/inl: -DWO_LANES_INLINE_LEAF=1).
S=tools/gpu_session.sh
B="python bench.py --scene rtiow_cover --steps 10 --warmup 2 --no-cpu-baseline --no-count-work"
P=abtest/inl/libwololo.so
bash $S \
 "rt:200:$B > gpurun_out/ab_rt.json" \
 "rt_i:200:WOLOLO_LIB=$P $B > gpurun_out/ab_rt_i.json" \
 "rtb:200:$B > gpurun_out/ab_rtb.json" \
 "rt_ib:200:WOLOLO_LIB=$P $B > gpurun_out/ab_rt_ib.json" \
 "rt_ic:200:WOLOLO_LIB=$P python bench.py --scene rtiow_cover --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_rt_ic.json" \
 "par:500:WOLOLO_LIB=$P python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k 'lanes or rtiow'"
