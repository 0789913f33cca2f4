R="python tools/root_step.py --worlds 8 --map-back none"
tools/gpu_session.sh \
 "a:900:for s in csg32 csg32_nested csg256_balanced csg256_chain rtiow_cover; do $R --scene \$s; WOLOLO_TILE_WANT=3 $R --scene \$s; WOLOLO_TILE_WANT=3 $R --scene \$s --band 5:1; done > gpurun_out/nomap_n8.log 2>&1" \
 "d2h:120:python -c \"import torch,time; a=torch.empty(1920*1080*4,dtype=torch.uint8,device='cuda'); h=torch.empty_like(a,device='cpu').pin_memory(); [h.copy_(a) for _ in range(3)]; torch.cuda.synchronize(); t=time.perf_counter(); [h.copy_(a,non_blocking=True) for _ in range(50)]; torch.cuda.synchronize(); dt=(time.perf_counter()-t)/50; print('D2H 8.3 MB pinned: %.3f ms, %.1f GB/s'%(dt*1e3, a.numel()/dt/1e9))\" > gpurun_out/d2h.log 2>&1"
