cd "${GRAFT_REPO_ROOT}"
F1="WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=max-ilp"
bash tools/gpu_session.sh \
 "a0:200:bash tools/env_ab.sh 'csg32|X=0'" \
 "a1:200:bash tools/env_ab.sh 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=max-ilp'" \
 "a2:200:bash tools/env_ab.sh 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=iterative-ilp'" \
 "a3:200:bash tools/env_ab.sh 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=iterative-minreg'" \
 "a4:200:bash tools/env_ab.sh 'csg256_balanced|X=0' 'csg256_balanced|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=max-ilp' 'csg256_balanced|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-sched-strategy=iterative-ilp'" \
 "a5:200:bash tools/env_ab.sh 'csg32|X=0'"
