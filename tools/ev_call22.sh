cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "ab:600:bash tools/env_ab.sh 'csg32|X=0' 'csg32|WOLOLO_JIT_FLAGS=-O2' 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-use-amdgpu-trackers=1' 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-schedule-relaxed-occupancy=1' 'csg32|X=0' 'csg32|WOLOLO_JIT_FLAGS=-O2' 'csg32|WOLOLO_JIT_FLAGS=-mllvm%-amdgpu-use-amdgpu-trackers=1'"
