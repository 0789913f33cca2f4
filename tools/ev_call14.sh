cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "ab:600:bash tools/env_ab.sh 'csg32|X=0' 'csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_LAST_REG=1' 'csg32|X=0' 'csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_LAST_REG=1' 'csg256_balanced|X=0' 'csg256_balanced|WOLOLO_JIT_FLAGS=-DWO_LDS_LAST_REG=1' 'csg32|WOLOLO_JIT_FLAGS=-DWO_LDS_LAST_REG=1%-DWO_LDS_NEXT_EAGER=3'"
