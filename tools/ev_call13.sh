cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "ab:600:bash tools/env_ab.sh 'csg32|WOLOLO_JIT_LEAF_PC=0' 'csg32|WOLOLO_JIT_LEAF_PC=1' 'csg32|WOLOLO_JIT_LEAF_PC=0' 'csg32|WOLOLO_JIT_LEAF_PC=1' 'csg256_balanced|WOLOLO_JIT_LEAF_PC=0' 'csg256_balanced|WOLOLO_JIT_LEAF_PC=1' 'csg256_chain|WOLOLO_JIT_LEAF_PC=0' 'csg256_chain|WOLOLO_JIT_LEAF_PC=1'"
