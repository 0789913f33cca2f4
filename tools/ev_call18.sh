cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "knobs:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k 'culling_knobs'"
