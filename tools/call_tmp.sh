tools/gpu_session.sh "gt:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" && bash tools/evidence_r05.sh rs && bash tools/evidence_r05.sh rsnomap
