cd "${GRAFT_REPO_ROOT}"
bash tools/gpu_session.sh \
 "tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:200:python bench.py > gpurun_out/final_bench.json"
