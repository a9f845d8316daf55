set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?
tail -25 $O/pytest_gpu.log
exit $rc
