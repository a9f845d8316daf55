set -u
cd $GRAFT_REPO_ROOT; O=gpurun_out/r05g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_resample.py tests/test_gpu_env_trainer.py tests/test_gpu_timer.py -x -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 9; }
grep -E "passed|failed|resample_motions" $O/pytest.log | tail -5
timeout -k 10 300 python -u tools/host_timeline.py > $O/host_timeline.txt 2>&1 || { tail -20 $O/host_timeline.txt; exit 9; }
head -45 $O/host_timeline.txt
VARIANTS="libphc_hip.so libphc_hip.so+PHC_GEMM_DISCARD=1 libphc_hip.so+PHC_GEMM_DISCARD=2 libphc_hip.so+YONLY=1 libphc_hip.so+MAXWG=256 libphc_hip.so+MAXWG=512" ROUNDS=2 bash tools/gemm_ab.sh > $O/gemm_epi_ab.txt 2>&1 || { tail -20 $O/gemm_epi_ab.txt; exit 9; }
grep -E "^==|TOTAL" $O/gemm_epi_ab.txt
