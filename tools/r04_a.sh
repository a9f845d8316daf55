set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 4; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 120 python tools/gemm_mb_probe.py > $O/probe_full.log 2>&1 || { tail -5 $O/probe_full.log; exit 5; }
PHC_GEMM_DISCARD=1 timeout -k 10 120 python tools/gemm_mb_probe.py > $O/probe_main.log 2>&1 || { tail -5 $O/probe_main.log; exit 6; }
timeout -k 10 180 python tools/lib_ceiling.py > $O/lib_ceiling.log 2>&1 || { tail -5 $O/lib_ceiling.log; exit 7; }
grep TOTAL $O/*.log
