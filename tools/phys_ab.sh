#!/bin/bash
# Physics-step A/B on the box: tests/test_gpu_physics.py against puffer-phc_amd/lib/libphc_hip_$V.so, then
# tools/physics_probe.py at 4096 and 16384 envs, product library and variant alternating, two rounds.
#   bash tools/build_variants.sh x "-DSOME_FLAG=1" && V=x bash tools/phys_ab.sh   -> gpurun_out/x/{test.log,ab.txt}
set -e
V=${V:?}; O=gpurun_out/$V; mkdir -p $O
L=$PWD/puffer-phc_amd/lib
PHC_HIP_LIB=$L/libphc_hip_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_physics.py > $O/test.log 2>&1
for r in 1 2; do for v in libphc_hip.so libphc_hip_$V.so; do for n in 4096 16384; do
  echo "$v $n $(PHC_HIP_LIB=$L/$v timeout -k 10 120 python tools/physics_probe.py $n 100 | tail -1)"
done; done; done | tee $O/ab.txt
