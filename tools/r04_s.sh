#!/bin/bash
# round-4 pass s: phc_policy_act rows per block A/B (8 vs 4)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
for r in 1 2 3; do for so in libphc_hip.so libphc_hip_r4.so; do
  echo -n "$so: "; PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/act_probe.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 4
done; done
