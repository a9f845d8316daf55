#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"
for r in 1 2; do for so in ${VARIANTS}; do
  echo -n "$so: "; PHC_HIP_LIB=$ROOT/puffer-phc_amd/lib/$so timeout -k 10 120 python tools/act_probe.py 2>&1 | grep -v amdgpu.ids | tail -1
done; done
