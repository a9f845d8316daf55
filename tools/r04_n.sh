#!/bin/bash
# Round-4 pass l (final tree): the evidence pass of tools/r04_final.sh, then the kernel-trace idle-gap
# breakdown and the host profile of the PPO iteration.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$ROOT"; O=$ROOT/gpurun_out/r04n; mkdir -p "$O"; export TMPDIR=/tmp
TAG=r04n bash tools/r04_final.sh || exit 9
TAG=r04n/gaps bash tools/r04_gaps.sh > "$O/gaps_run.log" 2>&1 || { tail -5 "$O/gaps_run.log"; exit 5; }
head -40 "$O/gaps/gaps.txt"
timeout -k 10 300 python tools/host_profile.py 3 > "$O/host_profile.txt" 2>&1 || { tail -5 "$O/host_profile.txt"; exit 7; }
echo r04_l done
