set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for so in libphc_hip.so libphc_hip_noin.so libphc_hip_noout.so libphc_hip_nofk.so; do
  echo -n "$so: "; PHC_HIP_LIB=$PWD/puffer-phc_amd/lib/$so timeout -k 10 60 python tools/physics_probe.py 4096 30 2>&1 | grep -v amdgpu | tail -1
done
echo -n "no self-collision: "; PHC_SELF_COL=0 timeout -k 10 60 python tools/physics_probe.py 4096 30 2>&1 | grep -v amdgpu | tail -1
