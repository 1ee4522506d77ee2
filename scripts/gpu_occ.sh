cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_ab.sh occ libgkarray_hip.so libgkarray_hip_w5.so libgkarray_hip_w7.so || exit $?
