# one 10^7-value stream beside 10^5 short ones at eps = 0.01 (small class: one wave) and 0.001 (workgroup)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python tools/long_small_eps.py 10000000 100000 2>&1 | grep -v amdgpu.ids
