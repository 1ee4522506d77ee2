cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r03r
bash scripts/gpu_check.sh $TAG || exit $?
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 3 > gpurun_out/${TAG}_bench_cfg5.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_cfg5.log | cut -c1-400
bash scripts/lds_attrib.sh r03s libgkarray_hip.so $(for g in 1 2 3 4 5 6 7 8 9 10 11 12; do echo -n "libgkarray_hip_dup$g.so "; done)
