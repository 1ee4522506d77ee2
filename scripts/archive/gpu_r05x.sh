# priority A/B (wg / stats_long) + spec tests, then the host enqueue cost per step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/archive/gpu_r05w.sh r05x || exit $?
timeout -k 10 300 python tools/host_enqueue.py 125000 250000 1000000 > gpurun_out/r05x_host.txt 2>&1 || { tail -5 gpurun_out/r05x_host.txt; exit 1; }
cat gpurun_out/r05x_host.txt
