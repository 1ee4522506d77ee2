# rocprofv3 kernel trace + stats of a short bench run (no counters)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_$TAG/bench.log 2>&1 || exit $?
find gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \;
