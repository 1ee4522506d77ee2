# Session check: -m gpu parity, default bench line, cfg5 bench + its kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01e}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 400 python bench.py --workload cfg5 --no-cpu --steps 2 --warmup 1 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_cfg5.log | cut -c1-600
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 2 --warmup 1 > $D/bench_trace.log 2>&1 || exit $?
find $D -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200
