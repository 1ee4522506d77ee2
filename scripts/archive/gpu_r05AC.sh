# kernel trace of the 125k-stream cfg3 step (one rank's share at N = 8) after the >= 0.3 s warm-up
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AC}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --streams 125000 --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/${TAG}_timeline.txt; cat gpurun_out/${TAG}_timeline.txt
