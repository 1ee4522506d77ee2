# Kernel traces of the 125k-stream proxy step over (library, environment) pairs.
# Usage: gpu_r6_trace_env.sh TAG "lib1 ENV=a" "lib2" ...   (TRACE_ARGS: bench arguments)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
i=0
for cfg in "$@"; do
  read -r lib envs <<< "$cfg"
  i=$((i+1))
  env GK_LIB_PATH=$L/$lib $envs timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_${i}_kt -o run -- \
    python3 bench.py --no-cpu ${TRACE_ARGS:---proxy 8 --steps 30 --warmup 3} > gpurun_out/${TAG}_${i}_kt.log 2>&1 || { echo "trace failed $cfg"; tail -5 gpurun_out/${TAG}_${i}_kt.log; exit 1; }
  f=$(find gpurun_out/${TAG}_${i}_kt -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $f > gpurun_out/${TAG}_${i}_step.txt || exit 1
  echo "== $cfg"; tail -1 gpurun_out/${TAG}_${i}_kt.log | cut -c1-120; tail -16 gpurun_out/${TAG}_${i}_step.txt
done
