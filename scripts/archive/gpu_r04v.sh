# Round-4: the fixed reset test + a cfg5 kernel trace of the current library
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04v
timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_state.log 2>&1
echo "state tests rc=$?: $(tail -1 gpurun_out/${TAG}_state.log)" | tee gpurun_out/${TAG}_ab.txt
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
echo "cfg5 profile rc=$?" | tee -a gpurun_out/${TAG}_ab.txt
