# Round-end evidence on the GPU box: -m gpu tests, smoke, the default bench
# line (with the CPU baseline legs), cfg2 / cfg4 / cfg5 lines, the cfg3
# rocprofv3 trace + PMC passes (stamped pmc_traffic.json), and the cfg4
# allocation trace (allocations per step).  Usage: gpu_round.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-round}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-300
for W in cfg2 cfg5; do
  timeout -k 10 300 python bench.py --workload $W --no-cpu --steps 3 > gpurun_out/${TAG}_bench_$W.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_bench_$W.log | cut -c1-200
done
for K in 1 8; do
  timeout -k 10 300 python bench.py --workload cfg4 --virtual-shards $K --no-cpu --steps 3 > gpurun_out/${TAG}_bench_cfg4_k$K.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_bench_cfg4_k$K.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --memory-allocation-trace --kernel-trace --output-format csv -d gpurun_out/${TAG}_alloc -o run -- \
  python3 bench.py --workload cfg4 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_alloc.log 2>&1 || exit $?
python3 tools/alloc_steps.py gpurun_out/${TAG}_alloc 1 3 | tee gpurun_out/${TAG}_alloc_steps.txt
bash scripts/profile_cfg3.sh $TAG
