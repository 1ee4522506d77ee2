# Full round check on the GPU box: -m gpu parity tests, default bench line
# (with the CPU baseline leg), cfg2 line, then the rocprofv3 trace + PMC passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 python bench.py --workload cfg2 --no-cpu --steps 3 > gpurun_out/${TAG}_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_cfg2.log | cut -c1-400
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
bash scripts/profile_cfg3.sh $TAG
