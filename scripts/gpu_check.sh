# Round check on the GPU box: -m gpu tests (parity, configs, state files),
# smoke, default bench line, kernel trace of the bench.  Usage: gpu_check.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|error" gpurun_out/${TAG}_pytest.log | head -20; tail -40 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_trace.log | cut -c1-300
