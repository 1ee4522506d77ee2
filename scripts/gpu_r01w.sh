cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01w}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | head -30 | cut -c1-300; tail -40 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
bash scripts/gpu_merge.sh || exit $?
