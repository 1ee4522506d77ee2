cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/r2_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/r2_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/r2_bench.log 2>&1 || exit $?
cat gpurun_out/r2_bench.log
