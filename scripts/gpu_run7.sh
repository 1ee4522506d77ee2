cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r11}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 python bench.py --workload cfg2 --no-cpu --steps 3 > gpurun_out/${TAG}_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_cfg2.log | cut -c1-400
timeout -k 10 300 python bench.py --workload cfg4 --values 100000 --no-cpu --steps 3 > gpurun_out/${TAG}_cfg4.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_cfg4.log | cut -c1-400
