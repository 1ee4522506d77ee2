cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -ne 0 ]; then exit 1; fi
bash scripts/gpu_prof.sh $TAG || exit $?
tail -1 gpurun_out/prof_$TAG/bench.log
