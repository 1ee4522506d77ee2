cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/long_probe.py > gpurun_out/probe.log 2>&1; rc=$?
cat gpurun_out/probe.log | tail -20; exit $rc
