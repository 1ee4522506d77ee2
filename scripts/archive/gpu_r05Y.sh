# k_ingest_small launch timeline (variant build -DGK_TIMELINE): wave start / stats role / end and stream
# start / end stamps at 125k, 250k and 1M streams -- where the short launch's fixed ~95 us goes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05Y}
timeout -k 10 300 python3 tools/launch_timeline.py ${ARGS:-125000 250000 1000000} > gpurun_out/${TAG}_timeline.txt 2>&1; rc=$?
cat gpurun_out/${TAG}_timeline.txt
exit $rc
