# k_ingest_wg's shader clock and us per flush: in the cfg5 batch vs 23 streams of 10^7 values alone vs one
# alone (timeline variant build -DGK_TIMELINE)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AF}
TL_WARM=3 timeout -k 10 400 python3 tools/launch_timeline.py ${ARGS:-wg:cfg5 wg:23 wg:1} > gpurun_out/${TAG}_wg_clock.txt 2>&1; rc=$?
cat gpurun_out/${TAG}_wg_clock.txt
exit $rc
