# shader clock of the k_ingest_small launch vs warm-up length: is the short (125k-stream) launch's lower
# clock a ramp after idle or its steady state?  (timeline variant build; see tools/launch_timeline.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05Z}
for spec in "125000:4" "125000:100" "125000:1000" "1000000:1" "1000000:40" "250000:400"; do
  S=${spec%%:*}; W=${spec#*:}
  TL_WARM=$W timeout -k 10 300 python3 tools/launch_timeline.py $S > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  grep -E "warm-up|clock|last stream" gpurun_out/${TAG}.tmp | tee -a gpurun_out/${TAG}_clock.txt
done
