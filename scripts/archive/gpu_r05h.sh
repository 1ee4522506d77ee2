# Per-wave work / barrier-wait profile of the workgroup flush (k_ingest_wg),
# presort beside (default) and ahead (GK_WG_CONC=0).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05h}
GK_WG_PRESORT=1 timeout -k 10 300 python tools/prof_sections.py --workload wg --per-wave > gpurun_out/${TAG}_wg_perwave.txt 2>&1 || exit $?
GK_WG_CONC=0 GK_WG_PRESORT=1 timeout -k 10 300 python tools/prof_sections.py --workload wg --per-wave > gpurun_out/${TAG}_wg_perwave_seq.txt 2>&1 || exit $?
cat gpurun_out/${TAG}_wg_perwave.txt gpurun_out/${TAG}_wg_perwave_seq.txt
