# per-wave profile of the wg flush with the carry walk's DPP round count (profiling build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05D}
GK_WG_CONC=0 timeout -k 10 300 python tools/prof_sections.py --workload wg --per-wave > gpurun_out/${TAG}_wg_perwave.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/${TAG}_wg_perwave.txt | head -18
