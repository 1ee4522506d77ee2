# per-wave profile of k_ingest_wg inside the real cfg5 batch (profiling build), incl. the wait for the prefetched batch.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05L}
timeout -k 10 300 python tools/prof_sections.py --workload cfg5 --per-wave > gpurun_out/${TAG}_cfg5_perwave.txt 2>&1 || { tail -5 gpurun_out/${TAG}_cfg5_perwave.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cfg5_perwave.txt | head -20
timeout -k 10 300 python tools/prof_sections.py --workload wg --per-wave > gpurun_out/${TAG}_wg_perwave.txt 2>&1 || { tail -5 gpurun_out/${TAG}_wg_perwave.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_wg_perwave.txt | head -20
