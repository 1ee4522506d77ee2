# prefetch latency probe (GK_PROF_PFLAT profiling build): how long the wg's next-batch loads take to land.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05M}
GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip_pflat.so timeout -k 10 300 python tools/prof_sections.py --workload cfg5 --per-wave > gpurun_out/${TAG}_cfg5_pflat.txt 2>&1 || { tail -5 gpurun_out/${TAG}_cfg5_pflat.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_cfg5_pflat.txt | head -20
