cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_sections.py --workload cfg3 > gpurun_out/prof_cfg3.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/prof_cfg3.txt; exit $rc
