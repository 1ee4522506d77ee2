cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/prof_sections.py --workload long > gpurun_out/prof_long.txt 2>&1; rc=$?
cat gpurun_out/prof_long.txt | grep -v amdgpu.ids; exit $rc
