# Section profile of k_ingest_small (needs the profiling library built in-tree: make -C sketches-py_amd/csrc prof)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sec}
timeout -k 10 300 python3 tools/prof_sections.py --workload cfg3 > gpurun_out/${TAG}_cfg3.txt 2>&1 || exit $?
cat gpurun_out/${TAG}_cfg3.txt
timeout -k 10 300 python3 tools/prof_sections.py --workload cfg2 > gpurun_out/${TAG}_cfg2.txt 2>&1 || exit $?
cat gpurun_out/${TAG}_cfg2.txt
