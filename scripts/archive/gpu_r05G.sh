# k_ingest_small section cycles per stream at 1M vs 125k / 250k streams (profiling build): where does
# the small-S launch lose ~10 %?
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05G}
for S in 1000000 250000 125000; do
  timeout -k 10 300 python tools/prof_sections.py --workload cfg3 --streams $S > gpurun_out/${TAG}_S$S.txt 2>&1 || { tail -5 gpurun_out/${TAG}_S$S.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_S$S.txt
done
