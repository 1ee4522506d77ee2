# cfg5 strong-split proxies with the workgroups launched first (every rank's balanced_assignment share alone)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AH}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
line gpurun_out/${TAG}.tmp "cfg5 N=1" | tee -a gpurun_out/${TAG}_ab.txt
for N in 2 4 8; do
  for ((R=0; R<N; R++)); do
    timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 2 --proxy $N --proxy-rank $R > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 proxy N=$N rank=$R" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
