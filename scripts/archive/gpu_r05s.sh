# cfg5 kernel trace + step timeline, cfg5 strong-split proxies (every rank's
# balanced_assignment share alone), cfg3 proxies (S = 500k/250k/125k).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05s}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_cfg5trace -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_cfg5trace.log 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_cfg5trace -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/${TAG}_cfg5_timeline.txt 2>&1 || true
echo traced
for N in 2 4 8; do
  R=0
  while [ $R -lt $N ]; do
    timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 1 --proxy $N --proxy-rank $R > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 proxy N=$N rank=$R" | tee -a gpurun_out/${TAG}_proxy.txt
    R=$((R+1))
  done
done
for S in 1000000 500000 250000 125000; do
  timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams $S > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  line gpurun_out/${TAG}.tmp "cfg3 S=$S" | tee -a gpurun_out/${TAG}_proxy.txt
done
