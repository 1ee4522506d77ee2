# One rank's share of the N-GPU strong split run alone (bench.py --proxy N), N = 1 2 4 8, REPS rounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-proxies}
for rep in $(seq 1 ${REPS:-2}); do
  for N in 1 2 4 8; do
    if [ $N = 1 ]; then A=""; else A="--proxy $N"; fi
    timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 $A > gpurun_out/${TAG}.tmp 2>&1 || { echo "FAILED $N"; tail -20 gpurun_out/${TAG}.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); print('N=%s  ms/step %.4f  launch_ms %.4f  value %.2f G  projected node %.1f G' % (sys.argv[1], d['ms_per_step'], d['roofline']['launch_ms'], d['value']/1e9, 1e9/ (d['ms_per_step']*1e-3)/1e9))" $N | tee -a gpurun_out/${TAG}.txt
  done
done
