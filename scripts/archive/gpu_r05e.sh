# A/B of the small-class launch's tail controls (GK_TAIL_I: single-stream
# grabs at the end of a part; GK_TAIL_S: unpaced last stats batches) at the
# strong-split proxy sizes and the full batch.  Usage: gpu_r05e.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05e}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for S in 125000 1000000; do
    for cfg in "0 0" "2048 0" "0 28" "2048 28" "4096 64" "1024 16"; do
      set -- $cfg
      GK_TAIL_I=$1 GK_TAIL_S=$2 timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams $S > gpurun_out/${TAG}.tmp 2>&1 || { tail -20 gpurun_out/${TAG}.tmp; exit 1; }
      line gpurun_out/${TAG}.tmp "S=$S I=$1 S=$2" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
