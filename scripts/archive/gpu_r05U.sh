# do waves that start in lockstep slow the short (125k-stream) launch?  k_ingest_small variants whose waves
# start spread over 0..63*64*D cycles (GK_DESYNC=D: 4, 12, 30) vs the product library, cfg3 at 125k and 1M streams.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05U}
D=sketches-py_amd/gkarray_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for S in 125000 1000000; do
    for v in hip hip_ds4 hip_ds12 hip_ds30; do
      GK_LIB_PATH=$D/libgkarray_$v.so timeout -k 10 300 python bench.py --streams $S --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
      line gpurun_out/${TAG}.tmp "S=$S $v" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
