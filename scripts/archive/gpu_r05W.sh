# ablation ladder of the small-class flush (timing only: the ablated variants give wrong tables): each variant
# drops one section -- the in-gap rank loop (rank = atomic slot), the first flush's register sort, the fused
# quantiles, the carry rounds -- or three at once; plus the product library without the fused stats role.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05W}
D=sketches-py_amd/gkarray_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for v in hip hip_abl_rank hip_abl_sort1 hip_abl_quant hip_abl_carry hip_abl_all3; do
    GK_LIB_PATH=$D/lib${v/hip/gkarray_hip}.so timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg3 $v" | tee -a gpurun_out/${TAG}_ab.txt
  done
  GK_FUSED_STATS=0 timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  line gpurun_out/${TAG}.tmp "cfg3 hip GK_FUSED_STATS=0" | tee -a gpurun_out/${TAG}_ab.txt
done
