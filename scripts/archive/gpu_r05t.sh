# cfg5 A/B: GK_WG_EXCL=1 (wg workgroups alone on their CUs) vs default; wg parity with it on.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05t}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
GK_WG_EXCL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head; exit 1; }
echo "wg tests ok with GK_WG_EXCL=1"
for rep in 1 2; do
  for ex in 1 0; do
    GK_WG_EXCL=$ex timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 GK_WG_EXCL=$ex" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
