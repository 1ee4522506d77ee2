# Fused stats role A/B: GPU parity with the default, then cfg3/cfg2 bench lines per GK_FUSED_STATS
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-fused}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | head -30 | cut -c1-300; exit 1; fi
for f in ${FS_LIST:-0 1 2 3 4}; do
  for w in cfg3 cfg2; do
    GK_FUSED_STATS=$f timeout -k 10 300 python bench.py --workload $w --no-cpu --steps 5 > gpurun_out/${TAG}_${w}_f$f.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], 'Gv/s=%.2f ms/step=%.3f launch_ms=%.3f stats_ms=%.3f' % (d['value']/1e9, d['ms_per_step'], r['launch_ms'], r['stats_kernel_ms']))" gpurun_out/${TAG}_${w}_f$f.log $w f$f | tee -a gpurun_out/${TAG}_ab.txt
  done
done
