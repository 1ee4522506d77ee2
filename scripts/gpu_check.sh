# GPU check after a kernel change: -m gpu parity tests, then cfg3 / cfg2 bench lines (no CPU leg).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
for wl in cfg3 cfg2; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_$wl.log 2>&1 || exit $?
  grep '^{"metric"' gpurun_out/${TAG}_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl', 'Gv/s=%.2f'%(d['value']/1e9), 'ms/step=%.2f'%d['ms_per_step'], 'ingest_ms=%.2f'%r['launch_ms'], 'stats_ms=%.2f'%r['stats_kernel_ms'], 'GB/s=%.0f'%r['achieved'])"
done
