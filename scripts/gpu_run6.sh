cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
for cfg in "1000000 1000" "100000 10000" "10000000 100"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --streams $1 --values $2 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_bench_$2.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_bench_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1 x $2', 'Gv/s=%.2f'%(d['value']/1e9), 'ms/step=%.2f'%d['ms_per_step'], 'ingest_ms=%.2f'%r['launch_ms'], 'stats_ms=%.2f'%r['stats_kernel_ms'], 'GB/s=%.0f'%r['achieved'])"
done
