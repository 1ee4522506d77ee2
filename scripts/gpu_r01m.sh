cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01m}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | head -30 | cut -c1-300; tail -40 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
D=gpurun_out/prof_${TAG}_probe
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 -u tools/long_probe.py > $D/probe.log 2>&1 || exit $?
grep "^S=" $D/probe.log
grep -E "k_stats_long|k_ingest<|k_presort" $D/run_kernel_stats.csv | cut -c1-200
for wl in cfg5 cfg4 cfg3; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_$wl.log 2>&1 || exit $?
  grep '^{"metric"' gpurun_out/${TAG}_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$wl', 'Gv/s=%.3f'%(d['value']/1e9), 'ms/step=%.2f'%d['ms_per_step'], 'ingest_ms=%.2f'%r['launch_ms'], 'stats_ms=%.2f'%r['stats_kernel_ms'])"
done
