# Round-5 fixed per-call cost: -m gpu suite, cfg3 bench + kernel trace, the
# strong-split proxies (one rank's share alone), cfg5.  Usage: gpu_r05c.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05c}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-28s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}_cfg3.log 2>&1 || exit $?
  line gpurun_out/${TAG}_cfg3.log cfg3 | tee -a gpurun_out/${TAG}_ab.txt
  for S in 500000 250000 125000; do
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams $S > gpurun_out/${TAG}_s$S.log 2>&1 || exit $?
    line gpurun_out/${TAG}_s$S.log "cfg3 S=$S" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
for FS in 0 6 8; do
  GK_FUSED_STATS=$FS timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams 125000 > gpurun_out/${TAG}_fs$FS.log 2>&1 || exit $?
  line gpurun_out/${TAG}_fs$FS.log "cfg3 S=125000 FS=$FS" | tee -a gpurun_out/${TAG}_ab.txt
done
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit $?
line gpurun_out/${TAG}_cfg5.log cfg5 | tee -a gpurun_out/${TAG}_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace125k -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 2 --streams 125000 > gpurun_out/${TAG}_trace125k.log 2>&1 || exit $?
echo done
