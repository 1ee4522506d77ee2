# rocprofv3 evidence for the bench line: kernel trace + stats of the default
# bench command, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) on the
# same workload.  Counters are collected without any tracing domain.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
  python3 bench.py --no-cpu --steps 5 --warmup 2 > $D/bench_trace.log 2>&1 || exit $?
ARGS="python3 bench.py --steps 1 --warmup 0 --no-cpu"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_ingest|k_stats" --output-format csv \
  -d $D/fetch -o run -- $ARGS > $D/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_ingest|k_stats" --output-format csv \
  -d $D/write -o run -- $ARGS > $D/write.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  --kernel-include-regex "k_ingest" --output-format csv -d $D/sq -o run -- $ARGS > $D/sq.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D 1e9 1e6 $D/summary.json $D/pmc_traffic.json
tail -1 $D/bench_trace.log | cut -c1-300
