# PMC counters of k_ingest (separate passes, counters only; no tracing domains)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
mkdir -p gpurun_out/$TAG
rocprofv3 -L > gpurun_out/$TAG/counters_list.txt 2>&1 || true
ARGS="python3 bench.py --steps 1 --warmup 0 --no-cpu --streams 200000"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY \
  --kernel-include-regex "k_ingest|k_stats" --output-format csv -d gpurun_out/$TAG/p1 -o run -- $ARGS > gpurun_out/$TAG/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU \
  --kernel-include-regex "k_ingest|k_stats" --output-format csv -d gpurun_out/$TAG/p2 -o run -- $ARGS > gpurun_out/$TAG/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_ingest|k_stats" --output-format csv -d gpurun_out/$TAG/p3 -o run -- $ARGS > gpurun_out/$TAG/p3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_ingest|k_stats" --output-format csv -d gpurun_out/$TAG/p4 -o run -- $ARGS > gpurun_out/$TAG/p4.log 2>&1 || exit $?
ls -R gpurun_out/$TAG | head -30
