# SQ counter passes (one rocprofv3 --pmc run each, no tracing domains) on the
# default bench step, k_ingest_small only (KRX: another kernel regex, e.g.
# k_ingest_wg with a cfg5 bench command).  Usage: pmc_sq.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sq}
ARGS="python3 bench.py --steps 1 --warmup 1 --no-cpu"
i=0
for CNT in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_ATOMIC_RETURN SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_WAVES SQ_CYCLES SQ_INSTS_LDS_ATOMIC SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CNT --kernel-include-regex "${KRX:-k_ingest_small}" --output-format csv \
    -d gpurun_out/${TAG}_p$i -o run -- $ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
  echo "pass $i ok"
done
