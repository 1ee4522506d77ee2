# SQ counter passes of k_ingest_small on the default bench step for several
# library builds (A/B of instruction mix / waits).  Usage: pmc_ab.sh TAG lib...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
ARGS="python3 bench.py --steps 1 --warmup 1 --no-cpu"
for lib in "$@"; do
  i=0
  for CNT in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL"; do
    i=$((i+1))
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -s KILL 180 rocprofv3 --pmc $CNT --kernel-include-regex "k_ingest_small" --output-format csv \
      -d gpurun_out/${TAG}_${lib%.so}_p$i -o run -- $ARGS > gpurun_out/${TAG}_${lib%.so}_p$i.log 2>&1 || { echo "pass $i failed ($lib)"; tail -5 gpurun_out/${TAG}_${lib%.so}_p$i.log; exit 1; }
  done
  echo "$lib ok"
done
