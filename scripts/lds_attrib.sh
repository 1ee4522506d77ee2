# LDS cost attribution of k_ingest_small's flush: one SQ_LDS_* PMC pass per
# attribution build (-DGK_DUP=1<<g issues access group g twice, results
# unchanged) and the product library; tools/lds_attrib.py prints the deltas.
# Usage: lds_attrib.sh TAG lib...   (libs in sketches-py_amd/gkarray_amd)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
ARGS="python3 bench.py --steps 1 --warmup 0 --no-cpu"
for lib in "$@"; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC \
    --kernel-include-regex "k_ingest_small" --output-format csv \
    -d gpurun_out/${TAG}_${lib%.so} -o run -- $ARGS > gpurun_out/${TAG}_${lib%.so}.log 2>&1 || { echo "pass failed ($lib)"; tail -5 gpurun_out/${TAG}_${lib%.so}.log; exit 1; }
  echo "$lib ok"
done
python3 tools/lds_attrib.py gpurun_out $TAG "$@" | tee gpurun_out/${TAG}_lds_attrib.txt
