# SQ counters (one pass) of k_ingest_wg in one cfg5 step, per listed build (GK_WG_EARLY=0: a counter pass
# serialises the kernels, and the early grid would wait its bounded 1 s for k_long_prep every call).  Usage: gpu_r6_wgsq.sh TAG lib1 [lib2 ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
for lib in "$@"; do
  n=${lib#libgkarray_hip}; n=${n%.so}; n=${n#_}; [ -z "$n" ] && n=prod
  GK_WG_EARLY=0 GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --kernel-include-regex k_ingest_wg --output-format csv -d gpurun_out/${TAG}_${n}_p1 -o run -- \
    python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu > gpurun_out/${TAG}_${n}_p1.log 2>&1 || { echo "SQ pass failed: $lib"; tail -5 gpurun_out/${TAG}_${n}_p1.log; exit 1; }
done
