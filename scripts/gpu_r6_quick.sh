# Quick parity subset (cfg3 full batch, goldens, stats role) on each listed build, then the cfg3 A/B.
# Usage: gpu_r6_quick.sh TAG lib1 [lib2 ...]   (A/B also over AB_EXTRA libs, which get no parity run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
for lib in "$@"; do
  GK_LIB_PATH=$L/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/${TAG}_${lib}_pq.log 2>&1 \
    || { echo "PARITY FAILED: $lib"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_${lib}_pq.log | head; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/${TAG}_${lib}_pq.log)"
done
NOTEST=1 SQ=${SQ:-0} bash scripts/gpu_r6.sh $TAG libgkarray_hip.so "$@" $AB_EXTRA
