cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 5 40 python -u tools/dbg_presort.py GK_HOST_CHAINS=0 GK_DBG_PRESORT_WAIT=1 > gpurun_out/dbgK4.log 2>&1; echo "K4 (presort complete before ingest, flags used) rc=$?"; tail -4 gpurun_out/dbgK4.log
grep -q DONE gpurun_out/dbgK4.log || exit 1
timeout -k 5 40 python -u tools/dbg_presort.py GK_HOST_CHAINS=0 GK_DBG_NOUSE=1 > gpurun_out/dbgK3.log 2>&1; echo "K3 (presort beside, ingest ignores it) rc=$?"; tail -4 gpurun_out/dbgK3.log
