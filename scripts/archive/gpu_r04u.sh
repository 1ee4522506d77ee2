# Debug the reset + deferral failure
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dbg/reset_defer.py > gpurun_out/r04u_dbg.txt 2>&1
echo "rc=$?" >> gpurun_out/r04u_dbg.txt
GK_TRACE=1 timeout -k 10 120 python -u -c "
import os, sys
os.environ['GK_POOL_SLOTS']='2'
sys.argv=['x']
exec(open('tools/dbg/reset_defer.py').read().replace('for mode in [\"fresh\", \"sync_reset\", \"async_reset\", \"reset_first\", \"async_reset_q\"]', 'for mode in [\"sync_reset\"]'))
" > gpurun_out/r04u_trace.txt 2>&1
echo "rc=$?" >> gpurun_out/r04u_trace.txt
