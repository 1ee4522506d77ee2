cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/prof_merge
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 -u tools/merge_probe.py > $D/probe.log 2>&1 || { tail -20 $D/probe.log; exit 1; }
grep "^S=" $D/probe.log
grep -E "k_merge|k_import|k_export|k_ingest" $D/run_kernel_stats.csv | cut -c1-160
