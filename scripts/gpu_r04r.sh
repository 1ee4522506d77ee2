# Round-4: host-side cost of a cfg3 step (HIP API trace beside the kernel
# trace) -- where the ~0.2 ms between launches goes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
D=gpurun_out/prof_${TAG}_api
mkdir -p $D
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/bench.log 2>&1
echo "api trace rc=$?" | tee gpurun_out/${TAG}_ab.txt
ls -R $D | head -20
