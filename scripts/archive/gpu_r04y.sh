# Round-4 final check on the committed tree: GPU suite, smoke, default bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04y
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
echo "full -m gpu rc=$?: $(tail -1 gpurun_out/${TAG}_pytest_gpu.log)" | tee gpurun_out/${TAG}_ab.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
echo "smoke rc=$?: $(tail -1 gpurun_out/${TAG}_smoke.log)" | tee -a gpurun_out/${TAG}_ab.txt
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench rc=$?: $(tail -1 gpurun_out/${TAG}_bench.json | cut -c1-300)" | tee -a gpurun_out/${TAG}_ab.txt
