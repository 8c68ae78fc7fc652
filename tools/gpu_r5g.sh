set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5g_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r5g_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5g_pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g_smoke.log 2>&1
tail -1 gpurun_out/r5g_smoke.log
bash tools/dp2_rehearsal.sh r05b
