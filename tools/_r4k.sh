set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1; tail -3 gpurun_out/r4k_pytest.log
grep -B5 -A25 "Error\|FAILED" gpurun_out/r4k_pytest.log | head -40
LIBS="O M O M" CONFIGS="1 2" KERNELS="enc_edge enc_node wgrad_ws" FIT=1 bash tools/ab.sh small
