set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_replay.py tests/test_gpu_training.py > gpurun_out/r5f_pytest.log 2>&1 || { tail -40 gpurun_out/r5f_pytest.log; exit 1; }
tail -2 gpurun_out/r5f_pytest.log
LIBS="G1 G3 G1 G3" CONFIGS="1 2" KERNELS="wgrad_ws edge_fwd" FIT=1 bash tools/ab.sh red
