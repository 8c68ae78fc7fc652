set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_team.py tests/test_gpu_replay.py tests/test_gpu_parity.py -k "team or replay or independent or backward_parity_small" > gpurun_out/r5f_pytest.log 2>&1 || { tail -40 gpurun_out/r5f_pytest.log; exit 1; }
tail -2 gpurun_out/r5f_pytest.log
LIBS="G1 G2 G1 G2" CONFIGS=1 KERNELS="enc_edge edge_fwd node_bwd enc_edge_bwd wgrad_ws" FIT=1 bash tools/ab.sh warm
