set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_team.py tests/test_gpu_replay.py tests/test_gpu_edge_cases.py tests/test_gpu_demolish.py tests/test_gpu_training.py > gpurun_out/r5a_pytest.log 2>&1 || { tail -40 gpurun_out/r5a_pytest.log; exit 1; }
tail -3 gpurun_out/r5a_pytest.log
LIBS="F0 F5 F6 F0 F5 F6" CONFIGS=1 KERNELS="enc_edge edge_fwd node_fwd node_bwd enc_edge_bwd wgrad_ws" FIT=1 bash tools/ab.sh fused
