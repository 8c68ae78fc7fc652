set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_team.py tests/test_gpu_parity.py tests/test_gpu_replay.py tests/test_gpu_edge_cases.py > gpurun_out/r5h_pytest.log 2>&1 || { tail -40 gpurun_out/r5h_pytest.log; exit 1; }
tail -2 gpurun_out/r5h_pytest.log
for L in H2 H3; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/dump_$L.npz; done
echo "== H2 vs H3"; python3 tools/cmp_npz.py gpurun_out/dump_H2.npz gpurun_out/dump_H3.npz | grep -c "bitwise=True"
LIBS="H2 H3 H2 H3" CONFIGS="1" KERNELS="edge_fwd node_bwd enc_edge_bwd" FIT=1 bash tools/ab.sh lds3
