set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "not bf16 and not config4" > gpurun_out/r5b_pytest.log 2>&1 || { tail -40 gpurun_out/r5b_pytest.log; exit 1; }
tail -3 gpurun_out/r5b_pytest.log
for L in F0 F3 F6; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/dump_$L.npz; done
echo "== F0 vs F6"; python3 tools/cmp_npz.py gpurun_out/dump_F0.npz gpurun_out/dump_F6.npz
echo "== F3 vs F6"; python3 tools/cmp_npz.py gpurun_out/dump_F3.npz gpurun_out/dump_F6.npz
LIBS="F3 F4 F6 F3 F4 F6" CONFIGS=0 KERNELS="edge_bwd dA wgrad_ws edge_fwd" bash tools/ab.sh dacc
SPWGNN_LIB=$R/abl/libD7.so timeout -k 10 120 python3 tools/fused_stamps.py
