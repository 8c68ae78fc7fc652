# The in-tree build (half tile off by default) against the previous build: GPU tests, bitwise dumps.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5r_pytest.log 2>&1 || { grep -E "^FAILED|passed|failed" gpurun_out/r5r_pytest.log; exit 1; }
tail -1 gpurun_out/r5r_pytest.log
SPWGNN_LIB=$R/abl/libA.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5r_dump_A.npz > gpurun_out/r5r_dump_A.log 2>&1
timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5r_dump_M.npz > gpurun_out/r5r_dump_M.log 2>&1
python3 tools/cmp_npz.py gpurun_out/r5r_dump_A.npz gpurun_out/r5r_dump_M.npz
# timing: previous build (A), half tile (H), padding-tile MFMAs skipped (P, diagnosis: wrong results)
LIBS="A H P A H P" KERNELS="node_fwd node_bwd enc_node enc_node_bwd" bash tools/ab.sh pad
