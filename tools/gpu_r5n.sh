# Half-tile precision probe: the GPU suite without -x (failure list), then dumps of the previous build
# (A), half tile only (H) and half tile + bf16 G3 (N = in-tree) compared per tensor.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5n_pytest.log 2>&1
grep -E "^FAILED|passed|failed" gpurun_out/r5n_pytest.log | cut -c1-200
set -e
for L in A H G; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5n_dump_$L.npz > gpurun_out/r5n_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5n_dump_$L.log; exit 1; }; done
echo "== H vs A"; python3 tools/cmp_npz.py gpurun_out/r5n_dump_A.npz gpurun_out/r5n_dump_H.npz
echo "== G vs A"; python3 tools/cmp_npz.py gpurun_out/r5n_dump_A.npz gpurun_out/r5n_dump_G.npz
