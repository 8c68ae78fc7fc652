# Half-tile node products and bf16 G3 (§3w): GPU tests on the in-tree build (both), a bitwise dump
# A/B of the bf16 G3 storage alone (abl/libG.so, half tile off) against the previous build
# (abl/libA.so), then same-box timing A/Bs: H = half tile only, P = padding-tile diagnosis,
# G = bf16 G3 only, N = both (the in-tree build).
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5m_pytest.log 2>&1 || { tail -30 gpurun_out/r5m_pytest.log; exit 1; }
tail -2 gpurun_out/r5m_pytest.log
for L in A G; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5m_dump_$L.npz > gpurun_out/r5m_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5m_dump_$L.log; exit 1; }; done
echo "== bf16 G3 vs previous"; python3 tools/cmp_npz.py gpurun_out/r5m_dump_A.npz gpurun_out/r5m_dump_G.npz
LIBS="A H P A H P" KERNELS="node_fwd node_bwd enc_node enc_node_bwd" bash tools/ab.sh ht
CONFIGS=3 LIBS="A G N A G N" KERNELS="node_bwd edge_bwd dA wgrad_w2" bash tools/ab.sh g3
CONFIGS=4 LIBS="A N A N" KERNELS="node_bwd edge_bwd dA wgrad_w2" bash tools/ab.sh g3
