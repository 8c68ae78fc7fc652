# Node forward, bf16 math: the bf16-stored H2s words handed to the W3 product as stored (N against A);
# C = N with the bf16 edge forward's ring 5 k-blocks deep instead of 2. Bitwise dumps, then timing.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A N C; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5zl_dump_$L.npz > gpurun_out/r5zl_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5zl_dump_$L.log; exit 1; }; done
for L in N C; do python3 tools/cmp_npz.py gpurun_out/r5zl_dump_A.npz gpurun_out/r5zl_dump_$L.npz | grep -c "bitwise=True"; done
LIBS="A N C A N C" CONFIGS="3 4" KERNELS="node_fwd edge_fwd" bash tools/ab.sh nodefwdw
