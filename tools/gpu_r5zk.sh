# bf16 batched weight gradient: 4 (A), 6 (B) or 8 (C) stage sets in flight on the staging waves;
# bitwise dumps B, C against A, then same-box timing at configs 3 and 4.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A B C; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5zk_dump_$L.npz > gpurun_out/r5zk_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5zk_dump_$L.log; exit 1; }; done
for L in B C; do python3 tools/cmp_npz.py gpurun_out/r5zk_dump_A.npz gpurun_out/r5zk_dump_$L.npz | grep -c "bitwise=True"; done
LIBS="A B C A B C" CONFIGS="3 4" KERNELS="wgrad_ws" bash tools/ab.sh nset
