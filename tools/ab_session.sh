set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A B; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r6f_dump_$L.npz > gpurun_out/r6f_dump_$L.log 2>&1 || { tail -20 gpurun_out/r6f_dump_$L.log; exit 1; }; done
python3 tools/cmp_npz.py gpurun_out/r6f_dump_A.npz gpurun_out/r6f_dump_B.npz | grep -c "bitwise=True" || true
python3 tools/cmp_npz.py gpurun_out/r6f_dump_A.npz gpurun_out/r6f_dump_B.npz | grep -v "bitwise=True" | head -5 || true
LIBS="A B A B" CONFIGS="0 3 4" KERNELS="dA edge_bwd" bash tools/ab.sh dalock
