set -e
R=$GRAFT_REPO_ROOT; cd $R
for L in A B; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/dump_$L.npz > gpurun_out/dump_$L.log 2>&1 || { tail -20 gpurun_out/dump_$L.log; exit 1; }; done
python3 tools/cmp_npz.py gpurun_out/dump_A.npz gpurun_out/dump_B.npz
LIBS="A B A B" CONFIGS="0 3" KERNELS="wgrad_ws wgrad_w2 edge_fwd" bash tools/ab.sh r5ring
