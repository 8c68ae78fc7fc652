# First-layer weight gradient: 16 bf16 / 8 fp32 blocks in flight (N) against 8 / 4 (A): bitwise
# dumps, then kernel profiles at the headline (x6) and config 3 (bf16).
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A N; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5zj_dump_$L.npz > gpurun_out/r5zj_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5zj_dump_$L.log; exit 1; }; done
python3 tools/cmp_npz.py gpurun_out/r5zj_dump_A.npz gpurun_out/r5zj_dump_N.npz | grep -c "bitwise=True"
python3 tools/cmp_npz.py gpurun_out/r5zj_dump_A.npz gpurun_out/r5zj_dump_N.npz | grep "bitwise=False" || true
for C in 0 3; do LIBS="A N A N" CONFIGS="$C" KERNELS="wgrad_ws" PROF=1 bash tools/ab.sh pos3d$C | grep "^c\|pos3\|=="; done
