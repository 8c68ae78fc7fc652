# Encoder backward, bf16 math: the bf16-stored dA words handed to the first product as stored:
# bitwise dumps against the previous build (A), then same-box timing at configs 3 and 4 (N = new).
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A N; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5zh_dump_$L.npz > gpurun_out/r5zh_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5zh_dump_$L.log; exit 1; }; done
python3 tools/cmp_npz.py gpurun_out/r5zh_dump_A.npz gpurun_out/r5zh_dump_N.npz | grep -c "bitwise=True"
python3 tools/cmp_npz.py gpurun_out/r5zh_dump_A.npz gpurun_out/r5zh_dump_N.npz | grep "bitwise=False" || true
LIBS="A N A N" CONFIGS="3 4" KERNELS="enc_edge_bwd enc_edge" bash tools/ab.sh encbwd
