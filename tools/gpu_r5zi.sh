# First-layer weight gradient, bf16 rows: twice the blocks in flight (same per-thread order):
# bitwise dumps against the previous build (A), then same-box timing at configs 3 and 4 (N = new).
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in A N; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/r5zi_dump_$L.npz > gpurun_out/r5zi_dump_$L.log 2>&1 || { tail -20 gpurun_out/r5zi_dump_$L.log; exit 1; }; done
python3 tools/cmp_npz.py gpurun_out/r5zi_dump_A.npz gpurun_out/r5zi_dump_N.npz | grep -c "bitwise=True"
python3 tools/cmp_npz.py gpurun_out/r5zi_dump_A.npz gpurun_out/r5zi_dump_N.npz | grep "bitwise=False" || true
LIBS="A N A N" CONFIGS="3" KERNELS="wgrad_ws" PROF=1 bash tools/ab.sh pos3ub
