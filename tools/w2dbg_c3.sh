# usage: bash tools/w2dbg_c3.sh — config 3 (bf16) W2-gradient kernel time under SPWGNN_W2G_DBG variants
# of the diagnosis library tools/diag/libD.so (wrong results; timing only)
set -e
R=$GRAFT_REPO_ROOT
cd $R
for v in ${VARIANTS:-0 1 2 4 32 33 36}; do
  SPWGNN_LIB=$R/tools/diag/libD.so SPWGNN_W2G_DBG=$v timeout -k 10 200 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel wgrad_w2 > gpurun_out/w2dbg3_$v.json 2> gpurun_out/w2dbg3_$v.err
  echo "dbg=$v $(python3 -c "import json;d=json.load(open('gpurun_out/w2dbg3_$v.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
