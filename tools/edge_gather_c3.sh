# usage: bash tools/edge_gather_c3.sh — config 3 (bf16) edge forward / backward per-launch time with the
# node-row gathers as built (0) and from one cached row (3), plus A rows from 8 cached blocks (1);
# diagnosis library tools/diag/libD.so (wrong results, timing only)
set -e
R=$GRAFT_REPO_ROOT
cd $R
for v in 0 1 3; do
  SPWGNN_LIB=$R/tools/diag/libD.so SPWGNN_EFWD_DBG=$v timeout -k 10 200 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel edge_fwd > gpurun_out/egc3_f$v.json 2> gpurun_out/egc3_f$v.err
  echo "fwd dbg=$v $(python3 -c "import json;d=json.load(open('gpurun_out/egc3_f$v.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
for v in 0 3; do
  SPWGNN_LIB=$R/tools/diag/libD.so SPWGNN_EBWD_DBG=$v timeout -k 10 200 python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel edge_bwd > gpurun_out/egc3_b$v.json 2> gpurun_out/egc3_b$v.err
  echo "bwd dbg=$v $(python3 -c "import json;d=json.load(open('gpurun_out/egc3_b$v.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
