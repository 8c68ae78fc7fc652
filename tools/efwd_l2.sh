# usage: bash tools/efwd_l2.sh — headline edge forward with the W2 image in LDS (SPWGNN_EFWD_DBG=0) vs
# streamed from L2 with the LDS left free (2), in the diagnosis library tools/diag/libD.so
set -e
R=$GRAFT_REPO_ROOT
cd $R
for v in 0 2; do
  SPWGNN_LIB=$R/tools/diag/libD.so SPWGNN_EFWD_DBG=$v timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg --no-kernel-table --roofline-kernel edge_fwd > gpurun_out/efwd_l2_$v.json 2> gpurun_out/efwd_l2_$v.err
  echo "dbg=$v $(python3 -c "import json;d=json.load(open('gpurun_out/efwd_l2_$v.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
