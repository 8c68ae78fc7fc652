# usage: bash tools/w2dbg.sh — W2-gradient kernel time under SPWGNN_W2G_DBG variants (one box)
set -e
R=$GRAFT_REPO_ROOT
cd $R
for v in ${VARIANTS:-0 1 2 4 6}; do
  SPWGNN_W2G_DBG=$v timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg --roofline-kernel wgrad_w2 > gpurun_out/w2dbg_$v.json 2> gpurun_out/w2dbg_$v.err
  echo "dbg=$v $(python3 -c "import json;d=json.load(open('gpurun_out/w2dbg_$v.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
done
