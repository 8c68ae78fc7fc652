# usage: ENVS="A=1 B=2" KERNEL=edge_bwd bash tools/envab.sh — bench + kernel stats per env setting
set -e
R=$GRAFT_REPO_ROOT
cd $R
i=0
for e in "none=0" $ENVS; do
  env $e timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg --roofline-kernel ${KERNEL:-edge_bwd} > gpurun_out/envab_$i.json 2> gpurun_out/envab_$i.err
  echo "$e $(python3 -c "import json;d=json.load(open('gpurun_out/envab_$i.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
  i=$((i+1))
done
