# Config 1: replayed graph (G) against the same launch sequence issued eagerly (E), alternating.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for m in G E G E; do
  F=$([ $m = E ] && echo --eager || echo "")
  timeout -k 10 300 python3 bench.py --config 1 --no-cpu-baseline $F > gpurun_out/r5w_c1_$m.json 2> gpurun_out/r5w_c1_$m.err
  echo "$m $(python3 -c "import json; d=json.load(open('gpurun_out/r5w_c1_$m.json')); print(d['ms_per_step'], d['loss'], d['config']['step_mode'])")"
done
