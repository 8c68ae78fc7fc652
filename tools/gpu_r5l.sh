# Round-5 bench lines of every config (with cpu_baseline) after the intensity-based roofline.
set -e
R=$GRAFT_REPO_ROOT; cd $R; O=$R/gpurun_out/r5l; mkdir -p $O
for c in ${CS:-0 1 2 3 4 5}; do
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_c$c.json 2> $O/bench_c$c.err
  cat $O/bench_c$c.json
done
