# Quick bench lines of every config (no CPU baseline), each step time-limited.
# usage: bash tools/bench_all.sh TAG [configs...]
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}; shift; CS=${@:-0 1 2 3 4 5}
cd $R
for c in $CS; do
  timeout -k 10 300 python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg > gpurun_out/${T}_bench_c$c.json 2> gpurun_out/${T}_bench_c$c.err
  cat gpurun_out/${T}_bench_c$c.json
done
