# usage: CONFIGS="3 4" bash tools/ab_cfg.sh TAG — A/B of tools/diag/libA.so vs libB.so on one box: step
# time and the kernel table (ms per launch) of each config, A and B interleaved twice
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
for c in ${CONFIGS:-3 4}; do
  for rep in 1 2; do
    for v in A B; do
      SPWGNN_LIB=$R/tools/diag/lib$v.so timeout -k 10 300 python3 bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline --no-f32-leg > gpurun_out/abc_${T}_c${c}_$v$rep.json 2> gpurun_out/abc_${T}_c${c}_$v$rep.err
      python3 - gpurun_out/abc_${T}_c${c}_$v$rep.json $c $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d.get("kernels", {})
print(f"c{sys.argv[2]} {sys.argv[3]} step {d['ms_per_step']} " + " ".join(f"{n}={v['avg_launch_ms']}" for n, v in k.items()))
PY
    done
  done
done
