# usage: [CONFIGS="0 3"] bash tools/lib_ab.sh — same-box A/B of tools/diag/libA.so vs libB.so: step time
# and the weight-gradient kernels' ms per step per config (bench kernel table), each run time-limited
set -e
R=$GRAFT_REPO_ROOT
cd $R
for c in ${CONFIGS:-0 3}; do
  for L in ${LIBS:-A B A B}; do
    SPWGNN_LIB=$R/tools/diag/lib$L.so timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-f32-leg > gpurun_out/ab_c${c}_$L.json 2> gpurun_out/ab_c${c}_$L.err
    echo "c$c $L $(python3 -c "import json;d=json.load(open('gpurun_out/ab_c${c}_$L.json'));k=d['kernels'];g=lambda n:(k.get(n,{}).get('ms_per_step'));print(d['ms_per_step'], 'ws', g('wgrad_ws'), 'w2', g('wgrad_w2'), 'ef', g('edge_fwd'), 'loss', d.get('loss'))")"
  done
done
