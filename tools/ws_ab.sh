# usage: [SKIP_TESTS=1] [CONFIGS="0 1"] [VARIANTS="env;env;..."] bash tools/ws_ab.sh — GPU tests, then per
# config and library/env variant: step time, the k_wgrad_ws family's and enc_edge's ms per step, loss.
# Default variants: libA (tools/diag, previous commit), the tree's library, and the -DSPWGNN_DIAG
# library with the team kernels off / also one launch per weight gradient.
set -e
R=$GRAFT_REPO_ROOT
cd $R
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ws_pytest.log 2>&1 || { tail -30 gpurun_out/ws_pytest.log; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -1 gpurun_out/ws_pytest.log
D=$R/tools/diag/libD.so
VARIANTS=${VARIANTS:-"SPWGNN_LIB=$R/tools/diag/libA.so;X=tree;SPWGNN_NO_TEAM=1 SPWGNN_LIB=$D;SPWGNN_NO_TEAM=1 SPWGNN_WS_UNBATCHED=1 SPWGNN_LIB=$D"}
for c in ${CONFIGS:-0 1 3}; do
  i=0
  IFS=';' read -ra VS <<< "$VARIANTS"
  for e in "${VS[@]}"; do
    env $e timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-f32-leg > gpurun_out/ws_c${c}_v$i.json 2> gpurun_out/ws_c${c}_v$i.err
    echo "c$c v$i [$(echo $e | sed "s#$R/##g")] $(python3 -c "import json;d=json.load(open('gpurun_out/ws_c${c}_v$i.json'));k=d['kernels'];g=lambda n:(k.get(n,{}).get('ms_per_step'));print(d['ms_per_step'], 'ws', g('wgrad_ws'), 'enc', g('enc_edge'), g('enc_edge_bwd'), 'loss', d['loss'])")"
    i=$((i+1))
  done
done
