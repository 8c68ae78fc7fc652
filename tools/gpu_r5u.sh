# BCE folded into the backward (§3x): GPU tests, then config 1 and Keras fit at batch 32
# with the BCE folded (F) and as its own launch (S: SPWGNN_NO_BCE_FOLD=1), same box, alternating.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5u_pytest.log 2>&1 || { grep -E "^FAILED|passed|failed|Error" gpurun_out/r5u_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5u_pytest.log
for v in 1 0 1 0; do
  L=$([ $v = 1 ] && echo S || echo F)
  SPWGNN_NO_BCE_FOLD=$v timeout -k 10 300 python3 bench.py --config 1 --no-cpu-baseline > gpurun_out/r5u_c1_$L.json 2> gpurun_out/r5u_c1_$L.err
  SPWGNN_NO_BCE_FOLD=$v timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/r5u_fit_$L.json 2> gpurun_out/r5u_fit_$L.err
  echo "$L c1 $(python3 -c "import json; print(json.load(open('gpurun_out/r5u_c1_$L.json'))['ms_per_step'])") fit $(tail -1 gpurun_out/r5u_fit_$L.json | cut -c1-160)"
done
