# usage: bash tools/w2tile_ab.sh — bf16 GPU tests, then configs 3 and 4: W2-gradient kernel and step
# time with the LDS node-row kernel (default) and the per-edge gather kernel (SPWGNN_W2G_GATHER=1 in the
# -DSPWGNN_DIAG library tools/diag/libD.so)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "bf16 or config3 or config4" > gpurun_out/w2t_pytest.log 2>&1 || { tail -30 gpurun_out/w2t_pytest.log; exit 1; }
tail -1 gpurun_out/w2t_pytest.log
for c in 3 4; do
  for e in "SPWGNN_W2G_GATHER=0" "SPWGNN_W2G_GATHER=1 SPWGNN_LIB=$R/tools/diag/libD.so"; do
    env $e timeout -k 10 300 python3 bench.py --config $c --steps 4 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel wgrad_w2 > gpurun_out/w2t_c${c}_${e%% *}.json 2> gpurun_out/w2t_c${c}_${e%% *}.err
    echo "c$c $e $(python3 -c "import json;d=json.load(open('gpurun_out/w2t_c${c}_${e%% *}.json'));print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['loss'])")"
  done
done
