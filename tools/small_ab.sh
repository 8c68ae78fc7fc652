# usage: bash tools/small_ab.sh — GPU tests on the in-tree library, then a same-box A/B of
# tools/diag/libA.so vs libB.so on the small-batch paths: config 1 (replayed steps) and Keras fit at
# batch 32 (tools/fit_bench.py); each run time-limited, stops at the first failure
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sab_pytest.log 2>&1 || { tail -40 gpurun_out/sab_pytest.log; exit 1; }
tail -1 gpurun_out/sab_pytest.log
CONFIGS=1 LIBS="A B A B" bash tools/lib_ab.sh
for L in A B A B; do
  SPWGNN_LIB=$R/tools/diag/lib$L.so timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/sab_fit_$L.json 2> gpurun_out/sab_fit_$L.err
  echo "fit $L $(tail -1 gpurun_out/sab_fit_$L.json | cut -c1-400)"
done
