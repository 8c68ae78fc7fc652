# usage: bash tools/ws_cap_ab.sh — GPU tests on the in-tree library, then a same-box A/B of
# tools/diag/libA.so vs libB.so on configs 2 and 1 (step time, weight-gradient kernels per step)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wsc_pytest.log 2>&1 || { tail -40 gpurun_out/wsc_pytest.log; exit 1; }
tail -1 gpurun_out/wsc_pytest.log
CONFIGS="2 1" LIBS="A B A B" bash tools/lib_ab.sh
# then the committed per-config artifacts with the in-tree library
if [ $# -gt 0 ]; then SKIP_TESTS=1 bash tools/refresh_round.sh "$@"; fi
