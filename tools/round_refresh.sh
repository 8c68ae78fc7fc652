# usage: bash tools/round_refresh.sh TAG CONFIG... — GPU tests, smoke, then the committed per-config
# artifacts (tools/config_artifacts.sh); each step time-limited, stops at the first failure
set -e
R=$GRAFT_REPO_ROOT; T=$1; shift
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -1 gpurun_out/${T}_smoke.log
SKIP_TESTS=1 bash tools/refresh_round.sh $T "$@"
