# Refresh the round's committed artifacts on the GPU box (each step time-limited, stops at the first
# failure): GPU tests, smoke, then tools/config_artifacts.sh for the given configs.
# usage: bash tools/refresh_round.sh TAG CONFIG...
set -e
R=$GRAFT_REPO_ROOT; T=${1:-r02}; shift
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
  tail -1 gpurun_out/${T}_pytest_gpu.log
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  tail -1 gpurun_out/${T}_smoke.log
fi
for c in "$@"; do
  bash tools/config_artifacts.sh $c $T > gpurun_out/${T}_c$c.log 2>&1
  grep '^{' gpurun_out/${T}_c$c/bench.json | tail -1 | cut -c1-300
done
