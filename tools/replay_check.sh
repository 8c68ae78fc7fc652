# usage: bash tools/replay_check.sh TAG — replay GPU tests, the config-1 probe (aux streams vs one
# stream), the config-1 bench line and the Keras fit bench
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "replay or keras or fit" > gpurun_out/${T}_rp_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_rp_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_rp_pytest.log
timeout -k 10 200 python3 tools/replay_probe.py 200 > gpurun_out/${T}_probe.json 2> gpurun_out/${T}_probe.err || { tail gpurun_out/${T}_probe.err; exit 1; }
cat gpurun_out/${T}_probe.json
timeout -k 10 300 python3 bench.py --config 1 --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/${T}_c1.json 2> gpurun_out/${T}_c1.err || { tail gpurun_out/${T}_c1.err; exit 1; }
cut -c1-300 gpurun_out/${T}_c1.json
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/${T}_fit.json 2> gpurun_out/${T}_fit.err || { tail gpurun_out/${T}_fit.err; exit 1; }
cat gpurun_out/${T}_fit.json
