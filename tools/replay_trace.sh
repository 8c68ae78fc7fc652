# usage: bash tools/replay_trace.sh TAG — kernel trace of the config-1 replay probe (overlap check)
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/${T}_trace -o run --output-format csv -- python3 $R/tools/replay_probe.py 30 > $R/gpurun_out/${T}_trace.log 2>&1
ls $R/gpurun_out/${T}_trace
