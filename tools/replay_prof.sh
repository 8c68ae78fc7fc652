# usage: bash tools/replay_prof.sh TAG — config-1 replay probe and its kernel trace
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
true

cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_rprof -o run --output-format csv -- python3 $R/tools/replay_probe.py 50 > $R/gpurun_out/${T}_rprof.log 2>&1
cd $R && python3 tools/profsum.py gpurun_out/${T}_rprof > gpurun_out/${T}_rprof_summary.txt
head -40 gpurun_out/${T}_rprof_summary.txt
