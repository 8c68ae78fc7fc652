# Round artifacts: full bench (with cpu_baseline), kernel-trace stats, HBM PMC passes.
# usage: bash tools/round_artifacts.sh TAG
set -e
R=$GRAFT_REPO_ROOT; T=${1:-r01}
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
tail -1 gpurun_out/${T}_pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/${T}_pmcA -o run --output-format csv -- python3 $B > $R/gpurun_out/${T}_pmcA.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/${T}_pmcB -o run --output-format csv -- python3 $B > $R/gpurun_out/${T}_pmcB.log 2>&1
cd $R && python3 tools/pmcsum.py gpurun_out/${T}_pmc_summary.json gpurun_out/${T}_pmcA gpurun_out/${T}_pmcB > /dev/null
cp gpurun_out/${T}_pmc_summary.json profiles/pmc_summary.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_stats -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-leg > $R/gpurun_out/${T}_stats_bench.json 2> $R/gpurun_out/${T}_stats_bench.err
cd $R && timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
cat gpurun_out/${T}_bench.json
python3 tools/profsum.py gpurun_out/${T}_stats > gpurun_out/${T}_kernel_summary.txt
head -8 gpurun_out/${T}_kernel_summary.txt
