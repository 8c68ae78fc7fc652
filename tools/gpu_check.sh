# usage: bash tools/gpu_check.sh TAG  — GPU tests, bench, kernel-trace stats (each step time-limited)
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_$T.log 2>&1 || { tail -30 gpurun_out/pytest_$T.log; exit 1; }
tail -2 gpurun_out/pytest_$T.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
cat gpurun_out/bench_$T.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$T -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg > $R/gpurun_out/prof_$T.log 2>&1
cd $R && python3 tools/profsum.py gpurun_out/prof_$T
