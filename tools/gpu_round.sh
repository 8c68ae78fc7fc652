# usage: bash tools/gpu_round.sh TAG [pytest-args...] — GPU tests, smoke, bench (with CPU baseline) and
# a kernel-trace stats profile of the bench step; each step time-limited, stops at the first failure.
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}; shift || true
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_stats -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-f32-leg --no-kernel-table --roofline-kernel edge_fwd > $R/gpurun_out/${T}_stats_bench.json 2> $R/gpurun_out/${T}_stats_bench.err
cd $R && python3 tools/profsum.py gpurun_out/${T}_stats > gpurun_out/${T}_kernel_summary.txt
head -12 gpurun_out/${T}_kernel_summary.txt
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/${T}_fit_bench.json 2> gpurun_out/${T}_fit_bench.err || { tail -20 gpurun_out/${T}_fit_bench.err; exit 1; }
cat gpurun_out/${T}_fit_bench.json
timeout -k 10 300 python3 bench.py --config 1 --steps 200 --warmup 20 > gpurun_out/${T}_bench_c1.json 2> gpurun_out/${T}_bench_c1.err || { tail -20 gpurun_out/${T}_bench_c1.err; exit 1; }
cut -c1-400 gpurun_out/${T}_bench_c1.json
