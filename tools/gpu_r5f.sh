# Small-batch double-buffered replay: replay tests, Keras fit, config 1, and the fit step gaps
set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_replay.py > gpurun_out/r5f_replay_tests.log 2>&1 || { tail -30 gpurun_out/r5f_replay_tests.log; exit 1; }
tail -1 gpurun_out/r5f_replay_tests.log
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/r5f_fit_bench.json 2> gpurun_out/r5f_fit_bench.err || { tail -20 gpurun_out/r5f_fit_bench.err; exit 1; }
cut -c1-300 gpurun_out/r5f_fit_bench.json
timeout -k 10 300 python3 bench.py --config 1 --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/r5f_bench_c1.json 2> gpurun_out/r5f_bench_c1.err || { tail -20 gpurun_out/r5f_bench_c1.err; exit 1; }
cut -c1-200 gpurun_out/r5f_bench_c1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r5f_fit_trace -o run --output-format csv -- python3 $R/tools/fit_bench.py 2048 1 > $R/gpurun_out/r5f_fit_trace.log 2>&1
cd $R && python3 tools/step_gaps.py gpurun_out/r5f_fit_trace | tee gpurun_out/r5f_fit_step_gaps.txt
