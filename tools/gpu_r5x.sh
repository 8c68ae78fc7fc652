# After making eager issue the small-batch default: GPU tests, config 1's bench line (with
# cpu_baseline) and kernel-trace stats, Keras fit bench.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5x_pytest.log 2>&1 || { grep -E "^FAILED|passed|failed|Error" gpurun_out/r5x_pytest.log | head -20; exit 1; }
tail -1 gpurun_out/r5x_pytest.log
timeout -k 10 400 python3 bench.py --config 1 > gpurun_out/r5x_c1.json 2> gpurun_out/r5x_c1.err
python3 -c "import json; d=json.load(open('gpurun_out/r5x_c1.json')); print(d['ms_per_step'], d['value'], d['config']['step_mode'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5x_c1_stats -o run --output-format csv -- python3 $R/bench.py --config 1 --steps 100 --warmup 10 --no-cpu-baseline --no-f32-leg > $R/gpurun_out/r5x_c1_stats.log 2>&1
cd $R && python3 tools/profsum.py gpurun_out/r5x_c1_stats > gpurun_out/r5x_kernel_summary_config1.txt
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/r5x_fit_bench.json 2> gpurun_out/r5x_fit_bench.err
tail -1 gpurun_out/r5x_fit_bench.json | cut -c1-300
