# Round-5 refresh after the step prologue: config 1's artifacts (bench line with cpu_baseline,
# kernel-trace stats, HBM PMC summary) and the Keras fit bench + step gaps.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/config_artifacts.sh 1 r05v
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/r05v_fit_bench.json 2> gpurun_out/r05v_fit_bench.err
tail -1 gpurun_out/r05v_fit_bench.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05v_fit_trace -o run --output-format csv -- python3 $R/tools/fit_bench.py 4096 1 > $R/gpurun_out/r05v_fit_trace.log 2>&1
cd $R && python3 tools/profsum.py gpurun_out/r05v_fit_trace > gpurun_out/r05v_kernel_summary_fit.txt && python3 tools/step_gaps.py gpurun_out/r05v_fit_trace > gpurun_out/r05v_fit_step_gaps.txt
head -3 gpurun_out/r05v_fit_step_gaps.txt
