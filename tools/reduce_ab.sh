# usage: bash tools/reduce_ab.sh — GPU tests on the in-tree library, then a same-box A/B of
# tools/diag/libA.so vs libB.so on configs 2 and 0 (step time, weight-gradient kernels per step)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rab_pytest.log 2>&1 || { tail -40 gpurun_out/rab_pytest.log; exit 1; }
tail -1 gpurun_out/rab_pytest.log
CONFIGS="2 0" LIBS="A B A B" bash tools/lib_ab.sh
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rab_s2 -o run --output-format csv -- python3 $R/bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg --no-kernel-table > $R/gpurun_out/rab_s2.json 2> $R/gpurun_out/rab_s2.err
cd $R && python3 tools/profsum.py gpurun_out/rab_s2 > gpurun_out/rab_ks2.txt && grep reduce gpurun_out/rab_ks2.txt
