# usage: bash tools/quick_check.sh TAG [CONFIGS] — GPU tests, then per config a bench line (no CPU
# baseline) and a kernel-trace stats summary; each step time-limited, stops at the first failure.
set -e
R=$GRAFT_REPO_ROOT; T=${1:-q}; CONFIGS=${2:-"0 3"}
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for c in $CONFIGS; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-f32-leg > gpurun_out/${T}_c$c.json 2> gpurun_out/${T}_c$c.err || { tail -20 gpurun_out/${T}_c$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${T}_c$c.json'));print('c$c', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_s$c -o run --output-format csv -- python3 $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg --no-kernel-table > $R/gpurun_out/${T}_s$c.json 2> $R/gpurun_out/${T}_s$c.err
  cd $R && python3 tools/profsum.py gpurun_out/${T}_s$c > gpurun_out/${T}_ks$c.txt && head -16 gpurun_out/${T}_ks$c.txt
done
