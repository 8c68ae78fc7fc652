# Per-config artifacts on the GPU box: the bench line (with cpu_baseline), kernel-trace stats and the two
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE) of the same workload, summarised into profiles/.
# usage: bash tools/config_artifacts.sh CONFIG TAG   (CONFIG 0 = headline; 1-5 = BASELINE.json configs)
set -e
R=$GRAFT_REPO_ROOT; C=${1:-0}; T=${2:-r02}
O=$R/gpurun_out/${T}_c$C
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg"
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmcA -o run --output-format csv -- python3 $B > $O/pmcA.json 2> $O/pmcA.err
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmcB -o run --output-format csv -- python3 $B > $O/pmcB.json 2> $O/pmcB.err
cd $R && python3 tools/pmcsum.py $O/pmc_summary.json --bench $O/pmcA.json $O/pmcA $O/pmcB > /dev/null
# the bench line below quotes this run's traffic: its summary goes where bench.py reads it
if [ "$C" = 0 ]; then cp $O/pmc_summary.json $R/profiles/pmc_summary.json; else cp $O/pmc_summary.json $R/profiles/pmc_summary_config$C.json; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline --no-f32-leg > $O/stats_bench.json 2> $O/stats_bench.err
cd $R && python3 tools/profsum.py $O/stats > $O/kernel_summary.txt
timeout -k 10 400 python3 bench.py --config $C > $O/bench.json 2> $O/bench.err
cat $O/bench.json
head -6 $O/kernel_summary.txt
