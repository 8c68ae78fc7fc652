set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python3 bench.py --config 1 > gpurun_out/r04_c1_bench2.json 2> gpurun_out/r04_c1_bench2.err
SKIP_TESTS=1 bash tools/refresh_round.sh r04 0 3
