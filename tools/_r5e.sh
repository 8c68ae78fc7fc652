set -e
R=$GRAFT_REPO_ROOT; cd $R
bash tools/refresh_round.sh r04 1
timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/r04_fit.json 2> gpurun_out/r04_fit.err
tail -1 gpurun_out/r04_fit.json | cut -c1-200
