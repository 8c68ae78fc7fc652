set -e
R=$GRAFT_REPO_ROOT; cd $R
for L in H0 H1 H0 H1 H0 H1; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/fit_$L.json 2> gpurun_out/fit_$L.err; echo "$L $(tail -1 gpurun_out/fit_$L.json | cut -c1-80)"; done
