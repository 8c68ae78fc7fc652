# Half-tile precision against the fp64 oracle: small batches on the chain kernels, half tile on (C)
# and off (D).
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for L in D C; do echo "== $L"; SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/ht_probe.py; done
