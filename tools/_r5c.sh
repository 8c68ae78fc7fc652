set -e
R=$GRAFT_REPO_ROOT; cd $R
for L in F0 F3 F5; do echo "== $L"; SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 120 python3 tools/_dbg_nan.py; done
