set -e
LIBS="E0 E2 E3 E4 E5 E0 E2 E3 E4 E5" CONFIGS="0 3" KERNELS="edge_fwd" bash tools/ab.sh efwd2
LIBS="E2 E5 E2 E5" CONFIGS="5" KERNELS="edge_fwd node_fwd" bash tools/ab.sh efwd5
