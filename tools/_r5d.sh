set -e
R=$GRAFT_REPO_ROOT; cd $R
LIBS="F3 F7 F3 F7" CONFIGS="0 2" KERNELS="edge_bwd dA wgrad_ws wgrad_w2 edge_fwd" bash tools/ab.sh rev
