# Same-box timing A/Bs: H = half tile only, G = bf16 G3 only, N = both (in-tree), A = previous build.
set -e
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
LIBS="A H A H" KERNELS="node_fwd node_bwd enc_node enc_node_bwd" bash tools/ab.sh ht
CONFIGS=3 LIBS="A G N A G N" KERNELS="node_fwd node_bwd edge_bwd dA wgrad_w2" bash tools/ab.sh g3
CONFIGS=4 LIBS="A N A N" KERNELS="node_fwd node_bwd edge_bwd dA wgrad_w2" bash tools/ab.sh g3
