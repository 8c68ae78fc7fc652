set -e
R=$GRAFT_REPO_ROOT; cd $R
LIBS="P32 P8 P16 P32 P8 P16" CONFIGS="1" KERNELS="wgrad_ws" FIT=1 bash tools/ab.sh prep
