set -e
R=$GRAFT_REPO_ROOT; cd $R
LIBS="M N M N" CONFIGS="3 4 0" KERNELS="edge_fwd edge_bwd dA wgrad_w2 wgrad_ws" bash tools/ab.sh r5nt
cd /tmp && export TMPDIR=/tmp
SPWGNN_LIB=$R/abl/libN.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/ntA -o run --output-format csv -- python3 $R/bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-table --roofline-kernel edge_fwd > $R/gpurun_out/ntA.log 2>&1
cd $R && python3 tools/pmcsum.py gpurun_out/nt.json gpurun_out/ntA | grep -E "edge_fwd|edge_bwd|k_dA|w2grad" | cut -c1-160
