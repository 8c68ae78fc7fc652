# SQ counters (two passes: issue/wait mix, MFMA busy; LDS and memory instruction mix) of one config's
# kernels, each pass its own rocprofv3 run; summary → gpurun_out/pmc_sq_c<CONFIG>.json
# usage: bash tools/pmc_sq.sh CONFIG
set -e
R=$GRAFT_REPO_ROOT; C=${1:-1}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg --no-kernel-table --roofline-kernel edge_fwd"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/sq${C}C -o run --output-format csv -- python3 $B > $R/gpurun_out/sq${C}C.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d $R/gpurun_out/sq${C}D -o run --output-format csv -- python3 $B > $R/gpurun_out/sq${C}D.log 2>&1
cd $R && python3 tools/pmcsum.py gpurun_out/pmc_sq_c$C.json gpurun_out/sq${C}C gpurun_out/sq${C}D > gpurun_out/pmc_sq_c$C.txt
