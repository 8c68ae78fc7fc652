# usage: KERNEL=name bash tools/pmc_one.sh TAG — SQ counter passes (C, D) for the bench step
set -e
R=$GRAFT_REPO_ROOT; TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg"
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmc${TAG}C -o run --output-format csv -- python3 $B > $R/gpurun_out/pmc${TAG}C.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR -d $R/gpurun_out/pmc${TAG}D -o run --output-format csv -- python3 $B > $R/gpurun_out/pmc${TAG}D.log 2>&1
cd $R && python3 tools/pmcsum.py gpurun_out/pmc${TAG}_all.json gpurun_out/pmc${TAG}C gpurun_out/pmc${TAG}D > gpurun_out/pmc${TAG}_all.txt
