# usage: bash tools/pmc_l2.sh TAG — TA/TCP/TCC busy and L2 request counters per kernel
set -e
R=$GRAFT_REPO_ROOT; TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg"
timeout -k 10 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES -d $R/gpurun_out/pmc${TAG}E -o run --output-format csv -- python3 $B > $R/gpurun_out/pmc${TAG}E.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --pmc TCP_TCP_TA_DATA_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES -d $R/gpurun_out/pmc${TAG}F -o run --output-format csv -- python3 $B > $R/gpurun_out/pmc${TAG}F.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d $R/gpurun_out/pmc${TAG}G -o run --output-format csv -- python3 $B > $R/gpurun_out/pmc${TAG}G.log 2>&1
cd $R && python3 tools/pmcsum.py gpurun_out/pmc${TAG}_l2.json gpurun_out/pmc${TAG}E gpurun_out/pmc${TAG}F gpurun_out/pmc${TAG}G > gpurun_out/pmc${TAG}_l2.txt
