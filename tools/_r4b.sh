set -o pipefail
export SPWGNN_LIB_DIAG=$GRAFT_REPO_ROOT/ab/libD.so
timeout -k 10 300 python3 tools/bf16_band_probe.py > gpurun_out/r4b_probe.txt 2>&1; cat gpurun_out/r4b_probe.txt | grep -v amdgpu.ids
SPWGNN_LIB=$SPWGNN_LIB_DIAG timeout -k 10 200 python3 tools/ws_jobs.py 0 3 > gpurun_out/r4b_wsjobs_c0.txt 2>&1 && head -16 gpurun_out/r4b_wsjobs_c0.txt
SPWGNN_LIB=$SPWGNN_LIB_DIAG timeout -k 10 200 python3 tools/ws_jobs.py 3 3 > gpurun_out/r4b_wsjobs_c3.txt 2>&1 && head -16 gpurun_out/r4b_wsjobs_c3.txt
