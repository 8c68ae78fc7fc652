# PMC of the team/fused kernels at the headline (team limit lifted, abl/libT.so) and of the chain;
# then the N>1 rehearsals. usage: bash tools/gpu_r5e.sh
set -e
R=$GRAFT_REPO_ROOT; cd $R
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-f32-leg --no-kernel-table --roofline-kernel edge_fwd"
for L in T M; do
  if [ $L = T ]; then export SPWGNN_LIB=$R/abl/libT.so; else unset SPWGNN_LIB; fi
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/fz${L}C -o run --output-format csv -- python3 $B > $R/gpurun_out/fz${L}C.log 2>&1
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/fz${L}D -o run --output-format csv -- python3 $B > $R/gpurun_out/fz${L}D.log 2>&1
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/fz${L}A -o run --output-format csv -- python3 $B > $R/gpurun_out/fz${L}A.log 2>&1
done
unset SPWGNN_LIB
cd $R
python3 tools/pmcsum.py gpurun_out/fz_T.json gpurun_out/fzTA gpurun_out/fzTC gpurun_out/fzTD > gpurun_out/fz_T.txt
python3 tools/pmcsum.py gpurun_out/fz_M.json gpurun_out/fzMA gpurun_out/fzMC gpurun_out/fzMD > gpurun_out/fz_M.txt
for L in T M; do python3 - gpurun_out/fz_$L.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1])
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0) if isinstance(kv[1], dict) else 0):
    if not isinstance(v, dict) or "SQ_WAVE_CYCLES" not in v:
        continue
    w = v["SQ_WAVE_CYCLES"]; gui = v.get("GRBM_GUI_ACTIVE", 0) / 8
    print(f"{k[:44]:44s} n={v['dispatches']:3d} gui_cyc {gui:9.3e} wait {v['SQ_WAIT_ANY']/w:.2f} issue {v['SQ_ACTIVE_INST_ANY']/w:.2f} "
          f"mfma_busy {v['SQ_VALU_MFMA_BUSY_CYCLES']/1024/max(gui,1):.2f} vmem_rd {v['SQ_INSTS_VMEM_RD']:.3e} "
          f"L2_rd_req {v.get('TCP_TCC_READ_REQ_sum',0):.3e} L2_hit {v.get('TCC_HIT_sum',0):.3e} L2_miss {v.get('TCC_MISS_sum',0):.3e} "
          f"hbm_rd {v.get('hbm_read_bytes',0)/1e9:.2f}GB")
PY
done
bash tools/dp2_rehearsal.sh r05
