# Bisect the chain-path gradient error (B8 N12 fc S5, tools/ht_probe.py case 2; B24 N12 case 6) with
# per-kernel f32 fallbacks (SPWGNN_X6_KERNELS, diagnosis build abl/libE.so: team kernels off, half tile off).
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for M in 127 126 125 123 119 111 95 63; do
  echo "== mask $M"; SPWGNN_X6_KERNELS=$M SPWGNN_LIB=$R/abl/libE.so PROBE_FIRST=2 PROBE_LAST=3 timeout -k 10 120 python3 tools/ht_probe.py || exit 1
done
