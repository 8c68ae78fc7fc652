# Same-box A/B of two library builds with a bitwise check first: abl/libA.so vs abl/libB.so dump every
# logit and gradient of tools/b16_dump.py's shapes (compared with tools/cmp_npz.py), then tools/ab.sh
# times them. Build the libraries with SPWGNN_BUILD_OUT=abl/libX.so (SPWGNN_CFLAGS for the variant) and
# drop ./abl from .gpurunignore for the session. usage: [CONFIGS="0 3 4"] [KERNELS="..."] bash tools/ab_session.sh TAG
set -e
R=$GRAFT_REPO_ROOT; T=${1:-ab}; cd $R; mkdir -p gpurun_out
U=$(echo ${LIBS:-A B} | tr ' ' '\n' | sort -u | tr '\n' ' ')
for L in $U; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/${T}_dump_$L.npz > gpurun_out/${T}_dump_$L.log 2>&1 || { tail -20 gpurun_out/${T}_dump_$L.log; exit 1; }; done
for L in $U; do
  [ "$L" = A ] && continue
  echo "A vs $L bitwise-equal entries: $(python3 tools/cmp_npz.py gpurun_out/${T}_dump_A.npz gpurun_out/${T}_dump_$L.npz | grep -c 'bitwise=True' || true)"
  python3 tools/cmp_npz.py gpurun_out/${T}_dump_A.npz gpurun_out/${T}_dump_$L.npz | grep -v "bitwise=True" | head -5 || true
done
LIBS="${LIBS:-A B A B}" CONFIGS="${CONFIGS:-0 3 4}" KERNELS="${KERNELS:-dA edge_bwd edge_fwd wgrad_ws wgrad_w2}" bash tools/ab.sh $T
