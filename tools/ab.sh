# Same-box A/B of library builds: abl/lib<L>.so for each L in LIBS (build them with
# `SPWGNN_CFLAGS=... python -m spwgnn_amd.build` and build into abl/ (SPWGNN_BUILD_OUT=abl/libA.so); delete abl/ afterwards, it
# ships with every gpurun push). Per config: step time, loss and the kernel table's ms per step of
# the kernels named in KERNELS. FIT=1 adds Keras fit at batch 32 (tools/fit_bench.py); PROF=1 adds a
# rocprofv3 kernel-trace summary per library. Every run is time-limited; stops at the first failure.
# usage: [LIBS="A B A B"] [CONFIGS="0 3"] [KERNELS="wgrad_ws edge_fwd"] [FIT=1] [PROF=1] bash tools/ab.sh TAG
set -e
R=$GRAFT_REPO_ROOT; T=${1:-x}
cd $R
for c in ${CONFIGS:-0}; do
  for L in ${LIBS:-A B A B}; do
    SPWGNN_LIB=$R/${AB_DIR:-abl}/lib$L.so timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-f32-leg \
      > gpurun_out/ab_${T}_c${c}_$L.json 2> gpurun_out/ab_${T}_c${c}_$L.err || { tail -20 gpurun_out/ab_${T}_c${c}_$L.err; exit 1; }
    echo "c$c $L $(KERNELS="${KERNELS:-wgrad_ws wgrad_w2 edge_fwd edge_bwd dA}" python3 -c "
import json, os
d = json.load(open('gpurun_out/ab_${T}_c${c}_$L.json'))
k = d.get('kernels', {})
print(d['ms_per_step'], ' '.join(f'{n} {k[n][\"ms_per_step\"]}' for n in os.environ['KERNELS'].split() if n in k), 'loss', d.get('loss'))")"
  done
done
if [ "${FIT:-0}" = 1 ]; then
  for L in ${LIBS:-A B A B}; do
    SPWGNN_LIB=$R/${AB_DIR:-abl}/lib$L.so timeout -k 10 300 python3 tools/fit_bench.py 4096 3 > gpurun_out/ab_${T}_fit_$L.json 2> gpurun_out/ab_${T}_fit_$L.err
    echo "fit $L $(tail -1 gpurun_out/ab_${T}_fit_$L.json | cut -c1-300)"
  done
fi
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  for L in $(echo ${LIBS:-A B} | tr ' ' '\n' | sort -u); do
    SPWGNN_LIB=$R/${AB_DIR:-abl}/lib$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_${T}_prof$L -o run \
      --output-format csv -- python3 $R/bench.py --config ${CONFIGS%% *} --steps 3 --warmup 1 --no-cpu-baseline --no-f32-leg \
      --no-kernel-table --roofline-kernel edge_fwd > $R/gpurun_out/ab_${T}_prof$L.log 2>&1
  done
  cd $R
  for L in $(echo ${LIBS:-A B} | tr ' ' '\n' | sort -u); do echo "== $L"; python3 tools/profsum.py gpurun_out/ab_${T}_prof$L | head -16; done
fi
