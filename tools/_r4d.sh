set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4d_pytest.log 2>&1; tail -3 gpurun_out/r4d_pytest.log
L=$GRAFT_REPO_ROOT/abl/libN.so
SPWGNN_LIB=$L SPWGNN_NODE_F32=1 timeout -k 10 200 python3 tools/b16_dump.py gpurun_out/r4d_A.npz > /dev/null 2>&1 && SPWGNN_LIB=$L timeout -k 10 200 python3 tools/b16_dump.py gpurun_out/r4d_B.npz > /dev/null 2>&1 && python3 tools/cmp_npz.py gpurun_out/r4d_A.npz gpurun_out/r4d_B.npz
for c in 3 4; do for v in 1 0 1 0; do
  SPWGNN_LIB=$L SPWGNN_NODE_F32=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-f32-leg > gpurun_out/r4d_c${c}_$v.json 2> gpurun_out/r4d_c${c}_$v.err || { tail -5 gpurun_out/r4d_c${c}_$v.err; exit 1; }
  echo "c$c node_f32=$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4d_c${c}_$v.json'));k=d['kernels'];print(d['ms_per_step'], ' '.join(f'{n} {k[n][\"ms_per_step\"]}' for n in ('wgrad_ws','edge_fwd','node_fwd','node_bwd','edge_bwd') if n in k), 'loss', d['loss'])")"
done; done
