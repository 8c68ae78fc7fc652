set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1; tail -3 gpurun_out/r4f_pytest.log
grep -B5 -A25 "Error\|FAILED" gpurun_out/r4f_pytest.log | head -60
L=$GRAFT_REPO_ROOT/abl/libR.so
for v in 1 0 1 0; do
  SPWGNN_LIB=$L SPWGNN_RB_ONEHOT=$v timeout -k 10 300 python3 bench.py --config 5 --no-cpu-baseline > gpurun_out/r4f_c5_$v.json 2> gpurun_out/r4f_c5_$v.err || { tail -5 gpurun_out/r4f_c5_$v.err; exit 1; }
  echo "c5 onehot=$v $(python3 -c "import json;d=json.load(open('gpurun_out/r4f_c5_$v.json'));k=d['kernels'];print(d['ms_per_step'], ' '.join(f'{n} {k[n][\"ms_per_step\"]} {k[n][\"frac\"]}' for n in ('edge_fwd','node_fwd','enc_edge') if n in k))")"
done
