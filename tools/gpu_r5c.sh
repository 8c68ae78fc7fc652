set -e
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k "band_probe_shape or receiver_block or bf16_math_against or config4" > gpurun_out/r5c_pytest.log 2>&1 || { tail -30 gpurun_out/r5c_pytest.log; exit 1; }
grep -E "passed|failed|logits rms" gpurun_out/r5c_pytest.log | cut -c1-220 | tail -14
timeout -k 10 600 python3 tools/bf16_band_probe.py > gpurun_out/r5c_bf16_band_probe.txt 2>&1 || { tail -20 gpurun_out/r5c_bf16_band_probe.txt; exit 1; }
cat gpurun_out/r5c_bf16_band_probe.txt
for L in A T; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/dump_$L.npz > gpurun_out/dump_$L.log 2>&1 || { tail -20 gpurun_out/dump_$L.log; exit 1; }; done
timeout -k 10 300 python3 tools/b16_dump.py gpurun_out/dump_M.npz > gpurun_out/dump_M.log 2>&1
echo "== main vs old tanh"; python3 tools/cmp_npz.py gpurun_out/dump_A.npz gpurun_out/dump_M.npz
echo "== main vs team-lifted"; python3 tools/cmp_npz.py gpurun_out/dump_M.npz gpurun_out/dump_T.npz
for L in T; do SPWGNN_LIB=$R/abl/lib$L.so timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-f32-leg > gpurun_out/r5c_bench_$L.json 2> gpurun_out/r5c_bench_$L.err || { tail -20 gpurun_out/r5c_bench_$L.err; exit 1; }; done
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-f32-leg > gpurun_out/r5c_bench_M.json 2> gpurun_out/r5c_bench_M.err
SPWGNN_LIB=$R/abl/libA.so timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-f32-leg > gpurun_out/r5c_bench_A.json 2> gpurun_out/r5c_bench_A.err
for L in M A T; do python3 -c "
import json; d=json.load(open('gpurun_out/r5c_bench_$L.json')); k=d['kernels']
print('$L', d['ms_per_step'], ' '.join(f'{n} {v[\"ms_per_step\"]}' for n,v in k.items()))"; done
