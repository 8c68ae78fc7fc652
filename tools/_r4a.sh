timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a_pytest.log 2>&1; tail -3 gpurun_out/r4a_pytest.log
timeout -k 10 200 python3 tools/ws_jobs.py 0 3 > gpurun_out/r4a_wsjobs_c0.txt 2>&1 && cat gpurun_out/r4a_wsjobs_c0.txt | head -20
timeout -k 10 200 python3 tools/ws_jobs.py 3 3 > gpurun_out/r4a_wsjobs_c3.txt 2>&1 && cat gpurun_out/r4a_wsjobs_c3.txt | head -20
SPWGNN_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --towers 16384 --buckets 2 > gpurun_out/r4a_dp2.json 2> gpurun_out/r4a_dp2.err && grep -o "\"allreduce\".*" gpurun_out/r4a_dp2.json | cut -c1-300
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-f32-leg > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err && cut -c1-400 gpurun_out/r4a_bench.json
