# The bench's N>1 control flow (torchrun, barrier, max-over-ranks timing, all-reduce) rehearsed with
# two gloo ranks time-sharing the one GPU of a gpurun box (the overlapped all-reduce, Trainer.reduce_split). usage: bash tools/dp2_rehearsal.sh TAG
set -e
R=$GRAFT_REPO_ROOT; T=${1:-r02}
cd $R
SPWGNN_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --towers 16384 > gpurun_out/${T}_dp2_c0.json 2> gpurun_out/${T}_dp2_c0.err
tail -1 gpurun_out/${T}_dp2_c0.json
SPWGNN_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config 4 --steps 2 --warmup 1 > gpurun_out/${T}_dp2_c4.json 2> gpurun_out/${T}_dp2_c4.err
tail -1 gpurun_out/${T}_dp2_c4.json
