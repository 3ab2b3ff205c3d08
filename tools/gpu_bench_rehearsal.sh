# Rehearsal of bench.py's N>1 path on a one-GPU box: torchrun with 2 ranks on
# device 0 over gloo (RCCL needs one GPU per rank), weak and strong modes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export FSDF_BENCH_BACKEND=gloo FSDF_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 > $O/weak2.json 2> $O/weak2.err || { tail -30 $O/weak2.err; exit 1; }
cat $O/weak2.json | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 10 --warmup 2 --global-points 1048576 > $O/strong2.json 2> $O/strong2.err || { tail -30 $O/strong2.err; exit 1; }
cat $O/strong2.json | cut -c1-300
