export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 120 python tools/stream_queue_probe.py && timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 tools/stream_queue_probe.py --nccl
