# HW-queue sharing probe, plain and under torch.distributed.run with an RCCL group
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 python tools/stream_queue_probe.py > gpurun_out/probe_plain.txt 2>&1 && timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 tools/stream_queue_probe.py --nccl > gpurun_out/probe_nccl.txt 2>&1 && grep -v amdgpu gpurun_out/probe_plain.txt && grep -A12 "matrix" gpurun_out/probe_nccl.txt
