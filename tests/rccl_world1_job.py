"""Run under torch.distributed.run with --nproc-per-node 1 by tests/test_gpu_dist.py: one
process, a real RCCL ("nccl") process group on cuda:0, and every collective of the
multi-GPU path executed over it on MI355X — dist.init(..., device=dev), the broadcast of
the real 63.5 MB packed weight arena, DetectionGather (both modes) on the pipelined
runner (side streams, two slots) and gather_outputs — each checked against the same work
done without a process group.  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dnn-inference-engine_amd"))

import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

import dist as D  # noqa: E402
import dnn_hip  # noqa: E402
import synth  # noqa: E402
import yolo_graph  # noqa: E402
import yolo_post  # noqa: E402


def main():
    rank, local_rank, world = D.env_rank()
    assert world == 1 and rank == 0
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    D.init("nccl", device=dev)
    assert tdist.get_backend() == "nccl"
    B = 8
    ws = synth.yolo_weights()
    g, _ = yolo_graph.build_graph(dnn_hip.DnnGraphBuilder, ws, in_shape=(B, 416, 416, 3))
    entries = dnn_hip.lower_graph(g)
    wb, sb = dnn_hip.Plan.memory(B, (416, 416, 3), entries)
    wbuf = torch.empty(wb, dtype=torch.uint8, device=dev)
    sbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
    plan = dnn_hip.Plan(B, (416, 416, 3), entries, device=0, weights_ptr=wbuf.data_ptr(),
                        workspace_ptr=sbuf.data_ptr(), upload=True)
    torch.cuda.synchronize()
    before = wbuf.clone()
    D.broadcast_weights(wbuf, src=0)  # RCCL broadcast of the packed arena
    torch.cuda.synchronize()
    arena_ok = bool(torch.equal(before, wbuf))

    frames = torch.from_numpy(synth.frames(list(range(B)))).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def compute(inp, out, n):
        plan.run_device(n, inp.data_ptr(), out.data_ptr(), stream)

    runner = D.ShardedRunner(compute, B, (416, 416, 3), (13, 13, 125), dev)
    full = runner.step(frames)  # gather_outputs over RCCL
    torch.cuda.synchronize()
    ref_out = full.clone()

    def post(out, n, slot, post_stream):
        dbufs[slot].run(out.data_ptr(), n, post_stream)
        return dbufs[slot].pack(n, post_stream)

    local = yolo_post.detect_batch(ref_out.cpu().numpy(), raise_errors=False)  # no process group
    n_det = sum(len(im) for im in local if not isinstance(im, int))
    res = {}
    for mode in ("sized", "fixed", "deferred"):
        runner = D.ShardedRunner(compute, B, (416, 416, 3), (13, 13, 125), dev, gather_mode=mode)
        dbufs = [yolo_post.DetectionBuffers(runner.shard_cap, dev) for _ in range(runner.slots)]
        got, pending = [], []
        for k in range(6):  # six steps through three or four slots: every slot reused
            pending.append(runner.launch_detections(frames, post, k % runner.slots))
            if len(pending) == runner.inflight:
                got.append(runner.finish_detections(pending.pop(0)))
        while pending:
            got.append(runner.finish_detections(pending.pop(0)))
        got.append(runner.flush_detections())
        got = [r for r in got if r is not None]  # deferred: the first finish returns nothing
        torch.cuda.synchronize()
        rows = [D.unpack_detections(*r) for r in got]
        res[mode] = {"ok": all(r == local for r in rows), "steps": len(got), "stats": runner.stats()}
    print(json.dumps({"backend": tdist.get_backend(), "arena_bytes": int(wb), "arena_ok": arena_ok,
                      "outputs_shape": list(full.shape), "detections": n_det, "modes": res}), flush=True)
    plan.close()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
