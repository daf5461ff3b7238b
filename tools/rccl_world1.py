"""The RCCL ("nccl") branches of the multi-GPU path, run for real on one GPU at world size 1.

A one-GPU box cannot host two RCCL ranks (one rank per device), so the N > 1 bench and the
GPU suite rehearse the rank path over gloo, whose branches stage device tensors through host
memory.  This script takes the branches only RCCL takes -- device tensors handed to
dist.broadcast / dist.gather / dist.all_gather / dist.all_reduce -- on a real RCCL
communicator of one rank, so API misuse (dtype, device, shape, list arguments) fails here
instead of on the driver's 8-GPU node:

  * distributed.broadcast_svo: the V1 Text pool and a V2 pool, device tensors, bytes equal;
  * distributed.gather_fixed_to_root / gather_parts: a device payload gathered into the
    root's parts list (the root's own part is the send tensor itself);
  * distributed.gather_to_root at world 1 (no peer: no transfer);
  * distributed.accumulate_samples: all_reduce of a device RGBA frame;
  * bench.rank_preflight: all_gather of the device identity, peer matrix, backend record;
  * the plugin renders the frame from the broadcast pool equal to the source pool's frame.

  MASTER_ADDR=127.0.0.1 MASTER_PORT=29555 python tools/rccl_world1.py
Prints one JSON line; exits non-zero on any mismatch.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29555")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.svo_data import SVOData
    import bench
    out = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    assert out["backend"] == "nccl", out

    z = np.load(os.path.join(ROOT, "tests", "golden", "text_svo.npz"))
    v1 = SVOData.from_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"], z["normal_code"])
    v2 = SVOData(nodes=v1.to_v2(), attachments=v1.attachments)
    for name, svo in (("v1", v1), ("v2", v2)):
        got = D.broadcast_svo(svo, 0, device=dev)
        words = svo.childDescriptors if svo.format == 1 else svo.nodes
        gw = got.childDescriptors if got.format == 1 else got.nodes
        assert got.format == svo.format and np.array_equal(np.asarray(gw), np.asarray(words)), name
        assert np.array_equal(got.attachments, svo.attachments), name
    # the other ranks' path of broadcast_svo (receive into fresh device tensors) is the same
    # dist.broadcast call on empty tensors of the announced shape: rank 0 covers its arguments
    out["broadcast_svo"] = "ok"

    send = torch.arange(4096, dtype=torch.uint8, device=dev)
    parts = [send]
    D.gather_fixed_to_root(send, parts, root=0)
    buf = torch.empty_like(send)
    D.gather_parts(send, [buf], dst=0)
    assert torch.equal(buf, send)
    D.gather_to_root(send, [None], root=0)
    out["gathers"] = "ok"

    rgba = torch.rand(64, 64, 4, device=dev)
    ref = rgba.clone()
    D.accumulate_samples(rgba, 1)
    assert torch.equal(rgba, ref)
    out["all_reduce"] = "ok"

    class A:   # rank_preflight reads nothing from args
        pass
    pre = bench.rank_preflight(A(), 0, 1, dev, dist)
    assert pre["backend"] == "nccl" and pre["process_group_world_size"] == 1 and pre["rccl_device_tensors"]
    out["preflight"] = {k: pre[k] for k in ("backend", "process_group_world_size", "rank_devices",
                                            "peer_access_matrix")}

    W, H = 256, 256
    frames = []
    for svo in (v2, D.broadcast_svo(v2, 0, device=dev)):
        rm = RaytracingMaster(capacity_nodes=len(svo))
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS["main"](), W, H)
        hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
        rm.render_device(W, H, hits_ptr=hits.data_ptr(), stack_mode=0)
        torch.cuda.synchronize()
        frames.append(hits.cpu().numpy())
        rm.close()
    assert np.array_equal(frames[0], frames[1])
    out["render_from_broadcast_pool"] = "identical"
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
