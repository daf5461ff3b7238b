"""Experiment: what the display rank's extra work costs per step in the N-rank
bench.  On one GPU, time rank 0's pipeline -- render its bands of
the weak-scaling frame straight into the display frame (stream R) while the
previous frame's N-1 received RGBA8 payloads are assembled around them
(stream G), double-buffered like bench.py's Gather -- against a plain rank's
step (render its bands into a payload only).  The RCCL receive itself is not
modelled (it lands in rank 0's HBM over xGMI concurrently).

  python tools/rank0_cost.py [--world 8] [--steps 40]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)
    for world in a.world:
        W, H = D.weak_frame(1920, 1080, world)
        rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS["flyover"](), W, H)
        per = D.max_band_len(H, world) * W
        R, G = torch.cuda.Stream(), torch.cuda.Stream()
        n_loc = D.band_len(H, 0, world) * W
        hits = torch.empty(n_loc * 24, dtype=torch.uint8, device="cuda")
        rgba = torch.empty(n_loc * 4, dtype=torch.float32, device="cuda")
        fh = [torch.empty(W * H * 24, dtype=torch.uint8, device="cuda") for _ in range(2)]
        fr = [torch.empty(W * H * 4, dtype=torch.float32, device="cuda") for _ in range(2)]
        f8 = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in range(2)]
        send = torch.empty(per, dtype=torch.int32, device="cuda")
        parts = [[None] + [torch.zeros(per, dtype=torch.int32, device="cuda") for _ in range(1, world)]
                 for _ in range(2)]
        ev_r = [torch.cuda.Event() for _ in range(2)]
        ev_g = [torch.cuda.Event() for _ in range(2)]

        def plain(i):   # a sending rank: band buffers + payload
            rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), rgba8=send.data_ptr(),
                            band=(8, 0, world), stream=R.cuda_stream)

        def display(i):   # rank 0: its rows into frame k, assemble the others' rows of frame k on G
            k = i & 1
            if i >= 2:
                R.wait_event(ev_g[k])
            rm.render_frame(W, H, hits=fh[k].data_ptr(), rgba=fr[k].data_ptr(), rgba8=f8[k].data_ptr(),
                            layout=_lib.LAYOUT_FRAME, band=(8, 0, world), stream=R.cuda_stream)
            ev_r[k].record(R)
            G.wait_event(ev_r[k])
            rm.assemble_frame(W, H, [None] + [p.data_ptr() for p in parts[k][1:]], _lib.PART_RGBA8,
                              rgba8=f8[k].data_ptr(), skip_part=0, stream=G.cuda_stream)
            ev_g[k].record(G)

        def frame_only(i):   # rank 0's render into the frame layout, no assemble
            k = i & 1
            rm.render_frame(W, H, hits=fh[k].data_ptr(), rgba=fr[k].data_ptr(), rgba8=f8[k].data_ptr(),
                            layout=_lib.LAYOUT_FRAME, band=(8, 0, world), stream=R.cuda_stream)

        def same_stream(i):   # render then assemble, both on R (no cross-stream events)
            k = i & 1
            rm.render_frame(W, H, hits=fh[k].data_ptr(), rgba=fr[k].data_ptr(), rgba8=f8[k].data_ptr(),
                            layout=_lib.LAYOUT_FRAME, band=(8, 0, world), stream=R.cuda_stream)
            rm.assemble_frame(W, H, [None] + [p.data_ptr() for p in parts[k][1:]], _lib.PART_RGBA8,
                              rgba8=f8[k].data_ptr(), skip_part=0, stream=R.cuda_stream)

        def assemble_only(i):
            k = i & 1
            rm.assemble_frame(W, H, [None] + [p.data_ptr() for p in parts[k][1:]], _lib.PART_RGBA8,
                              rgba8=f8[k].data_ptr(), skip_part=0, stream=R.cuda_stream)

        out = {}
        for name, fn in (("plain", plain), ("display", display), ("frame_only", frame_only),
                         ("same_stream", same_stream), ("assemble_only", assemble_only), ("plain", plain)):
            for i in range(5):
                fn(i)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(a.steps):
                fn(i)
            torch.cuda.synchronize()
            out[name] = (time.perf_counter() - t) / a.steps * 1e3
        print(f"world {world}: frame {W}x{H}, rank rows {n_loc // W}: plain rank {out['plain']:.4f} ms/step, "
              f"display rank {out['display']:.4f} ms/step ({out['display'] / out['plain']:.3f}x); frame layout only "
              f"{out['frame_only']:.4f}, render + assemble on one stream {out['same_stream']:.4f}, assemble alone "
              f"{out['assemble_only']:.4f}", flush=True)
        rm.close()


if __name__ == "__main__":
    main()
