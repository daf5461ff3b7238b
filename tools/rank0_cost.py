"""Experiment: what the display rank's extra work costs per step in the N-rank
bench, and what the weighted band deal recovers.  On one GPU,
time the two kinds of rank of bench.py's Gather pipeline for the C3
weak-scaling frame at N ranks:

  plain   : render its bands into band buffers + an RGBA8 payload;
  display : render its bands straight into display frame k, then (same stream)
            assemble frame k-1's rows of the other N-1 ranks from their parts.

for the round-robin deal and for the weighted deal bench.py calibrates
(distributed.weighted_owner).  The step of the whole job is the slower of the
two, so plain(round-robin) / max(display, plain) estimates the efficiency the
display rank leaves (the RCCL transfer, which lands in rank 0's HBM over xGMI
meanwhile, is not modelled).  --two-streams also times the display rank with
the assemble on a second stream beside the render.

  python tools/rank0_cost.py [--world 2 4 8] [--steps 40]
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
    ap.add_argument("--two-streams", action="store_true")
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)

    def timed(fn):
        for i in range(5):
            fn(i)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(a.steps):
            fn(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / a.steps * 1e3

    for world in a.world:
        W, H = D.weak_frame(1920, 1080, world)
        rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS["flyover"](), W, H)
        R, G = torch.cuda.Stream(), torch.cuda.Stream()
        fh = [torch.empty(W * H * 24, dtype=torch.uint8, device="cuda") for _ in range(2)]
        fr = [torch.empty(W * H * 4, dtype=torch.float32, device="cuda") for _ in range(2)]
        f8 = [torch.empty(W * H, dtype=torch.int32, device="cuda") for _ in range(2)]
        ev = [torch.cuda.Event() for _ in range(2)]

        def ranks(owner):
            per = D.max_band_len(H, world, owner=owner) * W
            n1 = D.band_len(H, 1, world, owner=owner) * W
            hits = torch.empty(n1 * 24, dtype=torch.uint8, device="cuda")
            rgba = torch.empty(n1 * 4, dtype=torch.float32, device="cuda")
            send = torch.empty(per, dtype=torch.int32, device="cuda")
            parts = [None] + [torch.zeros(per, dtype=torch.int32, device="cuda") for _ in range(1, world)]
            b0 = D.rank_band(0, world, owner=owner)
            b1 = D.rank_band(1, world, owner=owner)

            def plain(i):
                rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), rgba8=send.data_ptr(), band=b1,
                                stream=R.cuda_stream)

            def asm(k, stream):
                rm.assemble_frame(W, H, [None] + [p.data_ptr() for p in parts[1:]], _lib.PART_RGBA8,
                                  rgba8=f8[k].data_ptr(), skip_part=0, stream=stream.cuda_stream,
                                  owner=None if owner is None else list(owner))

            def display(i):
                k = i & 1
                rm.render_frame(W, H, hits=fh[k].data_ptr(), rgba=fr[k].data_ptr(), rgba8=f8[k].data_ptr(),
                                layout=_lib.LAYOUT_FRAME, band=b0, stream=R.cuda_stream)
                asm(k ^ 1, R)

            def display2(i):
                k = i & 1
                rm.render_frame(W, H, hits=fh[k].data_ptr(), rgba=fr[k].data_ptr(), rgba8=f8[k].data_ptr(),
                                layout=_lib.LAYOUT_FRAME, band=b0, stream=R.cuda_stream)
                ev[k].record(R)
                G.wait_event(ev[k])
                asm(k, G)

            def assemble_only(i):
                asm(i & 1, R)
            return plain, display, display2, assemble_only

        plain, display, display2, asm_only = ranks(None)
        rr = {"plain": timed(plain), "display": timed(display), "assemble": timed(asm_only)}
        if a.two_streams:
            rr["display_two_streams"] = timed(display2)
        rm.set_kernel_timing(True)
        rm.kernel_time()
        timed(plain)
        kern = rm.kernel_time()[0]
        rm.set_kernel_timing(False)
        share = max(1.0 / 8.0, 1.0 - (rr["assemble"] + 0.003) / kern)
        owner = D.weighted_owner(world, share)
        plain_w, display_w, _, _ = ranks(owner)
        wd = {"plain": timed(plain_w), "display": timed(display_w)}
        eff_rr = rr["plain"] / max(rr["plain"], rr["display"])
        eff_w = rr["plain"] / max(wd["plain"], wd["display"])
        extra = f", display on two streams {rr['display_two_streams']:.4f}" if a.two_streams else ""
        print(f"world {world}: frame {W}x{H}; round-robin: plain {rr['plain']:.4f}, display {rr['display']:.4f} "
              f"ms/step (assemble alone {rr['assemble']:.4f}{extra}) -> efficiency ~{eff_rr:.3f}; weighted "
              f"(display share {owner.count(0) / 8:.3f}): plain {wd['plain']:.4f}, display {wd['display']:.4f} "
              f"-> ~{eff_w:.3f}", flush=True)
        rm.close()


if __name__ == "__main__":
    main()
