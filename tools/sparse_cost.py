"""Experiment: what the sparse band payload costs on the GPUs.

For the C3 weak-scaling frame at N ranks, on one GPU: render every sending
rank's bands once (dense RGB + tile hit masks), then time
  pack     : svo_pack_hits of one sending rank (tile scan + pack), and
  assemble : rank 0's svo_assemble_frame of the other ranks' rows from sparse
             parts (their tile offsets travel in them: the assemble kernel only) beside the
             same rows from dense 3-byte RGB parts,
and report the bytes each sending rank would move.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

  python tools/sparse_cost.py [--world 2 4 8] [--steps 50] [--camera flyover]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--camera", default="flyover")
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)
    s = torch.cuda.Stream()
    sp = s.cuda_stream

    def timed(fn):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            fn()
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / a.steps

    for world in a.world:
        W, H = D.weak_frame(1920, 1080, world)
        rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS[a.camera](), W, H)
        frame = torch.empty(W * H, dtype=torch.int32, device="cuda")
        dense, sparse, counts, tiles = [None], [None], [None], [None]
        for r in range(1, world):
            band = D.rank_band(r, world)
            rows = D.band_len(H, r, world)
            nt = ((W + 7) // 8) * ((rows + 7) // 8)
            d = torch.empty(rows * W * 3, dtype=torch.uint8, device="cuda")
            p = torch.empty(_lib.sparse_part_bytes(nt, rows * W), dtype=torch.uint8, device="cuda")
            rm.render_frame(W, H, rgb8=d.data_ptr(), hitmask=p.data_ptr(), band=band, stream=sp)
            rm.pack_hits(W, H, band, d.data_ptr(), p.data_ptr(), stream=sp)
            s.synchronize()
            dense.append(d)
            sparse.append(p)
            tiles.append(nt)
            counts.append(int(p[12 * nt:12 * nt + 4].view(torch.int32).item()))
        b1 = D.rank_band(1, world)
        pack = timed(lambda: rm.pack_hits(W, H, b1, dense[1].data_ptr(), sparse[1].data_ptr(), stream=sp))
        asm_dense = timed(lambda: rm.assemble_frame(W, H, [None] + [d.data_ptr() for d in dense[1:]], _lib.PART_RGB8,
                                                    rgba8=frame.data_ptr(), skip_part=0, stream=sp))
        asm_sparse = timed(lambda: rm.assemble_frame(W, H, [None] + [p.data_ptr() for p in sparse[1:]],
                                                     _lib.PART_SPARSE_RGB8, rgba8=frame.data_ptr(), skip_part=0,
                                                     stream=sp))
        n1 = D.band_len(H, 1, world) * W
        print(f"world {world}: frame {W}x{H}, rank 1 {n1} px, hits {counts[1]} ({counts[1] / n1:.3f}); payload "
              f"dense {3 * n1} B, sparse {_lib.sparse_head_bytes(tiles[1]) + 3 * counts[1]} B "
              f"({(_lib.sparse_head_bytes(tiles[1]) + 3 * counts[1]) / (3 * n1):.3f}x); pack {pack * 1e3:.1f} us; assemble dense "
              f"{asm_dense * 1e3:.1f} us, sparse {asm_sparse * 1e3:.1f} us", flush=True)
        rm.close()


if __name__ == "__main__":
    main()
