"""Setup-phase breakdown of a wave log (tools/wave_log.py --out gpurun_out/wave_log.bin).
Word 11 of each record is a stamp taken once the wave's tile index is in hand; the committed
kernel leaves that word 0 -- r03y wrote it from a diagnostic patch of render_tile_kernel
(an `s_memrealtime` after the tile index, behind p.wave_log), built with tools/ab_lib.sh and
run through SVO_RT_LIB (profiles/r03y_setup_phase_breakdown.txt)."""
import numpy as np
L = np.fromfile("gpurun_out/wave_log.bin", np.uint32).reshape(-1, 12).astype(np.int64)
entry, tile, loop0, loop1, exitt = L[:, 8], L[:, 11], L[:, 0], L[:, 1], L[:, 9]
def q(a): return " ".join(f"{v*0.01:.2f}" for v in np.percentile(a, [10, 50, 90, 99]))
print("us p10/p50/p90/p99")
print("entry -> tile index  ", q(tile - entry))
print("tile -> loop start   ", q(loop0 - tile))
print("loop                 ", q(loop1 - loop0))
print("loop end -> exit     ", q(exitt - loop1))
tot = (exitt - entry).sum()
for name, a in (("tile load", tile - entry), ("setup compute", loop0 - tile), ("loop", loop1 - loop0), ("record", exitt - loop1)):
    print(f"{name:14s} {a.sum() / tot * 100:5.1f} % of wave time")
span = exitt.max() - entry.min()
print("span us", span * 0.01, "sum wave us", tot * 0.01, "-> mean resident", tot / span)
