"""Per-dispatch record of the bench's render launches from a rocprofv3 --kernel-trace CSV
(every kernel-time figure the docs quote recomputable from profiles/).

bench.py's measure_frame at N = 1 issues, in order: two instrumented launches (the fetch counts,
render_tile_kernel<..., COUNT>), W warmup launches, K timed launches (value; kernel_ms = their GPU
span over launches 2..K) and K more with the library's per-launch events (kernel_ms_events).  This
writes every primary render dispatch (render_seg_kernel / render_tile_kernel, not COUNT) with its
index, role and duration, and the mean duration of the timed launches 2..K beside the whole trace's.

  python tools/dispatch_summary.py <run_kernel_trace.csv> <warmup W> <steps K> <out.csv>
"""
import csv
import sys


def main():
    src, W, K, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    rows = []
    with open(src) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if "render_seg_kernel" not in name and "render_tile_kernel" not in name:
                continue
            targs = [a.strip() for a in name[name.index("<") + 1:name.index(">")].split(",")]
            if "render_tile_kernel" in name and len(targs) > 1 and targs[1] == "true":
                continue   # the instrumented fetch-count launch
            if "render_tile_kernel" in name and len(targs) > 3 and targs[3] == "true":
                continue   # the fused shadow-ray launches (bench.py's c3_plus_shadow_ray, after the timing)
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0].replace("void ", "")))
    rows.sort()
    roles = ["warmup"] * W + ["timed"] * K + ["events"] * K
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["index", "role", "kernel", "start_ns", "end_ns", "duration_ns"])
        for i, (a, b, n) in enumerate(rows):
            w.writerow([i, roles[i] if i < len(roles) else "other", n, a, b, b - a])
    timed = [b - a for (a, b, _), r in zip(rows, roles) if r == "timed"][1:]
    span = (rows[W + K - 1][1] - rows[W][1]) / (K - 1) if len(rows) >= W + K else None
    print(f"{len(rows)} render dispatches; timed launches 2..{K}: mean duration {sum(timed) / len(timed) / 1e3:.2f} us, "
          f"end-to-end span per launch {span / 1e3:.2f} us; all: {sum(b - a for a, b, _ in rows) / len(rows) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
