"""Summarise a tools/gpu_bench_profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/<tag> profiles/<round>_<tag>

Writes <dest>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
<dest>_bench.json (the bench lines) and profiles/pmc_summary.json (per-launch
HBM bytes of the render kernel, read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, are in KiB, and on gfx950 FETCH_SIZE reports half
the bytes of wide streaming reads; the correction (x2) is applied to the read
side as an upper bound and the raw value is kept beside it (this kernel's 8-byte
node gathers are not a calibrated access width).
"""
import csv
import json
import os
import shutil
import sys


def per_kernel(path):
    """Mean counters per launch of the primary-ray kernel: render_seg_kernel (the cost-ordered launch,
    every launch once an order exists) and render_tile_kernel without the instrumented and the fused
    shadow-ray instantiations."""
    vals = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if "render_tile_kernel" not in name and "render_seg_kernel" not in name:
                continue
            targs = [a.strip() for a in name[name.index("<") + 1:name.index(">")].split(",")]
            tile = "render_tile_kernel" in name
            if tile and len(targs) > 1 and targs[1] == "true":   # the instrumented (fetch-counting) launch
                continue
            if tile and len(targs) > 3 and targs[3] == "true":   # the fused shadow-ray launches (c3_plus_shadow_ray)
                continue
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    src, dest = sys.argv[1], sys.argv[2]
    os.makedirs(os.path.dirname(dest), exist_ok=True)
    shutil.copy(os.path.join(src, "prof", "run_kernel_stats.csv"), dest + "_kernel_stats.csv")
    lines = []
    for f in ("bench.json", "bench_overview.json"):
        p = os.path.join(src, f)
        if os.path.exists(p):
            lines += [json.loads(l) for l in open(p) if l.strip()]
    json.dump(lines, open(dest + "_bench.json", "w"), indent=1)
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    l2 = per_kernel(os.path.join(src, "pmc_l2", "run_counter_collection.csv"))
    fetch_b = fetch.get("FETCH_SIZE", 0.0) * 1024
    write_b = write.get("WRITE_SIZE", 0.0) * 1024
    hit, miss = l2.get("TCC_HIT_sum", 0.0), l2.get("TCC_MISS_sum", 0.0)
    summary = {
        "kernel": "render_seg_kernel / render_tile_kernel (hlsl stack, no fetch counting)",
        "workload": lines[0]["config"]["workload"] if lines else None,
        "fetch_bytes_raw": fetch_b,
        "write_bytes": write_b,
        "hbm_bytes_per_launch": 2 * fetch_b + write_b,
        "hbm_bytes_per_launch_raw": fetch_b + write_b,
        "l2_hit_rate": hit / (hit + miss) if hit + miss else None,
        "kernel_source_sha1": lines[0]["roofline"].get("kernel_source_sha1") if lines else None,
        "source": os.path.basename(dest),
        "note": "FETCH_SIZE x2 (gfx950 half-count correction, upper bound for 8-B gathers) + WRITE_SIZE",
    }
    json.dump(summary, open(os.path.join(os.path.dirname(dest), "pmc_summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
