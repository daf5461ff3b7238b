"""Per-kernel register / scratch / occupancy of libsvo_rt's kernels as the compiler reports them
(-Rpass-analysis=kernel-resource-usage, the build's own flags), one line per kernel.

  python tools/kernel_resources.py [--filter render_] [-D SVO_SEG_WAVES_PER_EU=1]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filter", default="render_")
    ap.add_argument("--source", default=os.path.join(ROOT, "raytracingtest_amd", "csrc", "svo_kernel.hip"))
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra -D definitions (A/B builds)")
    a = ap.parse_args()
    from raytracingtest_amd import build
    flags = [f for f in build.COMMON if f not in ("-shared", "-fPIC")]
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run([build.HIPCC, "--offload-arch=" + build.ARCH] + flags +
                           ["-D" + d for d in a.defines] + ["-c", a.source, "-o", os.path.join(td, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    cur = None
    rows = {}
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1).split(" ")[0]] = int(m.group(2))
    for name, v in rows.items():
        short = re.sub(r"^_ZN3svo(12_GLOBAL__N_1)?\d+", "", name)
        if a.filter and a.filter not in name:
            continue
        print(f"{short[:60]:60s} sgpr {v.get('TotalSGPRs', '?'):>3} vgpr {v.get('VGPRs', '?'):>3} "
              f"scratch {v.get('ScratchSize', '?'):>3} waves/SIMD {v.get('Occupancy', '?')}")


if __name__ == "__main__":
    main()
