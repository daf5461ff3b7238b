"""Table of bench lines from an A/B directory: kernel_ms per (case, variant), reps side by side.

  python tools/ab_table.py gpurun_out/r06sg sg_     (files <prefix><case>_<variant><rep>.json)
"""
import glob
import json
import os
import re
import sys


def main():
    d, pre = sys.argv[1], sys.argv[2]
    rows = {}
    for f in sorted(glob.glob(os.path.join(d, pre + "*.json"))):
        m = re.match(re.escape(pre) + r"([^_]+)_(.+?)([a-z])\.json$", os.path.basename(f))
        if not m or not os.path.getsize(f):
            continue
        x = json.load(open(f))
        x = x[0] if isinstance(x, list) else x
        rows.setdefault((m.group(1), m.group(2)), []).append(x["roofline"]["kernel_ms"])
    for (case, var), v in sorted(rows.items()):
        print(f"{case:6s} {var:10s} " + " ".join(f"{t:.4f}" for t in v) + f"   mean {sum(v) / len(v):.4f}")


if __name__ == "__main__":
    main()
