"""Generate tests/golden/text_svo.npz from the reference's `Text` SVO dump.

The reference file (Assets/Scripts/SVO/CompactSVO/Text) is an ASCII dump of a
64^3 (depth-6) compact SVO produced by an earlier NaiveCreator that stored
ABSOLUTE child pointers; each line prints the ChildDescriptor fields
(Util.cs:163-190 ToString) and the node's 16-bit normal code with its
decodeRawNormal16 (NaiveCreator.cs:573-595) + Vector3.Normalize value rounded
to one decimal (Unity Vector3.ToString "F1").

This script only reads that file as text and stores the parsed numbers (data,
not source): per descriptor the absolute child pointer, valid mask, non-leaf
mask, normal code and the printed normal.  Run it in a container that has
/root/reference; the resulting .npz is committed.

    python tests/golden/make_text_fixture.py [path/to/Text]
"""
import os
import re
import sys

import numpy as np

DEFAULT = "/root/reference/Assets/Scripts/SVO/CompactSVO/Text"
LINE = re.compile(
    r"CD: \[ChildDescriptor childPointer: (\d+), validMask: ([01]{8}), nonLeafMask: ([01]{8})\], "
    r"Normal: v\(([-\d.]+), ([-\d.]+), ([-\d.]+)\)([01]{16})\((\d+)\)")


def parse(path):
    ptr, valid, nonleaf, code, nrm = [], [], [], [], []
    with open(path, "r", encoding="utf-8", errors="replace") as fh:
        header = fh.readline().strip()
        for line in fh:
            line = line.strip()
            if not line:
                continue
            m = LINE.fullmatch(line)
            if m is None:
                raise ValueError(f"unparsed line: {line[:120]}")
            ptr.append(int(m.group(1)))
            valid.append(int(m.group(2), 2))
            nonleaf.append(int(m.group(3), 2))
            nrm.append([float(m.group(4)), float(m.group(5)), float(m.group(6))])
            bits = int(m.group(7), 2)
            c = int(m.group(8))
            if bits != c:
                raise ValueError("normal code binary/decimal mismatch")
            code.append(c)
    return header, (np.asarray(ptr, np.uint32), np.asarray(valid, np.uint8),
                    np.asarray(nonleaf, np.uint8), np.asarray(code, np.uint16),
                    np.asarray(nrm, np.float32))


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else DEFAULT
    header, (ptr, valid, nonleaf, code, nrm) = parse(src)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "text_svo.npz")
    np.savez_compressed(out, abs_child_ptr=ptr, valid_mask=valid, nonleaf_mask=nonleaf,
                        normal_code=code, normal_f1=nrm,
                        source=np.array("Assets/Scripts/SVO/CompactSVO/Text: " + header))
    print(f"wrote {out}: {len(ptr)} descriptors")


if __name__ == "__main__":
    main()
