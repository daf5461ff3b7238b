"""Generate tests/golden/opensimplex3d_table.json: the digest of the reference's
3D OpenSimplex contribution lookup (Assets/Scripts/Utility/Noise/Simplex.cs:
static constructor, base3D / p3D / lookupPairs3D, :103-138).

The script reads Simplex.cs as text, expands the lookup into the canonical
listing "hash:dx,dy,dz,..." (one line per populated hash, lattice offsets in
contribution order) and stores only its sha256 and sizes.  The native builder
generates the same table from the OpenSimplex region logic; the CPU test
tests/test_builder.py checks the two digests agree.  Run where /root/reference
exists:  python tests/golden/make_osn_digest.py
"""
import hashlib
import json
import os
import re
import sys

SRC = "/root/reference/Assets/Scripts/Utility/Noise/Simplex.cs"


def int_array(src, name):
    m = re.search(r"var " + name + r" = new int\[\] \{([^}]*)\}", src)
    return [int(v) for v in m.group(1).split(",")]


def base_sets(src):
    m = re.search(r"var base3D = new int\[\]\[\]\s*\{(.*?)\};", src, re.S)
    return [[int(v) for v in grp.split(",")] for grp in re.findall(r"new int\[\] \{([^}]*)\}", m.group(1))]


def main():
    src = open(sys.argv[1] if len(sys.argv) > 1 else SRC).read()
    base = base_sets(src)
    p3 = int_array(src, "p3D")
    pairs = int_array(src, "lookupPairs3D")
    lists = []
    for i in range(0, len(p3), 9):
        b = base[p3[i]]
        offs = [tuple(b[k + 1:k + 4]) for k in range(0, len(b), 4)]
        offs += [tuple(p3[i + 2:i + 5]), tuple(p3[i + 6:i + 9])]
        lists.append(offs)
    table = {pairs[i]: lists[pairs[i + 1]] for i in range(0, len(pairs), 2)}
    rows = [f"{h}:" + ",".join(str(v) for o in table[h] for v in o) for h in sorted(table)]
    digest = hashlib.sha256("\n".join(rows).encode()).hexdigest()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "opensimplex3d_table.json")
    json.dump({"source": "Assets/Scripts/Utility/Noise/Simplex.cs:103-138", "sha256": digest,
               "n_hashes": len(rows), "n_lists": len(lists)}, open(out, "w"), indent=1)
    print(out, digest, len(rows))


if __name__ == "__main__":
    main()
