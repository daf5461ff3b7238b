"""Compact-SVO node pool: the data contract of the hot path.

Mirrors `RT.SVOData` (Assets/Scripts/SVO/CompactSVO/CompactSVO.cs:22-35):
  childDescriptors : int32 per descriptor, (ptr16 << 16) | (valid8 << 8) | nonleaf8
                     with ptr RELATIVE to the descriptor (NaiveCreator.cs:164-165,184-187);
                     child slot c <-> offset (c&1, c>>1&1, c>>2&1) (Constants.cs:23-26).
  attachments      : 2 x uint32 per descriptor
                     [2i]   = colorA565 | colorB565 << 16
                     [2i+1] = choices(2 bits x 8 children) | normal16 << 16  (NaiveCreator.cs:189-191,254)

The reference's 16-bit relative pointer overflows at ~512^3 (SURVEY.md
Appendix B); such pools are held in the wide V2 form instead:
  nodes            : uint64, low 32 = valid8 << 8 | nonleaf8, high 32 = absolute
                     index of the first non-leaf child (0 when the descriptor word is 0).

Also implements the on-disk formats of SURVEY.md 5 / 8(f) #3:
  - the reference's raw int32 dump (CompactSVO.SaveToDisk, CompactSVO.cs:80-86),
  - the reference's `Text` debug dump (absolute pointers, printed normals),
  - a native binary pool file ("SVOP" header + nodes + attachments).
"""
import re
import struct

import numpy as np

FILE_MAGIC = b"SVOP"
FILE_VERSION = 1
_TEXT_LINE = re.compile(
    r"CD: \[ChildDescriptor childPointer: (\d+), validMask: ([01]{8}), nonLeafMask: ([01]{8})\], "
    r"Normal: v\([^)]*\)[01]{16}\((\d+)\)")


class SVOFormatError(ValueError):
    pass


def _popcount8(x):
    x = x.astype(np.uint32)
    x = x - ((x >> 1) & 0x55)
    x = (x & 0x33) + ((x >> 2) & 0x33)
    return (x + (x >> 4)) & 0x0F


class SVOData:
    """Node pool in V1 (reference) or V2 (wide) form, plus attachments."""

    def __init__(self, childDescriptors=None, attachments=None, nodes=None):
        if (childDescriptors is None) == (nodes is None):
            raise ValueError("give exactly one of childDescriptors (V1) or nodes (V2)")
        if childDescriptors is not None:
            self.childDescriptors = np.ascontiguousarray(childDescriptors, dtype=np.int32)
            self.nodes = None
            n = len(self.childDescriptors)
        else:
            self.childDescriptors = None
            self.nodes = np.ascontiguousarray(nodes, dtype=np.uint64)
            n = len(self.nodes)
        if attachments is None:
            attachments = np.zeros(2 * n, np.uint32)
        self.attachments = np.ascontiguousarray(attachments, dtype=np.uint32)
        if len(self.attachments) != 2 * n:
            raise SVOFormatError(f"attachments must hold 2 words per descriptor ({len(self.attachments)} != {2 * n})")

    # ------------------------------------------------------------------ views
    @property
    def format(self):
        return 1 if self.childDescriptors is not None else 2

    def __len__(self):
        return len(self.childDescriptors) if self.childDescriptors is not None else len(self.nodes)

    def masks_and_first(self):
        """(valid8<<8|nonleaf8, absolute first-child index) per descriptor."""
        if self.childDescriptors is not None:
            cd = self.childDescriptors.view(np.uint32)
            idx = np.arange(len(cd), dtype=np.uint64)
            first = np.where(cd != 0, idx + (cd >> 16).astype(np.uint64), 0)
            return (cd & 0xFFFF).astype(np.uint32), first.astype(np.uint64)
        lo = (self.nodes & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        return lo, (self.nodes >> np.uint64(32)).astype(np.uint64)

    def to_v2(self):
        """Wide nodes (resolves relative pointers to absolute)."""
        if self.nodes is not None:
            return self.nodes
        lo, first = self.masks_and_first()
        return (first.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)

    def as_v2(self):
        return SVOData(nodes=self.to_v2(), attachments=self.attachments)

    def levels(self):
        """Descriptor level of every node reachable from node 0 (1 = root), -1 if unreachable.
        Raises SVOFormatError on out-of-range child pointers."""
        n = len(self)
        lo, first = self.masks_and_first()
        nonleaf = (lo & 0xFF).astype(np.uint32)
        level = np.full(n, -1, np.int32)
        if n == 0:
            return level
        cur = np.array([0], np.int64)
        level[0] = 1
        depth = 1
        while len(cur):
            m = nonleaf[cur]
            kids = []
            for c in range(8):
                has = ((m >> c) & 1).astype(bool)
                if not has.any():
                    continue
                rank = _popcount8(m[has] & ((1 << c) - 1))
                kids.append(first[cur[has]].astype(np.int64) + rank.astype(np.int64))
            if not kids:
                break
            nxt = np.concatenate(kids)
            if nxt.size and (nxt.max() >= n or nxt.min() < 0):
                raise SVOFormatError("child pointer outside the node pool")
            nxt = nxt[level[nxt] < 0]
            depth += 1
            if depth > 22:
                raise SVOFormatError("node pool deeper than 22 levels")
            level[nxt] = depth
            cur = np.unique(nxt)
        return level

    def depth(self):
        return int(self.levels().max()) if len(self) else 0

    def max_relative_pointer(self):
        lo, first = self.masks_and_first()
        has = (lo & 0xFF) != 0
        if not has.any():
            return 0
        idx = np.arange(len(self), dtype=np.int64)
        return int((first.astype(np.int64) - idx)[has].max())

    def to_v1(self):
        """Reference (relative 16-bit pointer) form; raises if a pointer does not fit."""
        if self.childDescriptors is not None:
            return self
        lo, first = self.masks_and_first()
        idx = np.arange(len(self), dtype=np.int64)
        rel = np.where(first != 0, first.astype(np.int64) - idx, 0)
        if rel.size and (rel.max() > 0xFFFF or rel.min() < 0):
            raise SVOFormatError(f"relative child pointer {int(rel.max())} does not fit 16 bits; keep the V2 form")
        cd = ((rel.astype(np.uint32) << 16) | lo.astype(np.uint32)).view(np.int32)
        return SVOData(childDescriptors=cd, attachments=self.attachments)

    # ------------------------------------------------------------ constructors
    @classmethod
    def from_absolute(cls, abs_child_ptr, valid_mask, nonleaf_mask, normal_code=None, color_words=None):
        """Pool from absolute-pointer descriptors (the reference `Text` dump and
        SVOCreator.cs.disabled layout).  Attachments: normal code in the high half
        of word 2i+1, colour words (A|B<<16, choices) when given, else 0."""
        ptr = np.asarray(abs_child_ptr, np.int64)
        n = len(ptr)
        valid = np.asarray(valid_mask, np.uint32)
        nonleaf = np.asarray(nonleaf_mask, np.uint32)
        lo = (valid << 8) | nonleaf
        first = np.where(nonleaf != 0, ptr, 0).astype(np.uint64)
        nodes = (first << np.uint64(32)) | lo.astype(np.uint64)
        att = np.zeros(2 * n, np.uint32)
        if normal_code is not None:
            att[1::2] = np.asarray(normal_code, np.uint32) << 16
        if color_words is not None:
            cw = np.asarray(color_words, np.uint32).reshape(n, 2)
            att[0::2] = cw[:, 0]
            att[1::2] |= cw[:, 1] & 0xFFFF
        v2 = cls(nodes=nodes, attachments=att)
        try:
            return v2.to_v1()
        except SVOFormatError:
            return v2

    @classmethod
    def parse_text_dump(cls, path):
        """Import the reference's `Text` dump (Assets/Scripts/SVO/CompactSVO/Text)."""
        ptr, valid, nonleaf, code = [], [], [], []
        with open(path, "r", encoding="utf-8", errors="replace") as fh:
            fh.readline()
            for line in fh:
                line = line.strip()
                if not line:
                    continue
                m = _TEXT_LINE.fullmatch(line)
                if not m:
                    raise SVOFormatError(f"unparsed line: {line[:80]}")
                ptr.append(int(m.group(1)))
                valid.append(int(m.group(2), 2))
                nonleaf.append(int(m.group(3), 2))
                code.append(int(m.group(4)))
        return cls.from_absolute(ptr, valid, nonleaf, code)

    # -------------------------------------------------------------- file I/O
    def save_int32_dump(self, path):
        """CompactSVO.SaveToDisk (CompactSVO.cs:80-86): raw little-endian int32 descriptors."""
        self.to_v1().childDescriptors.astype("<i4").tofile(path)

    @classmethod
    def load_int32_dump(cls, path):
        desc = np.fromfile(path, dtype="<i4")
        return cls(childDescriptors=desc)

    def save(self, path):
        """Native pool file: 'SVOP', u32 version, u32 format, u64 count, nodes, attachments."""
        with open(path, "wb") as fh:
            fh.write(FILE_MAGIC + struct.pack("<IIQ", FILE_VERSION, self.format, len(self)))
            if self.format == 1:
                fh.write(self.childDescriptors.astype("<i4").tobytes())
            else:
                fh.write(self.nodes.astype("<u8").tobytes())
            fh.write(self.attachments.astype("<u4").tobytes())

    @classmethod
    def load(cls, path):
        with open(path, "rb") as fh:
            head = fh.read(20)
            if len(head) != 20 or head[:4] != FILE_MAGIC:
                raise SVOFormatError("not an SVOP node-pool file")
            version, fmt, n = struct.unpack("<IIQ", head[4:])
            if version != FILE_VERSION or fmt not in (1, 2):
                raise SVOFormatError(f"unsupported SVOP version/format {version}/{fmt}")
            width = 4 if fmt == 1 else 8
            raw_body, raw_att = fh.read(width * n), fh.read(8 * n)
            if len(raw_body) != width * n or len(raw_att) != 8 * n or fh.read(1):
                raise SVOFormatError("truncated or oversized SVOP file")
            body = np.frombuffer(raw_body, "<i4" if fmt == 1 else "<u8")
            att = np.frombuffer(raw_att, "<u4")
        if fmt == 1:
            return cls(childDescriptors=body.copy(), attachments=att.copy())
        return cls(nodes=body.copy(), attachments=att.copy())

    # ------------------------------------------------------------- analysis
    def leaf_voxels(self):
        """All leaf voxels as rows (node index, child slot, L, ix, iy, iz): the
        voxel spans [1 + i * 2^-L, 1 + (i + 1) * 2^-L] per axis of the [1,2]^3
        cube, its shader scale is 23 - L.  Test helper for
        brute-force first-hit checks; O(total leaves)."""
        n = len(self)
        lo, first = self.masks_and_first()
        valid = (lo >> 8) & 0xFF
        nonleaf = lo & 0xFF
        coord = np.zeros((n, 3), np.int64)   # integer position of each node at its level
        level = self.levels()
        order = np.argsort(level, kind="stable")
        order = order[level[order] > 0]
        leaves = []
        for li in np.unique(level[order]):
            cur = order[level[order] == li]
            for c in range(8):
                off = np.array([c & 1, (c >> 1) & 1, (c >> 2) & 1], np.int64)
                v = ((valid[cur] >> c) & 1).astype(bool)
                nl = ((nonleaf[cur] >> c) & 1).astype(bool)
                child_xyz = coord[cur] * 2 + off
                is_leaf = v & ~nl
                if is_leaf.any():
                    sel = cur[is_leaf]
                    leaves.append(np.column_stack([sel, np.full(len(sel), c), np.full(len(sel), li),
                                                   child_xyz[is_leaf]]))
                if nl.any():
                    sel = cur[nl]
                    rank = _popcount8(nonleaf[sel] & ((1 << c) - 1)).astype(np.int64)
                    kid = first[sel].astype(np.int64) + rank
                    coord[kid] = child_xyz[nl]
        if not leaves:
            return np.zeros((0, 6), np.int64)
        return np.concatenate(leaves).astype(np.int64)
