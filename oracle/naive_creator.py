"""Pure-Python restatement of the reference SVO builder -- TEST INFRASTRUCTURE ONLY.

An object-recursive transcription of RT.CS.NaiveCreator.Create(sampler, maxLevel)
(Assets/Scripts/SVO/CompactSVO/NaiveCreator.cs) used to check the native,
level-parallel builder (libsvo_build.so) on small trees:
  BuildTree        NaiveCreator.cs:52-118      IsEdge        :121-130
  CompressSVO(Aux) NaiveCreator.cs:132-193     GetAttachment :195-257
  CompressColor    NaiveCreator.cs:351-356     encodeRawNormal16 :547-571
with the Custom1 / Simplex samplers (SampleFunctions.cs:20-47) over an
OpenSimplex 3D (Noise/Simplex.cs:190-324, seed 7) written independently here.
C# float arithmetic is emulated with numpy.float32 scalars (one rounding per
operation); the noise runs in Python floats (IEEE double), as in C#.
Only small maxLevel values (<= 6) are practical.
"""
import math

import numpy as np

F = np.float32

# ---------------------------------------------------------------- OpenSimplex
STRETCH_3D = -1.0 / 6.0
SQUISH_3D = 1.0 / 3.0
NORM_3D = 1.0 / 103.0


def _lcg(seed):
    return (seed * 6364136223846793005 + 1442695040888963407) & 0xFFFFFFFFFFFFFFFF


def _signed(v):
    return v - (1 << 64) if v >= (1 << 63) else v


class OpenSimplex3:
    def __init__(self, seed=7):
        s = seed & 0xFFFFFFFFFFFFFFFF
        for _ in range(3):
            s = _lcg(s)
        source = list(range(256))
        self.perm = [0] * 256
        self.perm3 = [0] * 256
        for i in range(255, -1, -1):
            s = _lcg(s)
            v = _signed((s + 31) & 0xFFFFFFFFFFFFFFFF)
            r = (abs(v) % (i + 1)) * (1 if v >= 0 else -1)   # C# long % : sign of the dividend
            if r < 0:
                r += i + 1
            self.perm[i] = source[r]
            self.perm3[i] = (self.perm[i] % 24) * 3
            source[r] = source[i]
        self.grad = []
        for k in range(8):
            sx = 1 if k & 1 else -1
            sy = -1 if k & 2 else 1
            sz = -1 if k & 4 else 1
            self.grad += [sx * 11, sy * 4, sz * 4, sx * 4, sy * 11, sz * 4, sx * 4, sy * 4, sz * 11]

    @staticmethod
    def _extras(xins, yins, zins):
        """Lattice offsets of the contributing vertices for a point of the unit
        cell (the OpenSimplex region decisions)."""
        s = xins + yins + zins
        if s <= 1:
            base = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1)]
            a_p, a_s, b_p, b_s = 1, xins, 2, yins
            if a_s >= b_s and zins > b_s:
                b_s, b_p = zins, 4
            elif a_s < b_s and zins > a_s:
                a_s, a_p = zins, 4
            w = 1 - s
            if w > a_s or w > b_s:
                c = b_p if b_s > a_s else a_p
                x0, x1 = (-1, 0) if not c & 1 else (1, 1)
                if not c & 2:
                    y0 = y1 = 0
                    if not c & 1:
                        y1 -= 1
                    else:
                        y0 -= 1
                else:
                    y0 = y1 = 1
                z0, z1 = (0, -1) if not c & 4 else (1, 1)
            else:
                c = a_p | b_p
                x0, x1 = (0, -1) if not c & 1 else (1, 1)
                y0, y1 = (0, -1) if not c & 2 else (1, 1)
                z0, z1 = (0, -1) if not c & 4 else (1, 1)
            return base + [(x0, y0, z0), (x1, y1, z1)]
        if s >= 2:
            base = [(1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1)]
            a_p, a_s, b_p, b_s = 6, xins, 5, yins
            if a_s <= b_s and zins < b_s:
                b_s, b_p = zins, 3
            elif a_s > b_s and zins < a_s:
                a_s, a_p = zins, 3
            w = 3 - s
            if w < a_s or w < b_s:
                c = b_p if b_s < a_s else a_p
                x0, x1 = (2, 1) if c & 1 else (0, 0)
                if c & 2:
                    y0 = y1 = 1
                    if c & 1:
                        y1 += 1
                    else:
                        y0 += 1
                else:
                    y0 = y1 = 0
                z0, z1 = (1, 2) if c & 4 else (0, 0)
            else:
                c = a_p & b_p
                x0, x1 = (1, 2) if c & 1 else (0, 0)
                y0, y1 = (1, 2) if c & 2 else (0, 0)
                z0, z1 = (1, 2) if c & 4 else (0, 0)
            return base + [(x0, y0, z0), (x1, y1, z1)]
        base = [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (1, 0, 1), (0, 1, 1)]
        p1 = xins + yins
        a_s, a_p, a_f = (p1 - 1, 3, True) if p1 > 1 else (1 - p1, 4, False)
        p2 = xins + zins
        b_s, b_p, b_f = (p2 - 1, 5, True) if p2 > 1 else (1 - p2, 2, False)
        p3 = yins + zins
        if p3 > 1:
            sc = p3 - 1
            if a_s <= b_s and a_s < sc:
                a_s, a_p, a_f = sc, 6, True
            elif a_s > b_s and b_s < sc:
                b_s, b_p, b_f = sc, 6, True
        else:
            sc = 1 - p3
            if a_s <= b_s and a_s < sc:
                a_s, a_p, a_f = sc, 1, False
            elif a_s > b_s and b_s < sc:
                b_s, b_p, b_f = sc, 1, False

        def p110(c):
            return (-1, 1, 1) if not c & 1 else (1, -1, 1) if not c & 2 else (1, 1, -1)

        def p002(c):
            return (2, 0, 0) if c & 1 else (0, 2, 0) if c & 2 else (0, 0, 2)

        if a_f == b_f:
            e = [(1, 1, 1), p002(a_p & b_p)] if a_f else [(0, 0, 0), p110(a_p | b_p)]
        else:
            c1, c2 = (a_p, b_p) if a_f else (b_p, a_p)
            e = [p110(c1), p002(c2)]
        return base + e

    @staticmethod
    def _hash(xins, yins, zins):
        s = xins + yins + zins
        return (int(yins - zins + 1) | int(xins - yins + 1) << 1 | int(xins - zins + 1) << 2 | int(s) << 3 |
                int(s + zins) << 5 | int(s + yins) << 7 | int(s + xins) << 9)

    def evaluate(self, x, y, z):
        """Noise/Simplex.cs:268-324 (contributions in lookup order, dx = dx0 + c.dx)."""
        so = (x + y + z) * STRETCH_3D
        xs, ys, zs = x + so, y + so, z + so

        def ffloor(v):
            vi = int(v)
            return vi - 1 if v < vi else vi
        xsb, ysb, zsb = ffloor(xs), ffloor(ys), ffloor(zs)
        sq = (xsb + ysb + zsb) * SQUISH_3D
        dx0, dy0, dz0 = x - (xsb + sq), y - (ysb + sq), z - (zsb + sq)
        xins, yins, zins = xs - xsb, ys - ysb, zs - zsb
        # the lookup is keyed by the hash; regions are decided at the cell's
        # representative point for that hash (ties resolve like the C# table)
        offs = self._offsets_for_hash(self._hash(xins, yins, zins))
        value = 0.0
        for (ox, oy, oz) in offs:
            m = float(ox + oy + oz)
            cdx, cdy, cdz = -ox - m * SQUISH_3D, -oy - m * SQUISH_3D, -oz - m * SQUISH_3D
            dx, dy, dz = dx0 + cdx, dy0 + cdy, dz0 + cdz
            attn = 2 - dx * dx - dy * dy - dz * dz
            if attn > 0:
                px, py, pz = xsb + ox, ysb + oy, zsb + oz
                i = self.perm3[(self.perm[(self.perm[px & 0xFF] + py) & 0xFF] + pz) & 0xFF]
                vp = self.grad[i] * dx + self.grad[i + 1] * dy + self.grad[i + 2] * dz
                attn *= attn
                value += attn * attn * vp
        return value * NORM_3D

    _table = None

    @classmethod
    def _offsets_for_hash(cls, h):
        if cls._table is None:
            rng = np.random.default_rng(12345)
            t = {}
            for p in rng.random((200000, 3)):
                hh = cls._hash(*p)
                if hh not in t:
                    t[hh] = cls._extras(*p)
            cls._table = t
        return cls._table.get(h, [])


_SIMPLEX = None


def simplex():
    global _SIMPLEX
    if _SIMPLEX is None:
        _SIMPLEX = OpenSimplex3(7)
    return _SIMPLEX


def _qmul(lhs, rhs):   # UnityEngine.Quaternion operator* (x, y, z, w), float steps left to right
    lx, ly, lz, lw = lhs
    rx, ry, rz, rw = rhs
    return (F(F(F(F(lw * rx) + F(lx * rw)) + F(ly * rz)) - F(lz * ry)),
            F(F(F(F(lw * ry) + F(ly * rw)) + F(lz * rx)) - F(lx * rz)),
            F(F(F(F(lw * rz) + F(lz * rw)) + F(lx * ry)) - F(ly * rx)),
            F(F(F(F(lw * rw) - F(lx * rx)) - F(ly * ry)) - F(lz * rz)))


def unity_rotation_matrix(ex, ey, ez):
    """Matrix4x4.Rotate(Quaternion.Euler(ex, ey, ez)) in single precision, rows of the
    3x3 rotation (SampleFunctions.cs:56).  Euler: each half angle (deg * Mathf.Deg2Rad) / 2
    with its sine / cosine correctly rounded to float, q = (qY * qX) * qZ (Unity's Z, X, Y
    order); Rotate: Matrix4x4.Rotate's products and sums.  Unity's native Euler
    conversion is not public, so bit parity with Unity itself is unpinned."""
    deg2rad = F(math.pi * 2 / 360)
    half = [F(F(F(v) * deg2rad) / F(2)) for v in (ex, ey, ez)]
    c = [F(math.cos(float(h))) for h in half]
    s_ = [F(math.sin(float(h))) for h in half]
    z0 = F(0)
    qx, qy, qz = (s_[0], z0, z0, c[0]), (z0, s_[1], z0, c[1]), (z0, z0, s_[2], c[2])
    x_, y_, z_, w_ = _qmul(_qmul(qy, qx), qz)
    x, y, z = F(x_ * F(2)), F(y_ * F(2)), F(z_ * F(2))
    xx, yy, zz = F(x_ * x), F(y_ * y), F(z_ * z)
    xy, xz, yz = F(x_ * y), F(x_ * z), F(y_ * z)
    wx, wy, wz = F(w_ * x), F(w_ * y), F(w_ * z)
    one = F(1)
    return [[F(one - F(yy + zz)), F(xy - wz), F(xz + wy)],
            [F(xy + wz), F(one - F(xx + zz)), F(yz - wx)],
            [F(xz - wy), F(yz + wx), F(one - F(xx + yy))]]


def rotated_cuboid(x, y, z, radius=0.6):
    """SampleFunctions.functions[3] (SampleFunctions.cs:35-38,54-68)."""
    m = unity_rotation_matrix(45, 45, 45)
    p = [F(F(F(v) - F(1.5)) * F(2)) for v in (x, y, z)]
    r = [F(F(F(row[0] * p[0]) + F(row[1] * p[1])) + F(row[2] * p[2])) for row in m]   # MultiplyVector
    d = [F(F(abs(v)) - F(radius)) for v in r]
    myz = d[1] if d[1] > d[2] else d[2]                 # Mathf.Max
    mx = d[0] if d[0] > myz else myz
    mag = F(math.sqrt(float(F(F(F(d[0] * d[0]) + F(d[1] * d[1])) + F(d[2] * d[2])))))   # Vector3.Magnitude
    return mx if mx < mag else mag                      # Mathf.Min


def sampler(kind):
    """SampleFunctions.functions[kind] (SampleFunctions.cs:20-47)."""
    if kind == 3:   # RotatedCuboid
        return rotated_cuboid
    if kind == 4:   # Custom1
        def f(x, y, z):
            result = F(y) - F(1.5)
            r = F(3.0)
            r2 = F(r * F(8))
            result = F(result + F(F(0.5) * F(simplex().evaluate(float(F(x) * r), float(F(y) * r), float(F(z) * r)))))
            result = F(result + F(F(0.15) * F(simplex().evaluate(float(F(x) * r2), float(F(y) * r2),
                                                                  float(F(z) * r2)))))
            return result
        return f
    if kind == 2:
        def f(x, y, z):
            r = F(1132.0)
            return F(simplex().evaluate(float(F(x) * r), float(F(y) * r), float(F(z) * r)))
        return f
    if kind == 0:
        return lambda x, y, z: F(F(0.5) - F(y))
    raise ValueError("sampler not restated")


# ------------------------------------------------------------- Unity helpers
def v3(x, y, z):
    return np.array([x, y, z], F)


def normalize(v):   # Vector3.Normalize
    mag = F(math.sqrt(float(F(F(v[0] * v[0]) + F(v[1] * v[1])) + F(v[2] * v[2]))))
    if mag > F(1e-5):
        return np.array([F(v[0] / mag), F(v[1] / mag), F(v[2] / mag)], F)
    return v3(0, 0, 0)


def dist(a, b):   # Vector3.Distance
    d = (a - b).astype(F)
    return F(math.sqrt(float(F(F(d[0] * d[0]) + F(d[1] * d[1])) + F(d[2] * d[2]))))


def cs_int(f):   # C# (int)float
    f = float(f)
    if not math.isfinite(f) or f >= 2147483648.0 or f < -2147483648.0:
        return -2147483648
    return int(f)


def clamp(v, lo, hi):   # Mathf.Clamp keeps NaN
    if v < lo:
        return F(lo)
    if v > hi:
        return F(hi)
    return F(v)


VFOFFSETS = [v3(c & 1, (c >> 1) & 1, (c >> 2) & 1) for c in range(8)]   # Constants.cs:23-26
VDIRECTIONS = [v3(1, 0, 0), v3(-1, 0, 0), v3(0, 1, 0), v3(0, -1, 0), v3(0, 0, 1), v3(0, 0, -1)]


class Node:
    def __init__(self, position, size, level, leaf):
        self.position = np.asarray(position, F)
        self.size = F(size)
        self.level = level
        self.leaf = leaf
        self.children = None
        self.normal = v3(0, 1, 0)            # Vector3.up (Util.cs Node ctor)
        self.color = np.array([1, 0, 0], F)  # Color.red

    def center(self):
        return (self.position + np.ones(3, F) * F(self.size / F(2))).astype(F)


def build_tree(node, level, sample, max_level):   # NaiveCreator.cs:52-118
    if node.leaf:
        p = (node.position + (np.ones(3, F) * node.size).astype(F) / F(2)).astype(F)
        if sample(p[0], p[1], p[2]) <= 0 and is_edge(node, sample):
            h = F(0.001)
            s0 = sample(p[0], p[1], p[2])
            n = v3(F(sample(F(p[0] - h), p[1], p[2]) - s0), F(sample(p[0], F(p[1] - h), p[2]) - s0),
                   F(sample(p[0], p[1], F(p[2] - h)) - s0))
            node.normal = (-normalize(n)).astype(F)
            node.color = np.array([node.position[0] - F(1), node.position[1] - F(1), node.position[2] - F(1)], F)
            return node
        return None
    node.children = [None] * 8
    half = F(node.size / F(2))
    exists = False
    for i in range(8):
        child = Node((node.position + (VFOFFSETS[i] * half).astype(F)).astype(F), half, level + 1,
                     level + 1 == max_level)
        node.children[i] = build_tree(child, level + 1, sample, max_level)
        exists = exists or node.children[i] is not None
    if exists:
        num = 0
        cx = F(0)
        nsum = v3(0, 0, 0)
        for c in node.children:
            if c is not None:
                num += 1
                cx = F(cx + c.color[0])
                nsum = (nsum + c.normal).astype(F)
        inv = F(F(1) / F(num))
        node.color = np.array([F(cx * inv), F(0) * inv, F(0) * inv], F)
        node.normal = normalize(nsum)
        return node
    return None


def is_edge(node, sample):   # NaiveCreator.cs:121-130
    for d in VDIRECTIONS:
        pos = (node.center() + (d * node.size).astype(F)).astype(F)
        if sample(pos[0], pos[1], pos[2]) > 0:
            return True
    return False


def compress_color(c):   # NaiveCreator.cs:351-356
    col = cs_int(F(F(32) * F(c[0] - F(0.00001))))
    col |= cs_int(F(F(64) * F(c[1] - F(0.00001)))) << 5
    col |= cs_int(F(F(32) * F(c[2] - F(0.00001)))) << 11
    return col & 0xFFFFFFFF


def encode_normal16(n):   # NaiveCreator.cs:547-571
    a = np.abs(n).astype(F)
    axis = 0 if a[0] >= max(a[1], a[2]) else (1 if a[1] >= a[2] else 2)
    tuv = n if axis == 0 else (v3(n[1], n[2], n[0]) if axis == 1 else v3(n[2], n[0], n[1]))
    sign = 0 if tuv[0] >= 0 else 0x8000
    with np.errstate(all="ignore"):
        at = F(abs(tuv[0]))
        u = (cs_int(clamp(F(F(tuv[1] / at) * F(63)), -64, 63)) & 0x7F) << 6
        v = cs_int(clamp(F(F(tuv[2] / at) * F(31)), -32, 31)) & 0x3F
    return (sign | (axis << 13) | u | v) & 0xFFFF


def get_attachment(node):   # NaiveCreator.cs:195-257
    A = v3(0, 0, 0)
    B = v3(0, 0, 0)
    num = 0
    for c in node.children:
        if c is None:
            continue
        num += 1
        col = np.array(c.color, F)
        if num == 1:
            A = col
        elif dist(A, col) > F(0):
            B = col
    cand = [A, B, (F(0.667) * A + F(0.333) * B).astype(F), (F(0.333) * A + F(0.667) * B).astype(F)]
    choices = 0
    for i, c in enumerate(node.children):
        if c is None:
            continue
        col = np.array(c.color, F)
        best, choice = F(100), 0
        for j in range(4):
            d = dist(col, cand[j])
            if d < best:
                best, choice = d, j
        choices |= choice << (2 * i)
    att = compress_color(A) | (compress_color(B) << 16) | (choices << 32) | (encode_normal16(node.normal) << 48)
    return att & 0xFFFFFFFF, (att >> 32) & 0xFFFFFFFF


def compress(root, get_leaf=None):   # CompressSVO / CompressSVOAux, NaiveCreator.cs:132-193
    """get_leaf: NaiveCreator.GetLeaf (:28-29, used at :156-159): every leaf child
    becomes a link -- its valid bit stays, its leaf bit is not set (so the
    shader takes it as a non-leaf child), and the node's child pointer is
    overwritten with get_leaf(child) - nodeIndex for each leaf child in slot
    order (the last one wins).  The reference passes (int)position and size
    (a Vector4Int); here the callback gets the child's integer coordinates at
    its level and the level: get_leaf(ix, iy, iz, level)."""
    nodes = [0]
    att = [0, 0]

    def aux(node, idx):
        if node is None or node.leaf:
            return
        ptr = 0
        valid = 0
        leaf_mask = 0
        for c in range(8):
            ch = node.children[c]
            if ch is None:
                continue
            valid |= 1 << c
            if ch.leaf:
                if get_leaf is not None:
                    scale = F(2) ** (ch.level - 1)
                    ix, iy, iz = (int(F(F(ch.position[k] - F(1)) * scale)) for k in range(3))
                    ptr = get_leaf(ix, iy, iz, ch.level) - idx
                else:
                    leaf_mask |= 1 << c
            else:
                if ptr == 0:
                    ptr = len(nodes) - idx
                nodes.append(0)
                att.extend([0, 0])
        k = ptr
        for c in range(8):
            ch = node.children[c]
            if ch is not None and not ch.leaf:
                aux(ch, idx + k)
                k += 1
        nonleaf = (leaf_mask ^ 255) & valid
        nodes[idx] = ((ptr << 16) | (valid << 8) | nonleaf) & 0xFFFFFFFF
        a0, a1 = get_attachment(node)
        att[2 * idx] = a0
        att[2 * idx + 1] = a1

    aux(root, 0)
    return np.array(nodes, np.uint32).view(np.int32), np.array(att, np.uint32)


def create(sample_kind, max_level, get_leaf=None):
    """NaiveCreator.Create(SampleFunctions.functions[kind], maxLevel) -> (descriptors,
    attachments); with get_leaf, the tree built that way is compressed as by
    NaiveCreator.Create(root, getLeaf) (NaiveCreator.cs:30-42)."""
    root = Node(v3(1, 1, 1), 1, 1, False)
    build_tree(root, 1, sampler(sample_kind), max_level)
    return compress(root, get_leaf)
