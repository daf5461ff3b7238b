"""Second, independent restatement of the traversal: the reference's C# CPU
tracer `NVIDIAIterativeNaiveTracer.RayStep`
(Assets/Scripts/SVO/CompactSVO/NVIDIAIterativeTracer.cs:72-290), vectorised
over rays with numpy float32 (one IEEE rounding per operation, no FMA).

TEST INFRASTRUCTURE ONLY.  It shares no code with the C oracle
(oracle/svo_oracle.c, the HLSL restatement) and follows the C# semantics,
which differ from the HLSL ones:

* caller-space ray: no world->SVO transform (the test feeds o/32 + 1.5);
* t_max clamped to 1 (:112) -- so only voxels within t_svo <= 1 are reachable;
* ABSOLUTE child pointers: parent = (cd >> 16) + popc8(child_masks & 0x7F)
  (:195-197), i.e. the reference `Text` dump's native form;
* exact stack of StackData(int, float) (:62-70, :188), null-initialised, and a
  pop from a never-written slot keeps parent / t_max (:238-242);
* popc8 through the 256-entry LUT (:319-342);
* Mathf.Min / Mathf.Max (params) as ordered comparisons (UnityEngine.Mathf:
  m = v[0]; if (v[i] < m) m = v[i]) -- NaN-order dependent, unlike HLSL min/max;
* no iteration cap (the loop ends when scale reaches s_max = 23, :135).

Output per ray: hit flag, parent, hit_idx = idx ^ octant_mask ^ 7 (:286),
scale, t_min (SVO units; the HLSL distance is 2048 * t_min).
"""
import numpy as np

S_MAX = 23
F32 = np.float32

# :319-337, generated (popcount of the 8-bit index)
POPC8_LUT = np.array([bin(i).count("1") for i in range(256)], np.int32)


def _f2i(x):
    return np.asarray(x, F32).view(np.int32)


def _i2f(x):
    return np.asarray(x, np.int32).view(F32)


def _min2(a, b):
    # Mathf.Min(float a, float b) => a < b ? a : b
    return np.where(a < b, a, b)


def _max2(a, b):
    # Mathf.Max(float a, float b) => a > b ? a : b
    return np.where(a > b, a, b)


def _min3(a, b, c):
    # Mathf.Min(params float[]): m = v[0]; for i >= 1: if (v[i] < m) m = v[i]
    m = a
    m = np.where(b < m, b, m)
    return np.where(c < m, c, m)


def _max3(a, b, c):
    m = a
    m = np.where(b > m, b, m)
    return np.where(c > m, c, m)


def descriptors_absolute(abs_child_ptr, valid_mask, nonleaf_mask):
    """C# descriptor words ptr16 << 16 | valid8 << 8 | nonleaf8 with an ABSOLUTE
    pointer (ChildDescriptor, Util.cs:60-87; the `Text` dump's form)."""
    ptr = np.asarray(abs_child_ptr, np.int64)
    assert ptr.min() >= 0 and ptr.max() < 32768
    w = (ptr << 16) | (np.asarray(valid_mask, np.int64) << 8) | np.asarray(nonleaf_mask, np.int64)
    return w.astype(np.int32)


def ray_step(svo, origins, dirs):
    """Trace rays (origins, dirs: [n, 3] float32, caller space) through the int32
    descriptor list `svo`.  Returns a dict of per-ray arrays: hit (bool), parent,
    hit_idx, scale, t_min (float32), iterations."""
    svo = np.asarray(svo, np.int32)
    o = np.asarray(origins, F32)
    d = np.asarray(dirs, F32)
    n = len(o)
    one, half_c, two, three, zero = F32(1.0), F32(0.5), F32(2.0), F32(3.0), F32(0.0)

    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        # :86-92
        coef = [F32(1.0) / -np.abs(d[:, k]) for k in range(3)]
        bias = [coef[k] * o[:, k] for k in range(3)]
        # :94-106
        octant = np.full(n, 7, np.int32)
        for k in range(3):
            pos_dir = d[:, k] > zero
            octant = np.where(pos_dir, octant ^ (1 << k), octant)
            bias[k] = np.where(pos_dir, three * coef[k] - bias[k], bias[k])
        # :108-112
        t_min = _max3(two * coef[0] - bias[0], two * coef[1] - bias[1], two * coef[2] - bias[2])
        t_max = _min3(coef[0] - bias[0], coef[1] - bias[1], coef[2] - bias[2])
        h = t_max.copy()
        t_min = _max2(t_min, zero)
        t_max = _min2(t_max, one)

        # :115-131
        parent = np.zeros(n, np.int64)
        cd = np.zeros(n, np.int32)
        idx = np.zeros(n, np.int32)
        pos = [np.full(n, one, F32) for _ in range(3)]
        scale = np.full(n, S_MAX - 1, np.int32)
        scale_exp2 = np.full(n, half_c, F32)
        for k in range(3):
            c = (F32(1.5) * coef[k] - bias[k]) > t_min
            idx = np.where(c, idx ^ (1 << k), idx)
            pos[k] = np.where(c, F32(1.5), pos[k])

        stack_parent = np.zeros((n, S_MAX + 1), np.int64)
        stack_tmax = np.zeros((n, S_MAX + 1), F32)
        stack_set = np.zeros((n, S_MAX + 1), bool)   # StackData[] starts null

        active = scale < S_MAX
        hit = np.zeros(n, bool)
        iters = np.zeros(n, np.int64)
        rows = np.arange(n)
        while active.any():
            iters += active
            a = active
            # :149-151 fetch unless cached
            need = a & (cd == 0)
            cd = np.where(need, svo[np.where(need, parent, 0)], cd)
            # :157-160
            corner = [pos[k] * coef[k] - bias[k] for k in range(3)]
            tc_max = _min3(corner[0], corner[1], corner[2])
            # :162-164 (int shift, wraps)
            child_shift = idx ^ octant
            child_masks = ((cd.astype(np.int64) << child_shift) & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
            # :166-178
            valid = ((child_masks & 0x8000) != 0) & (t_min <= t_max)
            tv_max = _min2(t_max, tc_max)
            half = scale_exp2 * half_c
            center = [half * coef[k] + corner[k] for k in range(3)]
            descend = a & valid & (t_min <= tv_max)
            # :181-183 terminate on a leaf child
            leaf = descend & ((child_masks & 0x0080) == 0)
            hit |= leaf
            push = descend & ~leaf
            # :187-189
            store = push & (tc_max < h)
            if store.any():
                r, s = rows[store], scale[store]
                stack_parent[r, s] = parent[store]
                stack_tmax[r, s] = t_max[store]
                stack_set[r, s] = True
            h = np.where(push, tc_max, h)
            # :195-197 absolute pointer (arithmetic shift)
            ofs = (cd >> 16).astype(np.int64) + POPC8_LUT[child_masks & 0x7F]
            parent = np.where(push, ofs, parent)
            # :200-209
            idx = np.where(push, 0, idx)
            scale = np.where(push, scale - 1, scale)
            scale_exp2 = np.where(push, half, scale_exp2)
            for k in range(3):
                c = push & (center[k] > t_min)
                idx = np.where(c, idx ^ (1 << k), idx)
                pos[k] = np.where(c, pos[k] + scale_exp2, pos[k])
            t_max = np.where(push, tv_max, t_max)
            cd = np.where(push, 0, cd)
            # :214-223 ADVANCE
            adv = a & ~descend
            step = np.zeros(n, np.int32)
            for k in range(3):
                c = adv & (corner[k] <= tc_max)
                step = np.where(c, step ^ (1 << k), step)
                pos[k] = np.where(c, pos[k] - scale_exp2, pos[k])
            t_min = np.where(adv, tc_max, t_min)
            idx = np.where(adv, idx ^ step, idx)
            # :226-256 POP
            pop = adv & ((idx & step) != 0)
            if pop.any():
                diff = np.zeros(n, np.int32)
                for k in range(3):
                    c = pop & ((step & (1 << k)) != 0)
                    x = _f2i(pos[k]) ^ _f2i(pos[k] + scale_exp2)
                    diff = np.where(c, diff | x, diff)
                new_scale = (_f2i(diff.astype(F32)) >> 23) - 127
                scale = np.where(pop, new_scale, scale)
                assert not np.any(scale[pop] > S_MAX), "C# would index past stack[s_max] (IndexOutOfRange)"
                scale_exp2 = np.where(pop, _i2f(((scale - S_MAX + 127) << 23).astype(np.int32)), scale_exp2)
                sc = np.clip(scale, 0, S_MAX)
                got = pop & stack_set[rows, sc]
                parent = np.where(got, stack_parent[rows, sc], parent)
                t_max = np.where(got, stack_tmax[rows, sc], t_max)
                sh = [_f2i(pos[k]) >> sc for k in range(3)]
                for k in range(3):
                    pos[k] = np.where(pop, _i2f((sh[k] << sc).astype(np.int32)), pos[k])
                idx = np.where(pop, (sh[0] & 1) | ((sh[1] & 1) << 1) | ((sh[2] & 1) << 2), idx)
                h = np.where(pop, zero, h)
                cd = np.where(pop, 0, cd)
            active = a & ~hit & (scale < S_MAX)
    hit &= scale < S_MAX
    return {"hit": hit, "parent": parent, "hit_idx": (idx ^ octant ^ 7).astype(np.int32), "scale": scale,
            "t_min": t_min, "iterations": iters}
