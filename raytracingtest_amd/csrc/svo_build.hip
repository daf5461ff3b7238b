// svo_build.hip -- native SVO builder (include/svo_build.h).
//
// Restates the reference's RT.CS.NaiveCreator (Assets/Scripts/SVO/CompactSVO/
// NaiveCreator.cs) for MI355X:
//   * leaf classification (BuildTree leaf branch :54-73 + IsEdge :121-130) on
//     the GPU: every leaf centre of the 2^d grid (plus a one-cell halo for the
//     IsEdge probes) is sampled once per z-slab into a byte grid, surface
//     leaves are appended as Morton codes, and their finite-difference normals
//     (:58-63) are evaluated in a second kernel;
//   * tree + layout + attachments (BuildTree internal branch :77-115,
//     CompressSVOAux :138-193, GetAttachment :195-257) on the host, as a
//     direct restatement of the reference recursion over a Morton-sorted tree.
// Samplers: SampleFunctions.cs:13-48; OpenSimplex 3D with seed 7
// (Noise/Simplex.cs:190-218, :268-324).  The 3D contribution lookup is
// generated from the published OpenSimplex region logic (Kurt Spencer, 2014)
// and checked against the reference table's digest (tests/golden).
// Arithmetic: C# float/double semantics, one IEEE rounding per operation
// (-ffp-contract=off, no fast-math).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "svo_build.h"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string &m) { g_err = m; return code; }
constexpr int SVOB_OK = 0, SVOB_ERR_ARG = -1, SVOB_ERR_HIP = -4, SVOB_ERR_MEM = -6;

#define HIPB(expr)                                                                          \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) return fail(SVOB_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ------------------------------------------------------------------ OpenSimplex
constexpr double STRETCH_3D = -1.0 / 6.0;
constexpr double SQUISH_3D = 1.0 / 3.0;
constexpr double NORM_3D = 1.0 / 103.0;
constexpr int MAX_CONTRIB = 8;
constexpr int MAX_LISTS = 32;

struct ContribList {
    int count;
    int ox[MAX_CONTRIB], oy[MAX_CONTRIB], oz[MAX_CONTRIB];
    double dx[MAX_CONTRIB], dy[MAX_CONTRIB], dz[MAX_CONTRIB];
};

struct Simplex3 {
    uint8_t perm[256];
    uint8_t perm3D[256];
    int8_t list_of_hash[2048];   // -1: no entry (value 0)
    int nlists;
    ContribList lists[MAX_LISTS];
    double grad[72];
};

// Region logic of 3D OpenSimplex: lattice offsets of the two extra vertices.
// base 0: tetrahedron at (0,0,0); 1: tetrahedron at (1,1,1); 2: octahedron.
void region_contribs(double xins, double yins, double zins, int *base, int ext[2][3]) {
    const double inSum = xins + yins + zins;
    int x0, x1, y0, y1, z0, z1;
    if (inSum <= 1) {
        *base = 0;
        int aP = 1, bP = 2;
        double aS = xins, bS = yins;
        if (aS >= bS && zins > bS) { bS = zins; bP = 4; }
        else if (aS < bS && zins > aS) { aS = zins; aP = 4; }
        const double wins = 1 - inSum;
        if (wins > aS || wins > bS) {
            const int c = bS > aS ? bP : aP;
            if ((c & 1) == 0) { x0 = -1; x1 = 0; } else { x0 = x1 = 1; }
            if ((c & 2) == 0) { y0 = y1 = 0; if ((c & 1) == 0) y1 -= 1; else y0 -= 1; } else { y0 = y1 = 1; }
            if ((c & 4) == 0) { z0 = 0; z1 = -1; } else { z0 = z1 = 1; }
        } else {
            const int c = aP | bP;
            if ((c & 1) == 0) { x0 = 0; x1 = -1; } else { x0 = x1 = 1; }
            if ((c & 2) == 0) { y0 = 0; y1 = -1; } else { y0 = y1 = 1; }
            if ((c & 4) == 0) { z0 = 0; z1 = -1; } else { z0 = z1 = 1; }
        }
    } else if (inSum >= 2) {
        *base = 1;
        int aP = 6, bP = 5;
        double aS = xins, bS = yins;
        if (aS <= bS && zins < bS) { bS = zins; bP = 3; }
        else if (aS > bS && zins < aS) { aS = zins; aP = 3; }
        const double wins = 3 - inSum;
        if (wins < aS || wins < bS) {
            const int c = bS < aS ? bP : aP;
            if (c & 1) { x0 = 2; x1 = 1; } else { x0 = x1 = 0; }
            if (c & 2) { y0 = y1 = 1; if (c & 1) y1 += 1; else y0 += 1; } else { y0 = y1 = 0; }
            if (c & 4) { z0 = 1; z1 = 2; } else { z0 = z1 = 0; }
        } else {
            const int c = aP & bP;
            if (c & 1) { x0 = 1; x1 = 2; } else { x0 = x1 = 0; }
            if (c & 2) { y0 = 1; y1 = 2; } else { y0 = y1 = 0; }
            if (c & 4) { z0 = 1; z1 = 2; } else { z0 = z1 = 0; }
        }
    } else {
        *base = 2;
        double aS, bS;
        int aP, bP;
        bool aF, bF;
        const double p1 = xins + yins;
        if (p1 > 1) { aS = p1 - 1; aP = 3; aF = true; } else { aS = 1 - p1; aP = 4; aF = false; }
        const double p2 = xins + zins;
        if (p2 > 1) { bS = p2 - 1; bP = 5; bF = true; } else { bS = 1 - p2; bP = 2; bF = false; }
        const double p3 = yins + zins;
        if (p3 > 1) {
            const double s = p3 - 1;
            if (aS <= bS && aS < s) { aS = s; aP = 6; aF = true; }
            else if (aS > bS && bS < s) { bS = s; bP = 6; bF = true; }
        } else {
            const double s = 1 - p3;
            if (aS <= bS && aS < s) { aS = s; aP = 1; aF = false; }
            else if (aS > bS && bS < s) { bS = s; bP = 1; bF = false; }
        }
        auto perm110 = [](int c, int &x, int &y, int &z) {   // permutation of (1,1,-1) omitting c's axis
            if ((c & 1) == 0) { x = -1; y = 1; z = 1; } else if ((c & 2) == 0) { x = 1; y = -1; z = 1; } else { x = 1; y = 1; z = -1; }
        };
        auto perm002 = [](int c, int &x, int &y, int &z) {   // permutation of (0,0,2) on c's axis
            if (c & 1) { x = 2; y = 0; z = 0; } else if (c & 2) { x = 0; y = 2; z = 0; } else { x = 0; y = 0; z = 2; }
        };
        if (aF == bF) {
            if (aF) { x0 = y0 = z0 = 1; perm002(aP & bP, x1, y1, z1); }
            else { x0 = y0 = z0 = 0; perm110(aP | bP, x1, y1, z1); }
        } else {
            const int c1 = aF ? aP : bP, c2 = aF ? bP : aP;
            perm110(c1, x0, y0, z0);
            perm002(c2, x1, y1, z1);
        }
    }
    ext[0][0] = x0; ext[0][1] = y0; ext[0][2] = z0;
    ext[1][0] = x1; ext[1][1] = y1; ext[1][2] = z1;
}

__host__ __device__ inline int osn_hash(double xins, double yins, double zins) {
    const double inSum = xins + yins + zins;
    return (int)(yins - zins + 1) | (int)(xins - yins + 1) << 1 | (int)(xins - zins + 1) << 2 |
           (int)inSum << 3 | (int)(inSum + zins) << 5 | (int)(inSum + yins) << 7 | (int)(inSum + xins) << 9;
}

int init_simplex(Simplex3 *s, long long seed_in) {
    std::memset(s, 0, sizeof(*s));
    // Noise/Simplex.cs:190-218 permutation from the 64-bit LCG
    uint64_t seed = (uint64_t)seed_in;
    auto step = [](uint64_t v) { return v * 6364136223846793005ULL + 1442695040888963407ULL; };
    seed = step(step(step(seed)));
    uint8_t source[256];
    for (int i = 0; i < 256; ++i) source[i] = (uint8_t)i;
    for (int i = 255; i >= 0; --i) {
        seed = step(seed);
        const int64_t sv = (int64_t)(seed + 31ULL);
        int r = (int)(sv % (int64_t)(i + 1));
        if (r < 0) r += i + 1;
        s->perm[i] = source[r];
        s->perm3D[i] = (uint8_t)((s->perm[i] % 24) * 3);
        source[r] = source[i];
    }
    // gradient set: for sign pattern k, (+-11, +-4, +-4) and its two rotations
    for (int k = 0; k < 8; ++k) {
        const double sx = (k & 1) ? 1 : -1, sy = (k & 2) ? -1 : 1, sz = (k & 4) ? -1 : 1;
        const double g[9] = { sx * 11, sy * 4, sz * 4, sx * 4, sy * 11, sz * 4, sx * 4, sy * 4, sz * 11 };
        for (int j = 0; j < 9; ++j) s->grad[k * 9 + j] = g[j];
    }
    // contribution lists per hash, by sampling the region logic at interior points
    static const int base_sets[3][6][3] = {
        { {0, 0, 0}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1} },
        { {1, 1, 0}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1} },
        { {1, 0, 0}, {0, 1, 0}, {0, 0, 1}, {1, 1, 0}, {1, 0, 1}, {0, 1, 1} } };
    static const int base_count[3] = { 4, 4, 6 };
    for (int h = 0; h < 2048; ++h) s->list_of_hash[h] = -1;
    uint64_t rng = 0x9E3779B97F4A7C15ULL;
    auto uni = [&rng]() {
        rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
        return (double)(rng >> 11) * (1.0 / 9007199254740992.0);
    };
    for (int it = 0; it < 600000; ++it) {
        const double xi = uni(), yi = uni(), zi = uni();
        const int h = osn_hash(xi, yi, zi);
        int base, ext[2][3];
        region_contribs(xi, yi, zi, &base, ext);
        ContribList cl{};
        cl.count = base_count[base] + 2;
        for (int j = 0; j < cl.count; ++j) {
            const int *o = j < base_count[base] ? base_sets[base][j] : ext[j - base_count[base]];
            cl.ox[j] = o[0]; cl.oy[j] = o[1]; cl.oz[j] = o[2];
            const double m = (double)(o[0] + o[1] + o[2]);   // Contribution3(multiplier = sum, ...)
            cl.dx[j] = (double)(-o[0]) - m * SQUISH_3D;
            cl.dy[j] = (double)(-o[1]) - m * SQUISH_3D;
            cl.dz[j] = (double)(-o[2]) - m * SQUISH_3D;
        }
        int found = -1;
        for (int l = 0; l < s->nlists; ++l) {
            const ContribList &o = s->lists[l];
            if (o.count != cl.count) continue;
            bool same = true;
            for (int j = 0; j < cl.count && same; ++j)
                same = o.ox[j] == cl.ox[j] && o.oy[j] == cl.oy[j] && o.oz[j] == cl.oz[j];
            if (same) { found = l; break; }
        }
        if (found < 0) {
            if (s->nlists >= MAX_LISTS) return fail(SVOB_ERR_ARG, "opensimplex: too many contribution lists");
            s->lists[s->nlists] = cl;
            found = s->nlists++;
        }
        if (s->list_of_hash[h] >= 0 && s->list_of_hash[h] != found)
            return fail(SVOB_ERR_ARG, "opensimplex: hash does not determine the region");
        s->list_of_hash[h] = (int8_t)found;
    }
    return SVOB_OK;
}

__host__ __device__ inline int fast_floor(double x) {
    const int xi = (int)x;
    return x < xi ? xi - 1 : xi;
}

// Noise/Simplex.cs:268-324
__host__ __device__ inline double simplex_eval(const Simplex3 &s, double x, double y, double z) {
    const double stretchOffset = (x + y + z) * STRETCH_3D;
    const double xs = x + stretchOffset, ys = y + stretchOffset, zs = z + stretchOffset;
    const int xsb = fast_floor(xs), ysb = fast_floor(ys), zsb = fast_floor(zs);
    const double squishOffset = (double)(xsb + ysb + zsb) * SQUISH_3D;
    const double dx0 = x - ((double)xsb + squishOffset);
    const double dy0 = y - ((double)ysb + squishOffset);
    const double dz0 = z - ((double)zsb + squishOffset);
    const double xins = xs - (double)xsb, yins = ys - (double)ysb, zins = zs - (double)zsb;
    const int h = osn_hash(xins, yins, zins);
    const int li = (h >= 0 && h < 2048) ? s.list_of_hash[h] : -1;
    double value = 0.0;
    if (li < 0) return value * NORM_3D;
    const ContribList &c = s.lists[li];
    for (int j = 0; j < c.count; ++j) {
        const double dx = dx0 + c.dx[j];
        const double dy = dy0 + c.dy[j];
        const double dz = dz0 + c.dz[j];
        double attn = 2 - dx * dx - dy * dy - dz * dz;
        if (attn > 0) {
            const int px = xsb + c.ox[j], py = ysb + c.oy[j], pz = zsb + c.oz[j];
            const int i = s.perm3D[(s.perm[(s.perm[px & 0xFF] + py) & 0xFF] + pz) & 0xFF];
            const double valuePart = s.grad[i] * dx + s.grad[i + 1] * dy + s.grad[i + 2] * dz;
            attn *= attn;
            value += attn * attn * valuePart;
        }
    }
    return value * NORM_3D;
}

// RotatedCuboid's rotation, Matrix4x4.Rotate(Quaternion.Euler(45, 45, 45)) (SampleFunctions.cs:54-58),
// restated in single precision (oracle/naive_creator.py unity_rotation_matrix derives the same
// nine words and tests/test_builder.py pins them): the half angle (45 * Mathf.Deg2Rad) / 2, its
// sine and cosine correctly rounded to float, q = (qY * qX) * qZ (Unity's Z, X, Y order,
// Quaternion operator*), then Matrix4x4.Rotate's products and sums.  Unity's own native
// arithmetic for Euler -> quaternion is not public: parity with it is unpinned.
#define ROT45_M00 0x1.b504f4p-1f
#define ROT45_M01 -0x1.2bec30p-3f
#define ROT45_M02 0x1.000000p-1f
#define ROT45_M10 0x1.000000p-1f
#define ROT45_M11 0x1.fffffcp-2f
#define ROT45_M12 -0x1.6a09eap-1f
#define ROT45_M20 -0x1.2bec30p-3f
#define ROT45_M21 0x1.b504f6p-1f
#define ROT45_M22 0x1.fffffcp-2f

// SampleFunctions.cs:54-68: Cuboid(R p, radius); Mathf.Max / Mathf.Min as a > b ? a : b,
// Vector3.Magnitude as a float sum of squares through a double square root
__host__ __device__ inline float rotated_cuboid(float x, float y, float z) {
    const float px = (x - 1.5f) * 2.0f, py = (y - 1.5f) * 2.0f, pz = (z - 1.5f) * 2.0f;
    const float rx = ROT45_M00 * px + ROT45_M01 * py + ROT45_M02 * pz;   // MultiplyVector
    const float ry = ROT45_M10 * px + ROT45_M11 * py + ROT45_M12 * pz;
    const float rz = ROT45_M20 * px + ROT45_M21 * py + ROT45_M22 * pz;
    const float radius = 0.6f;
    const float dx = fabsf(rx) - radius, dy = fabsf(ry) - radius, dz = fabsf(rz) - radius;
    const float myz = dy > dz ? dy : dz;
    const float m = dx > myz ? dx : myz;
    const float mag = (float)sqrt((double)(dx * dx + dy * dy + dz * dz));
    return m < mag ? m : mag;
}

// SampleFunctions.cs:20-47 (float in, float out; C# single-precision steps)
__host__ __device__ inline float sample(const Simplex3 &s, int type, float x, float y, float z) {
    switch (type) {
    case 0:   // FlatGround (its Debug.LogFormat is dropped)
        return 0.5f - y;
    case 1: { // Sphere(p - 0.5, r = 0.25)
        const float px = x - 0.5f, py = y - 0.5f, pz = z - 0.5f;
        return px * px + py * py + pz * pz - 0.25f * 0.25f;
    }
    case 2: { // Simplex, r = 1132
        const float r = 1132.0f;
        return (float)simplex_eval(s, (double)(x * r), (double)(y * r), (double)(z * r));
    }
    case 3:   // RotatedCuboid, radius 0.6 (SampleFunctions.cs:35-38)
        return rotated_cuboid(x, y, z);
    default: { // 4: Custom1 simplex terrain
        float result = y - 1.5f;
        const float r = 3.0f;
        const float r2 = r * 8;
        result += 0.5f * (float)simplex_eval(s, (double)(x * r), (double)(y * r), (double)(z * r));
        result += 0.15f * (float)simplex_eval(s, (double)(x * r2), (double)(y * r2), (double)(z * r2));
        return result;
    }
    }
}

// ---------------------------------------------------------------- GPU kernels
// cell byte: bit0 = solid (s <= 0), bit1 = air (s > 0)
__global__ void sign_kernel(const Simplex3 *__restrict__ s, int type, int n, float size, int z_cell0, int z_cells,
                            uint8_t *__restrict__ cells) {
    const int np2 = n + 2;
    const size_t total = (size_t)np2 * np2 * z_cells;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int cx = (int)(i % np2);
        const int cy = (int)((i / np2) % np2);
        const int cz = z_cell0 + (int)(i / ((size_t)np2 * np2));
        // centre of leaf (c - 1): 1 + (c - 0.5) * size, exact dyadic
        const float px = 1.0f + ((float)cx - 0.5f) * size;
        const float py = 1.0f + ((float)cy - 0.5f) * size;
        const float pz = 1.0f + ((float)cz - 0.5f) * size;
        const float v = sample(*s, type, px, py, pz);
        cells[i] = (uint8_t)((v <= 0.0f ? 1 : 0) | (v > 0.0f ? 2 : 0));
    }
}

__device__ inline uint64_t spread3(uint32_t v) {
    uint64_t x = v & 0x1FFFFFu;
    x = (x | (x << 32)) & 0x1F00000000FFFFULL;
    x = (x | (x << 16)) & 0x1F0000FF0000FFULL;
    x = (x | (x << 8)) & 0x100F00F00F00F00FULL;
    x = (x | (x << 4)) & 0x10C30C30C30C30C3ULL;
    x = (x | (x << 2)) & 0x1249249249249249ULL;
    return x;
}

__device__ inline uint32_t compact3(uint64_t x) {
    x &= 0x1249249249249249ULL;
    x = (x ^ (x >> 2)) & 0x10C30C30C30C30C3ULL;
    x = (x ^ (x >> 4)) & 0x100F00F00F00F00FULL;
    x = (x ^ (x >> 8)) & 0x1F0000FF0000FFULL;
    x = (x ^ (x >> 16)) & 0x1F00000000FFFFULL;
    x = (x ^ (x >> 32)) & 0x1FFFFFULL;
    return (uint32_t)x;
}

// IsEdge: solid leaf with an air 6-neighbour (NaiveCreator.cs:56,121-130)
__global__ void classify_kernel(const uint8_t *__restrict__ cells, int n, int z0, int zc, uint64_t *__restrict__ out,
                                unsigned long long *__restrict__ counter, unsigned long long cap) {
    const int np2 = n + 2;
    const size_t plane = (size_t)np2 * np2;
    const size_t total = (size_t)n * n * zc;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % n);
        const int y = (int)((i / n) % n);
        const int zl = (int)(i / ((size_t)n * n));
        // slab cell buffer starts at padded z = z0 (leaf z0 - 1)
        const size_t c = (size_t)(zl + 1) * plane + (size_t)(y + 1) * np2 + (size_t)(x + 1);
        if (!(cells[c] & 1)) continue;
        const bool edge = (cells[c + 1] & 2) || (cells[c - 1] & 2) || (cells[c + np2] & 2) ||
                          (cells[c - np2] & 2) || (cells[c + plane] & 2) || (cells[c - plane] & 2);
        if (!edge) continue;
        const unsigned long long k = atomicAdd(counter, 1ULL);
        if (k < cap) {
            const uint32_t z = (uint32_t)(z0 + zl);
            out[k] = spread3((uint32_t)x) | (spread3((uint32_t)y) << 1) | (spread3(z) << 2);
        }
    }
}

__host__ __device__ inline void normalize_unity(float &x, float &y, float &z) {
    const float mag = (float)sqrt((double)(x * x + y * y + z * z));
    if (mag > 1e-5f) { x = x / mag; y = y / mag; z = z / mag; }
    else { x = 0.0f; y = 0.0f; z = 0.0f; }
}

// finite-difference normal, normal = -Normalize(n) (NaiveCreator.cs:58-63)
__global__ void normal_kernel(const Simplex3 *__restrict__ s, int type, float size, const uint64_t *__restrict__ codes,
                              size_t count, float *__restrict__ normals) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t code = codes[i];
        const float half = size / 2;
        const float px = (1.0f + (float)compact3(code) * size) + half;
        const float py = (1.0f + (float)compact3(code >> 1) * size) + half;
        const float pz = (1.0f + (float)compact3(code >> 2) * size) + half;
        const float h = 0.001f;
        float nx = sample(*s, type, px - h, py, pz) - sample(*s, type, px, py, pz);
        float ny = sample(*s, type, px, py - h, pz) - sample(*s, type, px, py, pz);
        float nz = sample(*s, type, px, py, pz - h) - sample(*s, type, px, py, pz);
        normalize_unity(nx, ny, nz);
        normals[3 * i + 0] = -nx;
        normals[3 * i + 1] = -ny;
        normals[3 * i + 2] = -nz;
    }
}

// ------------------------------------------------------------------ host layout
inline uint64_t spread3_h(uint32_t v) {
    uint64_t x = v & 0x1FFFFFu;
    x = (x | (x << 32)) & 0x1F00000000FFFFULL;
    x = (x | (x << 16)) & 0x1F0000FF0000FFULL;
    x = (x | (x << 8)) & 0x100F00F00F00F00FULL;
    x = (x | (x << 4)) & 0x10C30C30C30C30C3ULL;
    x = (x | (x << 2)) & 0x1249249249249249ULL;
    return x;
}
inline uint32_t compact3_h(uint64_t x) {
    x &= 0x1249249249249249ULL;
    x = (x ^ (x >> 2)) & 0x10C30C30C30C30C3ULL;
    x = (x ^ (x >> 4)) & 0x100F00F00F00F00FULL;
    x = (x ^ (x >> 8)) & 0x1F0000FF0000FFULL;
    x = (x ^ (x >> 16)) & 0x1F00000000FFFFULL;
    x = (x ^ (x >> 32)) & 0x1FFFFFULL;
    return (uint32_t)x;
}

struct V3 { float x, y, z; };

inline float dist3(const V3 &a, const V3 &b) {   // Vector3.Distance
    const float dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
    return (float)std::sqrt((double)(dx * dx + dy * dy + dz * dz));
}

inline int to_int_cs(float f) {   // C# (int)float: truncation, NaN/overflow -> int.MinValue
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int)f;
}

inline int compress_color(const V3 &c) {   // NaiveCreator.cs:351-356
    int color = to_int_cs(32.0f * (c.x - 0.00001f));
    color |= to_int_cs(64.0f * (c.y - 0.00001f)) << 5;
    color |= to_int_cs(32.0f * (c.z - 0.00001f)) << 11;
    return color;
}

inline float clampf_cs(float v, float lo, float hi) {   // Mathf.Clamp keeps NaN
    if (v < lo) v = lo; else if (v > hi) v = hi;
    return v;
}

inline uint32_t encode_normal16(const V3 &n) {   // NaiveCreator.cs:547-571
    const float ax = std::fabs(n.x), ay = std::fabs(n.y), az = std::fabs(n.z);
    const int axis = (ax >= std::max(ay, az)) ? 0 : (ay >= az) ? 1 : 2;
    V3 tuv;
    if (axis == 0) tuv = n;
    else if (axis == 1) tuv = { n.y, n.z, n.x };
    else tuv = { n.z, n.x, n.y };
    const uint32_t sign = tuv.x >= 0.0f ? 0u : 0x8000u;
    const uint32_t ab = (uint32_t)axis << 13;
    const float at = std::fabs(tuv.x);
    const uint32_t u = (uint32_t)((to_int_cs(clampf_cs((tuv.y / at) * 63.0f, -64.0f, 63.0f)) & 0x7F) << 6) & 0xFFFFu;
    const uint32_t v = (uint32_t)(to_int_cs(clampf_cs((tuv.z / at) * 31.0f, -32.0f, 31.0f)) & 0x3F);
    return (sign | ab | u | v) & 0xFFFFu;
}

// GetAttachment (NaiveCreator.cs:195-257)
inline void get_attachment(const bool present[8], const V3 color[8], const V3 &normal, uint32_t &w0, uint32_t &w1) {
    V3 A = { 0, 0, 0 }, B = { 0, 0, 0 };
    int numChildren = 0;
    const float bdist = 0.0f;
    for (int i = 0; i < 8; ++i) {
        if (!present[i]) continue;
        ++numChildren;
        if (numChildren == 1) A = color[i];
        else if (dist3(A, color[i]) > bdist) B = color[i];
    }
    const int ia = compress_color(A), ib = compress_color(B);
    const uint32_t inormal = encode_normal16(normal);
    V3 cand[4] = { A, B,
                   { 0.667f * A.x + 0.333f * B.x, 0.667f * A.y + 0.333f * B.y, 0.667f * A.z + 0.333f * B.z },
                   { 0.333f * A.x + 0.667f * B.x, 0.333f * A.y + 0.667f * B.y, 0.333f * A.z + 0.667f * B.z } };
    uint32_t choices = 0;
    for (int i = 0; i < 8; ++i) {
        if (!present[i]) continue;
        float best = 100.0f;
        int choice = 0;
        for (int j = 0; j < 4; ++j) {
            const float d = dist3(color[i], cand[j]);
            if (d < best) { best = d; choice = j; }
        }
        choices |= (uint32_t)choice << (i * 2);
    }
    const uint64_t att = (uint64_t)(uint32_t)ia | ((uint64_t)(uint32_t)ib << 16) | ((uint64_t)choices << 32) |
                         ((uint64_t)inormal << 48);
    w0 = (uint32_t)att;
    w1 = (uint32_t)(att >> 32);
}

struct Level {
    std::vector<uint64_t> key;
    std::vector<uint32_t> child_begin;   // into level k+1 (size = nodes + 1)
    std::vector<V3> normal, color;
};

struct Layout {
    int depth;
    std::vector<Level> lv;
    std::vector<uint64_t> nodes;
    std::vector<uint32_t> att;
    uint64_t count = 1;
    bool v1_ok = true;
};

void compress_aux(Layout &L, int k, uint32_t j, uint64_t nodeIndex) {   // CompressSVOAux
    const Level &cur = L.lv[k];
    const Level &kid = L.lv[k + 1];
    const bool kids_internal = (k + 1) < L.depth;
    const uint32_t b = cur.child_begin[j], e = cur.child_begin[j + 1];
    uint64_t childPointer = 0;
    uint32_t valid = 0;
    bool present[8] = { false };
    V3 colors[8] = {};
    for (uint32_t c = b; c < e; ++c) {
        const int slot = (int)(kid.key[c] & 7u);
        valid |= 1u << slot;
        present[slot] = true;
        colors[slot] = kid.color[c];
        if (kids_internal) {
            if (childPointer == 0) childPointer = L.count - nodeIndex;
            L.count++;
        }
    }
    if (kids_internal) {
        uint64_t cp = childPointer;
        for (uint32_t c = b; c < e; ++c) compress_aux(L, k + 1, c, nodeIndex + cp++);
    }
    const uint32_t nonleaf = kids_internal ? valid : 0u;
    if (childPointer > 0xFFFFu) L.v1_ok = false;
    const uint64_t first = nonleaf ? nodeIndex + childPointer : 0;
    L.nodes[nodeIndex] = (first << 32) | (uint64_t)((valid << 8) | nonleaf);
    get_attachment(present, colors, cur.normal[j], L.att[2 * nodeIndex], L.att[2 * nodeIndex + 1]);
}

int layout_from_sorted(int depth, std::vector<uint64_t> &codes, std::vector<V3> &normals, std::vector<V3> &colors,
                       svob_result *out) {
    Layout L;
    L.depth = depth;
    L.lv.resize(depth + 1);
    L.lv[depth].key = std::move(codes);
    L.lv[depth].normal = std::move(normals);
    L.lv[depth].color = std::move(colors);
    size_t total = 0;
    for (int k = depth - 1; k >= 0; --k) {   // BuildTree internal branch, bottom-up
        Level &cur = L.lv[k];
        const Level &kid = L.lv[k + 1];
        const size_t m = kid.key.size();
        for (size_t c = 0; c < m; ++c) {
            const uint64_t pk = kid.key[c] >> 3;
            if (cur.key.empty() || cur.key.back() != pk) {
                cur.key.push_back(pk);
                cur.child_begin.push_back((uint32_t)c);
            }
        }
        cur.child_begin.push_back((uint32_t)m);
        const size_t nn = cur.key.size();
        cur.normal.resize(nn);
        cur.color.resize(nn);
        for (size_t j = 0; j < nn; ++j) {
            V3 nsum = { 0, 0, 0 };
            float cx = 0.0f;
            int numChildren = 0;
            for (uint32_t c = cur.child_begin[j]; c < cur.child_begin[j + 1]; ++c) {
                ++numChildren;
                cx += kid.color[c].x;   // color.x += child.color.r (only r, NaiveCreator.cs:105)
                nsum.x = nsum.x + kid.normal[c].x;
                nsum.y = nsum.y + kid.normal[c].y;
                nsum.z = nsum.z + kid.normal[c].z;
            }
            const float inv = 1.0f / (float)numChildren;
            cur.color[j] = { cx * inv, 0.0f * inv, 0.0f * inv };
            normalize_unity(nsum.x, nsum.y, nsum.z);
            cur.normal[j] = nsum;
        }
        total += nn;
    }
    if (L.lv[0].key.size() != 1) return fail(SVOB_ERR_ARG, "internal: root level must hold one node");
    L.nodes.assign(total, 0);
    L.att.assign(2 * total, 0);
    compress_aux(L, 0, 0, 0);
    if (L.count != total) return fail(SVOB_ERR_ARG, "internal: layout count mismatch");

    out->n_nodes = total;
    out->depth = depth;
    out->v1_ok = L.v1_ok ? 1 : 0;
    out->n_leaves = L.lv[depth].key.size();
    out->nodes = (uint64_t *)std::malloc(total * sizeof(uint64_t));
    out->attachments = (uint32_t *)std::malloc(2 * total * sizeof(uint32_t));
    out->descriptors = (int32_t *)std::malloc(total * sizeof(int32_t));
    if (!out->nodes || !out->attachments || !out->descriptors) return fail(SVOB_ERR_MEM, "out of host memory");
    std::memcpy(out->nodes, L.nodes.data(), total * sizeof(uint64_t));
    std::memcpy(out->attachments, L.att.data(), 2 * total * sizeof(uint32_t));
    for (size_t i = 0; i < total; ++i) {
        const uint64_t nd = L.nodes[i];
        const uint32_t lo = (uint32_t)nd;
        const uint64_t first = nd >> 32;
        const uint32_t rel = (lo & 0xFFu) ? (uint32_t)(first - i) : 0u;
        out->descriptors[i] = (int32_t)((rel << 16) | lo);   // wraps exactly like C# when !v1_ok
    }
    return SVOB_OK;
}

int surface_leaves_gpu(int device, int type, int max_level, std::vector<uint64_t> &codes, std::vector<V3> &normals) {
    const int depth = max_level - 1;
    const int n = 1 << depth;
    const float size = std::ldexp(1.0f, -depth);
    Simplex3 hs;
    int rc = init_simplex(&hs, 7);   // SampleFunctions.cs:18 new OpenSimplexNoise(7)
    if (rc) return rc;
    HIPB(hipSetDevice(device));
    Simplex3 *ds = nullptr;
    uint8_t *cells = nullptr;
    uint64_t *dcodes = nullptr;
    unsigned long long *dcount = nullptr;
    auto cleanup = [&]() {
        if (ds) (void)hipFree(ds);
        if (cells) (void)hipFree(cells);
        if (dcodes) (void)hipFree(dcodes);
        if (dcount) (void)hipFree(dcount);
    };
    const size_t np2 = (size_t)n + 2;
    // slab height: keep the byte grid under ~512 MiB
    int slab = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, (512ull << 20) / (np2 * np2) - 2));
    size_t cap = std::max<size_t>(1 << 20, (size_t)n * n * 4);
    hipError_t e = hipMalloc(&ds, sizeof(Simplex3));
    if (e == hipSuccess) e = hipMemcpy(ds, &hs, sizeof(Simplex3), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&cells, np2 * np2 * (size_t)(slab + 2));
    if (e == hipSuccess) e = hipMalloc(&dcodes, cap * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&dcount, sizeof(unsigned long long));
    if (e != hipSuccess) { cleanup(); return fail(SVOB_ERR_HIP, std::string("builder alloc: ") + hipGetErrorString(e)); }
    codes.clear();
    for (int z0 = 0; z0 < n; z0 += slab) {
        const int zc = std::min(slab, n - z0);
        const int zcells = zc + 2;
        const size_t ncell = np2 * np2 * (size_t)zcells;
        const unsigned grid = (unsigned)std::min<size_t>((ncell + 255) / 256, 65536);
        hipLaunchKernelGGL(sign_kernel, dim3(grid), dim3(256), 0, 0, ds, type, n, size, z0, zcells, cells);
        e = hipGetLastError();
        if (e != hipSuccess) { cleanup(); return fail(SVOB_ERR_HIP, std::string("builder sign launch: ") + hipGetErrorString(e)); }
        for (;;) {
            e = hipMemset(dcount, 0, sizeof(unsigned long long));
            if (e != hipSuccess) break;
            const size_t nl = (size_t)n * n * zc;
            const unsigned g2 = (unsigned)std::min<size_t>((nl + 255) / 256, 65536);
            hipLaunchKernelGGL(classify_kernel, dim3(g2), dim3(256), 0, 0, cells, n, z0, zc, dcodes, dcount,
                               (unsigned long long)cap);
            e = hipGetLastError();
            if (e != hipSuccess) break;
            unsigned long long cnt = 0;
            e = hipMemcpy(&cnt, dcount, sizeof(cnt), hipMemcpyDeviceToHost);
            if (e != hipSuccess) break;
            if (cnt <= cap) {
                const size_t old = codes.size();
                codes.resize(old + cnt);
                e = hipMemcpy(codes.data() + old, dcodes, cnt * sizeof(uint64_t), hipMemcpyDeviceToHost);
                break;
            }
            (void)hipFree(dcodes);
            dcodes = nullptr;
            cap = (size_t)(cnt * 1.25) + 1024;
            e = hipMalloc(&dcodes, cap * sizeof(uint64_t));
            if (e != hipSuccess) break;
        }
        if (e != hipSuccess) { cleanup(); return fail(SVOB_ERR_HIP, std::string("builder classify: ") + hipGetErrorString(e)); }
    }
    std::sort(codes.begin(), codes.end());
    // normals of the sorted leaves
    normals.resize(codes.size());
    if (!codes.empty()) {
        float *dn = nullptr;
        if (codes.size() > cap) {
            (void)hipFree(dcodes);
            dcodes = nullptr;
            e = hipMalloc(&dcodes, codes.size() * sizeof(uint64_t));
        }
        if (e == hipSuccess) e = hipMemcpy(dcodes, codes.data(), codes.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&dn, codes.size() * 3 * sizeof(float));
        if (e == hipSuccess) {
            const unsigned g3 = (unsigned)std::min<size_t>((codes.size() + 255) / 256, 65536);
            hipLaunchKernelGGL(normal_kernel, dim3(g3), dim3(256), 0, 0, ds, type, size, dcodes, codes.size(), dn);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpy(normals.data(), dn, codes.size() * 3 * sizeof(float), hipMemcpyDeviceToHost);
        if (dn) (void)hipFree(dn);
        if (e != hipSuccess) { cleanup(); return fail(SVOB_ERR_HIP, std::string("builder normals: ") + hipGetErrorString(e)); }
    }
    cleanup();
    return SVOB_OK;
}

// Empty tree: CompressSVO's placeholder descriptor 0 stays 0; the root's
// attachment still encodes its default normal Vector3.up (Node ctor, Util.cs)
// with no children (NaiveCreator.cs:132-136, 195-257).
int empty_tree(int depth, svob_result *out) {
    out->n_nodes = 1; out->depth = depth; out->v1_ok = 1; out->n_leaves = 0;
    out->nodes = (uint64_t *)std::calloc(1, sizeof(uint64_t));
    out->attachments = (uint32_t *)std::calloc(2, sizeof(uint32_t));
    out->descriptors = (int32_t *)std::calloc(1, sizeof(int32_t));
    if (!out->nodes || !out->attachments || !out->descriptors) return fail(SVOB_ERR_MEM, "out of host memory");
    out->attachments[1] = encode_normal16({ 0.0f, 1.0f, 0.0f }) << 16;
    return SVOB_OK;
}

int check_sampler(int type, int max_level) {
    if (type < 0 || type > 4) return fail(SVOB_ERR_ARG, "unknown sampler");
    if (max_level < 2 || max_level > 22) return fail(SVOB_ERR_ARG, "max_level must be in [2, 22]");
    return SVOB_OK;
}

}  // namespace

extern "C" {

const char *svob_last_error(void) { return g_err.c_str(); }

void svob_free_ptr(void *p) { std::free(p); }

void svob_free(svob_result *r) {
    if (!r) return;
    std::free(r->descriptors);
    std::free(r->nodes);
    std::free(r->attachments);
    std::memset(r, 0, sizeof(*r));
}

int svob_opensimplex_table(int8_t *out) {
    if (!out) return fail(SVOB_ERR_ARG, "null out");
    static Simplex3 s;
    int rc = init_simplex(&s, 7);
    if (rc) return rc;
    std::memset(out, 0, 2048 * 25);
    for (int h = 0; h < 2048; ++h) {
        const int li = s.list_of_hash[h];
        if (li < 0) continue;
        const ContribList &c = s.lists[li];
        out[h * 25] = (int8_t)c.count;
        for (int j = 0; j < c.count; ++j) {
            out[h * 25 + 1 + 3 * j] = (int8_t)c.ox[j];
            out[h * 25 + 2 + 3 * j] = (int8_t)c.oy[j];
            out[h * 25 + 3 + 3 * j] = (int8_t)c.oz[j];
        }
    }
    return SVOB_OK;
}

int svob_eval_sampler(int sampler, size_t n, const float *xyz, float *out) {
    if (!xyz || !out) return fail(SVOB_ERR_ARG, "null argument");
    if (sampler < 0 || sampler > 4) return fail(SVOB_ERR_ARG, "unsupported sampler");
    static Simplex3 s;
    static bool ready = false;
    if (!ready) {
        int rc = init_simplex(&s, 7);
        if (rc) return rc;
        ready = true;
    }
    for (size_t i = 0; i < n; ++i) out[i] = sample(s, sampler, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    return SVOB_OK;
}

int svob_surface_leaves(int device, int sampler, int max_level, size_t *n_leaves, uint64_t **morton_out,
                        float **normals_out) {
    if (!n_leaves || !morton_out || !normals_out) return fail(SVOB_ERR_ARG, "null argument");
    int rc = check_sampler(sampler, max_level);
    if (rc) return rc;
    std::vector<uint64_t> codes;
    std::vector<V3> normals;
    rc = surface_leaves_gpu(device, sampler, max_level, codes, normals);
    if (rc) return rc;
    *n_leaves = codes.size();
    *morton_out = (uint64_t *)std::malloc(std::max<size_t>(1, codes.size()) * sizeof(uint64_t));
    *normals_out = (float *)std::malloc(std::max<size_t>(1, codes.size()) * 3 * sizeof(float));
    if (!*morton_out || !*normals_out) return fail(SVOB_ERR_MEM, "out of host memory");
    std::memcpy(*morton_out, codes.data(), codes.size() * sizeof(uint64_t));
    std::memcpy(*normals_out, normals.data(), codes.size() * 3 * sizeof(float));
    return SVOB_OK;
}

int svob_build_from_leaves(int depth, size_t n_leaves, const uint32_t *xyz, const float *normals, const float *colors,
                           svob_result *out) {
    if (!out || (n_leaves && (!xyz || !normals))) return fail(SVOB_ERR_ARG, "null argument");
    std::memset(out, 0, sizeof(*out));
    if (depth < 1 || depth > 21) return fail(SVOB_ERR_ARG, "depth must be in [1, 21]");
    const uint32_t n = 1u << depth;
    std::vector<std::pair<uint64_t, size_t>> order(n_leaves);
    for (size_t i = 0; i < n_leaves; ++i) {
        const uint32_t x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        if (x >= n || y >= n || z >= n) return fail(SVOB_ERR_ARG, "leaf coordinate outside the grid");
        order[i] = { spread3_h(x) | (spread3_h(y) << 1) | (spread3_h(z) << 2), i };
    }
    std::sort(order.begin(), order.end());
    for (size_t i = 1; i < n_leaves; ++i)
        if (order[i].first == order[i - 1].first) return fail(SVOB_ERR_ARG, "duplicate leaf coordinates");
    if (n_leaves == 0) return empty_tree(depth, out);
    std::vector<uint64_t> codes(n_leaves);
    std::vector<V3> nrm(n_leaves), col(n_leaves);
    const float inv = std::ldexp(1.0f, -depth);
    for (size_t i = 0; i < n_leaves; ++i) {
        const size_t s = order[i].second;
        codes[i] = order[i].first;
        nrm[i] = { normals[3 * s], normals[3 * s + 1], normals[3 * s + 2] };
        if (colors) col[i] = { colors[3 * s], colors[3 * s + 1], colors[3 * s + 2] };
        else col[i] = { (float)xyz[3 * s] * inv, (float)xyz[3 * s + 1] * inv, (float)xyz[3 * s + 2] * inv };
    }
    return layout_from_sorted(depth, codes, nrm, col, out);
}

int svob_build_sampler(int device, int sampler, int max_level, svob_result *out) {
    if (!out) return fail(SVOB_ERR_ARG, "null out");
    std::memset(out, 0, sizeof(*out));
    int rc = check_sampler(sampler, max_level);
    if (rc) return rc;
    std::vector<uint64_t> codes;
    std::vector<V3> normals;
    rc = surface_leaves_gpu(device, sampler, max_level, codes, normals);
    if (rc) return rc;
    const int depth = max_level - 1;
    if (codes.empty()) return empty_tree(depth, out);
    std::vector<V3> col(codes.size());
    const float inv = std::ldexp(1.0f, -depth);
    for (size_t i = 0; i < codes.size(); ++i)   // node.color = position - 1 (NaiveCreator.cs:66)
        col[i] = { (float)compact3_h(codes[i]) * inv, (float)compact3_h(codes[i] >> 1) * inv,
                   (float)compact3_h(codes[i] >> 2) * inv };
    return layout_from_sorted(depth, codes, normals, col, out);
}

}  // extern "C"
