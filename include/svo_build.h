/*
 * svo_build.h -- C-ABI of the native SVO builder (libsvo_build.so).
 *
 * Replaces the reference's CPU builder RT.CS.NaiveCreator
 * (Assets/Scripts/SVO/CompactSVO/NaiveCreator.cs) used by
 * RaytracingMaster.SetSVOBuffer() (RaytracingMaster.cs:90-109):
 *   Create(sampler, maxLevel)   NaiveCreator.cs:10-24
 *   BuildTree / IsEdge          NaiveCreator.cs:52-130   -> GPU leaf classification (HIP)
 *   CompressSVO / GetAttachment NaiveCreator.cs:132-257  -> host layout pass (C++)
 * Samplers: SampleFunctions.functions[] (SampleFunctions.cs:13-48) with the
 * seed-7 OpenSimplex noise (Noise/Simplex.cs).
 */
#ifndef SVO_BUILD_H
#define SVO_BUILD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SampleFunctions.Type (SampleFunctions.cs:4-11) */
typedef enum svob_sampler {
    SVOB_FLAT_GROUND = 0,
    SVOB_SPHERE = 1,
    SVOB_SIMPLEX = 2,
    SVOB_ROTATED_CUBOID = 3,   /* Cuboid(Rotate(Euler(45,45,45)) p, 0.6); the rotation restated in float */
    SVOB_CUSTOM1 = 4
} svob_sampler;

typedef struct svob_result {
    size_t    n_nodes;
    int       depth;          /* descriptor levels = maxLevel - 1 */
    int       v1_ok;          /* 1 if every relative child pointer fits 16 bits */
    int32_t  *descriptors;    /* V1 words (only meaningful when v1_ok) */
    uint64_t *nodes;          /* V2 nodes: first_child_abs << 32 | valid << 8 | nonleaf */
    uint32_t *attachments;    /* 2 words per node */
    size_t    n_leaves;       /* surface voxels */
} svob_result;

/* NaiveCreator.Create(SampleFunctions.functions[sampler], max_level): leaves
 * are classified on HIP device `device`. */
int svob_build_sampler(int device, int sampler, int max_level, svob_result *out);

/* Layout only (CompressSVO): surface leaves given as integer coordinates of a
 * 2^depth grid (x, y, z interleaved), per-leaf normals (float3) and optional
 * colours (float3, NULL = position - 1 as NaiveCreator.cs:66). */
int svob_build_from_leaves(int depth, size_t n_leaves, const uint32_t *xyz, const float *normals,
                           const float *colors, svob_result *out);

/* Surface leaves only (Morton-sorted 3*depth-bit codes + normals), malloc'd. */
int svob_surface_leaves(int device, int sampler, int max_level, size_t *n_leaves,
                        uint64_t **morton_out, float **normals_out);

/* Evaluate a sampler on the host (for tests): n points (x,y,z interleaved). */
int svob_eval_sampler(int sampler, size_t n, const float *xyz, float *out);

/* OpenSimplex 3D contribution table (2048 hashes x up to 8 lattice offsets):
 * out[h*25] = count (0 = no entry), then count x (dx, dy, dz) int8 offsets. */
int svob_opensimplex_table(int8_t *out /* 2048 * 25 */);

void svob_free(svob_result *r);
void svob_free_ptr(void *p);
const char *svob_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
