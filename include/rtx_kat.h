/*
 * rtx_kat.h — known-answer-test record layouts for rtx_kat() (GPU) and
 * rtx_oracle_kat() (CPU oracle).  Each kind evaluates one function of the hot
 * path over n fixed-size float records; integers travel as their float bit
 * patterns.  Fixtures come from the reference's own functions (oracle/ref_kat.c).
 *
 * kind               in (floats per record)                         out                        reference
 * KAT_MOLLER (0)     o3 d3 v0_3 e1_3 e2_3 eps          = 16          hit t                  = 2  object.c:422-441
 * KAT_SPHERE (1)     o3 d3 c3 r eps                    = 11          hit t n3               = 5  object.c:254-265,306-321
 * KAT_PLANE  (2)     o3 d3 n3 dd eps                   = 11          hit t n3               = 5  object.c:473-488
 * KAT_SLAB   (3)     o3 d3 lo3 hi3 eps                 = 13          hit tmin tmax          = 3  accel.c:112-158
 * KAT_NOISE  (4)     x y z                             = 3           noise                  = 1  SimplexNoise.c:99-194
 * KAT_TEXTURE(5)     type periodic c0_3 c1_3 scale mortar nfs ns fs P3 = 16  rgb3          = 3  material.c:152-200
 * KAT_SPH_LIGHT(6)   c3 r P3 u1 u2                     = 9           L3                     = 3  object.c:293-304
 * KAT_TRI_LIGHT(7)   v0_3 v1_3 v2_3 u1 u2              = 11          L3                     = 3  object.c:403-419
 * KAT_MORTON (8)     x y z (in [0,1])                  = 3           code(bits)             = 1  accel.c:72-88
 * KAT_U32    (9)     x                                 = 1           sat(bits) wrap(bits)   = 2  material.c:164
 * KAT_GI_DIR (10)    n3 eps u1 u2                      = 6           dir3                   = 3  render.c:240-281
 * KAT_REFRACT(11)    d3 n3 ior                         = 7           dir3                   = 3  render.c:320-335
 * -- the fast forms k_shadow actually runs (rtx_shadow.hip), checked against the exact ones --
 * KAT_ANY_TRI(12)    o3 d3 v0_3 e1_3 e2_3 eps tlim     = 17          hit                    = 1  object.c:422-441 (t < tlim)
 * KAT_SPH_LIGHT_SH(13) c3 r P3 u1 u2                   = 9           L3                     = 3  object.c:293-304
 * KAT_BOX_Q  (14)    o3 d3 lo3 hi3 qo3 qs3 tlim        = 19          hit(generic) hit(octant) = 2  accel.c:112-158
 *                    (the box is quantised on the device exactly as rtx_upload_scene quantises the
 *                     threaded BVH, rtx_quant.h, then tested by box_hit_q on the segment (0, tlim))
 * KAT_SPEC_POW(15)   x y                               = 2           fmaxf(0, pow(x, y))    = 1  render.c:224 (specular term,
 *                    x = specular_mul, y = shininess; the device runs sh_pow, the oracle glibc powf)
 * KAT_BOX_Q8 (16)   o3 d3 lo3 hi3 qo3 qs3 tlim org3 e3 = 25        hit(generic) hit(octant) = 2  accel.c:112-158
 *                    (the box quantised to 16 bits as for KAT_BOX_Q, then to 8 bits in an 8-wide node frame of
 *                     origin org (grid units, <= the 16-bit lo) and steps 2^e, rtx_quant.h rtx_quantise8, and
 *                     tested by the 8-wide walk's child test, rtx_shadow.hip w8_child)
 * Texture records use the params' u32conv for the float->uint32 conversion.
 */
#ifndef RTX_KAT_H
#define RTX_KAT_H

enum rtx_kat_kind {
	RTX_KAT_MOLLER = 0,
	RTX_KAT_SPHERE = 1,
	RTX_KAT_PLANE = 2,
	RTX_KAT_SLAB = 3,
	RTX_KAT_NOISE = 4,
	RTX_KAT_TEXTURE = 5,
	RTX_KAT_SPH_LIGHT = 6,
	RTX_KAT_TRI_LIGHT = 7,
	RTX_KAT_MORTON = 8,
	RTX_KAT_U32 = 9,
	RTX_KAT_GI_DIR = 10,
	RTX_KAT_REFRACT = 11,
	RTX_KAT_ANY_TRI = 12,
	RTX_KAT_SPH_LIGHT_SH = 13,
	RTX_KAT_BOX_Q = 14,
	RTX_KAT_SPEC_POW = 15,
	RTX_KAT_BOX_Q8 = 16,
	RTX_KAT_NKINDS = 17,
};
#define RTX_KAT_FIRST_SHADOW RTX_KAT_ANY_TRI /* kinds >= this run in rtx_shadow.hip */

static const int rtx_kat_in_width[RTX_KAT_NKINDS] = { 16, 11, 11, 13, 3, 16, 9, 11, 3, 1, 6, 7, 17, 9, 19, 2, 25 };
static const int rtx_kat_out_width[RTX_KAT_NKINDS] = { 2, 5, 5, 3, 1, 3, 3, 3, 1, 2, 3, 3, 1, 3, 2, 1, 2 };

#endif
