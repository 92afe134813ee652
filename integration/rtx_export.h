/*
 * rtx_export.h — the two accessors the drop-in (integration/rtx_render.c) needs from the
 * reference's private structs.  C-Raytracer keeps struct Sphere / Triangle / Plane private to
 * src/raytracer/object.c (object.c:25-44) and its texture structs private to material.c
 * (material.c:27-53), so each accessor is compiled inside that file: a maintainer appends
 *
 *     #include "object_export.inc"      at the end of src/raytracer/object.c
 *     #include "texture_export.inc"     at the end of src/raytracer/material.c
 *
 * and adds this directory and the MI355X library's include/ to the include path.
 */
#ifndef RTX_EXPORT_H
#define RTX_EXPORT_H

#include "rtx.h"

struct Object;
struct Texture;

/* object o (objects[i], object.h:48-53) as one rtx_object: type, num_lights, epsilon and the
 * geometry its *_postinit produced (object.c:231-237, 327-340, 448-466).  material is left for
 * the caller (an index into materials[]). */
void object_export(const struct Object *o, rtx_object *out);

/* the texture of a material (material.h:27-29) into out's texture fields (texture, periodic,
 * color, scale, mortar_width, noise_*, frequency_scale); returns 0, or -1 for an unknown kind */
int texture_export(const struct Texture *t, rtx_material *out);

#endif
