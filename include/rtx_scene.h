/*
 * rtx_scene.h — host glue kept outside the accelerated path (librtxscene).
 *
 * Plain-C re-implementations, with the reference's behaviour and error
 * messages, of the host code that feeds and drains the path:
 *   scene JSON loader  src/raytracer/scene.c:70-470   (replaces cJSON + scene.c)
 *   binary STL ingest  src/raytracer/object.c:521-587
 *   image plane setup  src/raytracer/image.c:34-56
 *   TIFF writer        src/raytracer/image.c:64-139   (8-bit or -f raw float + tag 65000 z)
 *   CLI flag parsing   src/core/argv.c, strhash.c, src/raytracer/render.c:61-116
 * The reference calls error() -> exit(1) on bad input; these return
 * RTX_ERR_SCENE / RTX_ERR_IO with the same message in rtx_scene_last_error().
 */
#ifndef RTX_SCENE_H
#define RTX_SCENE_H

#include "rtx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rtx_scene rtx_scene;

/* Load a scene file.  scale_arg = the value after -r ("norm" or a float), or
 * NULL for no scaling (scene.c:107-121).  Relative mesh paths are resolved
 * against base_dir, or against the CWD when base_dir is NULL (the reference). */
int rtx_scene_load(const char *path, const char *scale_arg, const char *base_dir, rtx_scene **out);
/* Same from an in-memory JSON document (name is used in messages only). */
int rtx_scene_parse(const char *json, size_t len, const char *name, const char *scale_arg, const char *base_dir,
		    rtx_scene **out);
const rtx_scene_desc *rtx_scene_desc_of(const rtx_scene *scene);
/* Number of JSON objects / mesh triangles, for logging like scene.c:305 */
uint32_t rtx_scene_num_json_objects(const rtx_scene *scene);
void rtx_scene_free(rtx_scene *scene);
const char *rtx_scene_last_error(void);

/* image_init (image.c:34-56) for resolution width x height. */
int rtx_frame_setup(const rtx_camera *camera, uint32_t width, uint32_t height, rtx_frame *out);

/* save_image (image.c:114-139): raw != 0 -> 32-bit float RGB + tag 65000 z. */
int rtx_tiff_write(const char *path, uint32_t width, uint32_t height, const float *rgb, const float *z, int raw);

/* hash_djb (strhash.c:14-20) */
uint32_t rtx_hash_djb(const char *s);

/* render_init (render.c:61-116) over argv: fills the renderer flags -b -a -s -g
 * -n -l -o into *p (other fields untouched).  Flags are matched anywhere in
 * argv by DJB hash (argv.c:38-55); unknown enum values keep the default. */
void rtx_params_from_argv(int argc, char **argv, rtx_params *p);

/* Write a binary STL (80-byte header, count, 50-byte records) — used by the
 * stand-in mesh generators; tris = n * 9 floats. */
int rtx_stl_write(const char *path, uint32_t n, const float *tris);

/* Read a raw TIFF as written by the reference's save_tiff_raw (-f) or by rtx_tiff_write(raw):
 * 3 x 32-bit float samples per pixel, contiguous, plus the z-buffer in private tag 65000
 * (what src/postprocess/image.c:29-75 image_load accepts, with its error checks).  *rgb and
 * *z are malloc'd; release them with rtx_buffer_free. */
int rtx_tiff_read_raw(const char *path, uint32_t *width, uint32_t *height, float **rgb, float **z);
void rtx_buffer_free(void *p);

/* The postprocessor's flags (src/postprocess/postproc.c:36-91, argv.c hashing semantics) into
 * *post; RTX_ERR_ARG with rtx_scene_last_error() for an unknown falloff name. */
int rtx_post_from_argv(int argc, char **argv, rtx_post *post);

#ifdef __cplusplus
}
#endif

#endif /* RTX_SCENE_H */
