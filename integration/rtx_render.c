/*
 * rtx_render.c — the MI355X drop-in for C-Raytracer's trace/intersect/shade path.
 *
 * Replaces src/raytracer/accel.c and src/raytracer/render.c: it defines what main.c calls
 * (main.c:76-79 accel_init / render_init / render, main.c:84 accel_deinit) and what scene.c
 * writes (render.c:53 global_ambient_light_intensity), and sends the scene the reference
 * loaded into its globals (object.h:79-86, material.h:59-60, camera.h:27, image.h:33) through
 * the C-ABI of include/rtx.h.  Everything else of the reference stays: main.c, scene.c + cJSON,
 * object.c (with object_export.inc appended), material.c (with texture_export.inc appended),
 * camera.c, image.c (save_image writes image.raster / image.z_buffer as before, -f included),
 * and src/core.
 *
 * Build (Makefile.rt, this file in place of accel.c and render.c):
 *     CFLAGS  += -I<repo>/integration -I<repo>/include
 *     LDFLAGS += -L<repo>/c-raytracer_amd/lib -lrtx -lrtxscene -Wl,-rpath,<repo>/c-raytracer_amd/lib
 * Flags: the reference's -b -a -s -g -n -l -o (render.c:61-116, parsed by rtx_params_from_argv),
 * plus --gpus N (N devices of this process, rtx_group_*; default 1).
 * Errors end the program through the reference's own error() (error.h:21-33).
 */
#include <stdlib.h>
#include <string.h>

#include "accel.h"
#include "argv.h"
#include "camera.h"
#include "error.h"
#include "image.h"
#include "material.h"
#include "object.h"
#include "render.h"
#include "system.h"

#include "rtx.h"
#include "rtx_export.h"
#include "rtx_scene.h"

v3 global_ambient_light_intensity = { 0 }; /* render.c:53, set by scene_load */

static rtx_ctx *ctx;     /* one device */
static rtx_group *group; /* --gpus N > 1 */
static rtx_params params;

static int gpus(void)
{
	const int i = argv_check_with_args("--gpus", 1);
	return i ? atoi(myargv[i + 1]) : 1;
}

/* accel_init (accel.c:266-315): the scene as the reference holds it, flattened into an
 * rtx_scene_desc, uploaded; the library builds its BVHs on the device */
void accel_init(void)
{
	printf_log("Uploading scene to the MI355X path.");
	rtx_material *m = calloc(num_materials ? num_materials : 1, sizeof(*m));
	rtx_object *o = calloc(num_objects ? num_objects : 1, sizeof(*o));
	uint32_t *e = calloc(num_emittant_objects ? num_emittant_objects : 1, sizeof(*e));
	error_check(m && o && e, "Failed to allocate the MI355X scene description.");
	for (size_t i = 0; i < num_materials; i++) {
		const struct Material *s = &materials[i];
		m[i].id = s->id;
		memcpy(m[i].ks, s->ks, sizeof(v3));
		memcpy(m[i].ka, s->ka, sizeof(v3));
		memcpy(m[i].kr, s->kr, sizeof(v3));
		memcpy(m[i].kt, s->kt, sizeof(v3));
		memcpy(m[i].ke, s->ke, sizeof(v3));
		m[i].shininess = s->shininess;
		m[i].refractive_index = s->refractive_index;
		m[i].emittant = s->emittant;
		m[i].reflective = s->reflective;
		m[i].transparent = s->transparent;
		error_check(!texture_export(s->texture, &m[i]), "Material [%d]: unknown texture.", s->id);
	}
	/* emittant_objects[] holds every emitter that is not a mesh triangle, in object order
	 * (scene.c:349-351); mesh emitters are counted but never registered (scene.c:314-316) */
	size_t num_emittant = 0;
	for (size_t i = 0; i < num_objects; i++) {
		object_export(objects[i], &o[i]);
		o[i].material = (int32_t)(objects[i]->material - materials);
		if (objects[i]->material->emittant)
			num_emittant++;
	}
	error_check(num_emittant == num_emittant_objects, "Emittant meshes are not supported by the MI355X path.");
	for (size_t k = 0; k < num_emittant_objects; k++) {
		size_t i = 0;
		while (i < num_objects && objects[i] != emittant_objects[k])
			i++;
		error_check(i < num_objects, "Emittant object %zu is not in the object list.", k);
		e[k] = (uint32_t)i;
	}
	rtx_scene_desc d;
	memset(&d, 0, sizeof(d));
	d.num_materials = (uint32_t)num_materials;
	d.materials = m;
	d.num_objects = (uint32_t)num_objects;
	d.objects = o;
	d.num_emitters = (uint32_t)num_emittant_objects;
	d.emitters = e;
	memcpy(d.ambient, global_ambient_light_intensity, sizeof(v3));
	memcpy(d.camera.position, camera.position, sizeof(v3));
	memcpy(d.camera.vectors, camera.vectors, sizeof(camera.vectors));
	d.camera.fov = camera.fov;
	d.camera.focal_length = camera.focal_length;
	const int n = gpus();
	int rc;
	if (n > 1)
		rc = rtx_group_open(n, NULL, &group) || rtx_group_upload_scene(group, &d);
	else
		rc = rtx_open(0, &ctx) || rtx_upload_scene(ctx, &d);
	free(m);
	free(o);
	free(e);
	if (rc)
		error("%s", rtx_last_error());
}

/* render_init (render.c:61-116): the same flags into rtx_params, plus the drop-in's own
 * --rng const|counter|strat (the library's light-sample streams; const = every rand_flt() draw
 * 0.5, the reference built with a constant rand()) and --seed N */
void render_init(void)
{
	rtx_params_default(&params);
	rtx_params_from_argv(myargc, myargv, &params);
	int i = argv_check_with_args("--rng", 1);
	if (i) {
		if (!strcmp(myargv[i + 1], "const"))
			params.rng = RTX_RNG_CONST;
		else if (!strcmp(myargv[i + 1], "counter"))
			params.rng = RTX_RNG_COUNTER;
		else if (!strcmp(myargv[i + 1], "strat"))
			params.rng = RTX_RNG_STRAT;
		else
			error("--rng %s: expected const, counter or strat.", myargv[i + 1]);
	}
	i = argv_check_with_args("--seed", 1);
	if (i)
		params.seed = strtoull(myargv[i + 1], NULL, 10);
}

/* render (render.c:345-368): the frame image_init (image.c:34-56) set up, into image.raster and
 * image.z_buffer (overwritten, not accumulated) */
void render(void)
{
	printf_log("Commencing raytracing.");
	rtx_frame f;
	memset(&f, 0, sizeof(f));
	f.width = image.resolution[X];
	f.height = image.resolution[Y];
	memcpy(f.corner, image.corner, sizeof(v3));
	memcpy(f.step_x, image.vectors[X], sizeof(v3));
	memcpy(f.step_y, image.vectors[Y], sizeof(v3));
	memcpy(f.origin, camera.position, sizeof(v3));
	const int rc = group ? rtx_group_render(group, &f, &params, &image.raster[0][0], image.z_buffer)
			     : rtx_render(ctx, &f, &params, &image.raster[0][0], image.z_buffer);
	if (rc)
		error("%s", rtx_last_error());
}

/* accel_deinit (accel.c:100-103) */
void accel_deinit(void)
{
	rtx_group_close(group);
	rtx_close(ctx);
	group = NULL;
	ctx = NULL;
}

/* the rest of accel.h (render.c was their only caller): the device path answers these queries
 * inside rtx_render, so they are never reached */
void accel_get_closest_intersection(const struct Ray *ray, struct Object **closest_object, v3 closest_normal,
				    float *closest_distance)
{
	(void)ray;
	(void)closest_normal;
	*closest_object = NULL;
	*closest_distance = 0.f;
	error("accel_get_closest_intersection: the MI355X path traces inside rtx_render.");
}

bool accel_is_light_blocked(const struct Ray *ray, const float distance, v3 light_intensity, const struct Object *emittant_object)
{
	(void)ray;
	(void)distance;
	(void)light_intensity;
	(void)emittant_object;
	error("accel_is_light_blocked: the MI355X path traces inside rtx_render.");
}
