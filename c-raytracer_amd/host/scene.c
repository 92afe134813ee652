/*
 * Scene loader: JSON scene -> rtx_scene_desc.
 *
 * Same schema, defaults, object order and error conditions as the reference's
 * scene_load (src/raytracer/scene.c:70-470), object/material initialisation
 * (object.c, material.c:70-84, camera.c:19-33) and STL ingest
 * (object.c:521-587).  Where the reference calls error() -> exit(1), this
 * returns RTX_ERR_SCENE (or RTX_ERR_IO) with the same message.
 */
#include <errno.h>
#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "json.h"
#include "rtx_scene.h"
#include "vmath.h"

/* strhash.c:14-20 */
uint32_t rtx_hash_djb(const char *cp)
{
	uint32_t hash = 5381;
	while (*cp)
		hash = 33 * hash ^ (uint8_t)*cp++;
	return hash;
}

static __thread char g_err[512];

const char *rtx_scene_last_error(void)
{
	return g_err;
}

static int set_err(int code, const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof(g_err), fmt, ap);
	va_end(ap);
	return code;
}

struct rtx_scene {
	rtx_scene_desc desc;
	rtx_material *materials;
	rtx_object *objects;
	uint32_t *emitters;
	uint32_t cap_objects;
	uint32_t num_json_objects;
};

/* -------------------------------------------------------------------------- */

typedef struct {
	const char *name; /* scene filename for messages */
	const char *base_dir;
	rtx_scene *s;
} loader;

#define SCENE_ERR(L, fmt, ...) set_err(RTX_ERR_SCENE, fmt " in scene [%s].", ##__VA_ARGS__, (L)->name)

/* GET_JSON_TYPECHECK (scene.c:30-34) */
static int get_typed(loader *L, const jval *parent, const char *token, enum jtype t, const char *tname, jval **out)
{
	jval *v = json_get(parent, token);
	int ok = v && (v->type == t || (t == J_FALSE && v->type == J_TRUE));
	if (!ok)
		return SCENE_ERR(L, "Expected token [%s] of type [%s]", token, tname);
	*out = v;
	return RTX_OK;
}

/* GET_JSON_ARRAY (scene.c:36-40) */
static int get_array(loader *L, const jval *parent, const char *token, int len, jval **out)
{
	int rc = get_typed(L, parent, token, J_ARRAY, "Array", out);
	if (rc)
		return rc;
	if (json_size(*out) != len)
		return SCENE_ERR(L, "Expected token [%s] of length [%d]", token, len);
	return RTX_OK;
}

/* cJSON_parse_float_array (scene.c:59-68) */
static int parse_floats(loader *L, const jval *arr, float *out)
{
	int i = 0;
	for (const jval *c = arr->child; c; c = c->next) {
		if (!json_is_number(c))
			return SCENE_ERR(L, "Expected token in Array of type [Number]");
		out[i++] = (float)c->num;
	}
	return RTX_OK;
}

static int get_v3(loader *L, const jval *parent, const char *token, float *out)
{
	jval *a;
	int rc = get_array(L, parent, token, 3, &a);
	return rc ? rc : parse_floats(L, a, out);
}

static int get_num(loader *L, const jval *parent, const char *token, jval **out)
{
	return get_typed(L, parent, token, J_NUMBER, "Number", out);
}

/* camera_load + camera_init (scene.c:124-147, camera.c:19-33) */
static int camera_load(loader *L, const jval *json)
{
	if (json_size(json) != 5)
		return set_err(RTX_ERR_SCENE, "Expected token [Camera] to contain 5 elements.");
	rtx_camera *c = &L->s->desc.camera;
	jval *jfov, *jfl;
	float v[2][3];
	int rc;
	if ((rc = get_v3(L, json, "position", c->position)) || (rc = get_v3(L, json, "vector_x", v[0])) ||
	    (rc = get_v3(L, json, "vector_y", v[1])) || (rc = get_num(L, json, "fov", &jfov)) ||
	    (rc = get_num(L, json, "focal_length", &jfl)))
		return rc;
	float fov = (float)jfov->num;
	float focal_length = (float)jfl->num;
	if (!(fov > 0.f && fov < 180.f))
		return set_err(RTX_ERR_SCENE, "Expected camera fov [%.2f] between [0.] and [180.].", (double)fov);
	c->fov = fov;
	c->focal_length = focal_length;
	vm_assign3(c->vectors[0], v[0]);
	vm_assign3(c->vectors[1], v[1]);
	vm_norm3(c->vectors[0]);
	vm_norm3(c->vectors[1]);
	vm_cross(c->vectors[0], c->vectors[1], c->vectors[2]);
	return RTX_OK;
}

/* texture_load (scene.c:195-293) */
static int texture_load(loader *L, const jval *json, rtx_material *m)
{
	jval *jtype;
	int rc = get_typed(L, json, "type", J_STRING, "String", &jtype);
	if (rc)
		return rc;
	switch (rtx_hash_djb(jtype->str)) {
	case 3226203393u: /* uniform */
		m->texture = RTX_TEX_UNIFORM;
		return get_v3(L, json, "color", m->color[0]);
	case 2234799246u: /* checkerboard */
	case 176032948u: { /* brick */
		int brick = rtx_hash_djb(jtype->str) == 176032948u;
		jval *jcolors, *jscale, *jmortar = NULL;
		if ((rc = get_array(L, json, "colors", 2, &jcolors)) || (rc = get_num(L, json, "scale", &jscale)))
			return rc;
		if (brick && (rc = get_num(L, json, "mortar width", &jmortar)))
			return rc;
		m->texture = brick ? RTX_TEX_BRICK : RTX_TEX_CHECKERBOARD;
		m->scale = (float)jscale->num;
		if (brick)
			m->mortar_width = (float)jmortar->num;
		int i = 0;
		for (const jval *c = jcolors->child; c; c = c->next) {
			if (!json_is_array(c))
				return SCENE_ERR(L, "Expected token in [colors] of type Array");
			if (json_size(c) != 3)
				return SCENE_ERR(L, "Expected token in [colors] of length 3");
			if ((rc = parse_floats(L, c, m->color[i])))
				return rc;
			i++;
		}
		return RTX_OK;
	}
	case 202158024u: { /* noisy periodic */
		jval *jnfs, *jns, *jfs, *jfunc;
		if ((rc = get_v3(L, json, "color", m->color[0])) || (rc = get_v3(L, json, "color gradient", m->color[1])) ||
		    (rc = get_num(L, json, "noise feature scale", &jnfs)) || (rc = get_num(L, json, "noise scale", &jns)) ||
		    (rc = get_num(L, json, "frequency scale", &jfs)) ||
		    (rc = get_typed(L, json, "function", J_STRING, "String", &jfunc)))
			return rc;
		m->texture = RTX_TEX_NOISY_PERIODIC;
		m->noise_feature_scale = (float)jnfs->num;
		m->noise_scale = (float)jns->num;
		m->frequency_scale = (float)jfs->num;
		switch (rtx_hash_djb(jfunc->str)) {
		case 193433777u: m->periodic = RTX_PERIODIC_SIN; break;
		case 193433504u: m->periodic = RTX_PERIODIC_SAW; break;
		case 837065195u: m->periodic = RTX_PERIODIC_TRIANGLE; break;
		case 2144888260u: m->periodic = RTX_PERIODIC_SQUARE; break;
		default:
			return SCENE_ERR(L, "Unexpected value [%s] of token [function]", jfunc->str);
		}
		return RTX_OK;
	}
	default:
		return SCENE_ERR(L, "Unrecognized token [%s] in texture", jtype->str);
	}
}

/* material_load + material_init (scene.c:165-193, material.c:70-84) */
static int material_load(loader *L, const jval *json, rtx_material *m)
{
	jval *jid, *jsh, *jri, *jtex;
	int rc;
	if ((rc = get_num(L, json, "id", &jid)) || (rc = get_num(L, json, "shininess", &jsh)) ||
	    (rc = get_num(L, json, "refractive_index", &jri)) ||
	    (rc = get_typed(L, json, "texture", J_OBJECT, "Object", &jtex)) || (rc = get_v3(L, json, "ks", m->ks)) ||
	    (rc = get_v3(L, json, "ka", m->ka)) || (rc = get_v3(L, json, "kr", m->kr)) ||
	    (rc = get_v3(L, json, "kt", m->kt)) || (rc = get_v3(L, json, "ke", m->ke)))
		return rc;
	m->id = json_int(jid);
	m->shininess = (float)jsh->num;
	m->refractive_index = (float)jri->num;
	if ((rc = texture_load(L, jtex, m)))
		return rc;
	/* MATERIAL_THRESHOLD 1e-6f, material.c:25,81-83 */
	m->emittant = vm_mag3(m->ke) > 1e-6f;
	m->reflective = vm_mag3(m->kr) > 1e-6f;
	m->transparent = vm_mag3(m->kt) > 1e-6f;
	return RTX_OK;
}

/* get_material (material.c:94-102): linear search, first match */
static int get_material(loader *L, int id, int *out)
{
	for (uint32_t i = 0; i < L->s->desc.num_materials; i++)
		if (L->s->materials[i].id == id) {
			*out = (int)i;
			return RTX_OK;
		}
	return set_err(RTX_ERR_SCENE, "Failed to get material id [%d].", id);
}

static rtx_object *push_object(loader *L)
{
	rtx_scene *s = L->s;
	if (s->desc.num_objects == s->cap_objects) {
		uint32_t cap = s->cap_objects ? s->cap_objects * 2 : 64;
		rtx_object *o = realloc(s->objects, sizeof(rtx_object) * cap);
		if (!o)
			return NULL;
		s->objects = o;
		s->cap_objects = cap;
	}
	rtx_object *o = &s->objects[s->desc.num_objects++];
	memset(o, 0, sizeof(*o));
	return o;
}

/* object_load (scene.c:363-376) */
static int object_header(loader *L, const jval *json, rtx_object *o, int type)
{
	jval *jmat;
	int rc = get_num(L, json, "material", &jmat);
	if (rc)
		return rc;
	jval *jeps = json_get(json, "epsilon");
	jval *jnl = json_get(json, "lights");
	o->type = type;
	o->epsilon = json_is_number(jeps) ? (float)jeps->num : -1.f;
	o->num_lights = json_is_number(jnl) ? (uint32_t)json_int(jnl) : 0u;
	return get_material(L, json_int(jmat), &o->material);
}

/* triangle_postinit (object.c:327-340) */
static void triangle_postinit(rtx_object *t)
{
	vm_sub3v(t->p1, t->p0, t->e1);
	vm_sub3v(t->p2, t->p0, t->e2);
	vm_cross(t->e1, t->e2, t->n);
	vm_norm3(t->n);
	if (t->epsilon == -1.f) {
		float magab = vm_mag3(t->e1) * vm_mag3(t->e2);
		t->epsilon = 0.003f * powf(0.5f * magab * sinf(acosf(vm_dot3(t->e1, t->e2) / magab)), 0.75f);
	}
}

static void mulmv(float m[3][3], const float *v, float *r)
{
	r[0] = vm_dot3(m[0], v);
	r[1] = vm_dot3(m[1], v);
	r[2] = vm_dot3(m[2], v);
}

/* mesh_load + mesh_to_objects + stl_load_objects (scene.c:437-457, object.c:521-587) */
static int mesh_load(loader *L, const jval *json)
{
	jval *jfile, *jscale;
	float position[3], rot[3];
	int rc;
	if ((rc = get_typed(L, json, "filename", J_STRING, "String", &jfile)) || (rc = get_v3(L, json, "position", position)) ||
	    (rc = get_v3(L, json, "rotation", rot)) || (rc = get_num(L, json, "scale", &jscale)))
		return rc;
	float scale = (float)jscale->num;
	rtx_object tmpl;
	memset(&tmpl, 0, sizeof(tmpl));
	if ((rc = object_header(L, json, &tmpl, RTX_TRIANGLE)))
		return rc;
	if (L->s->materials[tmpl.material].emittant)
		return SCENE_ERR(L, "Mesh [%s] has an emittant material: the reference counts but never registers mesh "
				    "emitters (scene.c:314-316 vs 349-351) and dereferences an unset emitter slot",
				 jfile->str);

	const char *fname = jfile->str;
	char path[4096];
	if (L->base_dir && fname[0] != '/')
		snprintf(path, sizeof(path), "%s/%s", L->base_dir, fname);
	else
		snprintf(path, sizeof(path), "%s", fname);
	FILE *f = fopen(path, "rb");
	if (!f)
		return set_err(RTX_ERR_IO, "Failed to open mesh file %s.", fname);

	char header[5];
	if (fread(header, 1, 5, f) != 5) {
		fclose(f);
		return set_err(RTX_ERR_IO, "Failed to read header of mesh file [%s].", fname);
	}
	if (!strncmp("solid", header, 5)) {
		fclose(f);
		return set_err(RTX_ERR_SCENE, "Mesh file [%s] does not use binary encoding.", fname);
	}
	/* ZYX rotation matrix, object.c:548-562 */
	float a = cosf(rot[2]) * sinf(rot[1]);
	float b = sinf(rot[2]) * sinf(rot[1]);
	float R[3][3] = {
		{ cosf(rot[2]) * cosf(rot[1]), a * sinf(rot[0]) - sinf(rot[2]) * cosf(rot[0]),
		  a * cosf(rot[0]) + sinf(rot[2]) * sinf(rot[0]) },
		{ sinf(rot[2]) * cosf(rot[1]), b * sinf(rot[0]) + cosf(rot[2]) * cosf(rot[0]),
		  b * cosf(rot[0]) - cosf(rot[2]) * sinf(rot[0]) },
		{ -sinf(rot[1]), cosf(rot[1]) * sinf(rot[0]), cosf(rot[1]) * cosf(rot[0]) },
	};
	uint32_t ntri;
	if (fseek(f, 80, SEEK_SET)) {
		fclose(f);
		return set_err(RTX_ERR_IO, "Failed to read header of mesh file.");
	}
	if (fread(&ntri, 4, 1, f) != 1) {
		fclose(f);
		return set_err(RTX_ERR_IO, "Failed to read triangle count in mesh file.");
	}
	unsigned char rec[50];
	for (uint32_t i = 0; i < ntri; i++) {
		if (fread(rec, 50, 1, f) != 1) {
			fclose(f);
			return set_err(RTX_ERR_IO, "Failed to read triangle in mesh file [%s].", fname);
		}
		float v[3][3];
		memcpy(v, rec + 12, sizeof(v));
		rtx_object *t = push_object(L);
		if (!t) {
			fclose(f);
			return set_err(RTX_ERR_NOMEM, "Unable to allocate mesh triangles.");
		}
		*t = tmpl;
		float *dst[3] = { t->p0, t->p1, t->p2 };
		for (int j = 0; j < 3; j++) {
			float tmp[3];
			mulmv(R, v[j], tmp);
			vm_mul3s(tmp, scale, dst[j]);
			vm_add3v(dst[j], position, dst[j]);
		}
		triangle_postinit(t);
	}
	fclose(f);
	return RTX_OK;
}

/* objects_load (scene.c:295-361) */
static int objects_load(loader *L, const jval *json)
{
	rtx_scene *s = L->s;
	uint32_t n = (uint32_t)json_size(json);
	if (!n)
		return SCENE_ERR(L, "Expected token [Objects] to contain nonzero element count");
	s->num_json_objects = n;

	/* first pass (scene.c:306-321): shape checks + emitter count */
	uint32_t num_emittant = 0;
	int rc;
	for (const jval *it = json->child; it; it = it->next) {
		if (!json_is_object(it))
			return SCENE_ERR(L, "Expected token in [Objects] of type Object");
		jval *jt, *jp, *jm;
		if ((rc = get_typed(L, it, "type", J_STRING, "String", &jt)) ||
		    (rc = get_typed(L, it, "parameters", J_OBJECT, "Object", &jp)) || (rc = get_num(L, jp, "material", &jm)))
			return rc;
		int mi;
		if ((rc = get_material(L, json_int(jm), &mi)))
			return rc;
		if (s->materials[mi].emittant)
			num_emittant++;
	}
	if (!num_emittant)
		return SCENE_ERR(L, "Expected non-zero number of emittant objects");

	s->emitters = calloc(num_emittant, sizeof(uint32_t));
	if (!s->emitters)
		return set_err(RTX_ERR_NOMEM, "Unable to allocate emitters.");

	/* second pass (scene.c:331-360) */
	for (const jval *it = json->child; it; it = it->next) {
		jval *jt = json_get(it, "type"), *jp = json_get(it, "parameters");
		rtx_object *o;
		switch (rtx_hash_djb(jt->str)) {
		case 3324768284u: { /* Sphere: sphere_load scene.c:378-395, sphere_postinit object.c:231-237 */
			jval *jr;
			float pos[3];
			if ((rc = get_num(L, jp, "radius", &jr)) || (rc = get_v3(L, jp, "position", pos)))
				return rc;
			if (!(o = push_object(L)))
				return set_err(RTX_ERR_NOMEM, "Unable to allocate objects.");
			o->radius = (float)jr->num;
			vm_assign3(o->p0, pos);
			if ((rc = object_header(L, jp, o, RTX_SPHERE)))
				return rc;
			if (o->epsilon == -1.f)
				o->epsilon = o->radius * 0.0003f;
		} break;
		case 103185867u: { /* Triangle: triangle_load scene.c:397-416 */
			float v[3][3];
			if ((rc = get_v3(L, jp, "vertex_1", v[0])) || (rc = get_v3(L, jp, "vertex_2", v[1])) ||
			    (rc = get_v3(L, jp, "vertex_3", v[2])))
				return rc;
			if (!(o = push_object(L)))
				return set_err(RTX_ERR_NOMEM, "Unable to allocate objects.");
			vm_assign3(o->p0, v[0]);
			vm_assign3(o->p1, v[1]);
			vm_assign3(o->p2, v[2]);
			if ((rc = object_header(L, jp, o, RTX_TRIANGLE)))
				return rc;
			triangle_postinit(o);
		} break;
		case 232719795u: { /* Plane: plane_load scene.c:418-435, plane_new/postinit object.c:448-466 */
			float pos[3], nrm[3];
			if ((rc = get_v3(L, jp, "position", pos)) || (rc = get_v3(L, jp, "normal", nrm)))
				return rc;
			if (!(o = push_object(L)))
				return set_err(RTX_ERR_NOMEM, "Unable to allocate objects.");
			vm_assign3(o->n, nrm);
			vm_norm3(o->n);
			o->d = vm_dot3(o->n, pos);
			vm_assign3(o->p0, pos);
			if ((rc = object_header(L, jp, o, RTX_PLANE)))
				return rc;
			if (s->materials[o->material].emittant)
				return set_err(RTX_ERR_SCENE, "Plane cannot be emittant");
			if (o->epsilon == -1.f)
				o->epsilon = 1.e-6f;
		} break;
		case 2088783990u: /* Mesh */
			if ((rc = mesh_load(L, jp)))
				return rc;
			continue;
		default:
			/* the reference leaves `object` uninitialised here (scene.c:334-347) */
			return SCENE_ERR(L, "Unrecognized object type [%s]", jt->str);
		}
		if (s->materials[o->material].emittant)
			s->emitters[s->desc.num_emitters++] = (uint32_t)(o - s->objects);
	}
	return RTX_OK;
}

/* get_objects_extents (object.c:200-225), FLT_MIN initial max kept */
static void objects_extents(const rtx_scene *s, float *mn, float *mx)
{
	mn[0] = mn[1] = mn[2] = FLT_MAX;
	mx[0] = mx[1] = mx[2] = FLT_MIN;
	for (uint32_t i = 0; i < s->desc.num_objects; i++) {
		const rtx_object *o = &s->objects[i];
		float c[2][3];
		if (o->type == RTX_PLANE)
			continue;
		if (o->type == RTX_SPHERE) {
			for (int j = 0; j < 3; j++) {
				c[0][j] = o->p0[j] - o->radius;
				c[1][j] = o->p0[j] + o->radius;
			}
		} else { /* triangle_get_corners object.c:375-388 */
			const float *v[3] = { o->p0, o->p1, o->p2 };
			vm_assign3(c[0], v[2]);
			vm_assign3(c[1], v[2]);
			for (int i2 = 0; i2 < 2; i2++)
				for (int j = 0; j < 3; j++) {
					if (c[0][j] > v[i2][j])
						c[0][j] = v[i2][j];
					else if (c[1][j] < v[i2][j])
						c[1][j] = v[i2][j];
				}
		}
		for (int j = 0; j < 3; j++) {
			if (c[0][j] < mn[j])
				mn[j] = c[0][j];
			if (c[1][j] > mx[j])
				mx[j] = c[1][j];
		}
	}
}

/* scene_scale (scene.c:459-470) with *_scale (object.c:239-246, 390-401, 500-514), camera_scale (camera.c:35-40) */
static int scene_scale(rtx_scene *s, float k)
{
	const float zero[3] = { 0.f, 0.f, 0.f };
	for (uint32_t i = 0; i < s->desc.num_objects; i++) {
		rtx_object *o = &s->objects[i];
		switch (o->type) {
		case RTX_SPHERE:
			o->epsilon *= k;
			o->radius *= k;
			vm_sub3v(o->p0, zero, o->p0);
			vm_mul3s(o->p0, k, o->p0);
			break;
		case RTX_TRIANGLE: {
			o->epsilon *= k;
			float *v[3] = { o->p0, o->p1, o->p2 };
			for (int j = 0; j < 3; j++) {
				vm_sub3v(v[j], zero, v[j]);
				vm_mul3s(v[j], k, v[j]);
			}
			vm_mul3s(o->e1, k, o->e1);
			vm_mul3s(o->e2, k, o->e2);
		} break;
		case RTX_PLANE: {
			float point[3] = { 1.f, 1.f, 1.f };
			int j;
			for (j = 0; j < 3; j++)
				if (fabsf(o->n[j]) > o->epsilon)
					break;
			if (j == 3)
				return set_err(RTX_ERR_SCENE, "Plane normal has no component above its epsilon; cannot scale");
			point[j] = 0.f;
			point[j] = (o->d - vm_dot3(point, o->n)) / o->n[j];
			vm_sub3v(point, zero, point);
			vm_mul3s(point, k, point);
			o->d = vm_dot3(o->n, point);
			o->epsilon *= k;
		} break;
		}
	}
	rtx_camera *c = &s->desc.camera;
	vm_sub3v(c->position, zero, c->position);
	vm_mul3s(c->position, k, c->position);
	c->focal_length *= k;
	return RTX_OK;
}

void rtx_scene_free(rtx_scene *s)
{
	if (!s)
		return;
	free(s->materials);
	free(s->objects);
	free(s->emitters);
	free(s);
}

int rtx_scene_parse(const char *text, size_t len, const char *name, const char *scale_arg, const char *base_dir,
		    rtx_scene **out)
{
	if (!text || !out)
		return set_err(RTX_ERR_ARG, "null argument");
	*out = NULL;
	loader L = { name ? name : "<memory>", base_dir, NULL };
	jval *json = json_parse(text, len);
	if (!json)
		return set_err(RTX_ERR_SCENE, "Failed to parse scene [%s].", L.name);
	int rc = RTX_OK;
	rtx_scene *s = calloc(1, sizeof(*s));
	if (!s) {
		json_free(json);
		return set_err(RTX_ERR_NOMEM, "Unable to allocate scene.");
	}
	L.s = s;
	if (!json_is_object(json)) {
		rc = set_err(RTX_ERR_SCENE, "Expected parent token of type Object in scene [%s].", L.name);
		goto done;
	}
	jval *jamb = json_get(json, "AmbientLight");
	jval *jmats, *jobjs, *jcam;
	if ((rc = get_typed(&L, json, "Materials", J_ARRAY, "Array", &jmats)) ||
	    (rc = get_typed(&L, json, "Objects", J_ARRAY, "Array", &jobjs)) ||
	    (rc = get_typed(&L, json, "Camera", J_OBJECT, "Object", &jcam)))
		goto done;
	if ((rc = camera_load(&L, jcam)))
		goto done;

	/* materials_load (scene.c:149-163) */
	uint32_t nm = (uint32_t)json_size(jmats);
	if (!nm) {
		rc = SCENE_ERR(&L, "Expected token [Materials] to contain nonzero element count");
		goto done;
	}
	s->materials = calloc(nm, sizeof(rtx_material));
	if (!s->materials) {
		rc = set_err(RTX_ERR_NOMEM, "Unable to allocate materials.");
		goto done;
	}
	for (const jval *it = jmats->child; it; it = it->next) {
		if (!json_is_object(it)) {
			rc = SCENE_ERR(&L, "Expected token in [Materials] of type Object");
			goto done;
		}
		if ((rc = material_load(&L, it, &s->materials[s->desc.num_materials])))
			goto done;
		s->desc.num_materials++;
	}

	if ((rc = objects_load(&L, jobjs)))
		goto done;

	if (json_is_array(jamb) && json_size(jamb) == 3 && (rc = parse_floats(&L, jamb, s->desc.ambient)))
		goto done;

	if (scale_arg) {
		float k;
		if (rtx_hash_djb(scale_arg) == 2087865883u) { /* norm */
			float mn[3], mx[3], range[3];
			objects_extents(s, mn, mx);
			vm_sub3v(mx, mn, range);
			float m = range[0];
			if (m < range[1])
				m = range[1];
			if (m < range[2])
				m = range[2];
			k = 1.f / m;
		} else {
			k = (float)atof(scale_arg);
		}
		if ((rc = scene_scale(s, k)))
			goto done;
	}
	s->desc.materials = s->materials;
	s->desc.objects = s->objects;
	s->desc.emitters = s->emitters;
done:
	json_free(json);
	if (rc) {
		rtx_scene_free(s);
		return rc;
	}
	*out = s;
	return RTX_OK;
}

int rtx_scene_load(const char *path, const char *scale_arg, const char *base_dir, rtx_scene **out)
{
	if (!path || !out)
		return set_err(RTX_ERR_ARG, "null argument");
	FILE *f = fopen(path, "rb");
	if (!f)
		return set_err(RTX_ERR_IO, "Unable to open scene file [%s].", path);
	fseek(f, 0, SEEK_END);
	long length = ftell(f);
	fseek(f, 0, SEEK_SET);
	char *buf = malloc((size_t)length + 1);
	if (!buf) {
		fclose(f);
		return set_err(RTX_ERR_NOMEM, "Unable to allocate [%ld] bytes on heap.", length + 1);
	}
	size_t nread = fread(buf, 1, (size_t)length, f);
	fclose(f);
	if (nread != (size_t)length) {
		free(buf);
		return set_err(RTX_ERR_IO, "Failed to read scene file [%s].", path);
	}
	buf[length] = '\0';
	int rc = rtx_scene_parse(buf, (size_t)length, path, scale_arg, base_dir, out);
	free(buf);
	return rc;
}

const rtx_scene_desc *rtx_scene_desc_of(const rtx_scene *s)
{
	return s ? &s->desc : NULL;
}

uint32_t rtx_scene_num_json_objects(const rtx_scene *s)
{
	return s ? s->num_json_objects : 0;
}

/* image_init (image.c:34-56) */
int rtx_frame_setup(const rtx_camera *c, uint32_t w, uint32_t h, rtx_frame *out)
{
	if (!c || !out || !w || !h)
		return set_err(RTX_ERR_ARG, "bad frame arguments");
	const float PI = 3.1415927f; /* type.h:32 */
	float size_x = 2 * c->focal_length * tanf(c->fov * PI / 360.f);
	float size_y = size_x * h / w;
	float focal[3], center[3], off_x[3], off_y[3];
	vm_mul3s(c->vectors[2], c->focal_length, focal);
	vm_add3v(focal, c->position, center);
	vm_mul3s(c->vectors[0], size_x / w, out->step_x);
	vm_mul3s(c->vectors[1], size_y / h, out->step_y);
	vm_mul3s(out->step_x, .5f - w / 2.f, off_x);
	vm_mul3s(out->step_y, .5f - h / 2.f, off_y);
	for (int j = 0; j < 3; j++)
		out->corner[j] = center[j] + off_x[j] + off_y[j];
	vm_assign3(out->origin, c->position);
	out->width = w;
	out->height = h;
	return RTX_OK;
}

/* argv_check_with_args (argv.c:38-55) */
static int argv_find(int argc, char **argv, const char *flag, int nargs)
{
	uint32_t h = rtx_hash_djb(flag);
	for (int i = 1; i < argc; i++)
		if (rtx_hash_djb(argv[i]) == h)
			return (i + nargs < argc) ? i : 0;
	return 0;
}

/* render_init (render.c:61-116) */
void rtx_params_from_argv(int argc, char **argv, rtx_params *p)
{
	int idx;
	if ((idx = argv_find(argc, argv, "-b", 1)))
		p->max_bounces = (uint32_t)abs(atoi(argv[idx + 1]));
	if ((idx = argv_find(argc, argv, "-a", 1))) {
		float a = (float)atof(argv[idx + 1]);
		p->min_intensity_sqr = a * a;
	}
	if ((idx = argv_find(argc, argv, "-s", 1)))
		switch (rtx_hash_djb(argv[idx + 1])) {
		case 187940251u: p->reflection = RTX_PHONG; break;
		case 175795714u: p->reflection = RTX_BLINN; break;
		}
	if ((idx = argv_find(argc, argv, "-g", 1)))
		switch (rtx_hash_djb(argv[idx + 1])) {
		case 354625309u: p->gi = RTX_GI_AMBIENT; break;
		case 2088095368u: p->gi = RTX_GI_PATH; break;
		}
	if ((idx = argv_find(argc, argv, "-n", 1)))
		p->samples = (uint32_t)abs(atoi(argv[idx + 1]));
	if ((idx = argv_find(argc, argv, "-l", 1)))
		switch (rtx_hash_djb(argv[idx + 1])) {
		case 2087865487u: p->attenuation = RTX_ATT_NONE; break;
		case 193412846u: p->attenuation = RTX_ATT_LIN; break;
		case 193433013u: p->attenuation = RTX_ATT_SQR; break;
		}
	if ((idx = argv_find(argc, argv, "-o", 1)))
		p->attenuation_offset = (float)atof(argv[idx + 1]);
}

int rtx_stl_write(const char *path, uint32_t n, const float *tris)
{
	FILE *f = fopen(path, "wb");
	if (!f)
		return set_err(RTX_ERR_IO, "Failed to open [%s] for writing.", path);
	unsigned char header[80];
	memset(header, 0, sizeof(header));
	memcpy(header, "binary STL written by rtx", 25);
	fwrite(header, 1, 80, f);
	fwrite(&n, 4, 1, f);
	unsigned char rec[50];
	for (uint32_t i = 0; i < n; i++) {
		memset(rec, 0, sizeof(rec));
		memcpy(rec + 12, tris + (size_t)i * 9, 36);
		if (fwrite(rec, 50, 1, f) != 1) {
			fclose(f);
			return set_err(RTX_ERR_IO, "Failed to write [%s].", path);
		}
	}
	fclose(f);
	return RTX_OK;
}

/* ---- postprocessor flags: src/postprocess/postproc.c:36-91 with argv.c:36-55 semantics ---- */
static int post_arg(int argc, char **argv, const char *flag, int nargs)
{
	const uint32_t hsh = rtx_hash_djb(flag);
	int idx = 0;
	for (int i = 1; i < argc; i++) /* argv_check: first argument (after argv[0]) with this hash */
		if (argv[i] && rtx_hash_djb(argv[i]) == hsh) {
			idx = i;
			break;
		}
	return idx + nargs < argc ? idx : 0; /* argv_check_with_args */
}

int rtx_post_from_argv(int argc, char **argv, rtx_post *post)
{
	if (!post || (argc > 0 && !argv))
		return set_err(RTX_ERR_ARG, "null argument");
	memset(post, 0, sizeof(*post));
	int idx = post_arg(argc, argv, "-b", 1);
	if (idx) {
		post->brighten = 1;
		post->brighten_factor = (float)atof(argv[idx + 1]);
	}
	if ((idx = post_arg(argc, argv, "--dof", 2))) {
		post->dof = RTX_DOF_SCALE_BIAS;
		post->dof_scale = (float)atof(argv[idx + 1]);
		post->dof_bias = (float)atof(argv[idx + 2]);
	} else if ((idx = post_arg(argc, argv, "--dof-camera", 3))) {
		post->dof = RTX_DOF_CAMERA;
		post->aperture = (float)atof(argv[idx + 1]);
		post->focal_length = (float)atof(argv[idx + 2]);
		post->plane_in_focus = (float)atof(argv[idx + 3]);
	}
	if ((idx = post_arg(argc, argv, "--mist", 6))) {
		post->mist = 1;
		post->mist_start = (float)atof(argv[idx + 1]);
		post->mist_depth = (float)atof(argv[idx + 2]);
		switch (rtx_hash_djb(argv[idx + 3])) {
		case 2088106052u: /* quad */
			post->mist_falloff = RTX_FALLOFF_QUAD;
			break;
		case 193412846u: /* lin */
			post->mist_falloff = RTX_FALLOFF_LIN;
			break;
		case 624812280u: /* inv-quad */
			post->mist_falloff = RTX_FALLOFF_INV_QUAD;
			break;
		default:
			return set_err(RTX_ERR_ARG, "Unrecognized falloff type [%s].", argv[idx + 3]);
		}
		for (int a = 0; a < 3; a++)
			post->mist_color[a] = (float)atof(argv[idx + 4 + a]);
	}
	return RTX_OK;
}
