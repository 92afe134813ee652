/*
 * engine — drop-in for the reference CLI (src/raytracer/main.c:57-89):
 *
 *   engine <input.json> <output.tif> <resX> <resY> [flags]
 *
 * Same flow: system_init -> scene_load -> image_init -> accel_init ->
 * render_init -> render -> save_image, with accel_init/render replaced by the
 * MI355X path (rtx_upload_scene / rtx_render) and the host glue from
 * librtxscene.  Reference flags: -m -b -a -s -n -r -l -o -p -g -f (HELPTEXT,
 * main.c:23-53; -o is undocumented there).  Extensions:
 *   --gpus N     render tile shards on N devices (one thread each)
 *   --device D   first device (default 0)
 *   --seed S     counter-RNG seed (default 1)
 *   --rng const  every rand_flt() draw = 0.5 (the oracle's REF_CONST_RNG)
 *   --u32 wrap   float->uint32 texture conversion of a generic x86-64 build
 *                (default: AVX-512 saturating, like -march=native on AVX-512 hosts)
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rtx.h"
#include "rtx_scene.h"

static const char *HELPTEXT =
	"Render a scene using raytracing (MI355X / gfx950 path).\n"
	"Usage: ./engine <input> <output> <resolution> [OPTIONAL_PARAMETERS]\n"
	"\n"
	"REQUIRED PARAMETERS:\n"
	"<input>      (string)            : .json scene file.\n"
	"<output>     (string)            : .tif file to which the image will be saved.\n"
	"<resolution> (integer) (integer) : resolution of the output image.\n"
	"OPTIONAL PARAMETERS:\n"
	"[-m] (integer | \"max\")           : accepted for compatibility (CPU threads; unused)\n"
	"[-b] (integer)                   : DEFAULT = 10      : maximum number of times that a light ray can bounce.\n"
	"[-a] (float)                     : DEFAULT = 0.01    : minimum light intensity for which a ray is cast.\n"
	"[-s] (\"phong\" | \"blinn\")         : DEFAULT = phong   : reflection model.\n"
	"[-n] (integer)                   : DEFAULT = 1       : number of samples which are rendered per pixel.\n"
	"[-r] (\"norm\" | float)            : DEFAULT = 1.0     : scene scaling factor.\n"
	"[-l] (\"none\" | \"lin\" | \"sqr\")    : DEFAULT = sqr     : light attenuation.\n"
	"[-o] (float)                     : DEFAULT = 1.0     : light attenuation offset.\n"
	"[-p] (\"real\" | \"cpu\")            : DEFAULT = real    : time to print with status messages.\n"
	"[-g] (string)                    : DEFAULT = ambient : global illumination model (ambient | path).\n"
	"[-f]                             : DEFAULT = OFF     : save raw output for post-processing.\n"
	"[--gpus N] [--device D] [--seed S] [--rng counter|const] [--u32 sat|wrap]\n";

static struct timespec t0;
static int log_cpu = 0;

static double now_s(void)
{
	if (log_cpu)
		return (double)clock() / CLOCKS_PER_SEC;
	struct timespec t;
	timespec_get(&t, TIME_UTC);
	return (t.tv_sec - t0.tv_sec) + (t.tv_nsec - t0.tv_nsec) * 1e-9;
}

#define LOG(fmt, ...) printf("[%08.3f] %10s:%18s:%3u: " fmt "\n", now_s(), "main.c", __func__, __LINE__, ##__VA_ARGS__)

static int argv_find(int argc, char **argv, const char *flag, int nargs)
{
	uint32_t h = rtx_hash_djb(flag);
	for (int i = 1; i < argc; i++)
		if (rtx_hash_djb(argv[i]) == h)
			return (i + nargs < argc) ? i : 0;
	return 0;
}

typedef struct {
	int device;
	const rtx_scene_desc *desc;
	const rtx_frame *frame;
	rtx_params params;
	float *rgb, *z;
	int rc;
	char err[512];
	rtx_stats stats;
} shard_job;

static void *shard_main(void *arg)
{
	shard_job *j = (shard_job *)arg;
	rtx_ctx *ctx = NULL;
	j->rc = rtx_open(j->device, &ctx);
	if (!j->rc)
		j->rc = rtx_upload_scene(ctx, j->desc);
	if (!j->rc)
		j->rc = rtx_render(ctx, j->frame, &j->params, j->rgb, j->z);
	if (!j->rc)
		rtx_get_stats(ctx, &j->stats);
	if (j->rc)
		snprintf(j->err, sizeof(j->err), "%s", rtx_last_error());
	rtx_close(ctx);
	return NULL;
}

int main(int argc, char **argv)
{
	timespec_get(&t0, TIME_UTC);
	if (argv_find(argc, argv, "--help", 0) || argv_find(argc, argv, "-h", 0)) {
		puts(HELPTEXT);
		return 0;
	} else if (argc < 5) {
		puts("Too few arguments. Use --help to find out which arguments are required to call this program.");
		return 1;
	}
	int idx;
	if ((idx = argv_find(argc, argv, "-p", 1)) && rtx_hash_djb(argv[idx + 1]) == 193416643u)
		log_cpu = 1;

	rtx_params p;
	rtx_params_default(&p);
	rtx_params_from_argv(argc, argv, &p);
	int ngpu = 1, dev0 = 0;
	if ((idx = argv_find(argc, argv, "--gpus", 1)))
		ngpu = atoi(argv[idx + 1]);
	if ((idx = argv_find(argc, argv, "--device", 1)))
		dev0 = atoi(argv[idx + 1]);
	if ((idx = argv_find(argc, argv, "--seed", 1)))
		p.seed = strtoull(argv[idx + 1], NULL, 10);
	if ((idx = argv_find(argc, argv, "--rng", 1)) && !strcmp(argv[idx + 1], "const"))
		p.rng = RTX_RNG_CONST;
	if ((idx = argv_find(argc, argv, "--u32", 1)) && !strcmp(argv[idx + 1], "wrap"))
		p.u32conv = RTX_U32_WRAP;
	if (ngpu < 1)
		ngpu = 1;

	LOG("Loading scene.");
	const char *scale = NULL;
	if ((idx = argv_find(argc, argv, "-r", 1)))
		scale = argv[idx + 1];
	rtx_scene *scene = NULL;
	if (rtx_scene_load(argv[1], scale, NULL, &scene)) {
		LOG("%s", rtx_scene_last_error());
		return 1;
	}
	const rtx_scene_desc *desc = rtx_scene_desc_of(scene);
	LOG("Loaded %u materials, %u objects (%u emitters).", desc->num_materials, desc->num_objects, desc->num_emitters);

	LOG("Initializing image.");
	uint32_t w = (uint32_t)abs(atoi(argv[3])), h = (uint32_t)abs(atoi(argv[4]));
	rtx_frame fr;
	if (rtx_frame_setup(&desc->camera, w, h, &fr)) {
		LOG("Invalid resolution.");
		return 1;
	}
	size_t px = (size_t)w * h;
	float *rgb = calloc(px * 3, sizeof(float)), *z = calloc(px, sizeof(float));
	shard_job *jobs = calloc((size_t)ngpu, sizeof(shard_job));
	pthread_t *th = calloc((size_t)ngpu, sizeof(pthread_t));
	if (!rgb || !z || !jobs || !th) {
		LOG("Unable to allocate the framebuffer.");
		return 1;
	}
	LOG("Commencing raytracing on %d GPU(s).", ngpu);
	for (int g = 0; g < ngpu; g++) {
		jobs[g].device = dev0 + g;
		jobs[g].desc = desc;
		jobs[g].frame = &fr;
		jobs[g].params = p;
		jobs[g].params.tile_offset = (uint32_t)g;
		jobs[g].params.tile_stride = (uint32_t)ngpu;
		jobs[g].rgb = ngpu == 1 ? rgb : calloc(px * 3, sizeof(float));
		jobs[g].z = ngpu == 1 ? z : calloc(px, sizeof(float));
		if (!jobs[g].rgb || !jobs[g].z) {
			LOG("Unable to allocate shard buffers.");
			return 1;
		}
		pthread_create(&th[g], NULL, shard_main, &jobs[g]);
	}
	uint64_t closest = 0, shadow = 0;
	double kms = 0;
	for (int g = 0; g < ngpu; g++) {
		pthread_join(th[g], NULL);
		if (jobs[g].rc) {
			LOG("GPU %d: %s", jobs[g].device, jobs[g].err);
			return 1;
		}
		closest += jobs[g].stats.closest_rays;
		shadow += jobs[g].stats.shadow_rays;
		if (jobs[g].stats.kernel_ms > kms)
			kms = jobs[g].stats.kernel_ms;
	}
	if (ngpu > 1) {
		/* gather: tile t belongs to shard t % ngpu */
		uint32_t tiles_x = (w + 7) / 8;
		for (uint32_t y = 0; y < h; y++)
			for (uint32_t x = 0; x < w; x++) {
				uint32_t t = (y / 8) * tiles_x + x / 8;
				const shard_job *j = &jobs[t % (uint32_t)ngpu];
				size_t i = (size_t)y * w + x;
				memcpy(rgb + 3 * i, j->rgb + 3 * i, 12);
				z[i] = j->z[i];
			}
	}
	LOG("Rays: %llu closest + %llu shadow in %.3f ms device time (%.1f Mrays/s).", (unsigned long long)closest,
	    (unsigned long long)shadow, kms, kms > 0 ? (closest + shadow) / (kms * 1e3) : 0.0);

	LOG("Saving image.");
	const char *out = argv[2];
	if (!strstr(out, ".tif"))
		LOG("Expected output file [%s] with extension .tif.", out);
	if (rtx_tiff_write(out, w, h, rgb, z, argv_find(argc, argv, "-f", 0) != 0)) {
		LOG("Failed to open output file [%s].", out);
		return 1;
	}
	LOG("Terminating.");
	rtx_scene_free(scene);
	return 0;
}
