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
 *   --gpus N     render on N devices (rtx_group: BVH built once, tiles dealt round-robin,
 *                shards gathered to the first device over RCCL)
 *   --device D   first device (default 0)
 *   --seed S     counter-RNG seed (default 1)
 *   --rng const  every rand_flt() draw = 0.5 (the oracle's REF_CONST_RNG)
 *   --rng counter  counter-based i.i.d. draws like rand_flt (the default)
 *   --rng strat    the same stream with the light samples stratified (opt-in, another estimator)
 *   --u32 wrap   float->uint32 texture conversion of a generic x86-64 build
 *                (default: AVX-512 saturating, like -march=native on AVX-512 hosts)
 */
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
	"[--gpus N] [--device D] [--seed S] [--rng counter|strat|const] [--u32 sat|wrap]\n";

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
	if ((idx = argv_find(argc, argv, "--rng", 1)) && !strcmp(argv[idx + 1], "counter"))
		p.rng = RTX_RNG_COUNTER;
	if ((idx = argv_find(argc, argv, "--rng", 1)) && !strcmp(argv[idx + 1], "strat"))
		p.rng = RTX_RNG_STRAT;
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
	int *devs = calloc((size_t)ngpu, sizeof(int));
	if (!rgb || !z || !devs) {
		LOG("Unable to allocate the framebuffer.");
		return 1;
	}
	for (int g = 0; g < ngpu; g++)
		devs[g] = dev0 + g;
	LOG("Commencing raytracing on %d GPU(s).", ngpu);
	rtx_group *grp = NULL;
	rtx_stats st;
	if (rtx_group_open(ngpu, devs, &grp) || rtx_group_upload_scene(grp, desc) ||
	    rtx_group_render(grp, &fr, &p, rgb, z) || rtx_group_get_stats(grp, &st)) {
		LOG("%s", rtx_last_error());
		rtx_group_close(grp);
		return 1;
	}
	rtx_group_close(grp);
	const uint64_t closest = st.closest_rays, shadow = st.shadow_rays;
	const double kms = st.kernel_ms;
	if (ngpu > 1)
		LOG("Gathered %d shards in %.3f ms.", ngpu, st.gather_ms);
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
