/*
 * postprocess — drop-in for the reference's postprocessor CLI
 * (src/postprocess/main.c:45-70):
 *
 *   postprocess <input raw .tif> <output .tif> [-b f] [--dof scale bias |
 *               --dof-camera aperture focal plane] [--mist start depth falloff r g b]
 *
 * Same flow: image_load -> postprocess -> save_image, with postprocess() run on the GPU
 * (rtx_postprocess, csrc/rtx_post.hip) and the host glue from librtxscene (raw-TIFF reader,
 * flag parser, 8-bit TIFF writer with save_image's clamp/truncate).
 * Extension: --device D (default 0).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rtx.h"
#include "rtx_scene.h"

static const char *HELPTEXT =
	"Apply post-processing effects to raytraced image (MI355X / gfx950 path).\n"
	"\n"
	"Usage: ./postprocess <input> <output> [OPTIONAL_PARAMETERS]\n"
	"\n"
	"REQUIRED PARAMETERS:\n"
	"<input>      (string)            : .tif raw file created by raytracer.\n"
	"<output>     (string)            : .tif file to which the image will be saved.\n"
	"OPTIONAL PARAMETERS:\n"
	"[-b] (float)                     : DEFAULT = 1.0     : brighten.\n"
	"[--dof] <scale> <bias>           : Apply depth of field effect (incompatible with --dof-camera).\n"
	"[--dof-camera] <aperture> <focal length> <plane in focus> : Apply depth of field effect (incompatible with --dof).\n"
	"[--mist] <start> <depth> <falloff> <color> : Apply colored mist based on distance.\n"
	"  <falloff> (\"quad\"|\"lin\"|\"inv-quad\") : Decay rate.\n"
	"[--device D]                     : HIP device (default 0).\n";

static struct timespec t0;

static double now_s(void)
{
	struct timespec t;
	timespec_get(&t, TIME_UTC);
	return (t.tv_sec - t0.tv_sec) + (t.tv_nsec - t0.tv_nsec) * 1e-9;
}

#define LOG(...)                                                   \
	do {                                                       \
		printf("[%08.3f] postprocess: ", now_s());         \
		printf(__VA_ARGS__);                               \
		printf("\n");                                      \
	} while (0)

int main(int argc, char **argv)
{
	timespec_get(&t0, TIME_UTC);
	for (int i = 1; i < argc; i++)
		if (!strcmp(argv[i], "--help") || !strcmp(argv[i], "-h")) {
			puts(HELPTEXT);
			return 0;
		}
	if (argc < 3) {
		puts("Too few arguments. Use --help to find out which arguments are required to call this program.");
		return 1;
	}
	int device = 0;
	for (int i = 3; i + 1 < argc; i++)
		if (!strcmp(argv[i], "--device"))
			device = atoi(argv[i + 1]);
	rtx_post post;
	if (rtx_post_from_argv(argc, argv, &post)) {
		fprintf(stderr, "ERROR: %s\n", rtx_scene_last_error());
		return 1;
	}
	LOG("Loading image.");
	uint32_t w = 0, h = 0;
	float *rgb = NULL, *z = NULL;
	int rc = rtx_tiff_read_raw(argv[1], &w, &h, &rgb, &z);
	if (rc) {
		fprintf(stderr, "ERROR: Failed to load raw input file [%s] (%d).\n", argv[1], rc);
		return 1;
	}
	rtx_ctx *ctx = NULL;
	if (rtx_open(device, &ctx)) {
		fprintf(stderr, "ERROR: %s\n", rtx_last_error());
		return 1;
	}
	LOG("Commencing Postprocessing");
	if (post.brighten)
		LOG("Brightening by factor %f.", (double)post.brighten_factor);
	if (post.dof == RTX_DOF_SCALE_BIAS)
		LOG("Applying depth of field with scale [%f] and bias [%f].", (double)post.dof_scale, (double)post.dof_bias);
	if (rtx_postprocess(ctx, w, h, &post, rgb, z)) {
		fprintf(stderr, "ERROR: %s\n", rtx_last_error());
		return 1;
	}
	LOG("Saving image.");
	if (!strstr(argv[2], ".tif"))
		LOG("Expected output file [%s] with extension .tif.", argv[2]);
	if (rtx_tiff_write(argv[2], w, h, rgb, NULL, 0)) {
		fprintf(stderr, "ERROR: Failed to open output file [%s].\n", argv[2]);
		return 1;
	}
	LOG("Terminating.");
	rtx_close(ctx);
	rtx_buffer_free(rgb);
	rtx_buffer_free(z);
	return 0;
}
