/*
 * ORACLE TEST INFRASTRUCTURE — not part of the product path.
 *
 * A main() for the reference's own postprocessor sources (src/postprocess/postproc.c,
 * src/postprocess/image.c, src/core/*.c, compiled unmodified from /root/reference by
 * oracle/Makefile): it runs the reference's image_load() and postprocess() exactly as
 * src/postprocess/main.c:45-70 does, then, instead of save_image()'s 8-bit quantisation,
 * dumps the float raster so the GPU postprocess can be checked bit for bit.
 *
 *   post_dump <input raw .tif> <output .f32> [reference postprocess flags...]
 * output: uint32 width, uint32 height, then width*height*3 float32 (row-major, RGB).
 */
#include <stdint.h>
#include <stdio.h>

#include "argv.h"
#include "image.h"
#include "postproc.h"
#include "system.h"

int main(int argc, char *argv[])
{
	myargc = argc;
	myargv = argv;
	argv_init();
	if (argc < 3)
		return 1;
	system_init();
	image_load();
	postprocess();
	FILE *f = fopen(argv[2], "wb");
	if (!f)
		return 2;
	uint32_t wh[2] = { image.resolution[0], image.resolution[1] };
	fwrite(wh, 4, 2, f);
	fwrite(image.raster, sizeof(float) * 3, image.pixels, f);
	fclose(f);
	argv_deinit();
	image_deinit();
	return 0;
}
