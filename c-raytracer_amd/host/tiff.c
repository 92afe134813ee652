/*
 * Minimal baseline-TIFF writer replacing the reference's libtiff use in
 * save_image / save_tiff / save_tiff_raw (src/raytracer/image.c:64-139):
 *   - tags: ImageWidth, ImageLength, BitsPerSample (8 or 32) x3,
 *     Compression none, Photometric RGB, StripOffsets, Orientation top-left,
 *     SamplesPerPixel 3, RowsPerStrip 1, StripByteCounts, PlanarConfig contig;
 *   - 8-bit mode: (uint8_t)fmaxf(fminf(v*255, 255), 0) per channel (image.c:96-98);
 *   - raw mode (-f): 32-bit float RGB samples with no SampleFormat tag, plus the
 *     private tag 65000 (FLOAT, count W*H) holding the z-buffer (image.c:64-85),
 *     which the postprocessor's image_load reads back.
 * Little-endian, one strip per row, like libtiff's output for these settings.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rtx_scene.h"

enum { T_SHORT = 3, T_LONG = 4, T_FLOAT = 11 };

typedef struct {
	uint16_t tag, type;
	uint32_t count, value; /* value or offset */
} ifd_entry;

static void put16(unsigned char *p, uint16_t v)
{
	p[0] = (unsigned char)v;
	p[1] = (unsigned char)(v >> 8);
}
static void put32(unsigned char *p, uint32_t v)
{
	p[0] = (unsigned char)v;
	p[1] = (unsigned char)(v >> 8);
	p[2] = (unsigned char)(v >> 16);
	p[3] = (unsigned char)(v >> 24);
}

int rtx_tiff_write(const char *path, uint32_t w, uint32_t h, const float *rgb, const float *z, int raw)
{
	if (!path || !rgb || !w || !h || (raw && !z))
		return RTX_ERR_ARG;
	const uint32_t bps = raw ? 32 : 8;
	const uint64_t row_bytes = (uint64_t)w * 3 * (bps / 8);
	const uint64_t img_bytes = row_bytes * h;
	const uint32_t n_entries = raw ? 12 : 11;

	/* layout: header | image strips | bps[3] | strip offsets | strip counts | z | IFD */
	uint64_t off = 8;
	const uint64_t off_img = off;
	off += img_bytes;
	off = (off + 3) & ~3ull;
	const uint64_t off_bps = off;
	off += 8;
	const uint64_t off_so = off;
	off += 4ull * h;
	const uint64_t off_sc = off;
	off += 4ull * h;
	const uint64_t off_z = off;
	if (raw)
		off += 4ull * w * h;
	const uint64_t off_ifd = off;
	off += 2 + 12ull * n_entries + 4;
	if (off > 0xFFFFFFFFull)
		return RTX_ERR_ARG; /* classic TIFF is 32-bit addressed */

	FILE *f = fopen(path, "wb");
	if (!f)
		return RTX_ERR_IO;
	unsigned char hdr[8] = { 'I', 'I', 42, 0 };
	put32(hdr + 4, (uint32_t)off_ifd);
	fwrite(hdr, 1, 8, f);

	unsigned char *row = malloc(row_bytes);
	if (!row) {
		fclose(f);
		return RTX_ERR_NOMEM;
	}
	for (uint32_t y = 0; y < h; y++) {
		const float *src = rgb + (size_t)y * w * 3;
		if (raw) {
			memcpy(row, src, row_bytes); /* host is little-endian x86-64 */
		} else {
			for (uint32_t i = 0; i < w * 3; i++)
				row[i] = (uint8_t)fmaxf(fminf(src[i] * 255.f, 255.f), 0.f);
		}
		fwrite(row, 1, row_bytes, f);
	}
	free(row);
	unsigned char pad[4] = { 0 };
	fwrite(pad, 1, (size_t)(off_bps - (off_img + img_bytes)), f);

	unsigned char b[8];
	put16(b, (uint16_t)bps);
	put16(b + 2, (uint16_t)bps);
	put16(b + 4, (uint16_t)bps);
	put16(b + 6, 0);
	fwrite(b, 1, 8, f);
	for (uint32_t y = 0; y < h; y++) {
		put32(b, (uint32_t)(off_img + row_bytes * y));
		fwrite(b, 1, 4, f);
	}
	for (uint32_t y = 0; y < h; y++) {
		put32(b, (uint32_t)row_bytes);
		fwrite(b, 1, 4, f);
	}
	if (raw)
		fwrite(z, 4, (size_t)w * h, f);

	ifd_entry e[12];
	int k = 0;
	e[k++] = (ifd_entry){ 256, T_LONG, 1, w };
	e[k++] = (ifd_entry){ 257, T_LONG, 1, h };
	e[k++] = (ifd_entry){ 258, T_SHORT, 3, (uint32_t)off_bps };
	e[k++] = (ifd_entry){ 259, T_SHORT, 1, 1 };
	e[k++] = (ifd_entry){ 262, T_SHORT, 1, 2 };
	e[k++] = (ifd_entry){ 273, T_LONG, h, h == 1 ? (uint32_t)off_img : (uint32_t)off_so };
	e[k++] = (ifd_entry){ 274, T_SHORT, 1, 1 };
	e[k++] = (ifd_entry){ 277, T_SHORT, 1, 3 };
	e[k++] = (ifd_entry){ 278, T_LONG, 1, 1 };
	e[k++] = (ifd_entry){ 279, T_LONG, h, h == 1 ? (uint32_t)row_bytes : (uint32_t)off_sc };
	e[k++] = (ifd_entry){ 284, T_SHORT, 1, 1 };
	if (raw)
		e[k++] = (ifd_entry){ 65000, T_FLOAT, w * h, w * h == 1 ? 0u : (uint32_t)off_z };
	unsigned char ent[12];
	put16(b, (uint16_t)k);
	fwrite(b, 1, 2, f);
	for (int i = 0; i < k; i++) {
		put16(ent, e[i].tag);
		put16(ent + 2, e[i].type);
		put32(ent + 4, e[i].count);
		if (e[i].type == T_SHORT && e[i].count == 1) {
			put16(ent + 8, (uint16_t)e[i].value);
			put16(ent + 10, 0);
		} else if (e[i].tag == 65000 && e[i].count == 1) {
			memcpy(ent + 8, z, 4);
		} else {
			put32(ent + 8, e[i].value);
		}
		fwrite(ent, 1, 12, f);
	}
	put32(b, 0);
	fwrite(b, 1, 4, f);
	int bad = ferror(f);
	fclose(f);
	return bad ? RTX_ERR_IO : RTX_OK;
}
