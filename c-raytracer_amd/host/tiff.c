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

/* ---- raw TIFF reader: what src/postprocess/image.c:29-75 (image_load) accepts ---- */
typedef struct {
	const unsigned char *p;
	size_t n;
	int be; /* big-endian file ("MM") */
} tbuf;

static uint32_t rd16(const tbuf *t, size_t o)
{
	if (o + 2 > t->n)
		return 0;
	const unsigned char *q = t->p + o;
	return t->be ? (uint32_t)(q[0] << 8 | q[1]) : (uint32_t)(q[1] << 8 | q[0]);
}
static uint32_t rd32(const tbuf *t, size_t o)
{
	if (o + 4 > t->n)
		return 0;
	const unsigned char *q = t->p + o;
	return t->be ? ((uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3])
		     : ((uint32_t)q[3] << 24 | (uint32_t)q[2] << 16 | (uint32_t)q[1] << 8 | q[0]);
}

typedef struct {
	uint32_t type, count, value; /* value = inline value or offset */
	size_t at;                   /* file offset of the 4-byte value field */
	int present;
} tfield;

static uint32_t tsize(uint32_t type) { return type == T_SHORT ? 2u : (type == 1 || type == 2 || type == 6 || type == 7) ? 1u : (type == 12 ? 8u : 4u); }

/* element i of a field (SHORT or LONG), inline or at its offset */
static uint32_t tget(const tbuf *t, const tfield *f, uint32_t i)
{
	const uint32_t sz = tsize(f->type);
	const size_t base = (uint64_t)f->count * sz <= 4 ? f->at : f->value;
	return f->type == T_SHORT ? rd16(t, base + 2 * (size_t)i) : rd32(t, base + 4 * (size_t)i);
}

int rtx_tiff_read_raw(const char *path, uint32_t *width, uint32_t *height, float **rgb, float **z)
{
	if (!path || !width || !height || !rgb || !z)
		return RTX_ERR_ARG;
	*rgb = NULL;
	*z = NULL;
	FILE *f = fopen(path, "rb");
	if (!f)
		return RTX_ERR_IO; /* image.c:37 "Failed to open input file" */
	fseek(f, 0, SEEK_END);
	long len = ftell(f);
	fseek(f, 0, SEEK_SET);
	unsigned char *buf = len > 8 ? malloc((size_t)len) : NULL;
	if (!buf || fread(buf, 1, (size_t)len, f) != (size_t)len) {
		free(buf);
		fclose(f);
		return RTX_ERR_IO;
	}
	fclose(f);
	tbuf t = { buf, (size_t)len, buf[0] == 'M' };
	int rc = RTX_ERR_IO;
	if (!((buf[0] == 'I' && buf[1] == 'I') || (buf[0] == 'M' && buf[1] == 'M')) || rd16(&t, 2) != 42)
		goto out;
	const uint32_t ifd = rd32(&t, 4);
	const uint32_t n = rd16(&t, ifd);
	tfield fw = { 0 }, fh = { 0 }, fbps = { 0 }, fcomp = { 0 }, fso = { 0 }, fspp = { 0 }, fsbc = { 0 }, fpc = { 0 },
	       fz = { 0 };
	for (uint32_t i = 0; i < n; i++) {
		const size_t e = ifd + 2 + 12 * (size_t)i;
		tfield x = { rd16(&t, e + 2), rd32(&t, e + 4), rd32(&t, e + 8), e + 8, 1 };
		if (x.type == T_SHORT && x.count == 1)
			x.value = rd16(&t, e + 8);
		switch (rd16(&t, e)) {
		case 256: fw = x; break;
		case 257: fh = x; break;
		case 258: fbps = x; break;
		case 259: fcomp = x; break;
		case 273: fso = x; break;
		case 277: fspp = x; break;
		case 279: fsbc = x; break;
		case 284: fpc = x; break;
		case 65000: fz = x; break;
		default: break;
		}
	}
	if (!fw.present || !fh.present || !fso.present)
		goto out;
	const uint32_t w = fw.type == T_SHORT ? fw.value & 0xFFFF : fw.value;
	const uint32_t h = fh.type == T_SHORT ? fh.value & 0xFFFF : fh.value;
	/* image.c:47-49: 3 samples, 32 bits, contiguous */
	if ((fspp.present ? fspp.value : 1) != 3 || !fbps.present || tget(&t, &fbps, 0) != 32 ||
	    (fpc.present && fpc.value != 1) || (fcomp.present && fcomp.value != 1) || !w || !h) {
		rc = RTX_ERR_ARG;
		goto out;
	}
	const size_t px = (size_t)w * h;
	/* image.c:70-73: "Corrupted Z-Buffer." unless the tag holds exactly W*H floats */
	if (!fz.present || fz.count != px || fz.type != T_FLOAT) {
		rc = RTX_ERR_ARG;
		goto out;
	}
	float *c = malloc(px * 12), *d = malloc(px * 4);
	if (!c || !d) {
		free(c);
		free(d);
		rc = RTX_ERR_NOMEM;
		goto out;
	}
	/* strips in order, rows contiguous */
	size_t at = 0;
	const size_t total = px * 12;
	for (uint32_t s = 0; s < fso.count && at < total; s++) {
		const uint32_t so = tget(&t, &fso, s);
		uint32_t sc = fsbc.present ? tget(&t, &fsbc, s) : (uint32_t)(total - at);
		if (sc > total - at)
			sc = (uint32_t)(total - at);
		if ((size_t)so + sc > t.n)
			break;
		memcpy((unsigned char *)c + at, buf + so, sc);
		at += sc;
	}
	const size_t zo = px == 1 ? fz.at : fz.value;
	if (at != total || zo + px * 4 > t.n) {
		free(c);
		free(d);
		goto out;
	}
	memcpy(d, buf + zo, px * 4);
	if (t.be) { /* byte-swap samples of a big-endian file */
		uint32_t *u = (uint32_t *)c, *v = (uint32_t *)d;
		for (size_t i = 0; i < px * 3; i++)
			u[i] = __builtin_bswap32(u[i]);
		for (size_t i = 0; i < px; i++)
			v[i] = __builtin_bswap32(v[i]);
	}
	*width = w;
	*height = h;
	*rgb = c;
	*z = d;
	rc = RTX_OK;
out:
	free(buf);
	return rc;
}

void rtx_buffer_free(void *p) { free(p); }
