/*
 * Recursive-descent JSON reader for scene files.  Behaviour that the scene
 * loader depends on mirrors cJSON as used by the reference (scene.c:87):
 *  - numbers are read with strtod into a double (cJSON parse_number);
 *  - "valueint" saturates to INT_MIN/INT_MAX;
 *  - object member lookup is case-sensitive and returns the first match;
 *  - content after the first complete value is ignored (cJSON_Parse does not
 *    require null termination).
 */
#include "json.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

#define MAX_DEPTH 1000

typedef struct {
	const char *p, *end;
	int depth;
} reader;

static void skip_ws(reader *r)
{
	while (r->p < r->end && (unsigned char)*r->p <= 32)
		r->p++;
}

static jval *new_val(enum jtype t)
{
	jval *v = calloc(1, sizeof(jval));
	if (v)
		v->type = t;
	return v;
}

static jval *parse_value(reader *r);

static int hexval(char c)
{
	if (c >= '0' && c <= '9')
		return c - '0';
	if (c >= 'a' && c <= 'f')
		return c - 'a' + 10;
	if (c >= 'A' && c <= 'F')
		return c - 'A' + 10;
	return -1;
}

static void put_utf8(char **o, unsigned cp)
{
	char *q = *o;
	if (cp < 0x80) {
		*q++ = (char)cp;
	} else if (cp < 0x800) {
		*q++ = (char)(0xC0 | (cp >> 6));
		*q++ = (char)(0x80 | (cp & 0x3F));
	} else if (cp < 0x10000) {
		*q++ = (char)(0xE0 | (cp >> 12));
		*q++ = (char)(0x80 | ((cp >> 6) & 0x3F));
		*q++ = (char)(0x80 | (cp & 0x3F));
	} else {
		*q++ = (char)(0xF0 | (cp >> 18));
		*q++ = (char)(0x80 | ((cp >> 12) & 0x3F));
		*q++ = (char)(0x80 | ((cp >> 6) & 0x3F));
		*q++ = (char)(0x80 | (cp & 0x3F));
	}
	*o = q;
}

static int read_hex4(const char *s, unsigned *out)
{
	unsigned v = 0;
	for (int i = 0; i < 4; i++) {
		int h = hexval(s[i]);
		if (h < 0)
			return 0;
		v = v * 16 + (unsigned)h;
	}
	*out = v;
	return 1;
}

static char *parse_string_raw(reader *r)
{
	if (r->p >= r->end || *r->p != '"')
		return NULL;
	const char *s = ++r->p;
	const char *e = s;
	while (e < r->end && *e != '"') {
		if (*e == '\\')
			e++;
		e++;
	}
	if (e >= r->end)
		return NULL;
	char *out = malloc((size_t)(e - s) + 1);
	if (!out)
		return NULL;
	char *o = out;
	const char *c = s;
	while (c < e) {
		if (*c != '\\') {
			*o++ = *c++;
			continue;
		}
		c++;
		switch (*c) {
		case 'b': *o++ = '\b'; c++; break;
		case 'f': *o++ = '\f'; c++; break;
		case 'n': *o++ = '\n'; c++; break;
		case 'r': *o++ = '\r'; c++; break;
		case 't': *o++ = '\t'; c++; break;
		case '"':
		case '\\':
		case '/': *o++ = *c++; break;
		case 'u': {
			unsigned cp;
			if (e - c < 5 || !read_hex4(c + 1, &cp))
				goto fail;
			c += 5;
			if (cp >= 0xD800 && cp <= 0xDBFF) {
				unsigned lo;
				if (e - c < 6 || c[0] != '\\' || c[1] != 'u' || !read_hex4(c + 2, &lo) || lo < 0xDC00 || lo > 0xDFFF)
					goto fail;
				c += 6;
				cp = 0x10000 + (((cp & 0x3FF) << 10) | (lo & 0x3FF));
			}
			put_utf8(&o, cp);
		} break;
		default:
			goto fail;
		}
	}
	*o = '\0';
	r->p = e + 1;
	return out;
fail:
	free(out);
	return NULL;
}

static jval *parse_number(reader *r)
{
	/* cJSON parse_number: take the run of number characters, strtod it */
	char buf[64];
	size_t n = 0;
	while (r->p + n < r->end && n < sizeof(buf) - 1) {
		char c = r->p[n];
		if ((c >= '0' && c <= '9') || c == '+' || c == '-' || c == 'e' || c == 'E' || c == '.')
			n++;
		else
			break;
	}
	if (n == 0)
		return NULL;
	memcpy(buf, r->p, n);
	buf[n] = '\0';
	char *endp;
	double d = strtod(buf, &endp);
	if (endp == buf)
		return NULL;
	jval *v = new_val(J_NUMBER);
	if (!v)
		return NULL;
	v->num = d;
	r->p += (endp - buf);
	return v;
}

static jval *parse_array(reader *r)
{
	jval *arr = new_val(J_ARRAY), *last = NULL;
	if (!arr)
		return NULL;
	r->p++; /* [ */
	skip_ws(r);
	if (r->p < r->end && *r->p == ']') {
		r->p++;
		return arr;
	}
	for (;;) {
		jval *item = parse_value(r);
		if (!item)
			goto fail;
		if (last)
			last->next = item;
		else
			arr->child = item;
		last = item;
		arr->count++;
		skip_ws(r);
		if (r->p >= r->end)
			goto fail;
		if (*r->p == ',') {
			r->p++;
			continue;
		}
		if (*r->p == ']') {
			r->p++;
			return arr;
		}
		goto fail;
	}
fail:
	json_free(arr);
	return NULL;
}

static jval *parse_object(reader *r)
{
	jval *obj = new_val(J_OBJECT), *last = NULL;
	if (!obj)
		return NULL;
	r->p++; /* { */
	skip_ws(r);
	if (r->p < r->end && *r->p == '}') {
		r->p++;
		return obj;
	}
	for (;;) {
		skip_ws(r);
		char *key = parse_string_raw(r);
		if (!key)
			goto fail;
		skip_ws(r);
		if (r->p >= r->end || *r->p != ':') {
			free(key);
			goto fail;
		}
		r->p++;
		jval *item = parse_value(r);
		if (!item) {
			free(key);
			goto fail;
		}
		item->key = key;
		if (last)
			last->next = item;
		else
			obj->child = item;
		last = item;
		obj->count++;
		skip_ws(r);
		if (r->p >= r->end)
			goto fail;
		if (*r->p == ',') {
			r->p++;
			continue;
		}
		if (*r->p == '}') {
			r->p++;
			return obj;
		}
		goto fail;
	}
fail:
	json_free(obj);
	return NULL;
}

static int match_lit(reader *r, const char *lit)
{
	size_t n = strlen(lit);
	if ((size_t)(r->end - r->p) >= n && !strncmp(r->p, lit, n)) {
		r->p += n;
		return 1;
	}
	return 0;
}

static jval *parse_value(reader *r)
{
	if (++r->depth > MAX_DEPTH)
		return NULL;
	skip_ws(r);
	jval *v = NULL;
	if (r->p >= r->end) {
		v = NULL;
	} else if (*r->p == '{') {
		v = parse_object(r);
	} else if (*r->p == '[') {
		v = parse_array(r);
	} else if (*r->p == '"') {
		char *s = parse_string_raw(r);
		if (s) {
			v = new_val(J_STRING);
			if (v)
				v->str = s;
			else
				free(s);
		}
	} else if (*r->p == '-' || (*r->p >= '0' && *r->p <= '9')) {
		v = parse_number(r);
	} else if (match_lit(r, "null")) {
		v = new_val(J_NULL);
	} else if (match_lit(r, "false")) {
		v = new_val(J_FALSE);
	} else if (match_lit(r, "true")) {
		v = new_val(J_TRUE);
	}
	r->depth--;
	return v;
}

jval *json_parse(const char *text, size_t len)
{
	reader r = { text, text + len, 0 };
	/* skip a UTF-8 BOM like cJSON does not; plain whitespace only */
	return parse_value(&r);
}

void json_free(jval *v)
{
	while (v) {
		jval *next = v->next;
		json_free(v->child);
		free(v->str);
		free(v->key);
		free(v);
		v = next;
	}
}

jval *json_get(const jval *obj, const char *key)
{
	if (!obj || obj->type != J_OBJECT)
		return NULL;
	for (jval *c = obj->child; c; c = c->next)
		if (c->key && !strcmp(c->key, key))
			return c;
	return NULL;
}

int json_size(const jval *v)
{
	return v ? v->count : 0;
}

int json_int(const jval *v)
{
	if (!v)
		return 0;
	if (v->num >= INT_MAX)
		return INT_MAX;
	if (v->num <= (double)INT_MIN)
		return INT_MIN;
	return (int)v->num;
}
