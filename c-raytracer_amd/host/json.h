/*
 * Minimal JSON DOM for the scene loader (replaces the reference's vendored
 * cJSON v1.7.14, lib/cJSON).  Only what scene.c needs: ordered object members,
 * arrays, numbers as double (strtod, like cJSON parse_number), strings.
 */
#ifndef RTX_JSON_H
#define RTX_JSON_H

#include <stddef.h>

enum jtype { J_NULL, J_FALSE, J_TRUE, J_NUMBER, J_STRING, J_ARRAY, J_OBJECT };

typedef struct jval {
	enum jtype type;
	double num;
	char *str;              /* J_STRING */
	char *key;              /* member name when inside an object */
	struct jval *child;     /* first element / member */
	struct jval *next;
	int count;
} jval;

/* Returns NULL on syntax error. */
jval *json_parse(const char *text, size_t len);
void json_free(jval *v);

/* cJSON_GetObjectItemCaseSensitive: first member named key, or NULL. */
jval *json_get(const jval *obj, const char *key);
/* cJSON_GetArraySize (works for objects too: member count). */
int json_size(const jval *v);
/* cJSON valueint: saturating (int) of the double. */
int json_int(const jval *v);

static inline int json_is_number(const jval *v) { return v && v->type == J_NUMBER; }
static inline int json_is_string(const jval *v) { return v && v->type == J_STRING; }
static inline int json_is_array(const jval *v) { return v && v->type == J_ARRAY; }
static inline int json_is_object(const jval *v) { return v && v->type == J_OBJECT; }

#endif
