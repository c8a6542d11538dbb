// internal.h -- shared between the translation units of libmapfx.so (not installed).
#ifndef MAPFX_INTERNAL_H
#define MAPFX_INTERNAL_H

#ifdef __cplusplus
extern "C" {
#endif
// sets the message returned by mapfx_last_error(); returns `code`
int mapfx_internal_error(int code, const char* msg);
#ifdef __cplusplus
}
#endif
#endif
