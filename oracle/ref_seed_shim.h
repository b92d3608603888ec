/*
 * ORACLE TEST INFRASTRUCTURE -- never shipped, never linked into the product.
 *
 * Force-included (g++ -include) into every reference translation unit when
 * oracle/Makefile builds oracle/_ref/refharness from /root/reference sources.
 *
 * Why: trace_math.h:34 declares `static int g_seed = rand();` in a header, so
 * every reference TU owns a private LCG stream seeded by whichever glibc rand()
 * call its static initialiser happens to make.  Only two streams matter:
 *   - Vector3.cpp's  (randomInsideSphere, Vector3.cpp:176-188)  -> "sphere seed"
 *   - Render.cpp's   (additive jitter,    Render.cpp:177-178)   -> "jitter seed"
 * This hook routes rand() through rfx_ref_seed(__BASE_FILE__) so the harness
 * can pin both seeds explicitly from the environment.  With no environment
 * override every call falls back to the real glibc rand(), i.e. the stock
 * behaviour of the unmodified sources.
 */
#pragma once
#include <stdlib.h>
#ifdef __cplusplus
extern "C"
#endif
int rfx_ref_seed(const char *translation_unit);
#define rand() rfx_ref_seed(__BASE_FILE__)
