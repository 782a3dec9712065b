/*
 * psx_debug.h — experiment hooks of libpsx (not part of the reference boundary).
 * Selects kernel variants at run time so A/B measurements run interleaved in one
 * process (cdna_hip_programming.md §5.4 rule 24).
 */
#ifndef PSX_DEBUG_H_
#define PSX_DEBUG_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { PSX_VARIANT_DENSE_INDEX = 0, PSX_VARIANT_DENSE_APPLY = 1, PSX_VARIANT_INV_LAYOUT = 2,
       PSX_VARIANT_ADA_APPLY = 3, PSX_VARIANT_H16_APPLY = 4,
       PSX_VARIANT_ORD_GRID = 5, PSX_VARIANT_ORD_SPLIT = 6 };

/* Returns the previous variant, or -1 for an unknown selector. */
int32_t psx_debug_set_variant(int32_t which, int32_t variant);
int32_t psx_debug_get_variant(int32_t which);

#ifdef __cplusplus
}
#endif
#endif
