/* Config override for building the UNMODIFIED reference sources in place.
 *
 * Test-oracle infrastructure only (see oracle/README.md).  Force-included
 * (`g++ -include oracle/ref_cfg.h`) in front of every reference translation
 * unit.  The reference's config.hh (/root/reference/config.hh:1-44) is
 * include-guarded, so after it has been pulled in here the render settings
 * can be re-pointed at the configuration under test, exactly as the reference
 * README invites ("You can change these freely", config.hh:10-13).  Nothing
 * else of the reference is altered.
 */
#ifndef PTG_REF_CFG_H
#define PTG_REF_CFG_H
#include "config.hh"

#ifndef REF_W
#define REF_W 640
#endif
#ifndef REF_H
#define REF_H 360
#endif
#ifndef REF_SPP
#define REF_SPP 256
#endif
#ifndef REF_BOUNCES
#define REF_BOUNCES 4
#endif

#undef IMAGE_WIDTH
#undef IMAGE_HEIGHT
#undef SAMPLES_PER_PIXEL
#undef MAX_BOUNCES
#define IMAGE_WIDTH REF_W
#define IMAGE_HEIGHT REF_H
#define SAMPLES_PER_PIXEL REF_SPP
#define MAX_BOUNCES REF_BOUNCES
#endif
