/*
 * isal_api.h — version surface of the MI355X erasure-code engine.
 *
 * Drop-in for the reference's include/isal_api.h (version macros at
 * isal_api.h:68-85, isal_get_version_str at :93, isal_get_version at :104).
 * The engine reports the ISA-L release whose erasure-code ABI it implements
 * (2.32.1), so callers that gate on ISAL_MAKE_VERSION keep working.
 */
#ifndef ISAL_HIP_ISAL_API_H
#define ISAL_HIP_ISAL_API_H

#ifdef __cplusplus
extern "C" {
#endif

#define ISAL_MAJOR_VERSION 2
#define ISAL_MINOR_VERSION 32
#define ISAL_PATCH_VERSION 1

#define ISAL_MAKE_VERSION(maj, min, patch) ((maj) * 0x10000 + (min) * 0x100 + (patch))
#define ISAL_VERSION ISAL_MAKE_VERSION(ISAL_MAJOR_VERSION, ISAL_MINOR_VERSION, ISAL_PATCH_VERSION)

/* "2.32.1": replaces isal_get_version_str (reference isal_api.h:93). */
const char *isal_get_version_str(void);

/* ISAL_VERSION as a number: replaces isal_get_version (reference isal_api.h:104). */
unsigned isal_get_version(void);

#ifdef __cplusplus
}
#endif

#endif /* ISAL_HIP_ISAL_API_H */
