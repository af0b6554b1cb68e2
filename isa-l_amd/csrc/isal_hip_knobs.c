/*
 * isal_hip_knobs.c — the engine's ISAL_HIP_* environment knobs.
 *
 * Every knob is read from the environment ONCE (first use) into a table, so
 * no launch or drop-in call pays a getenv; isal_hip_config_reload() re-reads
 * them (tests and tuning sweeps change knobs inside one process). The
 * reference has no runtime configuration beyond its CPU dispatch (SURVEY.md
 * §5 "Config / flags"); these knobs are the engine's own. Round 5 removed the
 * 18 that only selected variants measured flat or slower (their A/B results
 * stay in DESIGN.md §2b): every knob left either switches a default-on
 * mechanism off for an A/B or a fallback, or exists for a test.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "isal_hip.h"
#include "isal_hip_internal.h"

typedef struct {
        const char *name;
        /* string-valued knobs map their words to ints; NULL = integer knob */
        const char *const *words;
} knob_def;

static const char *const backend_words[] = {"auto", "gpu", "cpu", NULL};

static const knob_def defs[ISAL_HIP_KNOB_COUNT] = {
        [ISAL_HIP_KNOB_BACKEND] = {"ISAL_HIP_BACKEND", backend_words},
        [ISAL_HIP_KNOB_CPU_MAX_BYTES] = {"ISAL_HIP_CPU_MAX_BYTES", NULL},
        [ISAL_HIP_KNOB_LOG] = {"ISAL_HIP_LOG", NULL},
        [ISAL_HIP_KNOB_CPU_SIMD] = {"ISAL_HIP_CPU_SIMD", NULL},
        [ISAL_HIP_KNOB_STAGE_MB] = {"ISAL_HIP_STAGE_MB", NULL},
        [ISAL_HIP_KNOB_ENC_GLDS] = {"ISAL_HIP_ENC_GLDS", NULL},
        [ISAL_HIP_KNOB_CRC_TILES] = {"ISAL_HIP_CRC_TILES", NULL},
        [ISAL_HIP_KNOB_CRC_XROWS] = {"ISAL_HIP_CRC_XROWS", NULL},
        [ISAL_HIP_KNOB_FAULT] = {"ISAL_HIP_FAULT", NULL},
        [ISAL_HIP_KNOB_FAULT_CHUNK] = {"ISAL_HIP_FAULT_CHUNK", NULL},
        [ISAL_HIP_KNOB_CHUNK_KB] = {"ISAL_HIP_CHUNK_KB", NULL},
        [ISAL_HIP_KNOB_PIPE_CHUNKS] = {"ISAL_HIP_PIPE_CHUNKS", NULL},
        [ISAL_HIP_KNOB_PINNED_DIRECT] = {"ISAL_HIP_PINNED_DIRECT", NULL},
        [ISAL_HIP_KNOB_CPU_MAX_BYTES_PINNED] = {"ISAL_HIP_CPU_MAX_BYTES_PINNED", NULL},
        [ISAL_HIP_KNOB_PAR_COPY] = {"ISAL_HIP_PAR_COPY", NULL},
        [ISAL_HIP_KNOB_ENC_XOR] = {"ISAL_HIP_ENC_XOR", NULL},
        [ISAL_HIP_KNOB_ENC_LDS] = {"ISAL_HIP_ENC_LDS", NULL},
        [ISAL_HIP_KNOB_KARG] = {"ISAL_HIP_KARG", NULL},
        [ISAL_HIP_KNOB_MAX_HELPERS] = {"ISAL_HIP_MAX_HELPERS", NULL},
        [ISAL_HIP_KNOB_KARG_DONE] = {"ISAL_HIP_KARG_DONE", NULL},
        [ISAL_HIP_KNOB_ENC_GROUP] = {"ISAL_HIP_ENC_GROUP", NULL},
        [ISAL_HIP_KNOB_KARG_NARROW] = {"ISAL_HIP_KARG_NARROW", NULL},
        [ISAL_HIP_KNOB_ENC_WIDE5] = {"ISAL_HIP_ENC_WIDE5", NULL},
        [ISAL_HIP_KNOB_ENC_LDSX] = {"ISAL_HIP_ENC_LDSX", NULL},
};

static long long values[ISAL_HIP_KNOB_COUNT];
static pthread_once_t once = PTHREAD_ONCE_INIT;

static long long
parse(const knob_def *d)
{
        const char *e = getenv(d->name);
        int i;
        if (!e || !*e)
                return -1;
        if (!d->words)
                return strtoll(e, NULL, 10);
        for (i = 0; d->words[i]; i++)
                if (strcmp(e, d->words[i]) == 0)
                        return i;
        return -2; /* set, but not a known word */
}

/* ISAL_HIP_* names the library reads that are not knobs of the table */
static const char *const other_names[] = {"ISAL_HIP_SYSFS_ROOT", "ISAL_HIP_LIB", NULL};

extern char **environ;

/* An ISAL_HIP_* variable the library does not read — a knob removed in an
 * earlier round, or a typo — would silently leave an A/B arm on the default:
 * say so once per process, naming each such variable. */
static void
warn_unknown(void)
{
        static int warned;
        char **e;
        if (__atomic_exchange_n(&warned, 1, __ATOMIC_RELAXED) || !environ)
                return;
        for (e = environ; *e; e++) {
                const char *v = *e, *eq = strchr(v, '=');
                size_t n;
                int i, known = 0;
                if (strncmp(v, "ISAL_HIP_", 9) != 0 || !eq)
                        continue;
                n = (size_t) (eq - v);
                for (i = 0; i < ISAL_HIP_KNOB_COUNT && !known; i++)
                        known = strlen(defs[i].name) == n && strncmp(defs[i].name, v, n) == 0;
                for (i = 0; other_names[i] && !known; i++)
                        known = strlen(other_names[i]) == n && strncmp(other_names[i], v, n) == 0;
                if (!known)
                        fprintf(stderr, "isal_hip: ignoring unknown environment variable %.*s (not a knob of this "
                                        "library; see isal_hip_knobs.c)\n",
                                (int) n, v);
        }
}

static void
load(void)
{
        int i;
        for (i = 0; i < ISAL_HIP_KNOB_COUNT; i++)
                values[i] = parse(&defs[i]);
        warn_unknown();
}

long long
isal_hip_knob(int id)
{
        pthread_once(&once, load);
        return id >= 0 && id < ISAL_HIP_KNOB_COUNT ? values[id] : -1;
}

static unsigned generation;

void
isal_hip_config_reload(void)
{
        pthread_once(&once, load);
        load();
        __atomic_add_fetch(&generation, 1u, __ATOMIC_RELEASE);
}

unsigned
isal_hip_knob_generation(void)
{
        return __atomic_load_n(&generation, __ATOMIC_ACQUIRE);
}
