/* ref_redirect.c -- path redirection for the reference sampler build (see
 * ref_redirect.h).  Test infrastructure only. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* this file is compiled under the same -include: use the real functions */
#undef fopen
#undef access

static const char *k_prefix = "/scratch/ssolanski/HB_MCMC";

static const char *hbref_map(const char *path, char *buf, size_t cap) {
    const char *root = getenv("HBREF_ROOT");
    size_t lp = strlen(k_prefix);
    if (root && strncmp(path, k_prefix, lp) == 0) {
        snprintf(buf, cap, "%s%s", root, path + lp);
        return buf;
    }
    return path;
}

FILE *hbref_fopen(const char *path, const char *mode) {
    char buf[4096];
    return fopen(hbref_map(path, buf, sizeof buf), mode);
}

int hbref_access(const char *path, int mode) {
    char buf[4096];
    return access(hbref_map(path, buf, sizeof buf), mode);
}
