/* ref_redirect.h -- force-included (gcc -include) when compiling the
 * UNMODIFIED reference sampler src/mcmc_wrapper2.c from /root/reference.
 * The reference hard-codes "/scratch/ssolanski/HB_MCMC" as its data/output
 * root (mcmc_wrapper2.c:110,365,374); these two macros route fopen()/access()
 * through ref_redirect.c, which swaps that prefix for $HBREF_ROOT.  Nothing
 * else in the reference is altered.  Test infrastructure only. */
#ifndef HB_REF_REDIRECT_H
#define HB_REF_REDIRECT_H
#include <stdio.h>
#include <unistd.h>
FILE *hbref_fopen(const char *path, const char *mode);
int hbref_access(const char *path, int mode);
#define fopen(p, m) hbref_fopen((p), (m))
#define access(p, m) hbref_access((p), (m))
#endif
