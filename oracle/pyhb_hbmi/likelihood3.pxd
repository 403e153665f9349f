# Option B of INTEGRATION.md section 4: the reference's src/pyHB.pyx compiled
# unmodified against include/hbmi.h and linked to libhbmi.so, in place of the
# reference's likelihood3.pxd (which textually includes likelihood3.c).
# Test infrastructure: `make -C oracle pyhb_hbmi` builds it OUTSIDE the
# repository (tests/test_pyhb.py); nothing of it is shipped or travels.
# Nt is the C type of the header (long); the reference .pxd says double,
# which only works because it compiles likelihood3.c into the extension.
cdef extern from "hbmi.h":
    void calc_light_curve(double* times, long Nt, double* pars, double* template_)
    void calc_radii_and_Teffs(double* params, double* R1, double* R2, double* Teff1, double* Teff2)
    void calc_mags(double* params, double D, double* Gmg, double* BminusV, double* VminusG, double* GminusT)
    double _getT(double)
    double _getR(double)
    double envelope_Radius(double logM)
    double envelope_Temp(double logM)
