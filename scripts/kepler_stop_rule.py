"""CPU emulation of the eval kernels' cold Kepler solve (hb_device.hpp cold_start_k
+ newton_k) under two stopping rules: round 1-5's absolute one (predicted next
correction e d^2 / (2 den) <= 2^-52) and round 6's relative one (a quarter ulp
of E).  Per-lane (the kernel's wave-level exit only adds steps), exact libm
sin/cos in place of the rotations; E against an x87 long-double Newton root.

    python scripts/kepler_stop_rule.py
"""
import numpy as np
def root_ld(M, e, E0):
    Ml=M.astype(np.longdouble); El=E0.astype(np.longdouble); el=np.longdouble(e)
    for i in range(4): El=El-(El-el*np.sin(El)-Ml)/(1-el*np.cos(El))
    return El
def series(M,e):
    s=np.sin(M); c=np.cos(M); x=s*s
    e2=e*e;e3=e2*e;e4=e2*e2;e5=e4*e
    a0=e2+e4;a1=-8/3*e4;b0=(e+e3)+e5;b1=-(1.5*e3+17/3*e5);b2=125/24*e5
    return M + s*(c*(x*a1+a0)+(x*(x*b2+b1)+b0))
def solve(M,e,rule):
    E=series(M,e) if abs(e)<=0.25 else M+0.85*e*np.sign(np.sin(M))
    done=np.zeros(len(M),bool); steps=np.zeros(len(M),int)
    for it in range(5):
        den=1-e*np.cos(E)
        d=((E-e*np.sin(E))-M)/den
        En=E-d
        E=np.where(done,E,En); steps+=~done
        z=d*d
        if rule=='abs': conv=abs(e)*z<=2**-51*den
        else: conv=abs(e)*z<=2**-53*den*np.abs(E)
        done|=conv
    return E,steps
n=1<<20
M=(np.arange(n)+0.5)/n*4*np.pi-2*np.pi
for e in [0.01,0.05,0.1,0.15,0.2,0.226,0.25]:
    for rule in ['abs','rel']:
        E,st=solve(M,e,rule)
        r=root_ld(M,e,E)
        err=np.abs((E-r).astype(np.float64))/np.spacing(np.abs(E))
        print(e,rule,'max ulp %.2f'%err.max(),'mean steps %.3f'%st.mean(), 'max steps',st.max())
