"""CPU restatement of LAPACK dsyevd's 2x2 path (np.linalg.eigh), the
algorithm csrc/ellipse_api.hip runs per covariance (test infrastructure only):
dsteqr's splitting and iteration tests, dlaev2, the rotation of Z = I
(dlasr 'R','V'), and the selection sort.  Pinned against np.linalg.eigh in
tests/test_ellipse_restatement.py; mylib/error_ellipse.py:39-55 calls eigh.
"""
import math

import numpy as np

def dlaev2(a, b, c):
    sm=a+c; df=a-c; adf=abs(df); tb=b+b; ab=abs(tb)
    if abs(a)>abs(c): acmx,acmn=a,c
    else: acmx,acmn=c,a
    if adf>ab: q=ab/adf; rt=adf*math.sqrt(1.0+q*q)
    elif adf<ab: q=adf/ab; rt=ab*math.sqrt(1.0+q*q)
    else: rt=ab*math.sqrt(2.0)
    if sm<0: rt1=0.5*(sm-rt); s1=-1; rt2=(acmx/rt1)*acmn-(b/rt1)*b
    elif sm>0: rt1=0.5*(sm+rt); s1=1; rt2=(acmx/rt1)*acmn-(b/rt1)*b
    else: rt1=0.5*rt; rt2=-0.5*rt; s1=1
    if df>=0: cs=df+rt; s2=1
    else: cs=df-rt; s2=-1
    if abs(cs)>ab: ct=-tb/cs; sn1=1.0/math.sqrt(1.0+ct*ct); cs1=ct*sn1
    elif ab==0: cs1=1.0; sn1=0.0
    else: tn=-cs/tb; cs1=1.0/math.sqrt(1.0+tn*tn); sn1=tn*cs1
    if s1==s2: tn=cs1; cs1=-sn1; sn1=tn
    return rt1,rt2,cs1,sn1
def eig2(A):
    a,b,c=A[0,0],A[1,0],A[1,1]
    w=[a,c]; Z=np.eye(2)
    eps=2.0**-53; tst=abs(b)
    rot = tst!=0 and not (tst <= (math.sqrt(abs(a))*math.sqrt(abs(c)))*eps)
    if rot:
        t2=tst*tst
        lim=(2.0**-106*abs(c))*abs(a)+2.0**-1022 if abs(c)<abs(a) else (2.0**-106*abs(a))*abs(c)+2.0**-1022
        rot = not (t2<=lim)
    if rot:
        rt1,rt2,cs,sn=dlaev2(a,b,c); w=[rt1,rt2]; Z=np.array([[cs,-sn],[sn,cs]])
    if w[1]<w[0]:
        w=[w[1],w[0]]; Z=Z[:,::-1].copy()
    return np.array(w),Z
