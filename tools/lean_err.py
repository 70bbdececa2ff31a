"""Why the sweep's coefficients keep the reference's expression forms.

    python tools/lean_err.py

Random (w0, dtau, B1, B2, F1u, F2d) spanning thin to thick layers: propagate_fluxes
(twostream.py:139-176) in the reference's literal form, in rewritten forms — psi = -r Tr
("psi"), (xi + psi) - chi as -((chi - psi) - xi) ("vneg"), pi folded into B ("pi"), the
coefficients premultiplied by 1/chi ("pre") — and at 40 digits (mpmath).  Median errors are
all ~1e-15, but "psi", "vneg" and "pi" move the ill-conditioned thin-layer elements by up to
0.5 / 0.07 / 2e-8 relative against the literal form (the reference's chi, psi, xi rounding
errors are correlated and cancel in (chi - psi) - xi); "pre" stays within 6e-16.  The GPU
parity suite failed with the first three (profiles/r04/calls/r04c6/) and passes with "pre"
alone (FREI_LEAN).
"""
import numpy as np
from mpmath import mp, mpf
rng = np.random.default_rng(1)
n = 20000
w0 = 10**rng.uniform(-6, np.log10(0.5), n); w0[:n//2] = np.minimum(w0[:n//2], 0.1)
dtau = 10**rng.uniform(-9, 2, n)
B1 = 10**rng.uniform(5, 12, n); B2 = B1 * (1 + 10**rng.uniform(-8, -1, n) * rng.choice([-1, 1], n))
F1u = 10**rng.uniform(5, 12, n); F2d = 10**rng.uniform(3, 12, n)
def E(w): return np.where(w > 0.1, (1.225 - 0.1777*w) - 0.05582*(w*w), 1.0)
def ref(w0, dtau, B1, B2, F1u, F2d):
    e = E(w0); Emw = e - w0
    T = np.exp(-2*np.sqrt(e*Emw)*dtau)
    r = np.sqrt(Emw/e); zp = 0.5*(1+r); zm = 0.5*(1-r)
    chi = zm**2*T**2 - zp**2; xi = zp*zm*(1-T**2); psi = (zm**2 - zp**2)*T
    pi_w = np.pi*(1-w0)/Emw; Bp = (B1-B2)/dtau
    F2u = 1/chi*(psi*F1u - xi*F2d + pi_w*(B2*(chi+xi) - psi*B1 + Bp/(2*e)*(chi - psi - xi)))
    F1d = 1/chi*(psi*F2d - xi*F1u + pi_w*(B1*(chi+xi) - psi*B2 + Bp/(2*e)*(xi + psi - chi)))
    return F2u, F1d
def lean(w0, dtau, B1, B2, F1u, F2d, opts):
    e = E(w0); Emw = e - w0
    T = np.exp(-2*np.sqrt(e*Emw)*dtau)
    r = np.sqrt(Emw/e); zp = 0.5*(1+r); zm = 0.5*(1-r)
    zm2, zp2, T2 = zm*zm, zp*zp, T*T
    chi = zm2*T2 - zp2; xi = (zp*zm)*(1-T2)
    psi = -(r*T) if "psi" in opts else (zm2 - zp2)*T
    ic = 1/chi
    u = chi + xi
    v = (chi - psi) - xi
    vd = -v if "vneg" in opts else (xi + psi) - chi
    pi_w = (1-w0)/Emw if "pi" in opts else np.pi*(1-w0)/Emw
    b1, b2 = (np.pi*B1, np.pi*B2) if "pi" in opts else (B1, B2)
    q = ((b1-b2)/dtau)/(2*e)
    Xu = pi_w*((b2*u - psi*b1) + q*v); Xd = pi_w*((b1*u - psi*b2) + q*vd)
    if "pre" in opts:
        F2u = (ic*psi)*F1u - (ic*xi)*F2d + ic*Xu
        F1d = (ic*psi)*F2d - (ic*xi)*F1u + ic*Xd
    else:
        F2u = ic*((psi*F1u - xi*F2d) + Xu); F1d = ic*((psi*F2d - xi*F1u) + Xd)
    return F2u, F1d
# high precision reference with mpmath on a subset
mp.dps = 40
idx = np.arange(0, n, 20)
def exact(i):
    w=mpf(w0[i]); d=mpf(dtau[i]); b1=mpf(B1[i]); b2=mpf(B2[i]); fu=mpf(F1u[i]); fd=mpf(F2d[i])
    e = (mpf('1.225') - mpf('0.1777')*w) - mpf('0.05582')*w*w if w > mpf('0.1') else mpf(1)
    Emw = e-w; T = mp.exp(-2*mp.sqrt(e*Emw)*d); r = mp.sqrt(Emw/e); zp=(1+r)/2; zm=(1-r)/2
    chi = zm**2*T**2 - zp**2; xi = zp*zm*(1-T**2); psi=(zm**2-zp**2)*T; pw = mp.pi*(1-w)/Emw; Bp=(b1-b2)/d
    F2u = (psi*fu - xi*fd + pw*(b2*(chi+xi) - psi*b1 + Bp/(2*e)*(chi-psi-xi)))/chi
    F1d = (psi*fd - xi*fu + pw*(b1*(chi+xi) - psi*b2 + Bp/(2*e)*(xi+psi-chi)))/chi
    return float(F2u), float(F1d)
ex = np.array([exact(i) for i in idx])
R = ref(w0, dtau, B1, B2, F1u, F2d)
def err(F): return [np.max(np.abs(F[k][idx]-ex[:,k])/np.abs(ex[:,k])) for k in (0,1)], [np.median(np.abs(F[k][idx]-ex[:,k])/np.abs(ex[:,k])) for k in (0,1)]
print("ref  ", err(R))
for opts in [(), ("psi",), ("vneg",), ("pi",), ("pre",), ("psi","vneg","pi","pre")]:
    L = lean(w0, dtau, B1, B2, F1u, F2d, opts)
    print(opts, err(L), "vs ref max", [np.max(np.abs(L[k]-R[k])/np.abs(R[k])) for k in (0,1)])
