"""Fit of the fp32 atan polynomial in kinhip_device.h (atan2_pos_fast): atan(a) = a (1 + z P(z)),
z = a^2, a in [0, 1], P of degree 6, by iteratively reweighted least squares towards minimax
absolute error; prints the coefficients (z^0 first) and the max error in fp64 and fp32.
    python tools/atan_fit.py"""
import numpy as np

n = 7
t = np.cos(np.pi * (np.arange(20000) + 0.5) / 20000) * 0.5 + 0.5
t = t[t > 1e-4]
z = t * t
A = np.stack([z ** k for k in range(n)], 1)
w = np.ones_like(t)
coef = np.linalg.lstsq(A, (np.arctan(t) / t - 1) / z, rcond=None)[0]
for _ in range(50):
    r = t * (1 + z * (A @ coef)) - np.arctan(t)
    w = w * np.sqrt(np.abs(r) / np.abs(r).max() + 1e-3)
    coef = np.linalg.lstsq(A * (w * t * z)[:, None], (np.arctan(t) - t) * w, rcond=None)[0]
x = np.linspace(0, 1, 2000001)
zz = x * x
r64 = x * (1 + zz * sum(coef[k] * zz ** k for k in range(n)))
xf, cf = x.astype(np.float32), coef.astype(np.float32)
zf = xf * xf
p = cf[-1]
for k in range(n - 2, -1, -1):
    p = p * zf + cf[k]
r32 = xf * (np.float32(1) + zf * p)
print("coefficients z^0..z^6:", [float(c) for c in cf])
print(f"max abs error fp64 {np.abs(r64 - np.arctan(x)).max():.2e}  fp32 {np.abs(r32 - np.arctan(x)).max():.2e}")
