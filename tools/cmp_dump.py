import numpy as np, sys
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    x, y = a[k], b[k]
    d = np.abs(x - y)
    bad = np.argwhere(~np.isclose(x, y, rtol=1e-4, atol=1e-6 * (np.abs(x).max() + 1e-30)))
    print(k, x.shape, "max abs diff", float(np.nanmax(d)) if d.size else 0, "bad rows", sorted(set(bad[:, 0].tolist()))[:20] if bad.size else [])
