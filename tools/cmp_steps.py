import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for key in a.files:
    x, y = a[key], b[key]
    d = np.abs(x - y).max() / max(np.abs(y).max(), 1e-30)
    if d > 1e-6:
        print(f"{key:50s} rel {d:.3e}")
print("compared", len(a.files))
