import sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in sorted(a.files):
    same = np.array_equal(a[k], b[k])
    d = float(np.abs(a[k] - b[k]).max())
    print(f"{k:16s} bitwise={same} max|d|={d:.3e} max|a|={float(np.abs(a[k]).max()):.3e}")
