"""fx_pipe 4 device trace: per chain workgroup, chain cycles a key and the
cycles its chain waves spent at barriers / its loaders in a write (rows 4040 + c)."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(6, 4096, 8).astype(np.int64)[1][4040:4072]
for c, r in enumerate(t):
    if r[0] == 0:
        continue
    n = max(int(r[2]), 1)
    print(f"wg {c:2d}: chain {(r[1] - r[0]) / n:5.1f} cyc/key over {n} keys; barrier wait w0 {r[3] / n:5.1f} w1 {r[4] / n:5.1f} "
          f"cyc/key; loader write w2 {r[5]} w3 {r[6]} cyc")
