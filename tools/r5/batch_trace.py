"""Summarise a QASR_DEV_TRACE dump of a decode-batch step (decode_attn_seq_kernel<1>
marks: start, q/k/v ready, scores done, chain done; 100 MHz clock).  Dev tool."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(6, 4096, 8).astype(np.int64)[1]
x = t[(t[:, 0] > 0) & (t[:, 3] > 0)]
t0 = x[:, 0].min()
us = lambda v: (v - t0) / 100.0
print(f"workgroups {len(x)}: start {us(x[:, 0].min()):.2f}..{us(x[:, 0].max()):.2f} us, end {us(x[:, 3].min()):.2f}..{us(x[:, 3].max()):.2f}")
for name, a, b in (("q/k/v + norm/rope", 0, 1), ("K stream + scores", 1, 2), ("weights + chain", 2, 3), ("whole", 0, 3)):
    d = (x[:, b] - x[:, a]) / 100.0
    print(f"  {name:20s} median {np.median(d):6.2f}  p10 {np.percentile(d, 10):6.2f}  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f} us")
starts = np.sort(us(x[:, 0]))
print("start-time deciles (us):", " ".join(f"{v:.1f}" for v in np.percentile(starts, [0, 10, 25, 50, 75, 90, 100])))
