"""Default chain (fx1_chain_body) device trace: per kv group, each chain wave's
end (us after the group's start) and cycles a key (rows 4020 + g, 4030 + g)."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(6, 4096, 8).astype(np.int64)[1]
for g in range(8):
    st, n = t[4000 + g, 0], max(int(t[4010 + g, 2]), 1)
    if st == 0:
        continue
    ends = (t[4020 + g, :4] - st) / 100.0
    cyc = t[4030 + g, :4] / n
    print(f"g {g}: chain end per wave " + " ".join(f"{e:6.2f}" for e in ends) + " us;  cycles a key " +
          " ".join(f"{c:5.1f}" for c in cyc) + f";  published {(t[4000 + g, 5] - st) / 100.0:6.2f}")
    if t[4010 + g, 6]:
        print(f"      gather: {t[4010 + g, 5]} polls, the last issued at {(t[4010 + g, 6] - st) / 100.0:6.2f} us, "
              f"gathered at {(t[4000 + g, 2] - st) / 100.0:6.2f} us")
