"""Summarise a QASR_DEV_TRACE dump: per-block 100 MHz timestamps of one decode
layer's kernels (QKV GEMV, attention, o-proj, gate/up, down).  Dev tool only."""
import sys

import numpy as np

NAMES = ["qkv_gemv", "attention", "oproj_gemv", "gateup_gemv", "down_gemv"]


def main(path):
    t = np.fromfile(path, dtype=np.uint64).reshape(6, 4096, 8).astype(np.int64)
    wide = (t[1][4040:4072, 0] > 0).any()   # fx_pipe 2, 3, 4: chain blocks c = 0 .. 31 at rows 4000 + c, clocks at 4040 + c
    ch = t[1][4000:4040] if wide else t[1][4000:4008]
    ch = ch[ch[:, 0] > 0]
    ck = (t[1][4040:4072] if wide else t[1][4010:4018]).copy()   # chain workgroups: shader clock at chain start / end, keys
    t[1][4000:4080] = 0
    live = [t[k][t[k][:, 0] > 0] for k in range(5)]
    t0 = min(int(x[:, 0].min()) for x in live if len(x))
    us = lambda v: (v - t0) / 100.0
    prev_end = None
    for k, x in enumerate(live):
        if not len(x):
            continue
        st = x[:, 0]
        if k == 1 and len(ch):   # fused exact attention: split blocks (scores) + chain workgroups
            print(f"{NAMES[k]:12s} split blocks {len(x):4d} start {us(st.min()):7.2f}..{us(st.max()):7.2f}  "
                  f"scores published max {us(x[:, 3].max()):7.2f}")
            lab = ["start", "v ready", "scores gathered", "weights", "chain", "published", "w expf", "w stored"]
            nl = 8 if (ch[:, 6] > 0).all() else 6
            print(f"{'':12s} chain wgs {len(ch)}: " + "  ".join(f"{lab[i]} {us(np.median(ch[:, i])):6.2f}/{us(ch[:, i].max()):6.2f}"
                                                             for i in range(nl)))
            e = ch[:, 5].max()
            ok = ck[:, 1] > ck[:, 0]
            if ok.any() and len(ch) == len(ck[ok]):
                cyc = (ck[ok, 1] - ck[ok, 0]).astype(np.float64)
                dt = (ch[:, 4] - ch[:, 1]).astype(np.float64) / 100.0   # us, 'v ready' -> 'chain'
                print(f"{'':12s} chain: {np.median(cyc):.0f} shader cycles over {ck[ok, 2][0]} keys "
                      f"({np.median(cyc) / ck[ok, 2][0]:.1f} a key), {np.median(dt):.2f} us -> {np.median(cyc / dt) / 1e3:.2f} GHz; "
                      f"head 2g new-maximum keys {ck[ok, 3].tolist()}, slow 8-key groups {ck[ok, 4].tolist()}")
        elif k == 1:
            kv, rdy, cnt = x[:, 1], x[:, 2], x[:, 3]
            lastb = x[x[:, 4] > 0]
            print(f"{NAMES[k]:12s} blocks {len(x):4d} start {us(st.min()):7.2f}..{us(st.max()):7.2f}  "
                  f"kv-landed med +{np.median(kv - st) / 100:5.2f} max {us(kv.max()):7.2f}")
            print(f"{'':12s} scores +{np.median(x[:, 6] - kv) / 100:5.2f} softmax +{np.median(x[:, 7] - x[:, 6]) / 100:5.2f} "
                  f"pv +{np.median(rdy - x[:, 7]) / 100:5.2f}")
            print(f"{'':12s} partial-ready med +{np.median(rdy - kv) / 100:5.2f} max {us(rdy.max()):7.2f}  "
                  f"counted med +{np.median(cnt - rdy) / 100:5.2f} max {us(cnt.max()):7.2f}")
            print(f"{'':12s} combiners {len(lastb)}: burst landed +{np.median(lastb[:, 5] - lastb[:, 3]) / 100:5.2f}  "
                  f"end +{np.median(lastb[:, 4] - lastb[:, 5]) / 100:5.2f}  end max {us(lastb[:, 4].max()):7.2f}")
            e = lastb[:, 4].max()
        else:
            en = x[:, 1]
            print(f"{NAMES[k]:12s} blocks {len(x):4d} start {us(st.min()):7.2f}..{us(st.max()):7.2f}  "
                  f"end {us(en.min()):7.2f}..{us(en.max()):7.2f}  block-dur med {np.median(en - st) / 100:5.2f}")
            e = en.max()
        if prev_end is not None:
            print(f"{'':12s} gap from previous kernel's last block end to first start: {(st.min() - prev_end) / 100:5.2f} us")
        prev_end = e


if __name__ == "__main__":
    main(sys.argv[1])
