"""Host simulation of wide_stream_kernel's candidate buffer on 3*N(0,1) rows (api default: precision 16, temp 1,
V = 50,257, fp32 tiles of 256 ids, 4 sample tiles, 1,024-entry LDS buffer): how many segment entries a stream
writes for how many kept ids, under the flush policies measured in round 4 (wide path).
  all   -- flush the whole buffer when it stays more than half full after compaction (the kernel)
  mean  -- flush only the entries at or above the buffer's mean value (fewer stale writes, more instructions)
Usage: python tools/sim_wide_flush.py [rows]"""
import math
import sys

import numpy as np

V, TS, R, CW, NK = 50257, 256, 2 ** 16, 1024, 4


def simulate(x, policy):
    ntiles = (V + TS - 1) // TS
    space = ntiles // NK
    samp = [s * space + space - 1 for s in range(NK)]
    r = max(x[t * TS:(t + 1) * TS].max() for t in samp)

    def threshold(s_part):  # the kernel's running threshold from a partial sum against r
        L = math.log(s_part * 0.999 / R)
        return r + L - 1e-4 * (1 + abs(r) + abs(L))

    S = sum(np.exp(x[t * TS:(t + 1) * TS] - r).sum() for t in samp)
    tw = threshold(S)
    buf, flushed = np.empty(0), []

    def append(t):
        nonlocal buf
        v = x[t * TS:(t + 1) * TS]
        new = v[v >= tw]
        if len(buf) + len(new) > CW:
            buf = buf[buf >= tw]
            if len(buf) + len(new) > CW or 2 * len(buf) > CW:
                if policy == "mean":
                    up = buf[buf >= buf.mean()]
                    rest = buf[buf < buf.mean()]
                    if len(rest) + len(new) > CW:
                        up, rest = buf, np.empty(0)
                else:
                    up, rest = buf, np.empty(0)
                flushed.append(up)
                buf = rest
        buf = np.concatenate([buf, new])

    for t in samp:
        append(t)
    rest = [t for t in range(ntiles) if t not in samp]
    for i, t in enumerate(rest):
        S += np.exp(x[t * TS:(t + 1) * TS] - r).sum()
        append(t)
        if i % 4 == 3:
            tw = max(tw, threshold(S))
    m = x.max()
    Sf = np.exp(x - m).sum()
    L = math.log(Sf / R)
    xt = m + L - 1e-4 * (1 + abs(m) + abs(L))
    seg = np.concatenate(flushed + [buf[buf >= xt]])
    return len(seg), int((x >= xt).sum())


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    rng = np.random.default_rng(1)
    for _ in range(rows):
        x = 3.0 * rng.standard_normal(V)
        (na, k), (nm, _) = simulate(x, "all"), simulate(x, "mean")
        print(f"kept {k}: segment entries, flush all {na} ({na / k:.2f}x), mean pivot {nm} ({nm / k:.2f}x)")


if __name__ == "__main__":
    main()
