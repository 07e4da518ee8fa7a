"""Per-instantiation average duration of the decode kernels in a rocprofv3 --kernel-trace DB, over
the graph-replayed frames of attn_span_probe.py (the last 100-frame timing window of each variant is
not separable, so every dispatch counts).  Usage: python scripts/gemv_kernel_split.py <db>"""
import sqlite3
import sys
from collections import defaultdict

c = sqlite3.connect(sys.argv[1])
acc = defaultdict(lambda: [0, 0.0])
for name, s, e in c.execute("select name, start, end from kernels"):
    if not any(k in name for k in ("gemv_kernel", "attn_fd", "fast_attn2", "sample_fast")):
        continue
    k = name.split("(")[0].replace("void ", "")
    acc[k][0] += 1
    acc[k][1] += (e - s) / 1e3
for k, (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
    print(f"  {t / n:7.2f} us x {n:7d}  {k}")
