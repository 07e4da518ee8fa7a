"""Print the kernel sequence of one decode frame (and per-name totals per frame) from a
rocprofv3 --kernel-trace DB:  python scripts/frame_trace.py <db> [n_kernels]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
nk = int(sys.argv[2]) if len(sys.argv) > 2 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
fin = [i for i, r in enumerate(rows) if r[0].startswith("finish_kernel")]
a, b = fin[len(fin) // 2], fin[len(fin) // 2 + 1]
prev = rows[a][2]
for r in rows[a + 1:a + 1 + nk]:
    nm = r[0].split("(")[0].replace("void ", "")[:44]
    print(f"{nm:46s} blocks=({r[3] // r[6]},{r[4]},{r[5]}) dur={(r[2] - r[1]) / 1e3:7.2f}us gap={(r[1] - prev) / 1e3:5.2f}")
    prev = r[2]
tot = defaultdict(float)
for r in rows[a + 1:b + 1]:
    tot[r[0].split("(")[0].replace("void ", "")[:60]] += (r[2] - r[1]) / 1e3
span = (rows[b][2] - rows[a][2]) / 1e3
print(f"--- one frame: span {span:.1f} us, kernel sum {sum(tot.values()):.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {v:8.1f} us  {k}")
gaps = defaultdict(float)
cnt = defaultdict(int)
prev = rows[a][2]
for r in rows[a + 1:b + 1]:
    k = r[0].split("(")[0].replace("void ", "").split("<")[0][:40]
    gaps[k] += (r[1] - prev) / 1e3
    cnt[k] += 1
    prev = r[2]
print(f"--- gaps before each kernel class (sum {sum(gaps.values()):.1f} us over {sum(cnt.values())} launches)")
for k, v in sorted(gaps.items(), key=lambda kv: -kv[1]):
    print(f"  {v:8.1f} us  {cnt[k]:4d} x  {k}")
