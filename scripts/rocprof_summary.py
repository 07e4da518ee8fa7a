#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (rocpd sqlite `*_results.db`, or the CSV
`*_kernel_trace.csv`) into a markdown table + JSON for profiles/.

    python scripts/rocprof_summary.py <db-or-csv> <out-prefix> [--bench <bench-json-log>]

The JSON carries the aggregate of every decode-linear dispatch (the bench's roofline kernel:
the bf16 `gemv_kernel<..., QM = 0>` instantiations and `rowgemv_kernel<...>`): launch count and average duration, to be checked against bench.py's HIP-event figure.
With --pmc-fetch/--pmc-write (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs, separate passes) the
per-launch HBM traffic of that kernel is added, FETCH_SIZE doubled per the gfx950 correction in
MI355X_MICROARCH.md §HBM (wide coalesced reads are tallied at half their bytes).
"""
import argparse
import re
import csv
import json
import os
import sqlite3
from collections import defaultdict


def is_decode_linear(name):
    """bench.py's roofline kernel family: the bf16 decode GEMVs (gemv_kernel QM = 0, rowgemv_kernel)."""
    # bf16 instantiations only: both templates end in QM (0 bf16, 1 int8, 2 int4)
    return (name.startswith("void gemv_kernel") or name.startswith("void rowgemv_kernel")) and \
        re.search(r", 0>\(", name) is not None


def load_dispatches(path):
    """-> list of (name, duration_ns, grid) from a rocpd DB or a kernel_trace CSV."""
    out = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e, gx, gy, gz in c.execute("select name, start, end, grid_x, grid_y, grid_z from kernels"):
            out.append((name, e - s, (gx, gy, gz)))
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                out.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                            (int(r.get("Grid_Size_X", 0)), int(r.get("Grid_Size_Y", 0)),
                             int(r.get("Grid_Size_Z", 0)))))
    return out


def load_pmc(path, counter):
    """rocprofv3 --pmc run -> {kernel name: [values per dispatch]}"""
    vals = defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = "select name, counter_value from pmc_events where counter_name = ?"
        try:
            rows = c.execute(q, (counter,)).fetchall()
        except sqlite3.OperationalError:
            cols = [d[1] for d in c.execute("pragma table_info(pmc_events)")]
            raise SystemExit(f"unexpected pmc_events schema: {cols}")
        for n, v in rows:
            vals[n].append(float(v))
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") == counter:
                    vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def short(name, n=90):
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out_prefix")
    ap.add_argument("--bench", help="bench.py stdout of the profiled command (its JSON line)")
    ap.add_argument("--pmc-fetch")
    ap.add_argument("--pmc-write")
    ap.add_argument("--title", default="rocprofv3 --kernel-trace --stats")
    a = ap.parse_args()

    d = load_dispatches(a.trace)
    by = defaultdict(lambda: [0, 0])
    for name, ns, _ in d:
        by[name][0] += 1
        by[name][1] += ns
    total = sum(v[1] for v in by.values())
    rows = sorted(by.items(), key=lambda kv: -kv[1][1])
    # the bench's roofline kernel is the bf16 decode linear: gemv_kernel<..., QM = 0> (the int8 / int4
    # legs' instantiations end in 1> / 2> and are reported apart) and the row-block rowgemv_kernel
    gemv = [(n, ns) for n, ns, _ in d if is_decode_linear(n)]
    g_n = len(gemv)
    g_avg_us = sum(ns for _, ns in gemv) / max(g_n, 1) / 1e3
    summary = {"trace": os.path.basename(a.trace), "total_kernel_ms": total / 1e6,
               "gemv_kernel": {"launches": g_n, "avg_us": g_avg_us}}
    bench = None
    if a.bench:
        with open(a.bench) as fh:
            for line in fh:
                if line.startswith("{") and '"metric"' in line:
                    bench = json.loads(line)
        if bench:
            summary["bench_roofline"] = bench["roofline"]
            summary["gemv_kernel"]["bench_event_avg_us"] = bench["roofline"]["avg_launch_us"]
    if a.pmc_fetch:
        f = load_pmc(a.pmc_fetch, "FETCH_SIZE")
        fv = [v for n, vs in f.items() if is_decode_linear(n) for v in vs]
        if fv:
            # rocprofv3 reports FETCH_SIZE in KB; x2 = gfx950 wide-read correction
            summary["gemv_kernel"]["fetch_bytes_per_launch"] = 2 * 1024 * sum(fv) / len(fv)
    if a.pmc_write:
        w = load_pmc(a.pmc_write, "WRITE_SIZE")
        wv = [v for n, vs in w.items() if is_decode_linear(n) for v in vs]
        if wv:
            summary["gemv_kernel"]["write_bytes_per_launch"] = 1024 * sum(wv) / len(wv)
    g = summary["gemv_kernel"]
    if "fetch_bytes_per_launch" in g:
        g["hbm_bytes_per_launch"] = g["fetch_bytes_per_launch"] + g.get("write_bytes_per_launch", 0.0)

    if "hbm_bytes_per_launch" in g:
        with open(os.path.join(os.path.dirname(a.out_prefix), "pmc_gemv_r01.json"), "w") as fh:
            json.dump({"hbm_bytes_per_launch": round(g["hbm_bytes_per_launch"]),
                       "fetch_bytes_per_launch": round(g["fetch_bytes_per_launch"]),
                       "write_bytes_per_launch": round(g.get("write_bytes_per_launch", 0)),
                       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE of scripts/pmc_probe.py"}, fh)
    with open(a.out_prefix + ".json", "w") as fh:
        json.dump(summary, fh, indent=1)
    with open(a.out_prefix + ".md", "w") as fh:
        fh.write(f"# {a.title}\n\nsource: `{os.path.basename(a.trace)}`; {len(d)} dispatches, "
                 f"{total / 1e6:.1f} ms of kernel time\n\n")
        fh.write("| % time | launches | avg us | total ms | kernel |\n|---:|---:|---:|---:|---|\n")
        for name, (n, ns) in rows[:30]:
            fh.write(f"| {100 * ns / total:.1f} | {n} | {ns / n / 1e3:.2f} | {ns / 1e6:.1f} | `{short(name)}` |\n")
        fh.write(f"\ndecode linears (`gemv_kernel` bf16 instantiations, QM = 0, and `rowgemv_kernel`): {g_n} "
                 f"launches, average {g_avg_us:.3f} us")
        if bench:
            fh.write(f"; bench.py HIP-event average in the same run: {bench['roofline']['avg_launch_us']} us")
        fh.write("\n")
        if "hbm_bytes_per_launch" in g:
            fh.write(f"\nPMC (separate `--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` passes): per decode-linear launch "
                     f"{g['fetch_bytes_per_launch'] / 1e6:.2f} MB fetched (FETCH_SIZE KB x1024 x2, gfx950 "
                     f"wide-read correction) + {g['write_bytes_per_launch'] / 1e6:.3f} MB written = "
                     f"{g['hbm_bytes_per_launch'] / 1e6:.2f} MB HBM traffic\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
