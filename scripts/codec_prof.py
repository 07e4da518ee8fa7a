"""Codec GEMM shapes and per-launch times: runs one config-2 codec decode ([1,10,216] codes) with the
conv2 knob off and on, under rocprofv3 --kernel-trace, or (with a DB path) summarises a trace:
    rocprofv3 --kernel-trace -d DIR -o run -- python3 scripts/codec_prof.py
    python3 scripts/codec_prof.py <results.db>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))


def run():
    import numpy as np

    from fishmi import native
    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    ccfg = CodecConfig()
    codec = FishMICodec.synthetic(ccfg, 1, 0, "bf16", max_frames=216)
    codes = np.random.default_rng(0).integers(0, 1024, (ccfg.n_codebooks + 1, 216)).astype(np.int32)
    ref = None
    # fused decoder ResidualUnits (resunit_kernel) off / on, and its tile variants (resunit_cfg)
    for fuse, cfg in ((0, 0), (1, 0), (1, 1), (1, 2), (0, 0), (1, 0), (1, 1), (1, 2)):
        native.tune("codec_fuse", fuse)
        native.tune("resunit_cfg", cfg)
        for _ in range(3):
            w = codec.decode_codes(codes)
        ms0, n0, f0 = codec.profile()
        codec.decode_codes(codes)
        ms1, n1, f1 = codec.profile()
        same = "" if ref is None else f", bit-identical to fuse=0: {bool(np.array_equal(w, ref))}"
        ref = w if ref is None else ref
        print(f"codec_fuse={fuse} resunit_cfg={cfg}: {ms1 - ms0:.2f} ms, {n1 - n0} GEMM launches, "
              f"{(f1 - f0) / ((ms1 - ms0) * 1e-3) / 1e12:.1f} TFLOP/s{same}", flush=True)


def sequence(db, n_decodes):
    """the last decode's kernels in launch order (name, grid, us): maps times to layers"""
    import sqlite3

    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    per = len(rows) // n_decodes
    for r in rows[-per:]:
        print(f"{(r[2] - r[1]) / 1e3:9.2f} us  {r[0].split('(')[0].replace('void ', '')[:44]:44s} grid=({r[3] // r[6]},{r[4]},{r[5]})")


def summarise(db):
    import sqlite3
    from collections import defaultdict

    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        if "conv_gemm" not in r[0] and "resunit" not in r[0]:
            continue
        k = (r[0].split("(")[0].replace("void ", "")[:40], r[3] // r[6], r[4], r[5])
        agg[k][0] += 1
        agg[k][1] += (r[2] - r[1]) / 1e3
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{us:10.1f} us  n={n:4d}  avg {us / n:8.2f} us  {k[0]} grid=({k[1]},{k[2]},{k[3]})")


if __name__ == "__main__":
    if len(sys.argv) > 2:
        sequence(sys.argv[1], int(sys.argv[2]))
    elif len(sys.argv) > 1:
        summarise(sys.argv[1])
    else:
        run()
