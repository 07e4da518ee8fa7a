"""Codec decode for rocprofv3 --pmc passes (MFMA utilisation from the hardware counters, VERDICT r5
next #5): one config-2 codec decode of [1, 10, 216] codes (modded_dac.py:712-801 decoder behind the
RVQ decode and the window transformer; synthetic weights, bf16), after one warm-up decode.  The
last decode's dispatches are the measured ones (the warm-up's are the first half of the trace).

    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_VALU \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d DIR -o pmc -- python3 scripts/codec_pmc_probe.py
    python3 scripts/codec_pmc_probe.py --summary <counter_collection.csv or results.db>
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES",
            "GRBM_GUI_ACTIVE")
SIMDS = 256 * 4   # MI355X: 256 CUs x 4 SIMDs (MfmaUtil's SIMD_NUM, counter_defs.yaml)
XCDS = 8          # GRBM_GUI_ACTIVE is reported summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS note)
FRAMES = 216


def run():
    import numpy as np

    from fishmi.codec import FishMICodec
    from fishmi.config import CodecConfig

    ccfg = CodecConfig()
    codec = FishMICodec.synthetic(ccfg, 1, 0, "bf16", max_frames=FRAMES)
    codes = np.random.default_rng(0).integers(0, 1024, (ccfg.n_codebooks + 1, FRAMES)).astype(np.int32)
    codec.decode_codes(codes)
    ms0, _, f0 = codec.profile()
    codec.decode_codes(codes)
    ms1, _, f1 = codec.profile()
    print(f"codec decode: {ms1 - ms0:.3f} ms, {(f1 - f0) / 1e9:.1f} GFLOP (analytic, implicit-GEMM convs / linears)")


def family(name):
    for k in ("resunit_kernel", "conv_gemm2_kernel", "conv_gemm_kernel", "conv_splitk_epi_kernel", "window_attn",
              "dwconv_ln"):
        if k in name:
            return k
    return "other"


def load(path):
    """{dispatch id: (kernel name, {counter: value})} from a rocprofv3 --pmc run."""
    import csv
    import sqlite3
    from collections import defaultdict

    out = defaultdict(lambda: [None, {}])
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        cols = [d[1] for d in c.execute("pragma table_info(pmc_events)")]
        key = "dispatch_id" if "dispatch_id" in cols else ("event_id" if "event_id" in cols else cols[0])
        for d, n, cn, v in c.execute(f"select {key}, name, counter_name, counter_value from pmc_events"):
            out[d][0] = n
            out[d][1][cn] = out[d][1].get(cn, 0.0) + float(v)
    else:
        with open(path) as fh:
            for r in csv.DictReader(fh):
                d = r.get("Dispatch_Id") or r.get("Correlation_Id")
                out[d][0] = r["Kernel_Name"]
                out[d][1][r["Counter_Name"]] = out[d][1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def summarise(path, peak_tflops=2500.0):
    """Per kernel family over the measured (second) decode: MfmaUtil = sum MFMA busy cycles /
    (elapsed cycles x SIMDs), the bf16 MFMA work the counters saw (MOPS x 512 flops), VALU busy
    share, and the effective clock (GRBM_GUI_ACTIVE / 8 / kernel time is not available here: the
    elapsed cycles are GRBM_GUI_ACTIVE / 8).  Returns a dict (bench.py codec_roofline.mfma_busy)."""
    from collections import defaultdict

    disp = load(path)
    ids = sorted(disp, key=lambda x: int(x))
    names = [disp[d][0] for d in ids]
    # the probe's two identical decodes end the trace: the longest tail that repeats once is one
    # decode's dispatch sequence; the measured one is the second
    L = next((n for n in range(len(names) // 2, 0, -1) if names[-n:] == names[-2 * n:-n]), 0)
    if L == 0:
        raise SystemExit("no repeated decode sequence at the end of the trace")
    ids = ids[-L:]
    agg = defaultdict(lambda: defaultdict(float))
    for d in ids:
        name, cv = disp[d]
        for fam in (family(name), "all"):
            a = agg[fam]
            a["launches"] += 1
            for k, v in cv.items():
                a[k] += v
    out = {}
    for fam, a in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        cyc = a.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        if cyc <= 0:
            continue
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        mops = a.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) * 512.0
        out[fam] = {
            "launches": int(a["launches"]),
            "elapsed_Mcycles": round(cyc / 1e6, 4),
            "mfma_busy": round(busy / (cyc * SIMDS), 4),
            "bf16_mfma_gflop": round(mops / 1e9, 3),
            "mfma_flop_per_busy_cycle_per_simd": round(mops / busy, 1) if busy else None,
            # SQ_ACTIVE_INST_VALU counts quad-cycles per wave; / (elapsed x SIMDs) -> VALU issue share
            "valu_active": round(4.0 * a.get("SQ_ACTIVE_INST_VALU", 0.0) / (cyc * SIMDS), 4),
        }
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        import json

        print(json.dumps(summarise(sys.argv[2]), indent=1))
    else:
        run()
