"""Config 3's batched (B=32) decode kernels under rocprofv3: per bsacc_kernel
instantiation (each is one linear shape at S2-Pro widths) the average duration from a
--kernel-trace pass, its algorithmic bytes, the fraction of 8 TB/s, and the HBM traffic per launch
from separate --pmc FETCH_SIZE / WRITE_SIZE passes (FETCH_SIZE doubled: gfx950 wide-read correction,
MI355X_MICROARCH.md HBM section).

    python scripts/b32_profile.py run      # the workload (rocprofv3 runs it; eager frames)
    python scripts/b32_profile.py all OUT  # the three rocprofv3 passes + summary -> OUT.md / OUT.json
"""
import glob
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

B, T, FRAMES = 32, 128, 6
DIM, INTER, NQ, NQKV = 2560, 9728, 4096, 6144  # S2-Pro slow and fast stacks (same widths)
# bsacc_kernel<T, SPW, TPI, NTM, EPI, PRO> -> (matrix, N, K); EPI 4 = K-part slabs, 7 = SwiGLU8, 3 = F32
SHAPES = {"5, 2, 3, 4": ("wqkv (K-part slabs)", NQKV, DIM), "2, 4, 5, 4": ("wo (K-part slabs)", DIM, NQ),
          "10, 1, 5, 7": ("w1 || w3 (SwiGLU)", 2 * INTER, DIM), "5, 2, 5, 4": ("w2 (K-part slabs)", DIM, INTER)}


def run():
    sys.path.insert(0, os.path.join(ROOT, "fish-speech_amd"))
    import numpy as np

    from fishmi.config import S2_PRO_CONFIG, S2_PRO_IM_END_ID, DualARConfig
    from fishmi.llm import DualARModel

    cfg = DualARConfig._from_fish_qwen3_omni(S2_PRO_CONFIG)
    cfg.im_end_id = S2_PRO_IM_END_ID
    cfg.max_seq_len = 1024
    m = DualARModel.synthetic(cfg, seed=0, log2_half=5, device=0, precision="bf16", max_slots=B)
    m.use_graph(False)
    rng = np.random.default_rng(1)
    sp = DualARModel.sampling(temperature=0.7, top_p=0.9, top_k=30, seed=0, mask_im_end=True)
    for b in range(B):
        p = np.zeros((cfg.num_codebooks + 1, T), np.int32)
        p[0] = rng.integers(16, cfg.semantic_begin_id, T)
        m.prefill(b, p, sp)
    for _ in range(FRAMES):
        m.decode(list(range(B)))
    print("done")


def shape_of(name):
    mm = re.match(r"void \(anonymous namespace\)::bsacc_kernel<unsigned short, (\d+, \d+, \d+, \d+), 0>", name)
    return SHAPES.get(mm.group(1)) if mm else None


def passes(out):
    from rocprof_summary import load_dispatches, load_pmc

    res = {}
    for tag, extra in (("trace", ["--kernel-trace"]), ("fetch", ["--pmc", "FETCH_SIZE"]), ("write", ["--pmc", "WRITE_SIZE"])):
        d = tempfile.mkdtemp(prefix=f"b32_{tag}_", dir="/tmp")
        cmd = ["timeout", "-s", "KILL", "240", shutil.which("rocprofv3"), *extra, "--output-format", "csv", "-d", d,
               "-o", tag, "--", sys.executable, os.path.abspath(__file__), "run"]
        r = subprocess.run(cmd, cwd="/tmp", stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        csvs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv" if tag == "trace" else "*counter_collection.csv"),
                         recursive=True)
        if r.returncode != 0 or not csvs:
            raise SystemExit(f"rocprofv3 {tag} failed rc {r.returncode}: {r.stderr[-400:].decode(errors='replace')}")
        res[tag] = load_dispatches(csvs[0]) if tag == "trace" else load_pmc(csvs[0], "FETCH_SIZE" if tag == "fetch"
                                                                             else "WRITE_SIZE")
        shutil.rmtree(d, ignore_errors=True)
    rows = defaultdict(lambda: {"n": 0, "ns": 0})
    other = defaultdict(lambda: {"n": 0, "ns": 0})
    for name, ns, _ in res["trace"]:
        sh = shape_of(name)
        tgt = rows[sh] if sh else other[name.split("(")[0][:70]]
        tgt["n"] += 1
        tgt["ns"] += ns
    summary = {}
    lines = ["# B=32 decode (config 3) under rocprofv3: bsacc_kernel per linear shape", "",
             f"{FRAMES} eager batched frames of {B} slots at positions {T}..{T + FRAMES} (scripts/b32_profile.py); "
             "algorithmic bytes = N x K x 2 (weights) + R x K x 2 (X) + outputs (fp32 K-part slabs or bf16); "
             "traffic = FETCH_SIZE x 1024 x 2 (gfx950 wide-read correction) + WRITE_SIZE x 1024, separate passes", "",
             "| matrix | launches | avg us | algorithmic MB | TB/s | frac of 8 TB/s | HBM traffic MB | traffic / alg |",
             "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for sh, v in sorted(rows.items(), key=lambda kv: -kv[1]["ns"]):
        label, N, K = sh
        kp = 8 if "slabs" in label and K > 3000 else (2 if "wqkv" in label else 1)
        out_b = B * N * 4 * kp if "slabs" in label else B * (N // 2 if "SwiGLU" in label else N) * 2
        alg = N * K * 2 + B * K * 2 + out_b
        avg_us = v["ns"] / v["n"] / 1e3
        key = [n for n in res["fetch"] if shape_of(n) == sh]
        fv = [x for n in key for x in res["fetch"][n]]
        wv = [x for n in [n for n in res["write"] if shape_of(n) == sh] for x in res["write"][n]]
        traffic = (2 * 1024 * sum(fv) / len(fv) if fv else 0) + (1024 * sum(wv) / len(wv) if wv else 0)
        tbs = alg / avg_us / 1e6
        summary[label] = {"launches": v["n"], "avg_us": round(avg_us, 3), "alg_bytes": alg, "tb_s": round(tbs, 3),
                          "frac": round(tbs / 8, 4), "traffic_bytes": round(traffic), "traffic_ratio": round(traffic / alg, 3)}
        lines.append(f"| {label} | {v['n']} | {avg_us:.2f} | {alg / 1e6:.1f} | {tbs:.2f} | {tbs / 8:.3f} | "
                     f"{traffic / 1e6:.1f} | {traffic / alg:.3f} |")
    lines += ["", "Other kernels of the same frames:", "", "| kernel | launches | avg us |", "|---|---:|---:|"]
    for name, v in sorted(other.items(), key=lambda kv: -kv[1]["ns"])[:12]:
        lines.append(f"| `{name}` | {v['n']} | {v['ns'] / v['n'] / 1e3:.2f} |")
    with open(out + ".md", "w") as fh:
        fh.write("\n".join(lines) + "\n")
    with open(out + ".json", "w") as fh:
        json.dump(summary, fh, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        passes(sys.argv[2])
