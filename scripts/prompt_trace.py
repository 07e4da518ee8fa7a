"""Per-shape kernel times of the 64-token prompt pass under rocprofv3 --kernel-trace: every kernel
of scripts/prefill64_trace.py (four prefills) grouped by (name, grid), average us and the launch
count, with the weight bytes per launch for the prompt linears (grid -> N, K of S2-Pro).

    python scripts/prompt_trace.py OUT [fm_tune k=v ...]    # runs rocprofv3, writes OUT.md
"""
import glob
import os
import shutil
import subprocess
import sys
import tempfile
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main(out, knobs):
    from rocprof_summary import load_dispatches

    d = tempfile.mkdtemp(prefix="ptrace_", dir="/tmp")
    env = dict(os.environ, FISHMI_TUNE=",".join(knobs)) if knobs else dict(os.environ)
    cmd = ["timeout", "-s", "KILL", "240", shutil.which("rocprofv3"), "--kernel-trace", "--output-format", "csv",
           "-d", d, "-o", "t", "--", sys.executable, os.path.join(ROOT, "scripts", "prefill64_trace.py")]
    r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    csvs = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not csvs:
        raise SystemExit(f"rocprofv3 failed rc {r.returncode}: {r.stderr[-400:].decode(errors='replace')}")
    disp = load_dispatches(csvs[0])
    shutil.rmtree(d, ignore_errors=True)
    agg = defaultdict(lambda: [0, 0])
    for name, ns, grid in disp:
        if any(k in name for k in ("synth_kernel", "pack_kernel", "rocclr")):
            continue
        key = (name.replace("(anonymous namespace)::", "").split("(")[0][:60], grid)
        agg[key][0] += 1
        agg[key][1] += ns
    lines = [f"# 64-token prompt pass, per (kernel, grid) (scripts/prompt_trace.py{' ' + ' '.join(knobs) if knobs else ''})",
             "", "| kernel | grid | launches | avg us | total ms |", "|---|---|---:|---:|---:|"]
    for (name, grid), (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        lines.append(f"| `{name}` | {grid} | {n} | {ns / n / 1e3:.2f} | {ns / 1e6:.2f} |")
    open(out + ".md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
