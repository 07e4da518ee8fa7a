import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "fish-speech_amd"))
mode = sys.argv[1]
if mode == "torch_first":
    import torch
from fishmi import native
L = native.lib()
print("fm_device_count", L.fm_device_count())
import torch
print("torch avail", torch.cuda.is_available(), torch.cuda.device_count())
torch.cuda.set_device(0)
x = torch.ones(4, device="cuda")
print("ok", float(x.sum()))
for l in open("/proc/self/maps"):
    if "amdhip64" in l and "r-xp" in l:
        print(l.split()[-1])
