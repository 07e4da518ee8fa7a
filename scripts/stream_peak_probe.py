import sys; sys.path.insert(0, 'fish-speech_amd')
from fishmi import native
for _ in range(2):
    print(native.stream_peak(0, 2 << 30, 10))
