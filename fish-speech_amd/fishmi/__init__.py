"""fishmi -- MI355X-native Fish-Speech S2-Pro hot path (Dual-AR decode + modded-DAC decode).

Host-side mirror of the reference seams; compute lives in libfishmi.so (include/fishmi.h).
"""
__version__ = "0.1.0"
