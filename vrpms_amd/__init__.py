"""vrpms_amd -- MI355X-native solver core for the vrpms TSP/VRP service.

Layout:
  csrc/       hand-written gfx950 HIP kernels + the C-ABI (include/vrpms.h)
  _lib.py     ctypes binding of libvrpms.so (no CPU fallback)
  core.py     device context: instance upload, scoring, decode, argmin
  synth.py    seeded synthetic instances for the BASELINE.json configs
  build.py    in-tree hipcc build for gfx950
"""
__version__ = "0.1.0"
