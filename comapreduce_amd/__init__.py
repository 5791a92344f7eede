"""comapreduce_amd -- MI355X-native COMAP Level-1 -> Level-2 reduction and destriper.

The hot path runs in hand-written HIP kernels for gfx950 behind a
C ABI (``include/comap_hip.h``, ``comapreduce_amd/csrc``), loaded with ctypes by
``comapreduce_amd._native``.  The Python layers mirror the reference plugin API
(``PipelineFunction`` stages, ``Runner``, ``run_destriper``).
"""
__version__ = '0.1.0'
