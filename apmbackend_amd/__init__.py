"""apmbackend_amd -- an MI355X-native streaming APM engine.

tail -> parse -> join -> stats -> z-score -> alert -> DB, with the hot stages as hand-written
HIP kernels for gfx950 (csrc/kernels), a C++ host runtime (csrc/runtime) and RCCL over xGMI
for the multi-GPU fleet exchange.  Capabilities follow ztaylor797/APMBackend; see SURVEY.md.
"""
__version__ = "0.1.0"
