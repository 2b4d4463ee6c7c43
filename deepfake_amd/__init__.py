"""deepfake_amd — MI355X-native (gfx950) hot path of Polarisjame/DeepFake.

Hand-written HIP kernels behind a C ABI (include/dfk.h, libdfk.so), the
reference's nn.Module surface (deepfake_amd.models), and a one-process-per-GPU
RCCL data-parallel trainer (deepfake_amd.trainer).
"""
__version__ = "0.1.0"
