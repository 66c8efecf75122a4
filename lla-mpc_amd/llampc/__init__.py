"""llampc — MI355X-native (gfx950) drop-in for LLA-MPC's model-bank hot path.

Mirrors the reference's public API for that path (tianhao-stan-wu/LLA-MPC):
``llampc.models.Dynamic`` (batched Pacejka dynamics), ``llampc.mpc.evaluate_models_
vectorized`` (look-back scoring), the new fused tick ``llampc.mpc.plan`` and the
``llampc.mpc.ModelBank`` device handle, backed by hand-written HIP kernels in
``libllampc_hip.so`` (C ABI: include/llampc.h).  There is no CPU fallback.
"""
import os as _os

# Kernel arguments in device memory: the tick's blocks read their launch descriptors (and
# through them the inputs) with scalar loads first, and with kernargs in host memory every
# tick measured 5 us longer (31.3-32.3 vs 26.1-26.9 us).  Device kernargs are
# this ROCm's default; HIP_FORCE_DEV_KERNARG changes kernarg placement for EVERY HIP user of
# the process (torch included), so importing llampc only sets it when asked to
# (LLAMPC_SET_DEV_KERNARG=1, before the first HIP call; an explicit setting is kept).  bench.py
# and the tests set it themselves (INTEGRATION.md "Process environment").
if _os.environ.get("LLAMPC_SET_DEV_KERNARG") == "1":
    _os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

__version__ = "0.1.0"
