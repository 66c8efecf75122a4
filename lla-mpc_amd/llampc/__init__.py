"""llampc — MI355X-native (gfx950) drop-in for LLA-MPC's model-bank hot path.

Mirrors the reference's public API for that path (tianhao-stan-wu/LLA-MPC):
``llampc.models.Dynamic`` (batched Pacejka dynamics), ``llampc.mpc.evaluate_models_
vectorized`` (look-back scoring), the new fused tick ``llampc.mpc.plan`` and the
``llampc.mpc.ModelBank`` device handle, backed by hand-written HIP kernels in
``libllampc_hip.so`` (C ABI: include/llampc.h).  There is no CPU fallback.
"""
__version__ = "0.1.0"
