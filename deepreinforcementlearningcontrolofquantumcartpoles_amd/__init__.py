"""MI355X-native quantum-cartpole environment (env.step() hot path in HIP for gfx950).

Modules:
  _lib        ctypes binding of libqcart.so (include/qcart.h)
  config      physics presets of the four reference systems
  core        Stepper: one libqcart handle + device tensors
  simulation  drop-in surface of the reference `simulation` extension (B = 1)
  env         BatchedEnv: reset/step/observation semantics of the reference drivers, batched
  distributed env sharding over ranks + RCCL gather of episode returns
"""
from .config import DEFAULTS, HO, IHO, IQO, QO, Physics  # noqa: F401

__all__ = ["DEFAULTS", "HO", "IHO", "QO", "IQO", "Physics"]
