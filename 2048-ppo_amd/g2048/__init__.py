"""g2048: MI355X-native vectorised 2048 env + PPO hot path (HIP kernels behind a C ABI, PyTorch-ROCm host).

Public modules:
  g2048._lib        ctypes binding of libg2048.so (include/g2048.h)
  g2048.env         VecEnv: N boards in HBM, one kernel launch per step
  g2048.rollout     policy-driven rollouts into time-major device buffers
  g2048.advantage   reward / return-to-go / advantage scan + RTG moment tracking
  g2048.ppo         PPO-clip update (Muon + AdamW), optional RCCL gradient all-reduce
"""

__version__ = "0.1.0"
