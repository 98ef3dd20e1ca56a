"""voxnav -- MI355X-native batched voxel-grid exploration env.

The data-parallel hot path of Noimps/3D-Navigation-Reinforcement-Learning
(envs/CubicEnv.py step/reset batched as train/Grid_Train.py batches it),
rebuilt as hand-written HIP kernels for gfx950 behind the C-ABI in
include/voxnav.h.  Public API:

  rooms.*             room-file parser / room sets / synthetic boxes
  BatchedGridEnv      N agents per GPU, torch tensors in/out, SB3 auto-reset
  VoxnavVecEnv        SB3's VecEnv contract (SubprocVecEnv + Monitor) over BatchedGridEnv
  GridAgent           the reference's single-env gymnasium API (CubicEnv)
  SimpleGridAgent     the same for the goal-seeking simpleEnv variant
  RolloutCollector    on-device PPO rollout collection (policy in the loop)
  compute_gae         GAE advantage/return scan kernel
  PPOLearner          (Recurrent)PPO.train on the collector's device buffers (+ DDP)
  evaluate_policy     evaluate_grid.py's deterministic-episode metrics, batched
  save_checkpoint / load_checkpoint   SB3 .zip layout, Grid_Train naming
  sharding            multi-GPU agent sharding helpers
"""
from . import rooms  # noqa: F401
from ._native import VoxnavError, load as load_library  # noqa: F401

__all__ = ["rooms", "BatchedGridEnv", "VoxnavVecEnv", "GridAgent", "SimpleGridAgent", "RolloutCollector", "compute_gae",
           "PPOLearner", "evaluate_policy", "save_checkpoint", "load_checkpoint", "VoxnavError", "load_library"]


def __getattr__(name):
    # torch-dependent pieces are imported lazily
    if name == "BatchedGridEnv":
        from .env import BatchedGridEnv
        return BatchedGridEnv
    if name == "VoxnavVecEnv":
        from .vec_env import VoxnavVecEnv
        return VoxnavVecEnv
    if name == "GridAgent":
        from .gym_api import GridAgent
        return GridAgent
    if name == "SimpleGridAgent":
        from .gym_api import SimpleGridAgent
        return SimpleGridAgent
    if name == "RolloutCollector":
        from .collector import RolloutCollector
        return RolloutCollector
    if name == "compute_gae":
        from .gae import compute_gae
        return compute_gae
    if name == "PPOLearner":
        from .ppo import PPOLearner
        return PPOLearner
    if name == "evaluate_policy":
        from .evaluate import evaluate_policy
        return evaluate_policy
    if name in ("save_checkpoint", "load_checkpoint"):
        from . import checkpoint
        return getattr(checkpoint, name)
    raise AttributeError(name)
