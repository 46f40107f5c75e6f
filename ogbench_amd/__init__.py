"""ogbench_amd -- MI355X-native batched OGBench envs and offline replay.

Drop-in for the hot path of hliuson/ogbench:
  * ``make(env_id, num_envs=N, device=...)``  ~ ``gymnasium.make(env_id)`` for the
    locomaze (pointmaze) and powderworld registries, batched on one GPU;
  * ``make_env_and_datasets``/``load_dataset`` ~ ogbench/utils.py, returning
    HBM-resident dataset dicts of torch tensors;
  * ``datasets.GCDataset``/``HGCDataset`` ~ impls/utils/datasets.py, sampling with
    a fused HIP gather + hindsight-relabel kernel.
All compute runs in libogbx.so (HIP, gfx950); there is no CPU fallback.
"""

from .locomaze import MazeEnv, parse_env_id
from .powderworld import PowderworldEnv
from .registry import make, registered_env_ids
from .utils import load_dataset, make_env_and_datasets

__all__ = ['MazeEnv', 'PowderworldEnv', 'load_dataset', 'make', 'make_env_and_datasets', 'parse_env_id',
           'registered_env_ids']
