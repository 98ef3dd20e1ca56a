"""Checkpoints in the SB3 ``.zip`` layout and the reference's naming
(SURVEY.md 8(f) row 3).

train/Grid_Train.py saves ``model.save(path)`` every training segment under
``{SAVE_DIR}/rppo_hp{i}_arch_{arch_str}_lstm_{lstm_str}_s{steps}_view{L}.zip``
(:229-233) and Train_Further.py / evaluate_grid.py reload them.  An SB3 zip
holds ``policy.pth`` (the policy ``state_dict``), ``policy.optimizer.pth``,
``pytorch_variables.pth``, a ``data`` JSON with the constructor arguments
and counters, and ``_stable_baselines3_version``.

``save_checkpoint`` writes those members; the policy ``state_dict`` keys
are SB3's own (``lstm_actor.weight_ih_l0``, ``mlp_extractor.policy_net.0
.weight``, ``action_net.weight`` ...), so ``policy.pth`` moves between this
package and an SB3 ``RecurrentPPO`` in both directions.  ``data`` here is
plain JSON (SB3 stores cloudpickled objects there); ``load_checkpoint``
reads only JSON and ``torch.load(..., weights_only=True)`` -- nothing in a
checkpoint is executed.
"""
from __future__ import annotations

import io
import json
import zipfile
from pathlib import Path
from typing import Dict, Optional, Tuple, Union

import torch

from .policy import ActorCriticPolicy, RecurrentActorCriticPolicy

FORMAT_VERSION = "voxnav-sb3-layout-1"


def arch_str(net_arch: Dict[str, list]) -> str:
    """Grid_Train.py:154: ``pi[256, 256, 128]_vf[256, 256, 128]``."""
    return f"pi{list(net_arch['pi'])}_vf{list(net_arch['vf'])}"


def lstm_str(lstm_hidden_size: int, n_lstm_layers: int = 1, shared_lstm: bool = True) -> str:
    """Grid_Train.py:158-159 (the script labels the default as "shared")."""
    return f"h{lstm_hidden_size}l{n_lstm_layers}_{'shared' if shared_lstm else 'separate'}"


def checkpoint_name(hp_index: int, net_arch: Dict[str, list], lstm_hidden_size: int, steps: int, view: int,
                    n_lstm_layers: int = 1, shared_lstm: bool = True) -> str:
    """Grid_Train.py:232 (``hp_index`` is the 0-based ``hp_i``)."""
    return (f"rppo_hp{hp_index + 1}_arch_{arch_str(net_arch)}_lstm_"
            f"{lstm_str(lstm_hidden_size, n_lstm_layers, shared_lstm)}_s{steps}_view{view}.zip")


def eval_phase_for_steps(trained_steps: int) -> str:
    """evaluate_grid.py:146-151: which evaluation room set a checkpoint uses."""
    if trained_steps <= 1_000_000:
        return "P1_empty"
    if trained_steps <= 21_000_000:
        return "P2_small"
    return "P3_large"


def _policy_kwargs(policy) -> Dict[str, object]:
    ext = policy.mlp_extractor
    arch = dict(pi=[m.out_features for m in ext.linears("pi")], vf=[m.out_features for m in ext.linears("vf")])
    kw = dict(net_arch=arch, obs_dim=int(policy.obs_dim), n_actions=int(policy.n_actions))
    if policy.recurrent:
        kw.update(lstm_hidden_size=int(policy.lstm_hidden_size), n_lstm_layers=1)
    return kw


def save_checkpoint(path: Union[str, Path], policy, optimizer: Optional[torch.optim.Optimizer] = None,
                    num_timesteps: int = 0, hyperparams: Optional[Dict[str, object]] = None) -> Path:
    path = Path(path)
    if path.suffix != ".zip":
        path = path.with_suffix(".zip")
    path.parent.mkdir(parents=True, exist_ok=True)
    data = dict(policy_class="MlpLstmPolicy" if policy.recurrent else "MlpPolicy",
                algorithm="RecurrentPPO" if policy.recurrent else "PPO",
                policy_kwargs=_policy_kwargs(policy), num_timesteps=int(num_timesteps),
                hyperparams=dict(hyperparams or {}), format=FORMAT_VERSION)

    def blob(obj) -> bytes:
        b = io.BytesIO()
        torch.save(obj, b)
        return b.getvalue()

    sd = {k: v.detach().cpu() for k, v in policy.state_dict().items()}
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as z:
        z.writestr("data", json.dumps(data, indent=2))
        z.writestr("policy.pth", blob(sd))
        if optimizer is not None:
            z.writestr("policy.optimizer.pth", blob(optimizer.state_dict()))
        z.writestr("pytorch_variables.pth", blob({}))
        z.writestr("_stable_baselines3_version", FORMAT_VERSION)
    return path


def load_checkpoint(path: Union[str, Path], device="cpu") -> Tuple[torch.nn.Module, Dict[str, object]]:
    """-> (policy on ``device``, data dict).  The optimizer state is restored
    separately (``load_optimizer_state``) into an optimizer built over the
    returned policy's parameters."""
    with zipfile.ZipFile(path) as z:
        data = json.loads(z.read("data"))
        sd = torch.load(io.BytesIO(z.read("policy.pth")), map_location="cpu", weights_only=True)
    kw = dict(data["policy_kwargs"])
    kw.pop("n_lstm_layers", None)
    cls = RecurrentActorCriticPolicy if data.get("policy_class") == "MlpLstmPolicy" else ActorCriticPolicy
    pol = cls(ortho_init=False, **kw)
    pol.load_state_dict(sd, strict=True)
    return pol.to(device), data


def load_optimizer_state(path: Union[str, Path], optimizer: torch.optim.Optimizer) -> bool:
    """Restore ``policy.optimizer.pth`` into ``optimizer`` (False if absent)."""
    with zipfile.ZipFile(path) as z:
        if "policy.optimizer.pth" not in z.namelist():
            return False
        st = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), map_location="cpu", weights_only=True)
    optimizer.load_state_dict(st)
    return True
