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
.weight``, ``action_net.weight`` ...).  ``data`` here is plain JSON (SB3
stores cloudpickled objects there); ``load_checkpoint`` reads only JSON and
``torch.load(..., weights_only=True)`` -- nothing in a checkpoint is
executed.

Interop is one-way at the zip level: ``load_checkpoint`` reads the
reference's SB3 zips (policy.pth only, architecture from the tensor
shapes), but SB3's ``RecurrentPPO.load`` (Train_Further.py:145,
evaluate_grid.py:165) cannot read these zips' JSON ``data``; an SB3 model
takes this package's weights with
``model.policy.load_state_dict(torch.load(policy_pth, weights_only=True))``.
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
            osd = optimizer.state_dict()
            # the learner's fused-kernel flag is an execution choice of this build,
            # not part of sb3's Adam: saved as torch's default
            osd["param_groups"] = [{**g, "fused": None} if "fused" in g else g for g in osd["param_groups"]]
            z.writestr("policy.optimizer.pth", blob(osd))
        z.writestr("pytorch_variables.pth", blob({}))
        z.writestr("_stable_baselines3_version", FORMAT_VERSION)
    return path


# Keys an SB3 policy state_dict may hold that this package's modules do not:
# none carry parameters for MlpLstmPolicy / MlpPolicy (Flatten feature
# extractors), so this allow-list only guards against future SB3 versions
# registering buffers under these prefixes.  Anything else missing or
# unexpected is an error (strict load), never silently random weights.
SB3_IGNORED_PREFIXES = ("features_extractor.", "pi_features_extractor.", "vf_features_extractor.")


def load_policy_state(policy: torch.nn.Module, state_dict: Dict[str, torch.Tensor]) -> None:
    """``policy.load_state_dict`` for an SB3 (or voxnav) ``policy.pth``:
    strict over every parameter, after dropping only the allow-listed
    parameterless SB3 extractor keys."""
    sd = {k: v for k, v in state_dict.items() if not k.startswith(SB3_IGNORED_PREFIXES)}
    policy.load_state_dict(sd, strict=True)


def policy_from_state_dict(state_dict: Dict[str, torch.Tensor]) -> torch.nn.Module:
    """Build the policy a ``policy.pth`` describes from its tensor shapes
    alone (an SB3 zip's ``data`` member is cloudpickled and never read):
    LSTM hidden size from ``lstm_actor.weight_hh_l0``, MLP widths from
    ``mlp_extractor.{policy,value}_net.<i>.weight``, obs / action dims from
    the first layer and ``action_net``."""
    sd = state_dict

    def widths(branch):
        ks = sorted((int(k.split(".")[2]), k) for k in sd if k.startswith(f"mlp_extractor.{branch}.")
                    and k.endswith(".weight"))
        return [int(sd[k].shape[0]) for _, k in ks]

    arch = dict(pi=widths("policy_net"), vf=widths("value_net"))
    n_actions = int(sd["action_net.weight"].shape[0])
    if "lstm_actor.weight_ih_l0" in sd:
        H = int(sd["lstm_actor.weight_hh_l0"].shape[1])
        obs_dim = int(sd["lstm_actor.weight_ih_l0"].shape[1])
        pol = RecurrentActorCriticPolicy(obs_dim=obs_dim, n_actions=n_actions, lstm_hidden_size=H, net_arch=arch,
                                         ortho_init=False)
    else:
        first = sd["mlp_extractor.policy_net.0.weight"]
        pol = ActorCriticPolicy(obs_dim=int(first.shape[1]), n_actions=n_actions, net_arch=arch, ortho_init=False)
    load_policy_state(pol, sd)
    return pol


def load_checkpoint(path: Union[str, Path], device="cpu") -> Tuple[torch.nn.Module, Dict[str, object]]:
    """-> (policy on ``device``, data dict).

    Reads this package's zips (JSON ``data``) and SB3 / sb3_contrib zips
    (``model.save`` of the reference, train/Grid_Train.py:233): for those
    only ``policy.pth`` is loaded (``weights_only``) and the architecture is
    inferred from its shapes; ``data`` is returned as ``{"sb3": True}``
    without decoding SB3's cloudpickled fields.  The optimizer state is
    restored separately (``load_optimizer_state``) into an optimizer built
    over the returned policy's parameters."""
    with zipfile.ZipFile(path) as z:
        raw = z.read("data")
        sd = torch.load(io.BytesIO(z.read("policy.pth")), map_location="cpu", weights_only=True)
        ver = z.read("_stable_baselines3_version").decode(errors="replace").strip() \
            if "_stable_baselines3_version" in z.namelist() else ""
    try:
        data = json.loads(raw)
    except ValueError:
        data = None
    fmt = data.get("format") if isinstance(data, dict) else None
    ours = fmt is not None or ver.startswith("voxnav")
    if ours and fmt != FORMAT_VERSION:
        raise ValueError(f"{path}: voxnav checkpoint format {fmt or ver!r}, this build reads {FORMAT_VERSION!r}")
    if not ours:
        # an SB3 / sb3_contrib zip: JSON data with ``:serialized:`` (cloudpickled) fields and an SB3 version
        if not (isinstance(data, dict) and any(isinstance(v, dict) and ":serialized:" in v for v in data.values())) \
                and not ver:
            raise ValueError(f"{path}: neither a voxnav nor an SB3 checkpoint")
        return policy_from_state_dict(sd).to(device), {"sb3": True, "sb3_version": ver or None}
    kw = dict(data["policy_kwargs"])
    kw.pop("n_lstm_layers", None)
    cls = RecurrentActorCriticPolicy if data.get("policy_class") == "MlpLstmPolicy" else ActorCriticPolicy
    pol = cls(ortho_init=False, **kw)
    load_policy_state(pol, sd)
    return pol.to(device), data


def load_optimizer_state(path: Union[str, Path], optimizer: torch.optim.Optimizer) -> bool:
    """Restore ``policy.optimizer.pth`` into ``optimizer`` (False if absent).

    The file's hyperparameters and moments are loaded; the execution flags of
    the target groups (``fused`` / ``foreach`` / ``capturable``: how this
    build runs the step, saved as torch's defaults) are kept, and the
    per-parameter ``step`` counters are moved next to their parameters as
    f32 scalars -- what the learner's fused step (``PPOLearner._clip_step``,
    ``learn_ops.adam_step``) expects, so a resumed run stays on it."""
    with zipfile.ZipFile(path) as z:
        if "policy.optimizer.pth" not in z.namelist():
            return False
        st = torch.load(io.BytesIO(z.read("policy.optimizer.pth")), map_location="cpu", weights_only=True)
    flags = [{k: g[k] for k in ("fused", "foreach", "capturable") if k in g} for g in optimizer.param_groups]
    optimizer.load_state_dict(st)
    for g, f in zip(optimizer.param_groups, flags):
        g.update(f)
        if not g.get("fused"):
            continue
        for prm in g["params"]:
            s = optimizer.state.get(prm)
            if s and "step" in s and torch.is_tensor(s["step"]):
                s["step"] = s["step"].to(device=prm.device, dtype=torch.float32)
    return True
