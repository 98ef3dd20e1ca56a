"""Actor-critic policies of the rollout collector (the reference's SB3 policies).

``RecurrentActorCriticPolicy`` has the shape sb3_contrib's ``MlpLstmPolicy``
takes in train/Grid_Train.py (third-party; ``RecurrentPPO(policy=
"MlpLstmPolicy", policy_kwargs=dict(net_arch=dict(pi=[256, 256, 128],
vf=[256, 256, 128]), lstm_hidden_size=256, n_lstm_layers=1))`` at
train/Grid_Train.py:68-80, :196-204): Flatten(80) -> separate actor and
critic LSTM(80 -> 256) -> Tanh MLPs 256-256-256-128 -> action_net(128 -> 6)
and value_net(128 -> 1).  Parameter names follow SB3's state_dict keys
(``lstm_actor.weight_ih_l0``, ``mlp_extractor.policy_net.0.weight``,
``action_net.weight`` ...) so an SB3 checkpoint's ``policy.pth`` loads with
``voxnav.checkpoint.load_policy_state`` (strict, with an explicit allow-list
of parameterless SB3-only keys).

``ActorCriticPolicy`` is the feed-forward ``MlpPolicy`` of BASELINE config
C3 (PPO-MLP, same pi/vf MLPs on the observation).

The modules only hold the parameters; the rollout path that uses them is
``voxnav.collector`` (library GEMMs + the HIP kernels of
csrc/voxnav_collect.hip).  ``forward_torch`` is the plain-PyTorch f32
statement of the same forward, used by the tests as the fp32 reference.
"""
from __future__ import annotations

import math
from functools import partial
from typing import Dict, List, Optional, Tuple

import torch
from torch import nn

OBS_DIM = 80
NUM_ACTIONS = 6
DEFAULT_NET_ARCH = dict(pi=[256, 256, 128], vf=[256, 256, 128])   # train/Grid_Train.py:72
DEFAULT_LSTM_HIDDEN = 256                                         # train/Grid_Train.py:78


def _mlp(in_dim: int, widths: List[int]) -> nn.Sequential:
    layers: List[nn.Module] = []
    d = in_dim
    for w in widths:
        layers += [nn.Linear(d, w), nn.Tanh()]
        d = w
    return nn.Sequential(*layers)


class MlpExtractor(nn.Module):
    """SB3 ``MlpExtractor`` with ``net_arch=dict(pi=[...], vf=[...])``, Tanh."""

    def __init__(self, feature_dim: int, net_arch: Dict[str, List[int]]):
        super().__init__()
        self.policy_net = _mlp(feature_dim, list(net_arch["pi"]))
        self.value_net = _mlp(feature_dim, list(net_arch["vf"]))
        self.latent_dim_pi = net_arch["pi"][-1] if net_arch["pi"] else feature_dim
        self.latent_dim_vf = net_arch["vf"][-1] if net_arch["vf"] else feature_dim

    def linears(self, branch: str) -> List[nn.Linear]:
        seq = self.policy_net if branch == "pi" else self.value_net
        return [m for m in seq if isinstance(m, nn.Linear)]


def _init_weights(module: nn.Module, gain: float):
    # SB3 BasePolicy.init_weights: orthogonal weights, zero bias (Linear only)
    if isinstance(module, nn.Linear):
        nn.init.orthogonal_(module.weight, gain=gain)
        if module.bias is not None:
            module.bias.data.fill_(0.0)


class _ActorCriticBase(nn.Module):
    recurrent = False

    def _ortho_init(self):
        # SB3 ActorCriticPolicy._build: gains sqrt(2) / 0.01 / 1; the LSTMs
        # keep PyTorch's default init (sb3_contrib leaves them out).
        for module, gain in ((self.mlp_extractor, math.sqrt(2)), (self.action_net, 0.01), (self.value_net, 1.0)):
            module.apply(partial(_init_weights, gain=gain))

    @property
    def n_actions(self) -> int:
        return self.action_net.out_features


class ActorCriticPolicy(_ActorCriticBase):
    """PPO ``MlpPolicy`` (feed-forward) on the 80-float observation."""

    def __init__(self, obs_dim: int = OBS_DIM, n_actions: int = NUM_ACTIONS, net_arch=None, ortho_init: bool = True):
        super().__init__()
        net_arch = net_arch or DEFAULT_NET_ARCH
        self.obs_dim = obs_dim
        self.mlp_extractor = MlpExtractor(obs_dim, net_arch)
        self.action_net = nn.Linear(self.mlp_extractor.latent_dim_pi, n_actions)
        self.value_net = nn.Linear(self.mlp_extractor.latent_dim_vf, 1)
        if ortho_init:
            self._ortho_init()

    @torch.no_grad()
    def forward_torch(self, obs: torch.Tensor):
        """(logits [N, A], values [N]) in plain PyTorch f32."""
        lp = self.mlp_extractor.policy_net(obs)
        lv = self.mlp_extractor.value_net(obs)
        return self.action_net(lp), self.value_net(lv).squeeze(-1)


class RecurrentActorCriticPolicy(_ActorCriticBase):
    """sb3_contrib ``MlpLstmPolicy`` with separate actor / critic LSTMs
    (``enable_critic_lstm=True``, ``shared_lstm=False``, one layer)."""

    recurrent = True

    def __init__(self, obs_dim: int = OBS_DIM, n_actions: int = NUM_ACTIONS, lstm_hidden_size: int = DEFAULT_LSTM_HIDDEN,
                 net_arch=None, ortho_init: bool = True):
        super().__init__()
        net_arch = net_arch or DEFAULT_NET_ARCH
        if lstm_hidden_size % 4:
            raise ValueError("lstm_hidden_size must be a multiple of 4")
        self.obs_dim = obs_dim
        self.lstm_hidden_size = lstm_hidden_size
        self.lstm_actor = nn.LSTM(obs_dim, lstm_hidden_size, num_layers=1)
        self.lstm_critic = nn.LSTM(obs_dim, lstm_hidden_size, num_layers=1)
        self.mlp_extractor = MlpExtractor(lstm_hidden_size, net_arch)
        self.action_net = nn.Linear(self.mlp_extractor.latent_dim_pi, n_actions)
        self.value_net = nn.Linear(self.mlp_extractor.latent_dim_vf, 1)
        if ortho_init:
            self._ortho_init()

    def initial_state(self, n: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
        """(h, c), each [2 (actor, critic), n, H] zeros (RecurrentPPO._setup_model)."""
        z = torch.zeros((2, n, self.lstm_hidden_size), dtype=torch.float32, device=device)
        return z, z.clone()

    @torch.no_grad()
    def forward_torch(self, obs: torch.Tensor, h: torch.Tensor, c: torch.Tensor,
                      episode_starts: Optional[torch.Tensor] = None):
        """One step in plain PyTorch f32 (nn.LSTM), as
        RecurrentActorCriticPolicy.forward does it: the states are multiplied
        by (1 - episode_start) before the LSTM step.
        Returns (logits [N, A], values [N], h' [2, N, H], c' [2, N, H])."""
        if episode_starts is not None:
            m = (1.0 - episode_starts.float()).view(1, -1, 1)
            h, c = h * m, c * m
        x = obs.unsqueeze(0)
        out_pi, (hp, cp) = self.lstm_actor(x, (h[0:1].contiguous(), c[0:1].contiguous()))
        out_vf, (hv, cv) = self.lstm_critic(x, (h[1:2].contiguous(), c[1:2].contiguous()))
        lp = self.mlp_extractor.policy_net(out_pi[0])
        lv = self.mlp_extractor.value_net(out_vf[0])
        return (self.action_net(lp), self.value_net(lv).squeeze(-1), torch.cat([hp, hv], 0), torch.cat([cp, cv], 0))


def numpy_weights(policy: nn.Module) -> Dict[str, "object"]:
    """state_dict as float64 numpy arrays (for the CPU oracle in tests)."""
    return {k: v.detach().cpu().double().numpy() for k, v in policy.state_dict().items()}
