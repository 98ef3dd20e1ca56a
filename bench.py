#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of the batched CubicEnv step on MI355X.

Metric (BASELINE.json): "env-steps/sec at 65536 parallel agents, 32x32x8
room, 1/2/4/8 MI355X".  Workload (SURVEY.md 8(d), config C3 shape): per GPU
65,536 agents in a 32x32x8 walled-box room file (reference room grammar,
random.choice over the one-room set), local_map_length L=10
(train/Grid_Train.py:36), crash penalty -2.0, uniform random policy
(Philox4x32-10, seed 42), SB3 auto-reset with the pinned seed schedule
42 + global_agent_id + N_global * episode.  Inputs live in HBM before the
timed region; every step writes the full obs [N,80] f32, reward, terminated
and truncated tensors.

One "step" = one batched env step of all agents on the GPU.  The headline
resets a fresh env, runs exactly ``--warmup`` untimed steps, then times
exactly ``--steps`` steps (launches of ``--fuse`` F steps into a [F, N, 80]
rollout-chunk buffer; the last launch of each phase takes the remainder).
F = 128 by default: a 128-step rollout chunk per launch (the collector's
n_steps; the reference's rollouts are n_steps = 2048 per env,
train/Grid_Train.py:84); the same window at F = 16 is reported beside it
(``same_window_other_fuse``).
``roofline`` is computed from the same timed launches (HIP events on the
launch stream) and ``traffic`` from the PMC record of the same window
(profiles/pmc_traffic.json, keyed by room/L/N/F/warmup/steps).  When the
timed window is shorter than one whole 5,400-step episode of the 32x32x8
box, ``episode_window`` adds the same measurement over one full episode
from t=0 (every phase: early exploration, steady state, auto-reset).

``--gpus N`` (N > 1) without a launcher environment starts N ranks itself
(torch.distributed.run, one process per GPU, before any GPU call) and exits
with their status; every rank owns 65,536 agents with global ids (no
collective in the step), the timing is max-over-ranks, and the collector
leg all-gathers its trajectory buffers over RCCL at the rollout boundary.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--fuse F]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))

METRIC = "env-steps/sec at 65536 parallel agents, 32×32×8 room, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
EPISODE_WINDOW = 5408   # one whole 5,400-step episode of the 32x32x8 box, in F=16 launches


def algorithmic_bytes_per_step(L: int) -> int:
    """action 1 + window 64 + rays 6L + state 2*16 + obs 320 + reward 4 + flags 2."""
    return 1 + 64 + 6 * L + 32 + 320 + 4 + 2


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=EPISODE_WINDOW)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--agents", type=int, default=65536, help="agents per GPU")
    ap.add_argument("--room", default="32x32x8", help="WxDxH of the walled-box room")
    ap.add_argument("--L", type=int, default=10, help="local_map_length")
    ap.add_argument("--fuse", type=int, default=128,
                    help="env steps per kernel launch (headline): one launch fills a [F, N, 80] rollout chunk")
    ap.add_argument("--fuse-check", type=int, default=16,
                    help="also time the same window at this many steps per launch (0 = skip)")
    ap.add_argument("--episode-window", type=int, default=1,
                    help="when --steps < one episode, also time one whole episode (5,408 steps)")
    ap.add_argument("--single-step-check", type=int, default=1,
                    help="also time the drop-in one-step-per-launch call (vn_step_random k=1)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU baseline sample per leg in seconds (0 = skip)")
    ap.add_argument("--simple", type=int, default=1,
                    help="also time the simpleEnv variant (envs/simpleEnv.py) on the same agents/room, L=4")
    ap.add_argument("--room-sets", default="P2_training,P3_training",
                    help="env-only legs on these reference room sets (random policy, same launches), or none")
    ap.add_argument("--room-set-steps", type=int, default=1024, help="timed steps of each room-set leg")
    ap.add_argument("--collector", default="lstm,mlp",
                    help="policy-in-the-loop rollout collector legs: any of lstm (PPO-LSTM, P3_training, "
                         "BASELINE config C4) and mlp (PPO-MLP, P2_training, config C3), or none")
    ap.add_argument("--collector-T", type=int, default=128, help="rollout length (n_steps) of the collector leg")
    ap.add_argument("--collector-rollouts", type=int, default=2, help="timed rollouts of the collector leg")
    ap.add_argument("--collector-bf16", type=int, default=0,
                    help="also time the PPO-LSTM collector with bf16 policy GEMMs (an option: the reference's policy "
                         "is f32, so it is not a default leg)")
    ap.add_argument("--learner-batch", type=int, default=65536,
                    help="PPO learner legs: minibatch size (0 = skip); run on each f32 collector's buffer")
    ap.add_argument("--learner-minibatches", type=int, default=16, help="timed learner minibatch updates")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch/rendezvous rehearsal without a GPU: ranks init gloo, time a barrier, print the line")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


# ---------------------------------------------------------------- launch
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """``--gpus N`` without a launcher: start N ranks (one process per GPU)
    through torch.distributed.run as a child process -- nothing here has
    touched the GPU -- and return their exit status.  This replaces the
    reference's process-level env parallelism (train/Grid_Train.py:191-192)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve())]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def launches(total: int, F: int):
    """Launch sizes covering exactly ``total`` steps: F-step launches, the
    remainder last."""
    out = [F] * (total // F)
    if total % F:
        out.append(total % F)
    return out


# ---------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """CPU share of this job: the affinity set, capped by OMP_NUM_THREADS
    (the GPU box exposes the whole machine's CPUs but gives a job 16)."""
    cores = len(os.sched_getaffinity(0))
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))


def python_numpy_baseline(room, L, seconds, procs):
    """The reference's Python/NumPy step loop in its SubprocVecEnv shape
    (train/Grid_Train.py:191-192: one env per process): ``procs`` processes
    of oracle/py_cubic.py (a per-agent restatement of envs/CubicEnv.py, the
    reference itself cannot travel to this box), each one env under a
    uniform random policy with auto-reset, all stepping between the same two
    wall-clock instants.  Returns aggregate env-steps/s."""
    start = time.time() + 1.5 + 0.02 * procs   # let every child import numpy first
    stop = start + seconds
    ps = [subprocess.Popen([sys.executable, "-m", "oracle.py_cubic", "--room", room, "--L", str(L),
                            "--seed", str(42 + i), "--start-at", repr(start), "--stop-at", repr(stop)],
                           cwd=str(REPO), stdout=subprocess.PIPE, text=True) for i in range(procs)]
    steps = episodes = 0
    for p in ps:
        out, _ = p.communicate(timeout=seconds + 120)
        if p.returncode != 0:
            raise RuntimeError("python baseline child failed")
        rec = json.loads(out.strip().splitlines()[-1])
        steps += rec["steps"]
        episodes += rec["episodes"]
    return steps / (stop - start), steps, episodes


def c_port_baseline(room_whd, L, seconds, threads):
    """The C restatement (oracle/voxnav_oracle.c) of the same workload,
    OpenMP over agents: a second, stronger CPU reference point."""
    import numpy as np
    sys.path.insert(0, str(REPO))
    from oracle.oracle import OracleEnv, parse_room_text
    from voxnav.rooms import box_room, room_to_text
    N = 512 * threads
    W, D, H = room_whd
    env = OracleEnv([parse_room_text(room_to_text(box_room(W, D, H)))], n_agents=N, local_map_length=L,
                    use_room_draw=True)
    env.run_random(42 + np.arange(N), policy_seed=42, K=1, seed_stride=N, record=False, threads=threads)
    steps = 0
    t0 = time.perf_counter()
    k = 16
    while True:
        env.run_random(np.zeros(N, np.int64), policy_seed=42, K=k, t0=1 + steps // N, seed_stride=N,
                       initial_reset=False, record=False, threads=threads)
        steps += N * k
        el = time.perf_counter() - t0
        if el >= seconds:
            break
        k = min(1024, k * 2)
    return steps / el, N, steps // N, el


def cpu_baseline(room_whd, L, seconds):
    W, D, H = room_whd
    room = f"{W}x{D}x{H}"
    P = host_cores()
    v, steps, ep = python_numpy_baseline(room, L, seconds, P)
    v1, steps1, _ = python_numpy_baseline(room, L, max(2.0, seconds / 2), 1)
    cv, cn, ck, cel = c_port_baseline(room_whd, L, seconds, P)
    cv1, _, _, _ = c_port_baseline(room_whd, L, max(2.0, seconds / 4), 1)
    rec = {"value": round(v, 1), "unit": "env-steps/s", "cores": P, "kind": "port",
           "sample": f"{P} processes x 1 env (SubprocVecEnv shape), {steps} env-steps in {seconds:.0f} s, "
                     f"{ep} auto-resets: oracle/py_cubic.py, a per-agent Python/NumPy restatement of "
                     f"envs/CubicEnv.py (pinned bit-exact to the reference's golden trajectories), "
                     f"{room} box, L={L}, uniform random actions",
           "single_core_value": round(v1, 1), "cpu_model": cpu_model(),
           "c_openmp_port": {"value": round(cv, 1), "single_core_value": round(cv1, 1), "threads": P,
                             "sample": f"{cn} agents x {ck} steps ({cel:.1f} s) through oracle/voxnav_oracle.c "
                                       f"(C restatement of envs/CubicEnv.py, OpenMP over agents)"}}
    cal = REPO / "profiles" / "py_baseline_calibration.json"
    if cal.exists():
        c = json.loads(cal.read_text())
        ratio = float(c["restatement_over_reference"])
        rec["reference_equivalent_value"] = round(v / ratio, 1)
        rec["reference_equivalent_single_core_value"] = round(v1 / ratio, 1)
        rec["reference_calibration"] = {
            "restatement_over_reference": c["restatement_over_reference"],
            "reference_single_core_build_container": c["reference_envs_CubicEnv_steps_per_s"],
            "source": "tests/golden/calibrate_py_baseline.py: the unmodified envs/CubicEnv.py vs "
                      "oracle/py_cubic.py, one process each, build container " + c.get("cpu_model", "")}
    return rec


# ---------------------------------------------------------------- policy legs
def simple_bytes_per_step(L: int) -> int:
    """simpleEnv variant: action 1 + ray cells 6L + state 2*16 + goal 4 +
    obs 4*(6L+7) + reward 4 + flags 2."""
    return 1 + 6 * L + 32 + 4 + 4 * (6 * L + 7) + 4 + 2


def lstm_flops_per_agent_step(obs=80, H=256, arch=(256, 256, 128), A=6) -> int:
    """PPO-LSTM forward: x@W_ih for 2 LSTMs, h@W_hh for 2,
    the two Tanh MLPs and the heads, 2 FLOP per MAC."""
    macs = 2 * obs * 4 * H + 2 * H * 4 * H
    d = H
    for w in arch:
        macs += 2 * d * w
        d = w
    macs += d * (A + 1)
    return 2 * macs


def mlp_flops_per_agent_step(obs=80, arch=(256, 256, 128), A=6) -> int:
    macs, d = 0, obs
    for w in arch:
        macs += 2 * d * w
        d = w
    macs += d * (A + 1)
    return 2 * macs


def _max_over_ranks(torch, dist, dev, world, *vals):
    if world == 1:
        return vals
    t = torch.tensor(list(vals), dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return tuple(float(v) for v in t.tolist())


def collector_leg(args, torch, dist, dev, rank, world, N, kind, dtype="f32"):
    """Policy-in-the-loop rollouts (RecurrentPPO / PPO collect_rollouts +
    GAE) on the GPU at N agents per GPU: kind "lstm" = BASELINE config C4
    (P3_training rooms, PPO-LSTM, seq 128), "mlp" = config C3 (P2_training,
    PPO-MLP).  One untimed rollout, then timed ones; then the learner."""
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    from voxnav.rooms import load_archive_set
    rooms_name = "P3_training" if kind == "lstm" else "P2_training"
    rooms = load_archive_set(rooms_name)
    torch.manual_seed(42)
    pol = (RecurrentActorCriticPolicy() if kind == "lstm" else ActorCriticPolicy()).to(dev)
    env = BatchedGridEnv(num_agents=N, rooms=rooms, local_map_length=args.L, autoreset=True, device=dev,
                         agent_id_base=rank * N, seed_stride=N * world)
    col = RolloutCollector(env, pol, n_steps=args.collector_T, sample_seed=42, reset_seed=42, policy_dtype=dtype)
    col.collect()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.collector_rollouts):
        buf = col.collect()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el, = _max_over_ranks(torch, dist, dev, world, time.perf_counter() - t0)
    assert torch.isfinite(buf.advantages).all().item()
    gather = None
    if world > 1 and dtype == "f32" and dist.get_backend() == "nccl":   # not under the gloo rehearsal knob
        gather = allgather_leg(torch, dist, dev, rank, world, buf)
    learner = None
    if dtype == "f32" and args.learner_batch > 0:
        learner = learner_leg(args, torch, dist, dev, world, pol, buf, kind)
    steps = args.collector_T * args.collector_rollouts
    fl = lstm_flops_per_agent_step() if kind == "lstm" else mlp_flops_per_agent_step()
    tflops = fl * N * steps / el / 1e12
    name = ("PPO-LSTM (MlpLstmPolicy: actor+critic LSTM 256, pi/vf [256,256,128] Tanh)" if kind == "lstm"
            else "PPO-MLP (MlpPolicy: pi/vf [256,256,128] Tanh)")
    peak = 157.3 if dtype == "f32" else 2500.0     # dense MFMA peak for the GEMM dtype (MI355X_MICROARCH.md)
    env.close()
    del col, env
    out = {"value": round(N * world * steps / el, 1), "unit": "env-steps/s", "policy": name, "dtype": dtype,
           "config": "C4" if kind == "lstm" else "C3",
           "rooms": rooms_name, "agents_per_gpu": N, "rollout_steps": args.collector_T,
           "timed_rollouts": args.collector_rollouts, "ms_per_step": round(el * 1e3 / steps, 4),
           "includes": "policy forward, Categorical draw, env step + auto-reset, truncation bootstrap, "
                       + ("LSTM-state buffer stores, " if kind == "lstm" else "") + "last values, GAE",
           "policy_flops_per_agent_step": fl, "policy_tflops": round(tflops, 2),
           "policy_frac_of_mfma_peak": round(tflops / peak, 4), "mfma_peak_tflops": peak}
    if learner is not None:
        out["learner"] = learner
    if gather is not None:
        out["trajectory_allgather"] = gather
    return out


def allgather_leg(torch, dist, dev, rank, world, buf, reps=3):
    """the one exchange of the path -- the rollout's
    trajectory buffers all-gathered over RCCL (xGMI) at the rollout boundary
    (obs, actions, rewards, episode starts, values, log-probs, advantages,
    returns, and the LSTM states at the rollout's first step).  Timed
    max-over-ranks; bus bandwidth = algorithm bytes x (world-1)/world."""
    from voxnav.sharding import allgather_rollout
    bufs = {"obs": buf.obs, "actions": buf.actions, "rewards": buf.rewards, "episode_starts": buf.episode_starts,
            "values": buf.values, "log_probs": buf.log_probs, "advantages": buf.advantages,
            "returns": buf.returns}
    if buf.lstm_h is not None:
        bufs["lstm_h0"] = buf.lstm_h[:1]
        bufs["lstm_c0"] = buf.lstm_c[:1]
    dims = {k: (2 if k.startswith("lstm") else 1) for k in bufs}
    local_bytes = sum(t.numel() * t.element_size() for t in bufs.values())
    got = None
    times = []
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    for _ in range(reps):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        got = {}
        for k, t in bufs.items():
            got.update(allgather_rollout({k: t}, agent_dim=dims[k], flat=False))
        sync()
        el = time.perf_counter() - t0
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        times.append(float(tt.item()))
        if _ < reps - 1:
            del got
    # this rank's slice of the gathered buffers is its own data
    # [T, world, n_local, ...] views (no copy before or after the collective):
    # this rank's slice is its own data
    assert torch.equal(got["rewards"][:, rank], buf.rewards)
    assert torch.equal(got["obs"][:, rank], buf.obs)
    if buf.lstm_h is not None:
        assert torch.equal(got["lstm_h0"][:, :, rank], buf.lstm_h[:1])
    del got
    el = min(times)
    total = local_bytes * world
    return {"bytes_per_rank": local_bytes, "gathered_bytes": total, "seconds": round(el, 5),
            "algbw_GBps": round(total / el / 1e9, 2), "busbw_GBps": round(total * (world - 1) / world / el / 1e9, 2),
            "collective": "all_gather_into_tensor per buffer straight from the rollout buffer (RCCL over xGMI); "
                          "results as [T, world, n_local] views, no copies in the timed region", "reps": reps}


def learner_leg(args, torch, dist, dev, world, pol, buf, kind):
    """PPO learner: RecurrentPPO.train (kind lstm:
    packed-sequence LSTM re-run) / PPO.train (kind mlp) minibatch updates --
    clipped surrogate, value MSE, entropy, grad clip, Adam; gradient
    all-reduce over RCCL when N>1 -- on the collector's buffer, timed over a
    bounded number of minibatches."""
    from voxnav.ppo import PPOLearner
    T, N = buf.actions.shape
    B = min(args.learner_batch, T * N)
    n = max(1, min(args.learner_minibatches, (T * N) // B))
    ln = PPOLearner(pol, n_epochs=1, batch_size=B, seed=0,
                    process_group=dist.group.WORLD if world > 1 else None)
    perm = torch.roll(torch.arange(T * N, device=dev), -12345 % (T * N))
    if kind == "mlp":
        perm = torch.randperm(T * N, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    win = kind == "lstm"          # rolled contiguous windows, as train() cuts them
    ln.update_many(buf, [perm[m * B:(m + 1) * B] for m in range(2)], windows=win)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    nb = (T * N) // B
    ln.update_many(buf, [perm[(m % nb) * B:(m % nb + 1) * B] for m in range(n)], windows=win)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el, = _max_over_ranks(torch, dist, dev, world, time.perf_counter() - t0)
    sps = n * B * world / el
    fl = 3 * (lstm_flops_per_agent_step() if kind == "lstm" else mlp_flops_per_agent_step())  # fwd + bwd ~ 3x fwd
    inc = ("row layout (minibatch = whole env rollouts), actor+critic LSTM re-run in one persistent launch per "
           "direction (weight gradients inside the backward), MLPs (direct-load MFMA GEMMs), "
           if kind == "lstm" else "minibatch gather, actor/critic MLPs (direct-load MFMA GEMMs), ")
    return {"value": round(sps, 1), "unit": "samples/s", "batch_size": B, "minibatches": n,
            "ms_per_minibatch": round(el * 1e3 / n, 3), "tflops": round(fl * sps / 1e12, 2),
            "frac_of_f32_mfma_peak": round(fl * sps / 1e12 / 157.3, 4),
            "includes": inc + "heads + losses + their gradient (fused loss kernel), backward, gradient norm, Adam "
                        "(library kernels)"
            + (f", gradient all-reduce ({'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()})"
               if world > 1 else "")}


# ---------------------------------------------------------------- env window
def time_window(torch, dist, dev, world, env, N, F, warmup, steps, policy_seed=42, events=True):
    """Reset already done by the caller.  Run exactly ``warmup`` untimed
    steps, then time exactly ``steps`` steps in launches of F (remainder
    last).  Returns (elapsed_s max-over-ranks, kernel_ms_total max-over-ranks,
    launch sizes, out).  ``events=False``: no HIP event records in the timed
    region (kernel_ms is None)."""
    from voxnav.env import Rollout
    out = Rollout(torch.empty((F, N, env.obs_dim), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev), None)

    def view(k):
        return Rollout(out.obs[:k], out.reward[:k], out.terminated[:k], out.truncated[:k], None)

    for k in launches(warmup, F):
        env.step_random(k, policy_seed=policy_seed, out=view(k))
    timed = launches(steps, F)
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in timed]
    # the timed launches prepared up front (argument checks and conversions),
    # so the timed loop is the launches themselves
    fns, t = [], warmup
    for k in timed:
        fns.append(env.step_random_launcher(k, policy_seed, t, view(k)))
        t += k
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if events:
        for (a, b), fn in zip(ev, fns):
            a.record(stream)
            fn()
            b.record(stream)
    else:
        for fn in fns:
            fn()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not events:
        elapsed, = _max_over_ranks(torch, dist, dev, world, elapsed)
        return elapsed, None, timed, out
    kern_ms = sum(a.elapsed_time(b) for a, b in ev)
    elapsed, kern_ms = _max_over_ranks(torch, dist, dev, world, elapsed, kern_ms)
    return elapsed, kern_ms, timed, out


def roofline_block(bstep, N, F, steps, timed, kern_ms, traffic_rec, kernel_label):
    """Roofline of the dominant kernel over ONE window: algorithmic bytes of
    the window's env-steps / the window's summed launch time.  Per-launch
    figures are per F-step launch (window totals x F / steps)."""
    achieved = bstep * N * steps / (kern_ms * 1e-3) / 1e9
    full = [k for k in timed if k == F]
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "kernel": kernel_label,
            "kernel_avg_us": round(kern_ms * 1e3 / len(timed), 3),
            "kernel_us_per_F_launch": round(kern_ms * 1e3 * F / steps, 3),
            "launches": len(timed), "full_launches": len(full), "steps_per_launch": F,
            "algorithmic_bytes_per_env_step": bstep, "env_steps_per_launch": N * F}
    if traffic_rec is not None:
        roof["traffic"] = traffic_rec["hbm_bytes_per_launch"]
        # per env-step of the launches the record was taken over (a window
        # shorter than F runs shorter launches than N * F env-steps)
        roof["traffic_bytes_per_env_step"] = round(
            traffic_rec["hbm_bytes_per_launch"] / traffic_rec.get("env_steps_per_launch", N * F), 1)
        roof["traffic_source"] = traffic_rec.get("source")
    return roof


def traffic_for(W, D, H, L, N, F, warmup, steps, prefix=""):
    """The PMC traffic record of one window (profiles/pmc_traffic.json, written
    by scripts/traffic_record.py), keyed by room (WxDxH, or a room-set name in
    W with D = H = ""), L, N, launch size and window."""
    prof = REPO / "profiles" / "pmc_traffic.json"
    if not prof.exists():
        return None
    try:
        pm = json.loads(prof.read_text())
    except ValueError:
        return None
    room = f"{W}x{D}x{H}" if D != "" else str(W)
    return pm.get(f"{prefix}{room}_L{L}_N{N}_F{F}_W{warmup}_K{steps}")


# ---------------------------------------------------------------- main
def dry_run(args, world, rank):
    """Launch / rendezvous rehearsal on CPU (gloo): the --gpus N path up to
    the first GPU call, with the bench's barrier + max-over-ranks timing."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ranks = [rank]
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        got = [None] * world
        dist.all_gather_object(got, rank)
        ranks = got
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world, "steps": 0,
                          "warmup": 0, "dry_run": True, "ranks": ranks, "barrier_s": el,
                          "agents_global": args.agents * world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist
    # rehearsal knob for the multi-rank path on a one-GPU box: every rank on
    # cuda:0 over gloo (RCCL refuses two ranks on one device); not for numbers
    shared = os.environ.get("VOXNAV_BENCH_SHARED_DEVICE") == "1"
    if shared:
        local = 0
    if world > 1:
        if not shared and torch.cuda.device_count() < world:
            raise SystemExit(f"--gpus {world} needs {world} visible GPUs, found {torch.cuda.device_count()}")
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from voxnav.env import BatchedGridEnv
    from voxnav.rooms import box_room, single_room_set

    W, D, H = (int(v) for v in args.room.split("x"))
    N = args.agents
    F = max(1, args.fuse)
    if args.steps < 1 or args.warmup < 0:
        raise SystemExit("--steps must be >= 1 and --warmup >= 0")
    bstep = algorithmic_bytes_per_step(args.L)

    def make_env(L=args.L, variant="cubic"):
        e = BatchedGridEnv(num_agents=N, rooms=single_room_set(box_room(W, D, H)), local_map_length=L,
                           autoreset=True, device=dev, agent_id_base=rank * N, seed_stride=N * world,
                           variant=variant)
        e.reset(seed=42)
        return e

    # headline: a fresh env, exactly W warmup + K timed steps, nothing but the
    # launches between the two synchronizes; the roofline's kernel time from
    # HIP events on the launch stream over an identical re-run of the window
    # (fresh env, same seeds: the same work; the event records would add
    # ~15 us of host time to a one-launch window)
    env = make_env()
    label = env.kernel_label(F)
    elapsed, _, timed, out = time_window(torch, dist, dev, world, env, N, F, args.warmup, args.steps, events=False)
    assert torch.isfinite(out.obs).all().item()   # the trajectory buffer holds real observations
    env.close()
    del env, out
    env = make_env()
    ev_el, kern_ms, _, _ = time_window(torch, dist, dev, world, env, N, F, args.warmup, args.steps)
    env.close()
    del env
    roof = roofline_block(bstep, N, F, args.steps, timed, kern_ms,
                          traffic_for(W, D, H, args.L, N, F, args.warmup, args.steps), label)
    value = N * world * args.steps / elapsed
    # every agent starts at t=0 and a random-policy episode truncates at the
    # room's free-cell count: an auto-reset is inside the
    # window iff it reaches that step
    resets_in_window = args.warmup + args.steps >= box_room(W, D, H).total_free_cells

    episode = None
    if args.episode_window and args.steps < EPISODE_WINDOW:
        env = make_env()
        e_el, e_km, e_timed, _ = time_window(torch, dist, dev, world, env, N, F, 32, EPISODE_WINDOW)
        env.close()
        del env
        episode = {"value": round(N * world * EPISODE_WINDOW / e_el, 1), "unit": "env-steps/s",
                   "warmup": 32, "steps": EPISODE_WINDOW,
                   "ms_per_step": round(e_el * 1e3 / EPISODE_WINDOW, 5),
                   "window": "one whole 5,400-step episode of every agent from t=0 (incl. the auto-reset)",
                   "roofline": roofline_block(bstep, N, F, EPISODE_WINDOW, e_timed, e_km,
                                              traffic_for(W, D, H, args.L, N, F, 32, EPISODE_WINDOW), label)}

    fuse_alt = None
    if args.fuse_check and args.fuse_check != F:
        Fc = args.fuse_check
        env = make_env()
        c_el, c_km, c_timed, _ = time_window(torch, dist, dev, world, env, N, Fc, args.warmup, args.steps)
        fuse_alt = {"value": round(N * world * args.steps / c_el, 1), "steps_per_launch": Fc,
                    "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(c_el * 1e3 / args.steps, 5),
                    "roofline": roofline_block(bstep, N, Fc, args.steps, c_timed, c_km,
                                               traffic_for(W, D, H, args.L, N, Fc, args.warmup, args.steps),
                                               env.kernel_label(Fc))}
        env.close()
        del env

    single = None
    if args.single_step_check and F != 1:
        # kernel time from HIP events around each launch; the host-timed value
        # from a second window with no event markers between the launches
        # (an event record per launch adds a queue packet between steps)
        env = make_env()
        s_el, s_km, s_timed, _ = time_window(torch, dist, dev, world, env, N, 1, 10, 100)
        env.close()
        del env
        env = make_env()
        h_el, _, _, _ = time_window(torch, dist, dev, world, env, N, 1, 10, 400, events=False)
        single = {"value": round(N * world * 400 / h_el, 1), "steps": 400, "warmup": 10,
                  "us_per_call": round(h_el * 1e6 / 400, 3),
                  "us_per_call_with_events": round(s_el * 1e6 / 100, 3),
                  "kernel_avg_us": round(s_km * 1e3 / len(s_timed), 3),
                  "kernel": env.kernel_label(1)}
        env.close()
        del env

    simple = None
    if args.simple:
        senv = make_env(L=4, variant="simple")
        st_steps = max(args.steps, EPISODE_WINDOW if args.episode_window else 0)
        s_el, s_km, s_timed, _ = time_window(torch, dist, dev, world, senv, N, F, 32, st_steps)
        sb = simple_bytes_per_step(4)
        sach = sb * N * st_steps / (s_km * 1e-3) / 1e9
        simple = {"value": round(N * world * st_steps / s_el, 1), "unit": "env-steps/s",
                  "variant": "envs/simpleEnv.py", "room": f"{W}x{D}x{H}", "local_map_length": 4, "warmup": 32,
                  "steps": st_steps, "steps_per_launch": F, "kernel_avg_us": round(s_km * 1e3 / len(s_timed), 3),
                  "kernel": senv.kernel_label(F),
                  "roofline": {"bound": "hbm", "achieved": round(sach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(sach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_env_step": sb}}
        strf = traffic_for(W, D, H, 4, N, F, 32, st_steps, prefix="simple_")
        simple["roofline"]["traffic"] = strf["hbm_bytes_per_launch"] if strf else None
        if strf:
            simple["roofline"]["traffic_bytes_per_env_step"] = round(
                strf["read_bytes_per_env_step"] + strf["write_bytes_per_env_step"], 1)
            simple["roofline"]["traffic_source"] = strf["source"]
        senv.close()
        del senv

    # env-only legs on the room sets the reference trains on (train/Grid_Train.py:36-60):
    # P2_training (BASELINE C3's rooms) and P3_training (C4's), the same random-policy
    # window as the episode leg (the sets' rooms are 6-12 high: byte-mark kernels)
    room_sets = {}
    for rs in [r for r in args.room_sets.split(",") if r and r != "none"]:
        from voxnav.rooms import load_archive_set
        env = BatchedGridEnv(num_agents=N, rooms=load_archive_set(rs), local_map_length=args.L, autoreset=True,
                             device=dev, agent_id_base=rank * N, seed_stride=N * world)
        env.reset(seed=42)
        rlab = env.kernel_label(F)
        r_el, r_km, r_timed, _ = time_window(torch, dist, dev, world, env, N, F, 32, args.room_set_steps)
        env.close()
        del env
        room_sets[rs] = {"value": round(N * world * args.room_set_steps / r_el, 1), "unit": "env-steps/s",
                         "warmup": 32, "steps": args.room_set_steps, "steps_per_launch": F,
                         "roofline": roofline_block(bstep, N, F, args.room_set_steps, r_timed, r_km,
                                                   traffic_for(rs, "", "", args.L, N, F, 32, args.room_set_steps,
                                                               prefix="set_"), rlab)}

    legs = {}
    kinds = [k for k in args.collector.split(",") if k and k != "none"]
    for kind in kinds:
        if kind not in ("lstm", "mlp"):
            raise SystemExit(f"--collector: unknown leg {kind!r}")
        legs[f"collector_{kind}"] = collector_leg(args, torch, dist, dev, rank, world, N, kind)
        if kind == "lstm" and args.collector_bf16:
            legs["collector_lstm_bf16"] = collector_leg(args, torch, dist, dev, rank, world, N, kind, dtype="bf16")

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
            "data": "synthetic (walled-box room in the reference room-file grammar; Philox uniform random policy)",
            "config": {"workload": f"C3 env step: {N} agents/GPU, {W}x{D}x{H} room, L={args.L}, "
                                   f"random policy" + (", SB3 auto-reset in the window" if resets_in_window
                                                       else " (episode steps inside one episode: the "
                                                            "window holds no auto-reset)"),
                       "agents_per_gpu": N,
                       "global_agents": N * world, "room": f"{W}x{D}x{H}", "local_map_length": args.L,
                       "steps_per_launch": F,
                       "window": f"fresh env, {args.warmup} untimed steps, then exactly {args.steps} timed steps "
                                 f"in {len(timed)} launches (episode steps {args.warmup + 1}-"
                                 f"{args.warmup + args.steps}); roofline and traffic from the same launches of an "
                                 f"identical re-run of the window timed with HIP events "
                                 f"(wall {round(ev_el * 1e3 / args.steps, 5)} ms per step with the events)",
                       "parallelism": f"agent-sharded x{world} (no collective in the step)"},
            "roofline": roof,
        }
        if episode is not None:
            rec["episode_window"] = episode
        if fuse_alt is not None:
            rec["same_window_other_fuse"] = fuse_alt   # the same steps in launches of --fuse-check steps
        if single is not None:
            rec["drop_in_single_step"] = single   # vn_step-shaped call: one env step per launch
        if simple is not None:
            rec["simple_env"] = simple            # goal-seeking variant
        if room_sets:
            rec["env_room_sets"] = room_sets      # the reference's training room sets (P2 / P3)
        rec.update(legs)                          # policy in the loop
        if world == 1 and args.cpu_seconds > 0:
            rec["cpu_baseline"] = cpu_baseline((W, D, H), args.L, args.cpu_seconds)
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            Path(args.json_out).write_text(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
