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

One "step" = one batched env step of all agents on the GPU; the default
timed window is 5,408 steps, one full episode of the 32x32x8 box
(episodes truncate at total_free_cells = 5,400 steps), so the number is the
episode-average throughput rather than one phase of it.  ``--fuse F``
advances F steps per kernel launch (obs written for every step into a
[F, N, 80] trajectory buffer, i.e. the rollout-buffer shape); F=1 is the
drop-in VecEnv.step call.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--fuse F]
For N>1 launch one rank per GPU with torch.distributed.run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))

METRIC = "env-steps/sec at 65536 parallel agents, 32×32×8 room, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes_per_step(L: int) -> int:
    """action 1 + window 64 + rays 6L + state 2*16 + obs 320 + reward 4 + flags 2."""
    return 1 + 64 + 6 * L + 32 + 320 + 4 + 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 5408 = one whole 5,400-step episode of the 32x32x8 box (every agent
    # starts at t=0): the timed window covers every phase of an episode,
    # early exploration, steady state and the auto-reset
    ap.add_argument("--steps", type=int, default=5408)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--agents", type=int, default=65536, help="agents per GPU")
    ap.add_argument("--room", default="32x32x8", help="WxDxH of the walled-box room")
    ap.add_argument("--L", type=int, default=10, help="local_map_length")
    ap.add_argument("--fuse", type=int, default=16, help="env steps per kernel launch (headline)")
    ap.add_argument("--single-step-check", type=int, default=1,
                    help="also time the drop-in one-step-per-launch call (vn_step_random k=1)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (0 = skip)")
    ap.add_argument("--simple", type=int, default=1,
                    help="also time the simpleEnv variant (envs/simpleEnv.py) on the same agents/room, L=4")
    ap.add_argument("--collector", default="lstm", choices=["lstm", "mlp", "none"],
                    help="also time the policy-in-the-loop rollout collector (PPO-LSTM / PPO-MLP)")
    ap.add_argument("--collector-rooms", default="P3_training", help="reference room set for the collector leg")
    ap.add_argument("--collector-T", type=int, default=128, help="rollout length (n_steps) of the collector leg")
    ap.add_argument("--collector-rollouts", type=int, default=2, help="timed rollouts of the collector leg")
    ap.add_argument("--collector-bf16", type=int, default=1,
                    help="also time the collector with bf16 policy GEMMs (the reference's policy is f32)")
    ap.add_argument("--learner-batch", type=int, default=65536,
                    help="PPO learner leg: minibatch size (0 = skip); runs on the f32 PPO-LSTM collector's buffer")
    ap.add_argument("--learner-minibatches", type=int, default=16, help="timed learner minibatch updates")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(room_whd, L, seconds, threads_override=None):
    """The CPU oracle (C restatement of envs/CubicEnv.py step/reset) on the
    host cores, same room / L / policy / seed schedule, bounded sample."""
    import numpy as np
    sys.path.insert(0, str(REPO))
    from oracle.oracle import OracleEnv, parse_room_text
    from voxnav.rooms import box_room, room_to_text
    cores = len(os.sched_getaffinity(0))
    threads = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    if threads_override is not None:
        threads = int(threads_override)
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
    return {"value": steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{N} agents x {steps // N} steps of the same workload ({el:.1f} s) through "
                      f"oracle/voxnav_oracle.c (C restatement of envs/CubicEnv.py, OpenMP over agents)"}


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


def collector_leg(args, torch, dist, dev, rank, world, N, dtype="f32"):
    """Policy-in-the-loop rollouts (RecurrentPPO.collect_rollouts + GAE) on
    the GPU: BASELINE.json config C4 shape (P3_training rooms, PPO-LSTM,
    seq 128) at N agents per GPU.  One untimed rollout, then timed ones."""
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    from voxnav.rooms import load_archive_set
    rooms = load_archive_set(args.collector_rooms)
    torch.manual_seed(42)
    pol = (RecurrentActorCriticPolicy() if args.collector == "lstm" else ActorCriticPolicy()).to(dev)
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
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0].item())
    assert torch.isfinite(buf.advantages).all().item()
    gather = None
    if world > 1 and dtype == "f32" and dist.get_backend() == "nccl":   # not under the gloo rehearsal knob
        gather = allgather_leg(torch, dist, dev, rank, world, buf)
    learner = None
    if dtype == "f32" and args.collector == "lstm" and args.learner_batch > 0:
        learner = learner_leg(args, torch, dist, dev, world, pol, buf)
    steps = args.collector_T * args.collector_rollouts
    fl = lstm_flops_per_agent_step() if args.collector == "lstm" else mlp_flops_per_agent_step()
    tflops = fl * N * steps / el / 1e12
    name = ("PPO-LSTM (MlpLstmPolicy: actor+critic LSTM 256, pi/vf [256,256,128] Tanh)" if args.collector == "lstm"
            else "PPO-MLP (MlpPolicy: pi/vf [256,256,128] Tanh)")
    peak = 157.3 if dtype == "f32" else 2500.0     # dense MFMA peak for the GEMM dtype (MI355X_MICROARCH.md)
    env.close()
    del col, env
    out = {"value": round(N * world * steps / el, 1), "unit": "env-steps/s", "policy": name, "dtype": dtype,
            "rooms": args.collector_rooms, "agents_per_gpu": N, "rollout_steps": args.collector_T,
            "timed_rollouts": args.collector_rollouts, "ms_per_step": round(el * 1e3 / steps, 4),
            "includes": "policy forward, Categorical draw, env step + auto-reset, truncation bootstrap, "
                        "LSTM-state buffer stores, last values, GAE",
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
            got.update(allgather_rollout({k: t}, agent_dim=dims[k]))
        sync()
        el = time.perf_counter() - t0
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        times.append(float(tt.item()))
        if _ < reps - 1:
            del got
    # this rank's slice of the gathered buffers is its own data
    n = buf.rewards.shape[1]
    assert torch.equal(got["rewards"][:, rank * n:(rank + 1) * n], buf.rewards)
    assert torch.equal(got["obs"][:, rank * n:(rank + 1) * n], buf.obs)
    if buf.lstm_h is not None:
        assert torch.equal(got["lstm_h0"][:, :, rank * n:(rank + 1) * n], buf.lstm_h[:1])
    del got
    el = min(times)
    total = local_bytes * world
    return {"bytes_per_rank": local_bytes, "gathered_bytes": total, "seconds": round(el, 5),
            "algbw_GBps": round(total / el / 1e9, 2), "busbw_GBps": round(total * (world - 1) / world / el / 1e9, 2),
            "collective": "all_gather_into_tensor per buffer (RCCL over xGMI)", "reps": reps}


def learner_leg(args, torch, dist, dev, world, pol, buf):
    """PPO learner: sb3_contrib RecurrentPPO.train
    minibatch updates (packed-sequence LSTM re-run, clipped surrogate, value
    MSE, entropy, grad clip, Adam; gradient all-reduce over RCCL when N>1)
    on the collector's buffer.  Timed over a bounded number of minibatches."""
    from voxnav.ppo import PPOLearner
    T, N = buf.actions.shape
    B = min(args.learner_batch, T * N)
    n = max(1, min(args.learner_minibatches, (T * N) // B))
    ln = PPOLearner(pol, n_epochs=1, batch_size=B, seed=0,
                    process_group=dist.group.WORLD if world > 1 else None)
    perm = torch.roll(torch.arange(T * N, device=dev), -12345 % (T * N))
    for m in range(2):
        ln.update(buf, perm[m * B:(m + 1) * B])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for m in range(n):
        ln.update(buf, perm[(m % ((T * N) // B)) * B:(m % ((T * N) // B) + 1) * B])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t[0].item())
    sps = n * B * world / el
    fl = 3 * lstm_flops_per_agent_step()        # forward + backward ~ 3x forward
    return {"value": round(sps, 1), "unit": "samples/s", "batch_size": B, "minibatches": n,
            "ms_per_minibatch": round(el * 1e3 / n, 3), "tflops": round(fl * sps / 1e12, 2),
            "includes": "sequence packing, actor+critic LSTM re-run (dual-LSTM: library GEMMs + HIP cell kernels), MLPs, "
                        "losses, backward, "
                        "grad clip, Adam" + (", RCCL gradient all-reduce" if world > 1 else "")}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob for the multi-rank path on a one-GPU box: every rank on
    # cuda:0 over gloo (RCCL refuses two ranks on one device); not for numbers
    if os.environ.get("VOXNAV_BENCH_SHARED_DEVICE") == "1":
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if os.environ.get("VOXNAV_BENCH_SHARED_DEVICE") == "1":
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
    env = BatchedGridEnv(num_agents=N, rooms=single_room_set(box_room(W, D, H)), local_map_length=args.L,
                         autoreset=True, device=dev, agent_id_base=rank * N, seed_stride=N * world)
    env.reset(seed=42)
    from voxnav.env import Rollout

    def run(F, steps, warmup, env=env):
        out = Rollout(torch.empty((F, N, env.obs_dim), dtype=torch.float32, device=dev),
                      torch.empty((F, N), dtype=torch.float32, device=dev),
                      torch.empty((F, N), dtype=torch.uint8, device=dev),
                      torch.empty((F, N), dtype=torch.uint8, device=dev), None)
        launches_w = max(1, warmup // F)
        launches = max(1, steps // F)
        for _ in range(launches_w):
            env.step_random(F, policy_seed=42, out=out)
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(launches):
            ev[i][0].record(stream)
            env.step_random(F, policy_seed=42, out=out)
            ev[i][1].record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kern_ms = sum(a.elapsed_time(b) for a, b in ev) / launches
        if world > 1:
            t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed, kern_ms = float(t[0].item()), float(t[1].item())
        return out, launches_w * F, launches * F, elapsed, kern_ms

    single = None
    if args.single_step_check and F != 1:
        _, _, st1, el1, km1 = run(1, min(args.steps, 100), 10)
        single = {"value": round(N * world * st1 / el1, 1), "steps": st1, "kernel_avg_us": round(km1 * 1e3, 3)}
    out, warm_steps, steps_timed, elapsed, kern_ms = run(F, args.steps, args.warmup)
    simple = None
    if args.simple:
        senv = BatchedGridEnv(num_agents=N, rooms=single_room_set(box_room(W, D, H)), local_map_length=4,
                              autoreset=True, device=dev, agent_id_base=rank * N, seed_stride=N * world,
                              variant="simple")
        senv.reset(seed=42)
        _, _, st_s, el_s, km_s = run(F, args.steps, args.warmup, env=senv)
        sb = simple_bytes_per_step(4)
        sach = sb * N * F / (km_s * 1e-3) / 1e9
        simple = {"value": round(N * world * st_s / el_s, 1), "unit": "env-steps/s", "variant": "envs/simpleEnv.py",
                  "room": f"{W}x{D}x{H}", "local_map_length": 4, "steps": st_s, "steps_per_launch": F,
                  "kernel_avg_us": round(km_s * 1e3, 3),
                  "roofline": {"bound": "hbm", "achieved": round(sach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(sach / HBM_PEAK_GBS, 5), "algorithmic_bytes_per_env_step": sb}}
        senv.close()
        del senv
    coll = coll_bf = None
    if args.collector != "none":
        coll = collector_leg(args, torch, dist, dev, rank, world, N)
        if args.collector_bf16:
            coll_bf = collector_leg(args, torch, dist, dev, rank, world, N, dtype="bf16")

    # sanity: the trajectory buffer holds real observations
    assert torch.isfinite(out.obs).all().item()

    total_steps = N * world * steps_timed
    value = total_steps / elapsed
    bstep = algorithmic_bytes_per_step(args.L)
    achieved = bstep * N * F / (kern_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
            "kernel": "env_kernel<PH=8,EXT=false,FAST=true,RESET_ONLY=false,PCM=2> (plane-set mode)",
            "kernel_avg_us": round(kern_ms * 1e3, 3),
            "algorithmic_bytes_per_env_step": bstep, "env_steps_per_launch": N * F}
    prof = REPO / "profiles" / "pmc_traffic.json"
    if prof.exists():
        try:
            pm = json.loads(prof.read_text())
            key = f"{W}x{D}x{H}_L{args.L}_N{N}_F{F}"
            if key in pm:
                roof["traffic"] = pm[key]["hbm_bytes_per_launch"]
                roof["traffic_source"] = pm[key].get("source")
        except Exception:  # noqa: BLE001
            pass

    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": steps_timed, "warmup": warm_steps, "ms_per_step": round(elapsed * 1e3 / steps_timed, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
            "data": "synthetic (walled-box room in the reference room-file grammar; Philox uniform random policy)",
            "config": {"workload": f"C3 env step: {N} agents/GPU, {W}x{D}x{H} room, L={args.L}, "
                                   f"random policy, SB3 auto-reset", "agents_per_gpu": N,
                       "global_agents": N * world, "room": f"{W}x{D}x{H}", "local_map_length": args.L,
                       "steps_per_launch": F, "parallelism": f"agent-sharded x{world} (no collective in the step)"},
            "roofline": roof,
        }
        if single is not None:
            rec["drop_in_single_step"] = single   # vn_step-shaped call: one env step per launch
        if simple is not None:
            rec["simple_env"] = simple            # goal-seeking variant
        if coll_bf is not None:
            rec["collector_bf16"] = coll_bf
        if coll is not None:
            rec["collector"] = coll               # policy in the loop
        if world == 1 and args.cpu_seconds > 0:
            cb = cpu_baseline((W, D, H), args.L, args.cpu_seconds)
            one = cpu_baseline((W, D, H), args.L, max(2.0, args.cpu_seconds / 4), threads_override=1)
            cb["single_core_value"] = one["value"]
            cb["cpu_model"] = cpu_model()
            # the reference itself (Python, envs/CubicEnv.py) cannot travel to this
            # box; its step rate as measured in the build container
            cb["reference_python_build_container"] = {
                "single_core": 7.0e3, "eight_processes": 4.95e4, "unit": "env-steps/s",
                "workload": "32x32x8 box, L=10, random actions, 1 env per process",
                "source": "SURVEY.md §6 (Intel Xeon, 8 vCPU; not this box)"}
            rec["cpu_baseline"] = cb
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            Path(args.json_out).write_text(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
