#!/usr/bin/env python3
"""train.py's main loop (src/train.py:523-693) on the batched env, entirely on one GPU.

    reference                                   here
    ROS callbacks -> observe_* (:532-557)       obs = env.step(...) (device tensors, in place)
    agent.get_action (:572)                     brain.decide_action(obs, episode) for all envs
    rewarder2 + reach_times (:577-587)          env flags -> tracker.update_from(env)
    agent.memorize (:596)                       brain.memory.push_begin/push_end around the step
    agent.update_q_function (:597)              brain.replay() every --replay-every steps
    update_target every 2 episodes (:636-637)   every --target-every replays
    reach_rate > 0.8 -> save (:644-648)         tracker.summary()["any_complete"]

Usage: python examples/train_vec.py --envs 256 --steps 100
Prints one JSON line: env-steps/s of the whole loop, learner updates, losses, episode totals.
The loop is learner-bound: the reference Network costs ~6 GFLOP per sample forward (conv2:
32 -> 64 channels, 32x32 kernel, 38x38 outputs), ~20x that per replayed sample with backward.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from flow_field_based_motion_planner_amd import EpisodeTracker, FFMPConfig  # noqa: E402
from flow_field_based_motion_planner_amd.learner import Brain  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402


def conv_flops(grid: int, cin: int) -> dict:
    """Multiply-add FLOPs (x2) of the reference Network's convolutions per sample (train.py:234-237,
    :244-255: conv1 cin -> 32 k 32, conv2 32 -> 64 k 32, conv3 64 -> 64 k 8, conv4 64 -> 64 k 8 three
    times): forward, and backward = the data gradient of conv2-conv4 + the weight gradients of all."""
    layers, h = [], grid
    for c_in, c_out, k in [(cin, 32, 32), (32, 64, 32), (64, 64, 8), (64, 64, 8), (64, 64, 8), (64, 64, 8)]:
        h = h - k + 1
        layers.append(2.0 * h * h * c_out * c_in * k * k)
    fwd = sum(layers)
    return {"forward": fwd, "backward": 2 * fwd - layers[0]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=256)         # train.py:63 uses 1024
    ap.add_argument("--capacity", type=int, default=200_000)  # pfrl_train.py:65's; train.py:65 uses 20,000
    ap.add_argument("--reference-hparams", action="store_true",
                    help="the reference's own BATCH_SIZE = 1024 and CAPACITY = 20,000 (src/train.py:63-65), one "
                         "update per step")
    ap.add_argument("--replay-every", type=int, default=1)
    ap.add_argument("--target-every", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save", default="")
    ap.add_argument("--obs-format", default="f32", choices=["f32", "u8f16"],
                    help="u8f16: uint8 state_m / float16 potential (the Brain converts on input)")
    ap.add_argument("--amp", action="store_true", help="Q-network forwards in bfloat16 autocast (Brain(amp=True))")
    ap.add_argument("--no-mfma", action="store_true",
                    help="with --amp: conv2-conv4 through MIOpen instead of the MFMA kernel (conv_mfma.py)")
    ap.add_argument("--channels-last", action="store_true", help="NHWC Q-networks (Brain(channels_last=True))")
    ap.add_argument("--input-channels", type=int, default=2,
                    help="map input (train.py:66-69): 2 = [older, newest], 1 = newest, 3 = newest + flow xy, "
                         "12 = (occupancy + RGB flow) x 3 steps (FFMPVec.bev_maps); with --temporal-maps: that many frames")
    ap.add_argument("--temporal-maps", action="store_true",
                    help="make_temporal_maps over --input-channels mono frames (train.py:474-486), from the frame ring")
    ap.add_argument("--warmup", type=int, default=3, help="untimed loop iterations (MIOpen compiles each conv shape once)")
    args = ap.parse_args()
    if args.reference_hparams:
        args.batch, args.capacity, args.replay_every = 1024, 20_000, 1

    dev = torch.device("cuda:0")
    # the reference map: 100x100 cells of 5 cm (ffmp.py:14-19), 200-step episodes (train.py:60)
    cfg = FFMPConfig(grid=100, n_obst=4, n_beams=180, moving=True, max_steps=200, seed=args.seed,
                     flow=args.input_channels in (3, 12) and not args.temporal_maps)
    # k + 1 slots: enough on a wrapping ring too (the fallback on devices without HIP VMM), which
    # holds W - 1 distinct frames once it has wrapped (FFMPVec.max_temporal_frames)
    window = max(args.input_channels + 1, 3) if args.temporal_maps else None
    env = FFMPVec(args.envs, cfg, device=dev, keep_terminal=True, obs_format=args.obs_format, frame_window=window,
                  bev_series=3 if args.input_channels == 12 and not args.temporal_maps else 0)
    brain = Brain(env, capacity=args.capacity, batch_size=args.batch, seed=args.seed, amp=args.amp,
                  mfma=False if args.no_mfma else None,
                  channels_last=args.channels_last, input_channels=args.input_channels,
                  temporal_maps=args.temporal_maps)
    obs = env.reset()
    tracker = EpisodeTracker(args.envs, device=dev)
    losses, updates = [], 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    t_warm = None
    for step in range(args.warmup + args.steps):
        if step == args.warmup:
            torch.cuda.synchronize()
            t_warm = time.perf_counter()
        action = brain.decide_action(obs, tracker.episode)
        brain.memory.push_begin()
        obs, reward, done, info = env.step(action)
        brain.memory.push_end(action)
        tracker.update_from(env)
        if step % args.replay_every == 0:
            loss = brain.replay()
            if loss is not None:
                updates += 1
                if updates % 20 == 1:
                    losses.append(float(loss))
                if updates % args.target_every == 0:
                    brain.update_target_q_network()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dt = t1 - t_warm
    env.check_errors()
    summ = tracker.summary()
    timed_updates = sum(1 for s in range(args.warmup, args.warmup + args.steps) if s % args.replay_every == 0)
    fl = conv_flops(cfg.grid, args.input_channels)
    # acting: one forward of every env per step; a replay: Q(s) main, Q(s') main and target
    # forwards of the batch, and the backward of Q(s) (data + weight gradients; conv1 has no data gradient)
    conv_flop = args.steps * args.envs * fl["forward"] + timed_updates * args.batch * (3 * fl["forward"] +
                                                                                      fl["backward"])
    out = {"env_steps_per_s": args.envs * args.steps / dt, "seconds": dt, "warmup_seconds": t_warm - t0,
           "updates_per_s": timed_updates / dt, "conv_tflops_per_s": conv_flop / dt / 1e12,
           "conv_gflop_per_sample": {k: round(v / 1e9, 3) for k, v in fl.items()},
           "envs": args.envs, "steps": args.steps, "amp": args.amp, "mfma": bool(brain.mfma and args.amp), "channels_last": args.channels_last,
           "input_channels": args.input_channels, "temporal_maps": args.temporal_maps,
           "learner_updates": updates, "batch": args.batch, "loss_samples": losses[:10],
           "replay_bytes": brain.memory.hbm_bytes(), "replay_len": len(brain.memory), **summ}
    print(json.dumps(out))
    if args.save:
        torch.save(brain.main_q_network.state_dict(), args.save)


if __name__ == "__main__":
    main()
