"""The N>1 path on the GPU: two ranks (one process each, gloo — RCCL refuses two ranks on one
device, and the box has one) each step their own FFMPVec shard on cuda:0, keyed by global env
index, and all-gather the rollout scalars and per-env plane checksums with
distributed.gather_rollout / gather_env_rows.  The gathered result must equal ONE process stepping
every env, bit for bit: rewards, flags, and checksums of state_m (both frames), the potential
plane (bit patterns), the lidar and the raster record.  The shards are uneven (514 + 513 envs of
the C3 geometry) and use the seamless frame ring, like bench.py's ranks.  The reference has no
distribution at all: it runs one env on one device (/root/reference/src/train.py:43)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flow_field_based_motion_planner_amd.config import preset
from flow_field_based_motion_planner_amd.distributed import gather_env_rows, gather_rollout, shard_range

pytestmark = pytest.mark.gpu

TOTAL, STEPS = 1027, 12


def _cfg():
    return preset("C3", max_steps=5, seed=77)


def _actions():
    return np.random.default_rng(3).integers(0, 28, (STEPS, TOTAL))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _checksums(env) -> torch.Tensor:
    """(n, 4) int64 per env: sum of state_m cells (0/255), sums of the potential's, the lidar's and
    the record's float32 bit patterns (as int64, so any changed bit changes the sum)."""
    n = env.num_envs
    sm = env.state_m.reshape(n, -1).to(torch.int64).sum(1)
    pot = env.potential.reshape(n, -1).view(torch.int32).to(torch.int64).sum(1)
    lid = env.lidar.view(torch.int32).to(torch.int64).sum(1)
    rec = env.record.view(torch.int32).to(torch.int64).sum(1)
    return torch.stack([sm, pot, lid, rec], 1)


def _worker(rank, world, port, out_dir):
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    off, cnt = shard_range(TOTAL, world, rank)
    env = FFMPVec(cnt, _cfg(), device="cuda:0", env_offset=off, frame_window=8, seamless=True, autotune=False)
    env.reset()
    acts = torch.as_tensor(_actions(), device="cuda:0")
    rew, done, goal, cs = [], [], [], []
    for s in range(STEPS):
        env.step(acts[s, off:off + cnt])
        g = gather_rollout(env.reward, env.done, env.is_goal, total=TOTAL)
        assert g["reward"].device.type == "cuda"
        rew.append(g["reward"].cpu().numpy())
        done.append(g["done"].cpu().numpy())
        goal.append(g["is_goal"].cpu().numpy())
        cs.append(gather_env_rows(_checksums(env), total=TOTAL).cpu().numpy())
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"), rew=np.stack(rew), done=np.stack(done), goal=np.stack(goal),
                 cs=np.stack(cs), ring=np.array([env.ring == "seamless"]))
    dist.barrier()
    env.close()
    dist.destroy_process_group()


def test_two_gpu_ranks_equal_one_process(tmp_path):
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "dist.npz")
    assert bool(got["ring"][0])
    env = FFMPVec(TOTAL, _cfg(), device="cuda:0", frame_window=8, seamless=True, autotune=False)
    env.reset()
    acts = torch.as_tensor(_actions(), device="cuda:0")
    for s in range(STEPS):
        env.step(acts[s])
        assert np.array_equal(got["rew"][s], env.reward.cpu().numpy()), s
        assert np.array_equal(got["done"][s], env.done.cpu().numpy()), s
        assert np.array_equal(got["goal"][s], env.is_goal.cpu().numpy()), s
        assert np.array_equal(got["cs"][s], _checksums(env).cpu().numpy()), s
    assert got["done"].any()
    env.close()
