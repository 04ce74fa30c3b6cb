"""Batched learner (learner.Brain) on env tensors: one replay() update equals the reference
Brain's arithmetic (src/train.py:352-428, restated below on copies of the networks), and
decide_action follows the epsilon-greedy rule of :337-349.  The reference Brain itself needs
CUDA tensor types (torch.cuda.ByteTensor / LongTensor), so it is not run here: this
parity is against its restated formulas."""
import copy

import pytest
import torch
import torch.nn as nn

from flow_field_based_motion_planner_amd import FFMPConfig
from flow_field_based_motion_planner_amd.learner import Brain
from flow_field_based_motion_planner_amd.vec_env import FFMPVec

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _env(n=32):
    cfg = FFMPConfig(grid=100, n_obst=4, n_beams=64, moving=True, max_steps=6, seed=31)
    env = FFMPVec(n, cfg, device=DEV, keep_terminal=True)
    env.reset()
    return env


def _fill(brain, env, steps):
    g = torch.Generator(device="cpu").manual_seed(0)
    for _ in range(steps):
        brain.memory.push_begin()
        a = torch.randint(0, 28, (env.num_envs,), generator=g).to(DEV)
        env.step(a)
        brain.memory.push_end(a)


def test_replay_update_matches_reference_formulas():
    env = _env()
    brain = Brain(env, capacity=256, batch_size=48, seed=3)
    assert brain.replay() is None  # train.py:319-320: not enough memory yet
    _fill(brain, env, 3)
    idx = torch.randperm(len(brain.memory), device=DEV)[:48]
    main0 = copy.deepcopy(brain.main_q_network)
    targ0 = copy.deepcopy(brain.target_q_network)
    opt0 = torch.optim.Adam(main0.parameters(), lr=0.0005)
    b, ex = brain.memory.sample(48, index=idx)
    b = type(b)(*[t.clone() for t in b])
    loss = brain.replay(index=idx)
    # reference arithmetic (get_expected_state_action_values + update_main_q_network)
    main0.eval()
    targ0.eval()
    sav = main0(b.state_m, b.state_g, b.state_v, b.state_t).gather(1, b.action)
    a_m = main0(b.observe_m, b.observe_g, b.observe_v, b.observe_t).detach().max(1)[1].view(-1, 1)
    nxt = targ0(b.observe_m, b.observe_g, b.observe_v, b.observe_t).gather(1, a_m).detach().squeeze()
    expected = (b.reward.cpu() + 0.95 * nxt.cpu()).to(DEV)
    main0.train()
    ref_loss = nn.MSELoss()(sav, expected.unsqueeze(1))
    opt0.zero_grad()
    ref_loss.backward()
    opt0.step()
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=1e-5, atol=1e-5)
    # gradients agree to float32 reduction-order noise (MIOpen may pick different backward
    # algorithms for two identical calls); Adam's first step moves every parameter by at most
    # ~lr in the direction of sign(grad), so parameters agree within 2*lr and mostly far closer
    for (k, p), (_, q) in zip(brain.main_q_network.named_parameters(), main0.named_parameters()):
        gmax = float(q.grad.abs().max())
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-3, atol=1e-4 * gmax + 1e-12, msg=k)
        d = (p - q).detach().abs()
        assert float(d.max()) <= 2 * 0.0005 + 1e-6, k
        assert float((d <= 1e-6).float().mean()) > 0.9, k
    brain.update_target_q_network()
    for p, q in zip(brain.main_q_network.parameters(), brain.target_q_network.parameters()):
        assert torch.equal(p, q)


def test_decide_action_epsilon_greedy():
    env = _env(256)
    brain = Brain(env, capacity=512, batch_size=32, seed=4)
    obs = env.obs
    brain.main_q_network.eval()
    with torch.no_grad():
        greedy = torch.cat([brain.main_q_network(obs["state_m"][i:i + 1], obs["state_g"][i:i + 1],
                                                 obs["state_v"][i:i + 1], obs["state_t"][i:i + 1]).max(1)[1]
                            for i in range(256)])
    late = brain.decide_action(obs, torch.full((256,), 10 ** 9, device=DEV))
    assert torch.equal(late, greedy)  # epsilon ~ 0: always greedy, per-env B=1 semantics
    first = brain.decide_action(obs, torch.zeros(256, dtype=torch.int32, device=DEV))  # epsilon 0.5
    frac = float((first != greedy).float().mean())
    assert 0.3 < frac < 0.65 and first.dtype == torch.int64 and int(first.max()) < 28


@pytest.mark.parametrize("mfma", [True, False])
def test_amp_update_close_to_fp32(mfma):
    """Brain(amp=True): the same update with the Q-network forwards in bfloat16 autocast — conv2-4
    on the MFMA kernel (mfma=True, the default with amp) or MIOpen — loss within bf16 rounding of
    the fp32 update's on the same minibatch and weights, every parameter moved by Adam (fp32
    master weights), valid greedy actions."""
    env = _env()
    b32 = Brain(env, capacity=256, batch_size=48, seed=3)
    b16 = Brain(env, capacity=256, batch_size=48, seed=3, amp=True, mfma=mfma)
    assert b16.main_q_network.mfma == mfma
    b16.memory = b32.memory
    _fill(b32, env, 3)
    idx = torch.randperm(len(b32.memory), device=DEV)[:48]
    before = [p.detach().clone() for p in b16.main_q_network.parameters()]
    l32 = b32.replay(index=idx)
    l16 = b16.replay(index=idx)
    assert torch.isfinite(l16) and l16.dtype == torch.float32
    torch.testing.assert_close(l16, l32, rtol=5e-2, atol=5e-3)
    for p, q in zip(b16.main_q_network.parameters(), before):
        assert p.dtype == torch.float32 and not torch.equal(p, q)
    obs = env.obs
    a32 = b32.decide_action(obs, torch.full((env.num_envs,), 10 ** 9, device=DEV))
    a16 = b16.decide_action(obs, torch.full((env.num_envs,), 10 ** 9, device=DEV))
    assert a16.dtype == torch.int64 and int(a16.max()) < 28


@pytest.mark.parametrize("channels", [1, 3])
def test_replay_with_other_input_channels(channels):
    """Brain(input_channels=1 | 3): train.py:66-68's other map inputs (newest frame; newest frame +
    flow xy from the env's flow planes, replayed from the records) — one update equals the restated
    reference arithmetic on the same assembled inputs."""
    from flow_field_based_motion_planner_amd.network import map_channels
    cfg = FFMPConfig(grid=100, n_obst=4, n_beams=64, moving=True, max_steps=6, seed=32, flow=channels == 3)
    env = FFMPVec(32, cfg, device=DEV, keep_terminal=True)
    env.reset()
    brain = Brain(env, capacity=256, batch_size=48, seed=5, input_channels=channels)
    assert brain.main_q_network.conv1.in_channels == channels
    _fill(brain, env, 3)
    idx = torch.randperm(len(brain.memory), device=DEV)[:48]
    main0 = copy.deepcopy(brain.main_q_network)
    targ0 = copy.deepcopy(brain.target_q_network)
    b, ex = brain.memory.sample(48, index=idx)
    s_in = map_channels(b.state_m, ex.get("flow"), channels).clone()
    o_in = map_channels(b.observe_m, ex.get("observe_flow"), channels).clone()
    b = type(b)(*[t.clone() for t in b])
    loss = brain.replay(index=idx)
    main0.eval()
    targ0.eval()
    sav = main0(s_in, b.state_g, b.state_v, b.state_t).gather(1, b.action)
    a_m = main0(o_in, b.observe_g, b.observe_v, b.observe_t).detach().max(1)[1].view(-1, 1)
    nxt = targ0(o_in, b.observe_g, b.observe_v, b.observe_t).gather(1, a_m).detach().squeeze()
    ref_loss = nn.MSELoss()(sav, (b.reward + 0.95 * nxt).unsqueeze(1))
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=1e-5, atol=1e-5)
    a = brain.decide_action(env.obs, torch.zeros(32, dtype=torch.int32, device=DEV))
    assert a.shape == (32,) and int(a.max()) < 28


@pytest.mark.parametrize("amp", [False, True])
def test_temporal_maps_input(amp):
    """Brain(temporal_maps=True, input_channels=3): make_temporal_maps' code path for a mono BEV
    image (train.py:474-486, INPUT_CHANNELS frames): acting on env.temporal_maps(3), replaying
    3-frame series; one update equals the restated reference arithmetic on the sampled series
    (amp: the MFMA path, conv1's 3 channels folded with a zero fourth, within bf16 bounds)."""
    cfg = FFMPConfig(grid=100, n_obst=4, n_beams=64, moving=True, max_steps=6, seed=33)
    env = FFMPVec(32, cfg, device=DEV, keep_terminal=True, frame_window=4)
    env.reset()
    brain = Brain(env, capacity=256, batch_size=48, seed=6, input_channels=3, temporal_maps=True, amp=amp)
    assert brain.main_q_network.conv1.in_channels == 3 and brain.memory.series == 3
    _fill(brain, env, 4)
    idx = torch.randperm(len(brain.memory), device=DEV)[:48]
    main0 = copy.deepcopy(brain.main_q_network)
    targ0 = copy.deepcopy(brain.target_q_network)
    b, ex = brain.memory.sample(48, index=idx)
    assert b.state_m.shape == (48, 3, 100, 100)
    b = type(b)(*[t.clone() for t in b])
    loss = brain.replay(index=idx)
    main0.eval()
    targ0.eval()
    with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=amp):
        sav = main0(b.state_m, b.state_g, b.state_v, b.state_t).float().gather(1, b.action)
        a_m = main0(b.observe_m, b.observe_g, b.observe_v, b.observe_t).float().detach().max(1)[1].view(-1, 1)
        nxt = targ0(b.observe_m, b.observe_g, b.observe_v, b.observe_t).float().gather(1, a_m).detach().squeeze()
    ref_loss = nn.MSELoss()(sav, (b.reward + 0.95 * nxt).unsqueeze(1))
    tol = 2e-2 if amp else 1e-5
    torch.testing.assert_close(loss, ref_loss.detach(), rtol=tol, atol=tol)
    a = brain.decide_action(env.obs, torch.zeros(32, dtype=torch.int32, device=DEV))
    assert a.shape == (32,) and int(a.max()) < 28
    with pytest.raises(ValueError):
        Brain(env, capacity=256, input_channels=5, temporal_maps=True)  # more frames than the window


def test_amp_at_a_grid_outside_the_kernels_falls_back_per_layer():
    """Brain(amp=True) at G = 96 (the reference's Network accepts G > 90): the third conv4's weight
    gradient would have output rows of 6 < 8 positions, which the MFMA weight-gradient kernel does
    not take (ffmp_conv2d_check) — that layer runs F.relu(conv(x)) under autocast, the others stay
    on the matrix-core kernels, and the update completes (it raised FFMPBackendError before)."""
    from flow_field_based_motion_planner_amd import conv_mfma
    cfg = FFMPConfig(grid=96, n_obst=4, n_beams=64, moving=True, max_steps=6, seed=32)
    env = FFMPVec(32, cfg, device=DEV, keep_terminal=True)
    env.reset()
    b16 = Brain(env, capacity=128, batch_size=32, seed=5, amp=True)
    b32 = Brain(env, capacity=128, batch_size=32, seed=5)
    b16.memory = b32.memory
    _fill(b32, env, 2)
    calls = []
    real = conv_mfma.conv_relu

    def counting(conv, x):
        calls.append(tuple(x.shape))
        return real(conv, x)

    conv_mfma.conv_relu = counting
    try:
        idx = torch.arange(32, device=DEV)
        l16 = b16.replay(index=idx)
        l32 = b32.replay(index=idx)
    finally:
        conv_mfma.conv_relu = real
    assert torch.isfinite(l16)
    torch.testing.assert_close(l16, l32, rtol=5e-2, atol=5e-3)
    sides = sorted({s[2] for s in calls})
    assert {65, 34, 27, 20} <= set(sides) and 13 not in sides, sides  # conv2, conv3, conv4 x2 on MFMA
    assert not conv_mfma.supported(b16.main_q_network.conv4, (32, 64, 13, 13))


def test_amp_mfma_forward_tracks_fused_adam_updates():
    """fused Adam writes the weights without bumping _version, so the MFMA
    convolutions' cached bf16 packs went stale after the first update.  After two replay() updates
    under amp + mfma, the next MFMA conv forward must equal F.conv2d on the CURRENT weights (bf16
    autocast) — not on the initial ones."""
    import torch.nn.functional as F
    from flow_field_based_motion_planner_amd import conv_mfma
    env = _env()
    brain = Brain(env, capacity=256, batch_size=48, seed=7, amp=True, lr=5e-3)
    _fill(brain, env, 3)
    net = brain.main_q_network
    w0 = net.conv2.weight.detach().clone()
    x = torch.rand(4, 32, 69, 69, device=DEV)
    for _ in range(2):
        brain.replay(index=torch.randperm(len(brain.memory), device=DEV)[:48])
    torch.cuda.synchronize()
    assert not torch.equal(net.conv2.weight, w0)
    with torch.no_grad(), torch.autocast(device_type="cuda", dtype=torch.bfloat16):
        got = conv_mfma.conv_relu(net.conv2, x).float()
        ref = F.relu(F.conv2d(x, net.conv2.weight, net.conv2.bias)).float()
        stale = F.relu(F.conv2d(x, w0, net.conv2.bias)).float()
    scale = float(ref.abs().max()) + 1e-6
    err = float((got - ref).abs().max()) / scale
    err_stale = float((got - stale).abs().max()) / scale
    assert err < 2e-2, (err, err_stale)
    assert err < err_stale
