"""Pin the PPO update (agents/ppo.py:68-181) to the reference's own run: tests/golden/ppo_update.npz
was made by tests/golden/make_golden.py calling the reference's PPOAgent.update() on a 192-transition
buffer (5 episodes), with the sampler's permutations recorded (torch.manual_seed(1234) before
update(): SubsetRandomSampler draws torch.randperm(192) once per epoch and nothing else in update()
consumes the CPU RNG -- dropout is 0). It holds the weights before (w0) and after (w1) the update
and the mean losses over its 15 minibatch steps.

CPU: the torch restatement (uavhip.ppo.ppo_epochs on the drop-in module's forward, the reference's
GAE restated op for op) replaying the recorded permutations reproduces the reference's losses and
final weights bit for bit (the same torch CPU kernels run the same ops in the same order). The HIP training step is pinned to the same fixture in
tests/test_gpu_train.py::test_fused_update_replays_reference_update."""
import numpy as np
import torch

from conftest import load_golden


def reference_gae(rewards, dones, values, gamma=0.998, lam=0.95):
    """ppo.py:70-94 op for op (0-dim fp32 torch ops, Python-float rewards), CPU."""
    values = torch.from_numpy(np.asarray(values, np.float32))
    next_values = torch.cat([values[1:], torch.tensor([0.0])])
    gae, returns = 0, []
    for step in reversed(range(len(rewards))):
        done = bool(dones[step])
        v_next = next_values[step] if not done else 0.0
        delta = float(rewards[step]) + gamma * v_next - values[step]
        gae = delta + gamma * lam * gae * (1.0 - float(done))
        returns.insert(0, gae + values[step])
    returns = torch.tensor(returns, dtype=torch.float32)
    adv = returns - values
    return returns, (adv - adv.mean()) / (adv.std() + 1e-7)


def fixture_policy(f, key="w0"):
    from uavhip.policy import TransformerActorCritic
    net = TransformerActorCritic()
    net.load_state_dict({k[len(key) + 1:]: torch.from_numpy(f[k].copy()) for k in f.files if k.startswith(key + "/")})
    return net


def test_gae_restatement_matches_oracle():
    from oracle import gae as ogae
    f = load_golden("ppo_update.npz")
    ret, adv = reference_gae(f["rewards"], f["dones"], f["values"])
    r_o, a_o = ogae.gae_1d(f["rewards"], f["dones"], f["values"])
    np.testing.assert_array_equal(ret.numpy(), r_o)   # the oracle's bit-exact returns (gae.npz)
    np.testing.assert_allclose(adv.numpy(), ogae.normalize(a_o)[0], rtol=1e-5, atol=2e-6)


def test_torch_update_replays_reference_update():
    from uavhip.ppo import make_optimizer, ppo_epochs
    f = load_golden("ppo_update.npz")
    torch.manual_seed(0)
    net = fixture_policy(f)
    opt = make_optimizer(net)
    ret, adv = reference_gae(f["rewards"], f["dones"], f["values"])
    values = torch.from_numpy(f["values"])
    sa, sc, se, n = ppo_epochs(net, opt, torch.from_numpy(f["states"]), torch.from_numpy(f["actions"]),
                               torch.from_numpy(f["logprobs"]), values, ret, adv, perms=f["perms"])
    assert n == 5 * (192 // 64)
    got = np.array([sa, sc, se])
    want = np.array([f["loss_actor"], f["loss_critic"], f["entropy"]], dtype=np.float64)
    print("losses |d|:", np.abs(got - want))
    np.testing.assert_array_equal(got, want)
    worst = 0.0
    for k, v in net.state_dict().items():
        w1 = f["w1/" + k]
        d = float(np.abs(v.numpy() - w1).max())
        worst = max(worst, d)
        assert d == 0.0, (k, d)
    print(f"max |w1 - reference w1| = {worst:.3e}")
    # the update moved the weights by many times the bar
    moved = max(float(np.abs(f["w1/" + k] - f["w0/" + k]).max()) for k in net.state_dict())
    assert moved > 1e-3
