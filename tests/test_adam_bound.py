"""CPU: the teacher-forced Adam step bound (tests/adam_bound.py) that the GPU update tests use as
their bar.

Two torch CPU runs of the clipped-PPO update (uavhip.ppo.ppo_epochs, ppo.py:96-169) share the same
weights, Adam state and minibatches for k - 1 steps (bitwise identical so far); at step k the
second run's gradients are perturbed by up to 2e-5 of each tensor's max |grad| (below the GPU
gradient bar of 5e-5; independent random signs, worse than rounding). The step's parameter
difference stays inside the bound element for element, at t = 1 and at t = 4. The bound is not
vacuous: on most elements it is a small fraction of Adam's full step (lr), and a perturbation 100x
larger than the bound assumes breaks it."""
import copy

import pytest
import torch

from adam_bound import flatten_named, torch_adam_state, torch_step_bound, umax


def _bufs(n, g):
    states = torch.randn(n, 5, 14, generator=g) * 0.5
    states[: n // 3, :2] = 0
    acts = torch.randint(0, 2, (n,), generator=g)
    logp = -0.69 + 0.05 * torch.randn(n, generator=g)
    vals = torch.randn(n, generator=g)
    return states, acts, logp, vals, vals + 0.3 * torch.randn(n, generator=g), torch.randn(n, generator=g)


def test_umax_bounds_adam_step():
    assert umax(1, 0.9, 0.999) == pytest.approx(1.0)
    for t in (2, 4, 16, 100):
        assert 0.9 < umax(t, 0.9, 0.999) < 3.2


@pytest.mark.parametrize("k", [1, 4])
@pytest.mark.parametrize("scale,holds", [(2e-5, True), (1e-2, False)])
def test_step_bound_covers_perturbed_gradients(k, scale, holds):
    from uavhip.policy import TransformerActorCritic
    from uavhip.ppo import make_optimizer, ppo_epochs
    torch.manual_seed(3)
    ref = TransformerActorCritic()
    other = copy.deepcopy(ref)
    g = torch.Generator().manual_seed(4)
    bufs = _bufs(64 * k, g)
    perm = torch.randperm(64 * k, generator=g).tolist()
    opts = [make_optimizer(ref), make_optimizer(other)]
    if k > 1:  # identical history
        for net, opt in zip((ref, other), opts):
            ppo_epochs(net, opt, *bufs, epochs=1, batch_size=64, perms=[perm[:64 * (k - 1)]])
    p0, _ = flatten_named(ref.named_parameters())
    assert torch.equal(p0, flatten_named(other.named_parameters())[0])
    last = [perm[64 * (k - 1):]]
    ppo_epochs(ref, opts[0], *bufs, epochs=1, batch_size=64, perms=last)
    gen = torch.Generator().manual_seed(5)
    hooks = [p.register_hook(lambda grad: grad + (torch.rand(grad.shape, generator=gen) * 2 - 1) * scale *
                             grad.abs().max()) for p in other.parameters()]
    ppo_epochs(other, opts[1], *bufs, epochs=1, batch_size=64, perms=last)
    for h in hooks:
        h.remove()
    sb = torch_step_bound(ref, opts[0])
    t, gr, m, v = torch_adam_state(ref, opts[0])
    assert t == k
    got, _ = flatten_named(other.named_parameters())
    want, _ = flatten_named(ref.named_parameters())
    frac = float((sb.bound(t, gr, m, v) / sb.lr).median())
    print(f"t={t}: median bound / lr = {frac:.3e}")
    assert frac < 0.05  # not vacuous
    g_other = torch.cat([p.grad.reshape(-1) for p in other.parameters()])
    if holds:
        sb.check(t, gr, m, v, got, want, p0)  # the a-priori bound (rel = 1e-4 of max |g|)
        sb.check(t, gr, m, v, got, want, p0, g_other=g_other)  # the bound from the actual gradient difference
        sb.report()
    else:
        with pytest.raises(AssertionError):
            sb.check(t, gr, m, v, got, want, p0)
    # the actual-difference bound holds even for the large perturbation (the gradient bar is then
    # what catches it)
    with pytest.raises(AssertionError, match="gradient"):
        sb.check(t, gr, m, v, got, want, p0, g_other=g_other, grad_rel=scale / 10)
    sb.check(t, gr, m, v, got, want, p0, g_other=g_other, grad_rel=2 * scale)
