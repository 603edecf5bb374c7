"""How far can one Adam step of two implementations differ when their gradients differ only by
rounding? (Test infrastructure: the bar of the "HIP update vs torch update" step comparisons.)

torch.optim.Adam (agents/ppo.py:17-22, 153-169; torch's non-capturable formula) moves an element by
lr * u_t with u_t = m_hat_t / (s_t + eps), m_hat_t = m_t / (1 - b1^t), s_t = sqrt(v_t / (1 - b2^t)).
m_hat_t is a weighted MEAN of the (clipped) gradients g_1..g_t and s_t a weighted RMS of them; the
newest gradient's weights are w1 = (1 - b1) / (1 - b1^t) and w2 = (1 - b2) / (1 - b2^t). Teacher
forcing -- both sides enter step t with the same parameters and Adam moments, so only g_t differs,
by at most e per element -- gives |d m_hat_t| <= w1 e and |d s_t| <= sqrt(w2) e (the RMS is a
norm: triangle inequality), hence

    |d u_t| <= e (w1 + sqrt(w2) |u_t|) / (max(s_t - sqrt(w2) e, 0) + eps),

and never more than |u_t| + umax_t, where umax_t bounds |u| for ANY gradient sequence (Cauchy-Schwarz
on the two weighted sums; 1 at t = 1). The step's parameter difference is then at most lr times
that, plus the fp32 rounding of the update itself -- large where an element's gradient is small
against e (Adam normalises rounding noise up to a full lr-sized step: the in_proj key bias, whose
gradient softmax cancels exactly, is the extreme case), tiny where the gradient is large.

The in_proj key bias (in_proj_bias[D:2D] of every attention layer) gets a clause of its own: a
per-query constant added to every key's logit leaves softmax unchanged, so its gradient is zero in
exact arithmetic and BOTH sides' values are rounding noise of opposite sign as often as not. Adam
turns each into a step of up to lr * umax_t (at t = 1 exactly lr * sign(g)), so the two sides' steps
can differ by the full |u_t| + umax_t: the key-bias elements are checked against that cap and their
worst ratio is reported apart from every other element's (it sat at 0.97-0.99 of
the e-derived bound, which leaves no margin to read the rest of the step by).

The GPU tests give the bound the actual elementwise difference of the two sides' clipped gradients
of the step (and check that difference against the kernels' gradient bar separately), so the step
check is the update arithmetic against the gradients it was given; without a g_other, e is the
a-priori grad_error() below.

Without teacher forcing no such bound exists: an element Adam moved by a rounding-sized gradient
changes every later gradient (the feedback is first order through the Hessian, not negligible), so
multi-step comparisons are only meaningful between deterministic runs (measured + margin).

e comes from the gradient bar the kernels are tested to (tests/test_gpu_train.py: 5e-5 of each
tensor's max |grad|; measured <= 8.4e-6), used at twice that (rel = 1e-4), plus the clip
coefficient's error (clip_grad_norm_: the norm of the gradient error over the gradient's norm). The
reference side supplies g_t, m_t, v_t after its step."""
import math

import torch


def umax(t, b1, b2):
    """max |m_hat_t / s_t| over all gradient sequences (Adam's per-element step bound, in lr)."""
    r = b1 * b1 / b2
    geo = sum(r ** j for j in range(int(t)))
    return (1 - b1) / (1 - b1 ** t) * math.sqrt((1 - b2 ** t) / (1 - b2)) * math.sqrt(geo)


class AdamStepBound:
    """Per-element bound of one teacher-forced Adam step.

    segments: [(name, offset, numel)] of the parameter tensors in the flat vectors (per-tensor
    gradient maxima); lr: flat per-element learning rates."""

    def __init__(self, segments, lr, betas=(0.9, 0.999), eps=1e-8, rel=1e-4, abs_=1e-7, d_model=128):
        self.segs, self.lr = list(segments), lr.double()
        self.b1, self.b2, self.eps, self.rel, self.abs = betas[0], betas[1], eps, rel, abs_
        self.worst, self.worst_grad, self.worst_kb = {}, {}, {}
        self.d_model = d_model

    def key_bias(self, n):
        """Mask of the in_proj key-bias elements (in_proj_bias[D:2D], softmax-invariant) over a flat
        vector of n elements (flat buffers may pad between and after the tensors)."""
        kb = torch.zeros(n, dtype=torch.bool)
        for name, o, k in self.segs:
            if name.endswith("in_proj_bias"):
                assert k == 3 * self.d_model, (name, k)
                kb[o + self.d_model:o + 2 * self.d_model] = True
        return kb

    def grad_error(self, g):
        g = g.double().cpu()
        e = torch.zeros_like(g)
        err2 = 0.0
        for _, o, n in self.segs:
            d = self.rel * float(g[o:o + n].abs().max()) + self.abs
            e[o:o + n] = d
            err2 += n * d * d
        gn = float(g.norm())
        return e + g.abs() * (math.sqrt(err2) / gn if gn > 0 else 0.0)  # clip_grad_norm_ coefficient

    def bound(self, t, g, m, v, e=None):
        """The reference's state after its step t (1-based): clipped gradient g, exp_avg m,
        exp_avg_sq v; e: elementwise bound on how far the other side's g_t is off (default: the
        a-priori grad_error(g)) -> per-element bound on |d parameter| of this step."""
        g, m, v = g.double().cpu(), m.double().cpu(), v.double().cpu()
        e = self.grad_error(g) if e is None else e.double().cpu()
        w1 = (1 - self.b1) / (1 - self.b1 ** t)
        w2 = math.sqrt((1 - self.b2) / (1 - self.b2 ** t))
        s = (v / (1 - self.b2 ** t)).sqrt()
        u = (m / (1 - self.b1 ** t)) / (s + self.eps)
        du = e * (w1 + w2 * u.abs()) / ((s - w2 * e).clamp(min=0) + self.eps)
        du = torch.minimum(du, u.abs() + umax(t, self.b1, self.b2))
        return self.lr.cpu() * du

    def check(self, t, g, m, v, got, want, p_before, label="", g_other=None, grad_rel=5e-5):
        """|got - want| <= bound + fp32 rounding of both updates (2 ulp of the parameter before and
        after, 1e-6 lr), element by element; records the worst |d| / bound per tensor.
        g_other: the other side's clipped gradient of this step. Then (a) it must agree with g to
        grad_rel of each tensor's max |g| (the kernels' gradient bar) and (b) the bound is taken
        from the actual elementwise gradient difference (+ 1e-6 relative slack for the clip
        coefficient) -- the update arithmetic checked against the gradients it was given."""
        got, want, p0 = got.double().cpu(), want.double().cpu(), p_before.double().cpu()
        gd = g.double().cpu()
        e = None
        if g_other is not None:
            go = g_other.double().cpu()
            diff = (go - gd).abs()
            for name, o, n in self.segs:
                scale = float(gd[o:o + n].abs().max())
                err = float(diff[o:o + n].max())
                self.worst_grad[name] = max(self.worst_grad.get(name, 0.0), err / max(scale, 1e-30))
                assert err <= grad_rel * scale + 1e-7, f"{label} step {t} {name}: gradient |d| {err:.3e} vs max {scale:.3e}"
            e = diff + 1e-6 * gd.abs() + 1e-12
        b = self.bound(t, gd, m, v, e)
        # key bias: the cap for ANY gradient (its value is rounding noise on both sides)
        s_ = (v.double().cpu() / (1 - self.b2 ** t)).sqrt()
        u = (m.double().cpu() / (1 - self.b1 ** t)) / (s_ + self.eps)
        key_bias = self.key_bias(b.numel())
        b = torch.where(key_bias, self.lr.cpu() * (u.abs() + umax(t, self.b1, self.b2)), b)
        tol = b + 2.0 ** -22 * (want.abs() + p0.abs()) + 1e-6 * self.lr.cpu()
        d = (got - want).abs()
        ratio = d / tol
        for name, o, n in self.segs:
            kb = key_bias[o:o + n]
            r = ratio[o:o + n]
            self.worst[name] = max(self.worst.get(name, 0.0), float(r[~kb].max()))
            if bool(kb.any()):
                self.worst_kb[name] = max(self.worst_kb.get(name, 0.0), float(r[kb].max()))
            bad = d[o:o + n] > tol[o:o + n]
            if bool(bad.any()):
                i = o + int(bad.nonzero()[0])
                vs = float((v.double().cpu()[i] / (1 - self.b2 ** t)) ** 0.5)
                raise AssertionError(f"{label} step {t} {name}[{i - o}]: |d| {float(d[i]):.3e} > bound {float(tol[i]):.3e} "
                                     f"({int(bad.sum())} elements over; g {float(gd[i]):.3e}, s {vs:.3e}, "
                                     f"m {float(m[i]):.3e}, e {float(e[i]) if e is not None else float('nan'):.3e})")
        return tol

    def report(self):
        """Prints the worst |d| / bound over every element but the key biases, the key biases' own
        worst against their cap, and the gradient agreement; returns the first."""
        k = max(self.worst, key=self.worst.get)
        msg = f"Adam step: max |d| / bound = {self.worst[k]:.3e} ({k}; key biases excluded)"
        if self.worst_kb:
            kk = max(self.worst_kb, key=self.worst_kb.get)
            msg += f"; key bias (softmax-invariant, cap |u| + umax) max |d| / cap = {self.worst_kb[kk]:.3e} ({kk})"
        if self.worst_grad:
            kg = max(self.worst_grad, key=self.worst_grad.get)
            msg += f"; max gradient |d| / max |g| = {self.worst_grad[kg]:.3e} ({kg})"
        print(msg)
        return self.worst[k]


def flatten_named(params):
    """[(name, tensor)] -> (flat float64 tensor, [(name, offset, numel)])."""
    segs, flat, o = [], [], 0
    for k, p in params:
        n = p.numel()
        segs.append((k, o, n))
        flat.append(p.detach().reshape(-1).double())
        o += n
    return torch.cat(flat), segs


def torch_adam_state(policy, optimizer):
    """(t, flat clipped grad, flat exp_avg, flat exp_avg_sq) of a torch.optim.Adam right after its
    step, parameters in named_parameters order."""
    named = list(policy.named_parameters())
    st = [optimizer.state[p] for _, p in named]
    t = int(float(st[0]["step"]))
    g = torch.cat([p.grad.reshape(-1) for _, p in named])
    m = torch.cat([s["exp_avg"].reshape(-1) for s in st])
    v = torch.cat([s["exp_avg_sq"].reshape(-1) for s in st])
    return t, g, m, v


def torch_step_bound(policy, optimizer, **kw):
    named = list(policy.named_parameters())
    lr_of = {}
    for gr in optimizer.param_groups:
        for p in gr["params"]:
            lr_of[p] = gr["lr"]
    _, segs = flatten_named(named)
    lr = torch.cat([torch.full((p.numel(),), float(lr_of[p]), dtype=torch.float64) for _, p in named])
    gr = optimizer.param_groups[0]
    return AdamStepBound(segs, lr, betas=gr["betas"], eps=gr["eps"], **kw)


def trainer_step_bound(trainer, **kw):
    """AdamStepBound over FusedPPOTrainer flat buffers (after an UPDATE, grads holds the clipped
    gradient Adam consumed; state = (adam_step, grads, adam_m, adam_v))."""
    from uavhip.policy import layout
    offs, n = layout()
    named = list(trainer.policy.state_dict().items())
    segs = [(k, o, v.numel()) for (k, v), o in zip(named, offs)]
    d = trainer.desc
    lr = torch.full((n,), float(d.lr_critic), dtype=torch.float64)
    critic0 = min(o for k, o, _ in segs if k.startswith("critic"))
    lr[:critic0] = float(d.lr_actor)
    return AdamStepBound(segs, lr, betas=(d.beta1, d.beta2), eps=d.adam_eps, **kw)
