"""ORACLE (test infrastructure): explicit torch-fp32 restatement of networks/transformer_net.py.

Written as plain tensor algebra (no nn.TransformerEncoderLayer) so it is an independent
check of both the reference (pinned against tests/golden/policy.npz) and the HIP kernel:
  TransformerBlock.forward        transformer_net.py:47-64
    mask = (|x|.sum(-1) == 0); mask[:, -1] = False          (key padding mask)
    h = relu(x W_e^T + b_e) + pos[:, :S]
    post-LN encoder layer (nn.TransformerEncoderLayer defaults, norm_first=False, relu,
    dropout 0, LN eps 1e-5, 8 heads x 16, scale 1/sqrt(16)):
        h = LN1(h + MHA(h)),  h = LN2(h + W2 relu(W1 h + b1) + b2)
  get_action / evaluate           transformer_net.py:96-144 (last token -> MLP heads)
Weights are the reference state_dict (50 keys, transformer_net.py state_dict naming).
"""
import math

import torch

EPS = 1e-5
HEADS = 8


def _ln(x, w, b):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + EPS) * w + b


def block(sd, prefix, x, nlayers):
    B, S, _ = x.shape
    mask = x.abs().sum(-1) == 0
    mask[:, -1] = False
    h = torch.relu(x @ sd[f"{prefix}.embedding.0.weight"].T + sd[f"{prefix}.embedding.0.bias"])
    h = h + sd[f"{prefix}.pos_embedding"][:, :S, :]
    D = h.shape[-1]
    hd = D // HEADS
    bias = torch.zeros(B, 1, 1, S, dtype=h.dtype)
    bias = bias.masked_fill(mask[:, None, None, :], float("-inf"))
    for l in range(nlayers):
        p = f"{prefix}.transformer.layers.{l}"
        qkv = h @ sd[f"{p}.self_attn.in_proj_weight"].T + sd[f"{p}.self_attn.in_proj_bias"]
        q, k, v = qkv.split(D, dim=-1)
        q = q.view(B, S, HEADS, hd).transpose(1, 2)
        k = k.view(B, S, HEADS, hd).transpose(1, 2)
        v = v.view(B, S, HEADS, hd).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(hd) + bias
        a = torch.softmax(s, dim=-1) @ v
        a = a.transpose(1, 2).reshape(B, S, D)
        a = a @ sd[f"{p}.self_attn.out_proj.weight"].T + sd[f"{p}.self_attn.out_proj.bias"]
        h = _ln(h + a, sd[f"{p}.norm1.weight"], sd[f"{p}.norm1.bias"])
        f = torch.relu(h @ sd[f"{p}.linear1.weight"].T + sd[f"{p}.linear1.bias"])
        f = f @ sd[f"{p}.linear2.weight"].T + sd[f"{p}.linear2.bias"]
        h = _ln(h + f, sd[f"{p}.norm2.weight"], sd[f"{p}.norm2.bias"])
    return h


def heads(sd, x):
    """-> logits [B,2], value [B] (fp32)."""
    ha = block(sd, "actor_net", x, 1)[:, -1, :]
    logits = torch.relu(ha @ sd["actor_head.0.weight"].T + sd["actor_head.0.bias"])
    logits = logits @ sd["actor_head.2.weight"].T + sd["actor_head.2.bias"]
    hc = block(sd, "critic_net", x, 2)[:, -1, :]
    value = torch.relu(hc @ sd["critic_head.0.weight"].T + sd["critic_head.0.bias"])
    value = value @ sd["critic_head.2.weight"].T + sd["critic_head.2.bias"]
    return logits, value[:, 0]


def evaluate(sd, x, actions):
    """-> logp(a), value, entropy, logits (Categorical(softmax(logits)))."""
    with torch.no_grad():
        logits, value = heads(sd, x)
        logp_all = torch.log_softmax(logits, dim=-1)
        p = logp_all.exp()
        logp = logp_all.gather(1, actions.view(-1, 1).long())[:, 0]
        ent = -(p * logp_all).sum(-1)
    return logp, value, ent, logits


def state_dict_from_npz(npz, tag):
    pre = f"{tag}/w/"
    return {k[len(pre):]: torch.from_numpy(npz[k].copy()) for k in npz.files if k.startswith(pre)}
