"""Policy checkpoints in the reference's format: `torch.save(policy.state_dict(), path)`
(main_train.py:209-212, 231-232), read back by `torch.load` + `load_state_dict`
(test_visualize.py:21-22). The HIP policy keeps the reference's parameter names, so files of the
current architecture load strictly and are fragment-packed for the kernels on the next call
(TransformerActorCritic.packed_weights keys the pack on the parameters' versions).

The four `saved_models/*/best_model.pth` files shipped with the reference come from older
architectures (SURVEY.md §2, row saved_models; §8(f) row 3) and do not load strictly into the
current model -- not into the reference's own either:

    arch            actor / critic layers   pos_embedding   head input         parameters
    current         1 / 2                   yes             last token (128)   419,267
    actor2          2 / 2                   yes             last token (128)   551,747
    flat640         2 / 2                   no              5 x 128 flattened  616,003

`load_checkpoint(..., strict=False)` loads what matches in name and shape (torch's own
`strict=False` raises on a shape mismatch; here mismatched tensors are skipped and reported) and
returns a report naming the rest, so such a file can be inspected or partially reused. Files are
always read with `torch.load(weights_only=True)`: nothing in them is executed.
"""
import os
from dataclasses import dataclass, field

import torch

# (actor layers, critic layers, pos_embedding, head input width) -> architecture name
_ARCHS = {(1, 2, True, 128): "current", (2, 2, True, 128): "actor2", (2, 2, False, 640): "flat640"}


@dataclass
class LoadReport:
    arch: str                       # "current", "actor2", "flat640" or "unknown"
    params: int                     # parameters in the file
    loaded: list = field(default_factory=list)       # keys copied into the policy
    missing: list = field(default_factory=list)      # policy keys the file lacks
    unexpected: list = field(default_factory=list)   # file keys the policy lacks
    mismatched: list = field(default_factory=list)   # (key, file shape, policy shape)

    @property
    def complete(self):
        return not (self.missing or self.unexpected or self.mismatched)


def _layers(sd, trunk):
    idx = {int(k.split(".layers.")[1].split(".")[0]) for k in sd if k.startswith(f"{trunk}.transformer.layers.")}
    return max(idx) + 1 if idx else 0


def describe(state_dict):
    """Architecture of a reference-format state_dict: (name, fields) with fields actor_layers,
    critic_layers, pos_embedding, head_in, params."""
    sd = state_dict
    head = sd.get("actor_head.0.weight")
    f = {"actor_layers": _layers(sd, "actor_net"), "critic_layers": _layers(sd, "critic_net"),
         "pos_embedding": "actor_net.pos_embedding" in sd and "critic_net.pos_embedding" in sd,
         "head_in": int(head.shape[1]) if head is not None else 0,
         "params": int(sum(v.numel() for v in sd.values()))}
    key = (f["actor_layers"], f["critic_layers"], f["pos_embedding"], f["head_in"])
    return _ARCHS.get(key, "unknown"), f


def read_checkpoint(path):
    """The state_dict in a checkpoint file, on the CPU, without executing anything in the file."""
    if not os.path.isfile(path):
        raise FileNotFoundError(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(sd, dict) or not all(isinstance(v, torch.Tensor) for v in sd.values()):
        raise ValueError(f"{path}: not a state_dict of tensors (main_train.py:211 saves policy.state_dict())")
    return sd


def save_checkpoint(policy, path):
    """main_train.py:211 / :232 -- the reference's format (the policy's state_dict, nothing else)."""
    torch.save(policy.state_dict(), path)


def load_checkpoint(policy, source, strict=True):
    """Load a checkpoint file (or a state_dict) into a TransformerActorCritic.

    strict=True: the outcome of torch's `load_state_dict` (test_visualize.py:22): any missing,
    unexpected or mis-shaped key raises RuntimeError -- checked before anything is copied, so a
    refused file leaves the policy as it was (torch copies the matching tensors, then raises).
    strict=False: copies every tensor whose name and shape match, skips the rest; returns the
    LoadReport either way."""
    sd = read_checkpoint(source) if isinstance(source, (str, os.PathLike)) else source
    arch, f = describe(sd)
    own = policy.state_dict()
    rep = LoadReport(arch=arch, params=f["params"])
    rep.missing = [k for k in own if k not in sd]
    rep.unexpected = [k for k in sd if k not in own]
    rep.mismatched = [(k, tuple(sd[k].shape), tuple(own[k].shape)) for k in sd
                      if k in own and sd[k].shape != own[k].shape]
    if strict:
        if not rep.complete:
            raise RuntimeError(f"Error(s) in loading state_dict for {type(policy).__name__} ({arch} checkpoint, "
                               f"{rep.params} parameters): missing keys {rep.missing}, unexpected keys "
                               f"{rep.unexpected}, size mismatches {rep.mismatched}")
        policy.load_state_dict(sd, strict=True)
        rep.loaded = list(own)
        return rep
    bad = {k for k, _, _ in rep.mismatched}
    sub = {k: v for k, v in sd.items() if k in own and k not in bad}
    policy.load_state_dict(sub, strict=False)
    rep.loaded = list(sub)
    return rep
