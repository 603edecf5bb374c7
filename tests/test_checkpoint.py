"""Checkpoint format (main_train.py:209-212, 231-232; test_visualize.py:21-22):
the reference's torch.save(state_dict) files round-trip through the HIP policy, and the older
architectures of saved_models/*/best_model.pth are recognised, refused by a strict load and
partially loaded with a report by a non-strict one. CPU, and one GPU test of the repack."""
import glob
import os

import pytest
import torch

from uavhip.checkpoint import describe, load_checkpoint, read_checkpoint, save_checkpoint
from uavhip.policy import TransformerActorCritic

REF_MODELS = "/root/reference/saved_models"


def _legacy(kind, seed=3):
    """A state_dict of an older architecture, built from the current one's tensors: `actor2` adds a
    second actor encoder layer; `flat640` also drops the position embeddings and widens the head
    inputs to the flattened 5 x 128 window."""
    torch.manual_seed(seed)
    sd = dict(TransformerActorCritic().state_dict())
    pre = "actor_net.transformer.layers."
    for k in [k for k in sd if k.startswith(pre + "0.")]:
        sd[k.replace(pre + "0.", pre + "1.")] = sd[k].clone() + 0.5
    if kind == "flat640":
        for t in ("actor_net", "critic_net"):
            del sd[f"{t}.pos_embedding"]
        for h in ("actor_head", "critic_head"):
            sd[f"{h}.0.weight"] = torch.randn(64, 640)
    return sd


def test_round_trip_is_exact(tmp_path):
    torch.manual_seed(1)
    a = TransformerActorCritic()
    torch.manual_seed(2)
    b = TransformerActorCritic()
    path = str(tmp_path / "best_model.pth")
    save_checkpoint(a, path)
    rep = load_checkpoint(b, path)
    assert rep.arch == "current" and rep.complete and rep.params == 419267
    for (k, va), (_, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(va, vb), k
    # the file is exactly what the reference saves: a plain state_dict, readable without pickled code
    sd = torch.load(path, map_location="cpu", weights_only=True)
    assert list(sd) == list(a.state_dict())


def test_load_bumps_pack_key():
    """A load changes the parameters' versions, so the next kernel call repacks (packed_weights)."""
    torch.manual_seed(1)
    a = TransformerActorCritic()
    before = tuple(p._version for p in a.parameters())
    torch.manual_seed(2)
    load_checkpoint(a, TransformerActorCritic().state_dict())
    assert tuple(p._version for p in a.parameters()) != before


@pytest.mark.parametrize("kind,params", [("actor2", 551747), ("flat640", 616003)])
def test_legacy_architectures(kind, params):
    sd = _legacy(kind)
    arch, f = describe(sd)
    assert arch == kind and f["params"] == params
    torch.manual_seed(4)
    pol = TransformerActorCritic()
    ref = {k: v.clone() for k, v in pol.state_dict().items()}
    with pytest.raises(RuntimeError):  # the reference's own load (test_visualize.py:22) fails too
        load_checkpoint(pol, sd, strict=True)
    for k, v in pol.state_dict().items():  # a failed strict load leaves the policy untouched
        assert torch.equal(v, ref[k]), k
    rep = load_checkpoint(pol, sd, strict=False)
    assert not rep.complete and rep.arch == kind
    assert all(k.startswith("actor_net.transformer.layers.1.") for k in rep.unexpected)
    assert len(rep.unexpected) == 12
    if kind == "flat640":
        assert sorted(rep.missing) == ["actor_net.pos_embedding", "critic_net.pos_embedding"]
        assert sorted(k for k, _, _ in rep.mismatched) == ["actor_head.0.weight", "critic_head.0.weight"]
    else:
        assert not rep.missing and not rep.mismatched
    own = pol.state_dict()
    for k in rep.loaded:
        assert torch.equal(own[k], sd[k]), k
    for k, _, _ in rep.mismatched:
        assert torch.equal(own[k], ref[k]), k


def test_not_a_state_dict(tmp_path):
    path = str(tmp_path / "x.pth")
    torch.save({"a": 1}, path)
    with pytest.raises(ValueError):
        read_checkpoint(path)
    with pytest.raises(FileNotFoundError):
        read_checkpoint(str(tmp_path / "missing.pth"))


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference checkpoints not present (GPU box)")
def test_reference_saved_models_are_recognised():
    """The four files shipped with the reference (read with weights_only=True): SURVEY.md §2."""
    seen = {}
    for path in sorted(glob.glob(os.path.join(REF_MODELS, "*", "best_model.pth"))):
        arch, f = describe(read_checkpoint(path))
        seen.setdefault(arch, []).append(f["params"])
    assert seen == {"flat640": [616003, 616003], "actor2": [551747, 551747]}


@pytest.mark.gpu
def test_loaded_checkpoint_drives_the_kernels(tmp_path):
    """A policy that ran the fused forward, then loads another policy's file, repacks on its next
    call: its outputs equal the saving policy's bitwise (same packed weights, same kernel)."""
    torch.manual_seed(11)
    a = TransformerActorCritic().cuda()
    torch.manual_seed(12)
    b = TransformerActorCritic().cuda()
    x = torch.randn(256, 5, 14, device="cuda")
    x[:7, :3] = 0.0  # padded rows
    acts = torch.randint(0, 2, (256,), device="cuda")
    before = b.fused_forward(x, actions=acts)[1].clone()
    path = str(tmp_path / "final_model.pth")
    save_checkpoint(a, path)
    load_checkpoint(b, path)
    _, lp_b, v_b, _, _ = b.fused_forward(x, actions=acts)
    _, lp_a, v_a, _, _ = a.fused_forward(x, actions=acts)
    assert not torch.equal(before, lp_b)
    assert torch.equal(lp_a, lp_b) and torch.equal(v_a, v_b)
